// AWQ W4A16 checkpoint dequantisation (load time).
//
// The reference deploys Qwen/Qwen2.5-Coder-7B-Instruct-AWQ on vLLM
// (reference helm/values.yaml:67).  On MI355X the 7B model's
// bf16 weights are 15 GB of 288 GB HBM3E, so the engine serves AWQ
// checkpoints unquantised: every AutoAWQ "GEMM"-format linear
//   qweight int32 [K, N/8]   (8 x 4-bit, nibble i = column 8c + kOrder[i])
//   qzeros  int32 [K/G, N/8] (same packing)
//   scales  fp16  [K/G, N]
// is expanded once on the GPU into the torch Linear layout W[N, K] bf16,
//   W[n, k] = (q[k, n] - z[k/G, n]) * s[k/G, n]
// so every hot GEMM keeps its bf16 MFMA path.
//
// One block per 64(k) x 64(n) tile: 256 threads read the 64 x 8 packed words
// (coalesced along n), dequantise into an LDS tile stored n-major, then write
// 64 rows of 64 bf16 (128 B each) as 16 B per lane — the transpose happens in
// LDS, both HBM streams are contiguous.
#include "common.h"

using namespace grag;

namespace {
constexpr int kTile = 64;
constexpr int kThreads = 256;
constexpr int kPad = 8;  // bf16 elements of row padding (keeps 16 B row alignment, spreads banks)
// nibble i of a packed word holds column 8c + kOrder[i] (AutoAWQ pack order)
__constant__ int kOrder[8] = {0, 2, 4, 6, 1, 3, 5, 7};

__global__ __launch_bounds__(kThreads) void awq_dequant_kernel(const int32_t* __restrict__ qweight,
                                                               const int32_t* __restrict__ qzeros,
                                                               const __fp16* __restrict__ scales,
                                                               bf16* __restrict__ out, int K, int N, int G) {
  __shared__ bf16 tile[kTile][kTile + kPad];  // [n][k]
  const int n0 = blockIdx.x * kTile, k0 = blockIdx.y * kTile;
  const int NP = N >> 3;
  // load + dequantise: 64 k-rows x 8 packed words, 2 per thread
  for (int u = threadIdx.x; u < kTile * (kTile / 8); u += kThreads) {
    const int kr = u >> 3, c = u & 7;
    const int k = k0 + kr;
    const int pc = (n0 >> 3) + c;
    const uint32_t q = (uint32_t)qweight[(size_t)k * NP + pc];
    const int g = k / G;
    const uint32_t z = (uint32_t)qzeros[(size_t)g * NP + pc];
    const __fp16* srow = scales + (size_t)g * N + (pc << 3);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int col = kOrder[i];
      const float qv = (float)((q >> (4 * i)) & 0xF);
      const float zv = (float)((z >> (4 * i)) & 0xF);
      tile[c * 8 + col][kr] = f2bf((qv - zv) * (float)srow[col]);
    }
  }
  __syncthreads();
  // store: 64 n-rows x 8 chunks of 8 bf16 (16 B), 2 per thread
  for (int u = threadIdx.x; u < kTile * (kTile / 8); u += kThreads) {
    const int nr = u >> 3, ch = u & 7;
    *reinterpret_cast<bf16x8_t*>(out + (size_t)(n0 + nr) * K + k0 + ch * 8) =
        *reinterpret_cast<const bf16x8_t*>(&tile[nr][ch * 8]);
  }
}
}  // namespace

// Shapes are checked by the caller (ops/quant.py): K % 64 == 0, N % 64 == 0,
// G % 64 == 0 or 64 % G == 0 is not required (k / G per row), K % G == 0.
GRAG_API int grag_awq_dequant(const void* qweight, const void* qzeros, const void* scales, void* out, int K,
                              int N, int G, hipStream_t stream) {
  if (K % kTile || N % kTile || G <= 0 || K % G) return (int)hipErrorInvalidValue;
  dim3 grid(N / kTile, K / kTile);
  hipLaunchKernelGGL(awq_dequant_kernel, grid, dim3(kThreads), 0, stream, (const int32_t*)qweight,
                     (const int32_t*)qzeros, (const __fp16*)scales, (bf16*)out, K, N, G);
  return (int)hipGetLastError();
}
