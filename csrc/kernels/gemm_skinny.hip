// Weight-streaming skinny GEMM for decode-sized batches (SURVEY §2.7 N1c/N1h/
// N1i/N1j/N1k at M = batch <= 64 per row tile):
//
//   C[M, N] = A[M, K] · W[N, K]^T (+ bias[N])          bf16 in, fp32 acc
//
// Regime: every weight byte is read exactly once per step, so the kernel is
// HBM-bound on W (e.g. Qwen2-7B gate_up: 271 MB per layer).  Design (cdna
// guide §5 "GEMV / M <= 16 decode weights" row, extended to M <= 64):
//   * no LDS staging — both MFMA operands are K-contiguous rows, so A and W
//     fragments load straight into v_mfma_f32_16x16x32_bf16 operands;
//   * full-line weight reads: per 64-k step lane group h4 owns k = 16*h4 ..
//     16*h4+15 (two adjacent 16-B loads), i.e. a k-permutation applied to both
//     operands (the dot product is order-free), so the four lane groups of a
//     row consume one whole 128-B line in the same step — with the natural
//     8-k-per-group layout each line would be fetched in two halves on two
//     steps, and with nontemporal loads that doubles HBM traffic;
//   * W streamed nontemporal (read once); A stays L2-resident, shared by all
//     workgroups;
//   * a workgroup owns NT output columns x 16*MT rows; its 4 waves split K into
//     quarters (intra-WG split-K) so N = 3584 still yields >= 224 workgroups;
//     a 2-deep software pipeline keeps two 64-k steps of loads in flight; the
//     4 partial tiles are summed through LDS (+ optional bias) and written once.
#include "common.h"

using namespace grag;

namespace {

template <int MT, int NT>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const bf16* __restrict__ A, int lda,
                                                          const bf16* __restrict__ W, int ldw,
                                                          const bf16* __restrict__ bias, bf16* __restrict__ C,
                                                          int ldc, int M, int N, int K) {
  constexpr int NN = NT / 16;
  __shared__ __attribute__((aligned(16))) float red[4][MT * 16][NT + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h4 = lane >> 4, li = lane & 15;
  const int n0 = blockIdx.x * NT;
  const int m0 = blockIdx.y * (MT * 16);
  const int kq = ((K / 64 + 3) / 4) * 64;  // K quarter per wave, multiple of 64
  const int kb = wave * kq;
  const int ke = min(K, kb + kq);

  const bf16* ap[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int row = m0 + mt * 16 + li;
    row = row < M ? row : M - 1;
    ap[mt] = A + (size_t)row * lda + 16 * h4;
  }
  const bf16* wp[NN];
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    int col = n0 + nt * 16 + li;
    col = col < N ? col : N - 1;
    wp[nt] = W + (size_t)col * ldw + 16 * h4;
  }
  f32x4_t acc[MT][NN];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#define LOAD_STEP(aa, ww, kk)                                                                  \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                          \
    aa[mt][0] = *reinterpret_cast<const bf16x8_t*>(ap[mt] + (kk));                             \
    aa[mt][1] = *reinterpret_cast<const bf16x8_t*>(ap[mt] + (kk) + 8);                         \
  }                                                                                            \
  _Pragma("unroll") for (int nt = 0; nt < NN; ++nt) {                                          \
    ww[nt][0] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(wp[nt] + (kk)));  \
    ww[nt][1] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(wp[nt] + (kk) + 8)); \
  }
#define MMA_STEP(aa, ww)                                                                       \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                            \
  _Pragma("unroll") for (int nt = 0; nt < NN; ++nt) {                                          \
    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aa[mt][0], ww[nt][0], acc[mt][nt], 0, 0, 0); \
    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aa[mt][1], ww[nt][1], acc[mt][nt], 0, 0, 0); \
  }

  if (kb < ke) {
    bf16x8_t a0[MT][2], w0[NN][2], a1[MT][2], w1[NN][2];
    LOAD_STEP(a0, w0, kb)
    int k = kb;
    for (; k + 128 <= ke; k += 128) {
      LOAD_STEP(a1, w1, k + 64)
      MMA_STEP(a0, w0)
      if (k + 128 < ke) {
        LOAD_STEP(a0, w0, k + 128)
      }
      MMA_STEP(a1, w1)
    }
    if (k < ke) {
      MMA_STEP(a0, w0)
    }
  }
#undef LOAD_STEP
#undef MMA_STEP
  // C tile layout: row = 16*mt + 4*h4 + r, col = 16*nt + li
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NN; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][16 * mt + 4 * h4 + r][16 * nt + li] = acc[mt][nt][r];
  __syncthreads();
  for (int e = threadIdx.x; e < MT * 16 * NT; e += 256) {
    const int row = e / NT, col = e % NT;
    const int gm = m0 + row, gn = n0 + col;
    if (gm < M && gn < N) {
      float v = red[0][row][col] + red[1][row][col] + red[2][row][col] + red[3][row][col];
      if (bias) v += (float)bias[gn];
      C[(size_t)gm * ldc + gn] = f2bf(v);
    }
  }
}

template <int MT>
int launch_mt(const bf16* A, int lda, const bf16* W, int ldw, const bf16* bias, bf16* C, int ldc, int M, int N,
              int K, int nt, hipStream_t stream) {
  const int mtiles = (M + MT * 16 - 1) / (MT * 16);
  if (nt == 64) {
    dim3 g((N + 63) / 64, mtiles);
    gemm_skinny_kernel<MT, 64><<<g, 256, 0, stream>>>(A, lda, W, ldw, bias, C, ldc, M, N, K);
  } else if (nt == 32) {
    dim3 g((N + 31) / 32, mtiles);
    gemm_skinny_kernel<MT, 32><<<g, 256, 0, stream>>>(A, lda, W, ldw, bias, C, ldc, M, N, K);
  } else {
    dim3 g((N + 15) / 16, mtiles);
    gemm_skinny_kernel<MT, 16><<<g, 256, 0, stream>>>(A, lda, W, ldw, bias, C, ldc, M, N, K);
  }
  return (int)hipGetLastError();
}

}  // namespace

// nt: output columns per workgroup (16/32/64); 0 = auto.
GRAG_API int grag_gemm_skinny(const void* A, const void* W, const void* bias, void* C, int lda, int ldw,
                              int ldc, int M, int N, int K, int nt, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 64 != 0 || lda % 8 != 0 || ldw % 8 != 0) return (int)hipErrorInvalidValue;
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const int mtiles = (M + mt * 16 - 1) / (mt * 16);
  if (nt == 0) {
    nt = 16;
    const int maxnt = mt == 4 ? 32 : 64;  // keep VGPRs (and occupancy) in check at M > 32
    if (maxnt >= 64 && (long)(N / 64) * mtiles >= 512) nt = 64;
    else if ((long)(N / 32) * mtiles >= 512) nt = 32;
  }
  const bf16* a = (const bf16*)A;
  const bf16* w = (const bf16*)W;
  const bf16* b = (const bf16*)bias;
  bf16* c = (bf16*)C;
  if (mt == 1) return launch_mt<1>(a, lda, w, ldw, b, c, ldc, M, N, K, nt, stream);
  if (mt == 2) return launch_mt<2>(a, lda, w, ldw, b, c, ldc, M, N, K, nt, stream);
  return launch_mt<4>(a, lda, w, ldw, b, c, ldc, M, N, K, nt, stream);
}
