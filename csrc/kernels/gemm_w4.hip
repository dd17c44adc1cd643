// W4A16 decode GEMM at the reference's precision (AWQ: 4-bit weights, group-128 scales and zero points,
// 16-bit activations; the reference serves Qwen2.5-Coder-7B-Instruct-AWQ, helm/values.yaml:67;
// SURVEY §2.7 N1c/N1h/N1i/N1j):
//
//   D[M, N] = A[M, K] · Wq[N, K]^T,   Wq[n, k] = (q[n, k] - z[n, k/128]) * s[n, k/128]
//
// Same skeleton as gemm_decode.hip (W streamed HBM -> VGPRs by counted inline-asm loads, D+1-slot ring;
// A through an LDS-DMA ring shared by the workgroup's waves; one raw barrier per 64-deep K-step), with the
// weights a quarter of the bytes:
//   * packed layout (ops/quant.py pack_w4): per 32-row block and K-step, 64 lanes x 16 B — exactly the
//     MFMA fragments a wave needs, so one global_load_dwordx4 per lane per K-step brings both of its
//     16-row tiles' k-halves (16 nibbles per tile row) and the 1-KiB wave load is fully contiguous;
//   * dequantised in registers: nibbles spread to bytes (2 ALU ops per 8 values), v_cvt_f32_ubyte per
//     value, one fma with the row's (s, -z*s) of the group, v_cvt_pk_bf16_f32 — the scale is per W row,
//     and a lane's whole fragment is one row, so (s, -z*s) are two scalars per lane per tile per group;
//   * (s, -z*s) as float2 [rows][K/128], loaded per K-step (8 B per lane per tile, L2-resident);
//   * rows are stored in the order the waves consume them; for the SwiGLU gate/up weight each 32-row block
//     is [16 gate rows | the 16 matching up rows] so silu(g)*u forms in registers (EPI_SILU).
#include "common.h"

// Diagnostic builds only (scripts/dev/w4_diag.py, never the shipped library): GRAG_W4_DIAG bit 0 drains
// every load before each step's barrier (no loads in flight across compute), bit 1 pads the workgroup's LDS
// to 160 KB (one workgroup per CU), bit 2 loads the weights with plain (compiler-visible) loads instead of
// the inline-asm ring, bit 3 checks every fragment against global memory, bit 4 pads wait states between
// the dequant and the MFMAs.
#ifndef GRAG_W4_DIAG
#define GRAG_W4_DIAG 0
#endif

using namespace grag;

GRAG_API int grag_splitk_reduce(const void* ws, const void* bias, void* C, int ldc, int M, int N, int S, int epi,
                                int act, hipStream_t stream);

namespace {

enum { EPI_STORE = 0, EPI_SILU = 1, EPI_PARTIAL = 2 };
enum { ACT_NONE = 0, ACT_GELU = 1, ACT_GELU_TANH = 3 };
constexpr int kDepth = 4;   // K-steps issued ahead (ring of kDepth + 1 slots)

constexpr int kGroup = 128; // quantisation group along K

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_erf_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (2.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * u)));
}
template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if constexpr (ACT == ACT_GELU) return gelu_erf_f(x);
  else if constexpr (ACT == ACT_GELU_TANH) return gelu_tanh_f(x);
  else return x;
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// LDS-DMA piece through the compiler builtin (hipcc owns M0 and its hazards)
__device__ __forceinline__ void glds16(const void* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)lds_dst, 16, 0, 0);
}

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// one K-step of this lane's packed weights (16 B) and the (s, -z s) of its two rows for the step's group;
// inline asm so hipcc's waitcnt pass does not drain the ring beside the LDS-DMA (guide §5 trap (b)); the
// registers are consumed only after wait_w, which names them
__device__ __forceinline__ void ldw(u32x4_t& q, f32x2_t& sz0, f32x2_t& sz1, const void* pq, const void* p0,
                                    const void* p1) {
  if constexpr ((GRAG_W4_DIAG & 4) != 0) {  // diagnostic: plain compiler-visible loads (waits placed by hipcc)
    q = *reinterpret_cast<const u32x4_t*>(pq);
    sz0 = *reinterpret_cast<const f32x2_t*>(p0);
    sz1 = *reinterpret_cast<const f32x2_t*>(p1);
    return;
  }
  asm volatile(
      "global_load_dwordx4 %0, %3, off\n\t"
      "global_load_dwordx2 %1, %4, off\n\t"
      "global_load_dwordx2 %2, %5, off"
      : "=&v"(q), "=&v"(sz0), "=&v"(sz1)
      : "v"(pq), "v"(p0), "v"(p1)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_w(u32x4_t& q, f32x2_t& a, f32x2_t& b) {
  if constexpr ((GRAG_W4_DIAG & 4) != 0) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    return;
  }
  asm volatile("s_waitcnt vmcnt(%3)" : "+v"(q), "+v"(a), "+v"(b) : "n"(N) : "memory");
}

__device__ __forceinline__ void bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 8 nibbles (k = j at bits 4j) -> bf16x8 of (q - z) * s
__device__ __forceinline__ bf16x8_t dequant8(unsigned d, float s, float zs) {
  const unsigned lo = d & 0x0F0F0F0Fu, hi = (d >> 4) & 0x0F0F0F0Fu;
  float v[8];
  // (float)((x >> 8b) & 0xFF) selects v_cvt_f32_ubyte{b}
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    v[2 * b] = (float)((lo >> (8 * b)) & 0xFFu);
    v[2 * b + 1] = (float)((hi >> (8 * b)) & 0xFFu);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = __builtin_fmaf(v[j], s, zs);
  return pack8(v);
}

#if (GRAG_W4_DIAG & 8) != 0
// diagnostic: [0] A-fragment mismatches (LDS vs global), [1] W-word mismatches (ring vs global),
// [2..5] first A mismatch (step, mt, lane, k-half), [6..8] first W mismatch (step, lane, word)
__device__ unsigned g_w4_diag[16];
#endif

struct WArgs {
  const bf16* A;
  const unsigned* Wq;  // [N/32][K/64][64][4] dwords
  const float* sz;     // [N][K/128] x (s, -z s)
  const bf16* bias;    // in consumption row order
  void* C;
  int lda, ldc;
  int M, N, K;
  int ksplit, kt_split;
};

template <int EPI, int ACT, int MT, int D, int NWV>
__global__ __launch_bounds__(64 * NWV) void gemm_w4_kernel(WArgs p) {
  constexpr int NST = D + 1;
  constexpr int ABYTES = MT * 16 * 128;
  constexpr int GA = (MT * 2) / NWV;
  constexpr int GW = 3;  // W dwordx4 + two (s, -z s) dwordx2 per lane per K-step
  static_assert((MT * 2) % NWV == 0, "A pieces must split evenly over the waves");
  static_assert(NST * ABYTES <= 160 * 1024, "LDS ring exceeds 160 KB");
  __shared__ __attribute__((aligned(16))) char smem[(GRAG_W4_DIAG & 2) ? 160 * 1024 : NST * ABYTES];

  const int tid = threadIdx.x;
  const int L = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = L & 15, h4 = L >> 4;
  const int bidx = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bidx / p.ksplit, split = bidx % p.ksplit;
  const int blk = tile * NWV + w;  // this wave's 32-row block (consumption order)
  const int ks = p.K >> 6;
  const int G = p.K / kGroup;
  const int kb = split * p.kt_split;
  const int ke = min(ks, kb + p.kt_split);
  const int nsteps = ke - kb;

  const char* wq = reinterpret_cast<const char*>(p.Wq) + ((size_t)blk * ks + kb) * 1024 + L * 16;
  const int r0 = blk * 32 + li, r1 = r0 + 16;
  const float* sz0 = p.sz + ((size_t)r0 * G) * 2;
  const float* sz1 = p.sz + ((size_t)r1 * G) * 2;

  const bf16* ap[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int q = w * GA + i;
    const int row = q * 8 + (L >> 3);
    const int c = (L & 7) ^ ((row >> 1) & 7);
    ap[i] = p.A + (size_t)min(row, p.M - 1) * p.lda + (size_t)kb * 64 + c * 8;
  }

  u32x4_t wv[NST];
  f32x2_t s0[NST], s1[NST];
  f32x4_t acc[MT][2];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt][0] = acc[mt][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // steps past the range re-read the first step's bytes (L2-resident) so every iteration issues the same ops
  auto issue = [&](int step, int slot) {
    const bool live = step < nsteps;
    const int st = live ? step : 0;
    const int g = ((kb + st) * 64) / kGroup;
#pragma unroll
    for (int i = 0; i < GA; ++i) glds16(ap[i] + st * 64, smem + slot * ABYTES + (w * GA + i) * 1024);
    ldw(wv[slot], s0[slot], s1[slot], wq + (size_t)st * 1024, sz0 + 2 * g, sz1 + 2 * g);
  };

  const int sw = (li >> 1) & 7;
  const int aoff0 = li * 128 + ((h4 ^ sw) << 4);
  const int aoff1 = li * 128 + (((4 + h4) ^ sw) << 4);
  auto compute = [&](int slot, int step) {
#if (GRAG_W4_DIAG & 8) != 0
    {  // every fragment this lane is about to use, against the same bytes read straight from global memory
      const char* Ad = smem + slot * ABYTES;
      for (int mt = 0; mt < MT; ++mt) {
        for (int hh = 0; hh < 2; ++hh) {
          const bf16x8_t got = *reinterpret_cast<const bf16x8_t*>(Ad + mt * 2048 + (hh ? aoff1 : aoff0));
          const int row = min(mt * 16 + li, p.M - 1);
          const bf16x8_t want = *reinterpret_cast<const bf16x8_t*>(p.A + (size_t)row * p.lda +
                                                                    (size_t)(kb + step) * 64 + (4 * hh + h4) * 8);
          if (__builtin_bit_cast(u32x4_t, got)[0] != __builtin_bit_cast(u32x4_t, want)[0] ||
              __builtin_bit_cast(u32x4_t, got)[3] != __builtin_bit_cast(u32x4_t, want)[3]) {
            if (atomicAdd(&g_w4_diag[0], 1u) == 0u) {
              g_w4_diag[2] = step; g_w4_diag[3] = mt; g_w4_diag[4] = L; g_w4_diag[5] = hh;
            }
          }
        }
      }
      const u32x4_t wwant = *reinterpret_cast<const u32x4_t*>(wq + (size_t)step * 1024);
      for (int e = 0; e < 4; ++e)
        if (wv[slot][e] != wwant[e]) {
          if (atomicAdd(&g_w4_diag[1], 1u) == 0u) { g_w4_diag[6] = step; g_w4_diag[7] = L; g_w4_diag[8] = e; }
        }
    }
#endif
    bf16x8_t w00 = dequant8(wv[slot][0], s0[slot][0], s0[slot][1]);
    bf16x8_t w01 = dequant8(wv[slot][1], s0[slot][0], s0[slot][1]);
    bf16x8_t w10 = dequant8(wv[slot][2], s1[slot][0], s1[slot][1]);
    bf16x8_t w11 = dequant8(wv[slot][3], s1[slot][0], s1[slot][1]);
#if (GRAG_W4_DIAG & 16) != 0
    // diagnostic: pin the dequantised fragments, then 16 wait states, before any MFMA reads them
    asm volatile("" : "+v"(w00), "+v"(w01), "+v"(w10), "+v"(w11));
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#endif
    const char* As = smem + slot * ABYTES;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(As + mt * 2048 + aoff0);
      const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(As + mt * 2048 + aoff1);
      acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w00, a0, acc[mt][0], 0, 0, 0);
      acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w01, a1, acc[mt][0], 0, 0, 0);
      acc[mt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w10, a0, acc[mt][1], 0, 0, 0);
      acc[mt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w11, a1, acc[mt][1], 0, 0, 0);
    }
  };

#pragma unroll
  for (int d = 0; d < D; ++d) issue(d, d);
  // A K-step's LDS slot is READ one barrier interval after the wait that retires its LDS-DMA, never in
  // the same interval (cdna_hip_programming.md §5 "Read a staged buffer one phase AFTER the wait that
  // retires it"): iteration t waits for step t + 1 and computes step t.  Round 2 waited for step t and
  // read it right after one barrier; that passed for some row tilings and builds and returned 1-25 %
  // wrong results for others (scripts/dev/w4_diag.py: draining every load before the barrier, plain
  // loads instead of the inline-asm register ring, one workgroup per CU and in-kernel data checks did not
  // explain it; adding wait states moved which tilings failed): the DMA's LDS write is not ordered for a
  // same-interval ds_read by the vmcnt + barrier alone.
  wait_w<(D - 1) * (GA + GW)>(wv[0], s0[0], s1[0]);
  bar();
  for (int t0 = 0; t0 < nsteps; t0 += NST) {
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      if constexpr ((GRAG_W4_DIAG & 1) != 0) wait_w<0>(wv[(u + 1) % NST], s0[(u + 1) % NST], s1[(u + 1) % NST]);
      // retire step t + 1 (steps t + 2 .. t + D - 1 stay in flight)
      wait_w<(D - 2) * (GA + GW)>(wv[(u + 1) % NST], s0[(u + 1) % NST], s1[(u + 1) % NST]);
      bar();
      issue(t0 + u + D, (u + D) % NST);  // slot of step t - 1: its readers passed this barrier
      if (t0 + u < nsteps) compute(u, t0 + u);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: acc[mt][nt][r] = D[row 32 blk + 16 nt + 4 h4 + r][A row 16 mt + li]
  if constexpr (EPI == EPI_SILU) {
    bf16* C = (bf16*)p.C;
    const int oc = blk * 16 + 4 * h4;
    if (2 * (blk * 16) >= p.N) return;
    float bg[4], bu[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bg[r] = p.bias ? (float)p.bias[blk * 32 + 4 * h4 + r] : 0.f;
      bu[r] = p.bias ? (float)p.bias[blk * 32 + 16 + 4 * h4 + r] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + li;
      if (m >= p.M) continue;
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bits(silu_f(acc[mt][0][r] + bg[r]) * (acc[mt][1][r] + bu[r]));
      *reinterpret_cast<bf16x4_t*>(C + (size_t)m * p.ldc + oc) = o;
    }
  } else {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = blk * 32 + nt * 16 + 4 * h4;
      if (n >= p.N) continue;
      float bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = (EPI == EPI_STORE && p.bias) ? (float)p.bias[n + r] : 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = mt * 16 + li;
        if (m >= p.M) continue;
        if constexpr (EPI == EPI_PARTIAL) {
          float* ws = (float*)p.C + ((size_t)split * p.M + m) * p.N + n;
          *reinterpret_cast<f32x4_t*>(ws) = acc[mt][nt];
        } else {
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bits(act_f<ACT>(acc[mt][nt][r] + bv[r]));
          *reinterpret_cast<bf16x4_t*>((bf16*)p.C + (size_t)m * p.ldc + n) = o;
        }
      }
    }
  }
}

template <int MT, int NWV>
int launch_v(const WArgs& a, int epi, int act, int nwg, hipStream_t s) {
#define GO(E, AC) gemm_w4_kernel<E, AC, MT, kDepth, NWV><<<nwg, 64 * NWV, 0, s>>>(a)
  if (epi == EPI_PARTIAL) GO(EPI_PARTIAL, ACT_NONE);
  else if (epi == EPI_SILU) GO(EPI_SILU, ACT_NONE);
  else if (act == ACT_GELU) GO(EPI_STORE, ACT_GELU);
  else if (act == ACT_GELU_TANH) GO(EPI_STORE, ACT_GELU_TANH);
  else GO(EPI_STORE, ACT_NONE);
#undef GO
  return (int)hipGetLastError();
}

}  // namespace

// Variants: (mt, nwv) = (4, 4), (8, 4), (12, 4), (16, 4).  Round 2 shipped (16, 4) only: the others
// returned 1-15 % wrong results on dense operands.  Root cause (scripts/dev/w4_diag.py, GPU runs in
// profiles/w4_diag_r3.txt): each K-step's A slot was read in the same barrier interval as the vmcnt wait
// that retired its LDS-DMA; the ring now retires step t + 1 one interval before step t + 1 is read.
GRAG_API int grag_gemm_w4_has(int mt, int nwv) { return nwv == 4 && (mt == 4 || mt == 8 || mt == 12 || mt == 16); }

// y = epilogue(x @ dequant(wq)^T) for M <= 16 * mt rows.  wq / sz from ops/quant.py pack_w4 (rows in
// consumption order: natural, or gate/up 16-row pairs for epi 1 = silu*mul -> out [M, N/2]).  ksplit > 1
// (store epilogue only): fp32 planes into ws, then grag_splitk_reduce.  Requirements (checked):
// K % 256 == 0, N % (32 * nwv) == 0, lda % 8 == 0, ldc % 4 == 0.
GRAG_API int grag_gemm_w4(const void* A, const void* Wq, const void* sz, const void* bias, void* C, int lda,
                          int ldc, int M, int N, int K, int epi, int act, int mt, int nwv, int ksplit, void* ws,
                          hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (!grag_gemm_w4_has(mt, nwv) || M > 16 * mt) return (int)hipErrorInvalidValue;
  if (K % 256 != 0 || N % (32 * nwv) != 0 || lda % 8 != 0 || ldc % 4 != 0) return (int)hipErrorInvalidValue;
  if (epi != EPI_STORE && epi != EPI_SILU) return (int)hipErrorInvalidValue;
  if (act != ACT_NONE && act != ACT_GELU && act != ACT_GELU_TANH) return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU && (act != ACT_NONE || ksplit > 1)) return (int)hipErrorInvalidValue;
  const int kt = K / 64;
  if (ksplit < 1) ksplit = 1;
  const int kts = (kt + ksplit - 1) / ksplit;  // any split length: steps past a split's end are not computed
  ksplit = (kt + kts - 1) / kts;
  if (ksplit > 1 && ws == nullptr) return (int)hipErrorInvalidValue;
  WArgs a;
  a.A = (const bf16*)A;
  a.Wq = (const unsigned*)Wq;
  a.sz = (const float*)sz;
  a.bias = ksplit > 1 ? nullptr : (const bf16*)bias;
  a.C = ksplit > 1 ? ws : C;
  a.lda = lda; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K;
  a.ksplit = ksplit;
  a.kt_split = kts;
  const int nwg = (N / (32 * nwv)) * ksplit;
  const int e = ksplit > 1 ? EPI_PARTIAL : epi;
  int err;
  if (mt == 4) err = launch_v<4, 4>(a, e, act, nwg, stream);
  else if (mt == 8) err = launch_v<8, 4>(a, e, act, nwg, stream);
  else if (mt == 12) err = launch_v<12, 4>(a, e, act, nwg, stream);
  else err = launch_v<16, 4>(a, e, act, nwg, stream);
  if (err || ksplit == 1) return err;
  return grag_splitk_reduce(ws, bias, C, ldc, M, N, ksplit, epi, act, stream);
}
