// Weight-streaming stream-K GEMM for decode-batch shapes (SURVEY §2.7 N1c/N1h/
// N1i/N1j/N1k and N2b/N2d at small M):
//
//   C[M, N] = A[M, K] · W[N, K]^T (+ bias[N])          bf16 in, fp32 acc
//
// Regime: M = decode batch (17..128 per row tile: MT = 2, 4 or 8 sixteen-row
// MFMA tiles, so a batch of up to 128 rows streams the weights exactly once).  W (e.g. Qwen2-7B down_proj,
// 136 MB) is read once from HBM per step; A (M x K) is re-read from L2 by every
// column tile, so the A:W L2 traffic ratio is M / BN.
//
// Structure (cdna guide §5 "Projection GEMM at M = 256": x through LDS in full
// 128-B lines filled by LDS-DMA; "glds vs register staging"):
//   * one workgroup = 4 waves = BN output columns x 16*MT rows; every
//     workgroup walks an equal share of the flattened (tile, k-step) space
//     (stream-K: G = number of resident workgroups, so every CU streams the
//     same number of weight bytes whatever N / BN is);
//   * every 64-k step, the W tile (BN rows x 128 B) and the A tile (16*MT rows
//     x 128 B) arrive by global_load_lds_dwordx4 — one wave instruction moves
//     8 whole 128-B lines, so HBM sees only full-line requests — into an
//     NST-deep LDS ring; the k-chunk of each row is XOR-swizzled on the SOURCE
//     address (LDS stays lane-linear, rule 21) so the ds_read_b128 fragment
//     reads of 16 consecutive rows hit 16 distinct bank slots;
//   * counted `s_waitcnt vmcnt(N)` + raw s_barrier keep NST-2 stages in flight
//     across the barrier (a __syncthreads() would drain them);
//   * wave w owns columns [w*BN/4, (w+1)*BN/4) and all 16*MT rows, so A is read
//     from LDS by all four waves but fetched from L2 once per workgroup;
//   * a tile whose k range lies wholly inside one workgroup's share is written
//     directly (bias + bf16); a tile split across workgroups is combined
//     IN-LAUNCH (§5 item 2): each part writes an fp32 slab slot, drains, one
//     lane releases (agent fence) and takes a relaxed agent-scope ticket; the
//     part that draws the last ticket acquires, sums the slots + bias -> bf16
//     and resets the ticket word (the counter array is zero-initialised at
//     allocation, so graph replays need no memset).
// Measured: the library GEMMs (TunableOp-selected hipBLASLt) win at M >= 16-32
// on most Qwen2-7B shapes; ops/linear.py picks per shape from a table timed
// inside hipGraphs (tuning/gemm_dispatch_gfx950.json).
#include "common.h"

#include <algorithm>

using namespace grag;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

namespace {

__device__ __forceinline__ void glds16(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)l, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// byte offset of (row, logical 16-B chunk c) inside a [rows][128 B] swizzled image
__device__ __forceinline__ int swz(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }

template <int MT, int BN, int NST>
__global__ __launch_bounds__(256) void gemm_stream_kernel(const bf16* __restrict__ A, int lda,
                                                          const bf16* __restrict__ W, int ldw,
                                                          const bf16* __restrict__ bias, bf16* __restrict__ C,
                                                          int ldc, int M, int N, int K, int ntm, int pmax,
                                                          float* __restrict__ slab, unsigned* __restrict__ counters) {
  constexpr int AROWS = MT * 16;
  constexpr int WBYTES = BN * 128;
  constexpr int STAGE = (BN + AROWS) * 128;
  constexpr int NN = BN / 64;     // 16-column tiles per wave
  constexpr int GW = BN / 32;     // W glds per wave per stage
  constexpr int GA = MT / 2;      // A glds per wave per stage
  constexpr int GPS = GW + GA;
  constexpr int TILE = AROWS * BN;
  static_assert(MT == 2 || MT == 4 || MT == 8, "MT");
  static_assert(BN == 64 || BN == 128 || BN == 256, "BN");
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE + 16];
  unsigned* flag = reinterpret_cast<unsigned*>(smem + NST * STAGE);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h4 = lane >> 4, li = lane & 15;
  const int G = gridDim.x;
  const int b = xcd_remap(blockIdx.x, G);

  // ---- stream-K work split: (tile, k-step) iterations dealt in equal contiguous ranges
  // (32-bit: every planned shape has < 2^31 / G iterations; the launcher checks)
  const int ks = (K + 63) >> 6;
  const int ntn = (N + BN - 1) / BN;
  const int total = ntn * ntm * ks;
  const int it0 = (int)((long)b * total / G), it1 = (int)((long)(b + 1) * total / G);
  const int n = it1 - it0;
  const bool ktail = (K & 63) != 0;
  auto block_of = [&](int x) -> int { return (int)(((long)(x + 1) * G + total - 1) / total) - 1; };
  // ---- per-lane LDS-DMA geometry: lane L of instruction i fills row r0 + L/8, physical chunk L%8
  const int lr = lane >> 3, pc = lane & 7;
  int wrow[GW], wc[GW], arow[GA], ac[GA];
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    wrow[i] = (wave * GW + i) * 8 + lr;
    wc[i] = (pc ^ ((wrow[i] >> 1) & 7)) * 8;
  }
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    arow[i] = (wave * GA + i) * 8 + lr;
    ac[i] = (pc ^ ((arow[i] >> 1) & 7)) * 8;
  }

  // issue cursor: (tile, k-step) of the next stage to load, advanced incrementally
  int i_tile = it0 / ks, i_k = it0 % ks;
  auto issue = [&](int buf) {
    const int n0 = (i_tile / ntm) * BN, m0 = (i_tile % ntm) * AROWS;
    const int k0 = i_k * 64;
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < GW; ++i) {
      int gn = n0 + wrow[i];
      gn = gn < N ? gn : N - 1;
      // chunks past K (only in a K % 64 tail step) re-read the row start; their products are zeroed
      const int kc = (!ktail || k0 + wc[i] + 8 <= K) ? k0 + wc[i] : 0;
      glds16(W + (size_t)gn * ldw + kc, base + (wave * GW + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      int gm = m0 + arow[i];
      gm = gm < M ? gm : M - 1;
      const int kc = (!ktail || k0 + ac[i] + 8 <= K) ? k0 + ac[i] : 0;
      glds16(A + (size_t)gm * lda + kc, base + WBYTES + (wave * GA + i) * 1024);
    }
    if (++i_k == ks) { i_k = 0; ++i_tile; }
  };

  f32x4_t acc[MT][NN];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf, int kvalid) {  // kvalid: valid k in this step (64 except a tail)
    const char* Ws = smem + buf * STAGE;
    const char* As = Ws + WBYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + h4;
      bf16x8_t af[MT], wf[NN];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) af[mt] = *reinterpret_cast<const bf16x8_t*>(As + swz(mt * 16 + li, c));
#pragma unroll
      for (int nt = 0; nt < NN; ++nt)
        wf[nt] = *reinterpret_cast<const bf16x8_t*>(Ws + swz((wave * NN + nt) * 16 + li, c));
      if (kvalid < 64 && c * 8 + 8 > kvalid) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) af[mt] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NN; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], wf[nt], acc[mt][nt], 0, 0, 0);
    }
  };

  // C/acc map: row = 16*mt + 4*h4 + r, col = 16*(wave*NN + nt) + li
  auto flush = [&](int tile, int kbeg, int kend) {
    const int n0 = (tile / ntm) * BN, m0 = (tile % ntm) * AROWS;
    if (kbeg == 0 && kend == ks) {  // this workgroup owns the whole tile: write it directly
#pragma unroll
      for (int nt = 0; nt < NN; ++nt) {
        const int gn = n0 + (wave * NN + nt) * 16 + li;
        if (gn >= N) continue;
        const float bv = bias ? (float)bias[gn] : 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int gm = m0 + mt * 16 + 4 * h4 + r;
            if (gm < M) C[(size_t)gm * ldc + gn] = f2bf(acc[mt][nt][r] + bv);
          }
      }
      return;
    }
    // partial tile: slab slot = position of this workgroup among the tile's contributors
    const int tb = tile * ks;
    const int bfirst = block_of(tb), blast = block_of(tb + ks - 1);
    const int ncontrib = blast - bfirst + 1;
    float* my = slab + ((size_t)tile * pmax + (b - bfirst)) * TILE;
#pragma unroll
    for (int nt = 0; nt < NN; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          my[(mt * 16 + 4 * h4 + r) * BN + (wave * NN + nt) * 16 + li] = acc[mt][nt][r];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned tk = __hip_atomic_fetch_add(&counters[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tk >= (unsigned)ncontrib) report_index_error(ERR_TICKET, tk);  // stale / shared ticket word
      const unsigned last = tk == (unsigned)(ncontrib - 1) ? 1u : 0u;
      if (last) {
        __hip_atomic_store(&counters[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      flag[0] = last;
    }
    __syncthreads();
    if (flag[0] == 0u) return;
    // last arriver: sum the contributors' slabs (+bias) -> bf16, 4 consecutive columns per thread
    const float* base = slab + (size_t)tile * pmax * TILE;
    for (int e = threadIdx.x; e < TILE / 4; e += 256) {
      const int row = e / (BN / 4), c4 = (e % (BN / 4)) * 4;
      const int gm = m0 + row, gn = n0 + c4;
      if (gm >= M || gn >= N) continue;
      float4 s = *reinterpret_cast<const float4*>(base + row * BN + c4);
      int p = 1;
      for (; p + 2 <= ncontrib; p += 2) {
        const float4 t0 = *reinterpret_cast<const float4*>(base + (size_t)p * TILE + row * BN + c4);
        const float4 t1 = *reinterpret_cast<const float4*>(base + (size_t)(p + 1) * TILE + row * BN + c4);
        s.x += t0.x + t1.x; s.y += t0.y + t1.y; s.z += t0.z + t1.z; s.w += t0.w + t1.w;
      }
      if (p < ncontrib) {
        const float4 t0 = *reinterpret_cast<const float4*>(base + (size_t)p * TILE + row * BN + c4);
        s.x += t0.x; s.y += t0.y; s.z += t0.z; s.w += t0.w;
      }
      float v[4] = {s.x, s.y, s.z, s.w};
      if (bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += (float)bias[gn + j];
      }
      bf16x4_t o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bits(v[j]);
      *reinterpret_cast<bf16x4_t*>(C + (size_t)gm * ldc + gn) = o;
    }
  };

  // ---- NST-deep LDS-DMA ring over this workgroup's iterations (segments of several tiles)
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < n) issue(s);
  int c_tile = it0 / ks, c_k = it0 % ks, seg_k0 = c_k;
  int buf = 0, ibuf = NST - 1;
  for (int t = 0; t < n; ++t) {
    if (t + NST - 2 < n) wait_vm<GPS * (NST - 2)>();
    else wait_vm<0>();
    lds_barrier();  // stage t landed for every wave; every wave is done reading stage t-1
    if (t + NST - 1 < n) issue(ibuf);
    ibuf = ibuf == NST - 1 ? 0 : ibuf + 1;
    compute(buf, (ktail && c_k == ks - 1) ? (K & 63) : 64);
    buf = buf == NST - 1 ? 0 : buf + 1;
    if (c_k == ks - 1 || t == n - 1) {
      flush(c_tile, seg_k0, c_k + 1);
      seg_k0 = 0;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NN; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    if (++c_k == ks) { c_k = 0; ++c_tile; }
  }
}

template <int MT, int BN, int NST>
int launch(const bf16* A, int lda, const bf16* W, int ldw, const bf16* bias, bf16* C, int ldc, int M, int N, int K,
           int G, int pmax, float* slab, unsigned* counters, hipStream_t stream) {
  const int ntm = (M + MT * 16 - 1) / (MT * 16);
  gemm_stream_kernel<MT, BN, NST><<<G, 256, 0, stream>>>(A, lda, W, ldw, bias, C, ldc, M, N, K, ntm, pmax, slab,
                                                         counters);
  return (int)hipGetLastError();
}

}  // namespace

// Plan helper: out4 = {mt, bn, grid, pmax} and the slab floats needed
// (out4[4]).  grid = workgroups of the stream-K split (one per CU by default:
// a 4x128 workgroup holds 96 KB of LDS ring); pmax = max workgroups sharing a
// tile (slab slots per tile).
GRAG_API int grag_gemm_stream_plan(int M, int N, int K, int ncu, int* out5) {
  const int mt = M <= 32 ? 2 : (M <= 64 ? 4 : 8);
  const int bn = 256;
  const int ntm = (M + mt * 16 - 1) / (mt * 16);
  const long ks = (K + 63) / 64;
  const long tiles = (long)((N + bn - 1) / bn) * ntm;
  const long total = tiles * ks;
  long G = ncu > 0 ? ncu : 256;
  if (total < G * 4) G = (total + 3) / 4;  // >= 4 k-steps per workgroup
  if (G < 1) G = 1;
  const long per = total / G;              // >= 4
  const int pmax = (int)((ks + per - 1) / per) + 1;
  out5[0] = mt;
  out5[1] = bn;
  out5[2] = (int)G;
  out5[3] = pmax;
  out5[4] = (int)std::min<long>(tiles * pmax * (long)(mt * 16) * bn, 0x7fffffffL);
  return 0;
}

// counters: >= tiles zero-initialised uint32 words (each reset by its tile's
// last arriver); slab: >= tiles * pmax * (16*mt) * bn fp32.
GRAG_API int grag_gemm_stream(const void* A, const void* W, const void* bias, void* C, int lda, int ldw, int ldc,
                              int M, int N, int K, int mt, int bn, int G, int pmax, void* slab, void* counters,
                              hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 16 != 0 || lda % 8 != 0 || ldw % 8 != 0 || ldc % 4 != 0 || N % 4 != 0) return (int)hipErrorInvalidValue;
  if (G < 1 || pmax < 2 || slab == nullptr || counters == nullptr) return (int)hipErrorInvalidValue;
  {  // the slab must hold every contributor of the most-split tile
    const int ntm = (M + mt * 16 - 1) / (mt * 16);
    const long ks = (K + 63) / 64, total = (long)((N + bn - 1) / bn) * ntm * ks;
    if (total >= (1L << 31) / G || total / G < 1 || (ks + total / G - 1) / (total / G) + 1 > pmax)
      return (int)hipErrorInvalidValue;
  }
  const bf16* a = (const bf16*)A;
  const bf16* w = (const bf16*)W;
  const bf16* b = (const bf16*)bias;
  bf16* c = (bf16*)C;
  float* sl = (float*)slab;
  unsigned* cnt = (unsigned*)counters;
#define GO(MT_, BN_, NST_) return launch<MT_, BN_, NST_>(a, lda, w, ldw, b, c, ldc, M, N, K, G, pmax, sl, cnt, stream)
  if (mt <= 2) {
    if (bn == 64) GO(2, 64, 6);
    if (bn == 128) GO(2, 128, 7);
    GO(2, 256, 4);
  }
  if (mt <= 4) {
    if (bn == 64) GO(4, 64, 4);
    if (bn == 128) GO(4, 128, 6);
    GO(4, 256, 3);
  }
  // 128-row tiles (decode batches 65..128): 24 / 32 / 48 KB per ring stage
  if (bn == 64) GO(8, 64, 6);
  if (bn == 128) GO(8, 128, 4);
  GO(8, 256, 3);
#undef GO
}

GRAG_ERR_UNIT(gemm_stream)
