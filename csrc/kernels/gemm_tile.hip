// Owned bf16 MFMA GEMM for the prefill / encoder / decode projections
// (SURVEY §2.7 N1c, N1h, N1i, N1j, N1k, N2b, N2d):
//
//   D[M, N] = A[M, K] · W[N, K]^T        bf16 in, fp32 accumulate
//
// with the epilogue fused into the kernel:
//   EPI_STORE   bf16 out = act(acc + bias)                (act: none / gelu-erf / gelu-tanh)
//   EPI_SILU    bf16 out[M, N/2] = silu(g + bg) * (u + bu) (gate/up rows interleaved in 32-row
//               blocks by ops/gemm.py: rows [64j, 64j+32) = gate j*32.., [64j+32, 64j+64) = up)
//   EPI_PARTIAL fp32 split-K slab ws[split][M][N] (reduced + epilogued by splitk_reduce_kernel)
//
// Geometry (cdna_hip_programming.md §5 "The 256² 8-phase template", re-derived
// for this schedule): 256x256 output tile, BK = 64, 8 waves (512 threads) as
// 2 (M) x 4 (N); wave (wr, wc) owns rows [128 wr, +128) x cols [64 wc, +64) as
// 2x2 quadrants of 64x32.  Each K-tile is computed in 4 phases, one quadrant
// per phase (16 v_mfma_f32_16x16x32_bf16 each):
//     P1 (0,0)  reads A(q0) 8x b128 + B(q0) 4x b128
//     P2 (0,1)  reads B(q1) 4x b128            (A(q0) kept in registers)
//     P3 (1,1)  reads A(q1) 8x b128            (B(q1) kept)
//     P4 (1,0)  no LDS reads                    (A(q1), B(q0) kept)
// LDS = 2 K-tile buffers x 4 slots of 16 KB (A q0, A q1, B q0, B q1), each slot
// = the 128 rows (both wave rows / all 4 wave columns) one quadrant needs.  A
// slot is refilled by LDS-DMA (global_load_lds_dwordx4, 2 per thread) as soon
// as its last reader phase has passed a barrier:
//     P1(t): A q1 of tile t+1   P2(t): A q0 of t+2   P3(t): B q0 of t+2   P4(t): B q1 of t+2
// so every slot is in flight for 4 phases and ONE counted `s_waitcnt
// vmcnt(8)` per phase (never 0 in the main loop) retires exactly the slot the
// phase after next reads.  Waves 4-7 run one barrier interval behind waves 0-3
// (stagger, MI355X_MICROARCH.md "Two waves per SIMD" item 9): on every SIMD one
// wave is in its LDS/DMA segment while its partner runs its MFMA cluster; the
// waits are placed one phase early for exactly that reason (a reader in the
// leading group must not outrun a DMA the lagging group issued).
// Rows are 128 B; chunks XOR-swizzled by (row >> 1) & 7 on the SOURCE address
// (LDS image lane-linear, rule 21) — conflict-free for the b128 lane groups.
// The MFMA is issued with the W fragment as operand A, so each lane ends with
// 4 consecutive output columns of one row: 8-byte bf16 / 16-byte fp32 stores.
#include "common.h"

using namespace grag;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

namespace {

constexpr int kSlot = 128 * 128;  // 128 rows x 64 bf16
constexpr int kBuf = 4 * kSlot;   // one K-tile: A q0, A q1, B q0, B q1
constexpr int kThreads = 512;

enum { EPI_STORE = 0, EPI_SILU = 1, EPI_PARTIAL = 2 };
enum { ACT_NONE = 0, ACT_GELU = 1, ACT_SILU = 2, ACT_GELU_TANH = 3 };

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_erf_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (2.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * u)));
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)(uint16_t)f2bits(lo) | ((uint32_t)(uint16_t)f2bits(hi) << 16);
}
template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if constexpr (ACT == ACT_GELU) return gelu_erf_f(x);
  else if constexpr (ACT == ACT_SILU) return silu_f(x);
  else if constexpr (ACT == ACT_GELU_TANH) return gelu_tanh_f(x);
  else return x;
}

__device__ __forceinline__ void glds16(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)l, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// raw barrier: never drains the LDS-DMA in flight (a __syncthreads() would emit vmcnt(0))
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct Args {
  const bf16* A;
  const bf16* W;
  const bf16* bias;
  void* C;
  int lda, ldw, ldc;
  int M, N, K;
  int tiles_m, tiles_n, ksplit, kt_split;  // K-tiles (of 64) per split
  int dp_tiles;    // blockIdx < dp_tiles: one whole tile (or K-split) each
  int sk_grid;     // blockIdx >= dp_tiles: stream-K workgroups over the remaining tiles
  float* slab;     // split-K partial planes, or 2 x 256 KB stream-K slots per SK workgroup
  unsigned* cnt;   // stream-K arrival tickets, one per SK tile (zero at rest)
  int a_bytes, w_bytes;  // buffer-resource extents of A / W (SCHED 1; both < 2 GB)
};

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// MFMA shape of a 64x32 quadrant (cdna guide §5.4 rule 28: the chip holds different clocks on the two
// bf16 shapes, so both are built at the same output tile per wave and the faster one by wall is the
// default; grag_gemm_tile_mfma() selects).  LDS bytes per quadrant are the same for both: every A / B
// element a wave needs is read from LDS once per K-tile either way.
//   MF 16: 4 x 2 tiles of v_mfma_f32_16x16x32_bf16, 2 k-steps of 32   (16 MFMAs per quadrant)
//   MF 32: 2 x 1 tiles of v_mfma_f32_32x32x16_bf16, 4 k-steps of 16   ( 8 MFMAs per quadrant)
// A quadrant's accumulators are 8 "chunks" of 4 consecutive output columns of one lane row:
//   MF 16: chunk c = (mt, nt) = (c >> 1, c & 1): row 16 mt + (L & 15), col 16 nt + 4 (L >> 4)
//   MF 32: chunk c = (mt, i)  = (c >> 2, c & 3): row 32 mt + (L & 31), col 8 i + 4 (L >> 5)
template <int MF>
struct Shape;
template <>
struct Shape<16> {
  typedef f32x4_t Acc[4][2];  // [mt][nt]
  typedef bf16x8_t FA[4][2];  // [mt][k-step]
  typedef bf16x8_t FB[2][2];  // [nt][k-step]
  static constexpr int kRows = 4, kCpr = 2;  // row slots per quadrant, chunks per row slot
};
template <>
struct Shape<32> {
  typedef f32x16_t Acc[2];    // [mt]
  typedef bf16x8_t FA[2][4];  // [mt][k-step]
  typedef bf16x8_t FB[4];     // [k-step]
  static constexpr int kRows = 2, kCpr = 4;
};

template <int MF>
__device__ __forceinline__ void mma_cluster(typename Shape<MF>::Acc& acc, const typename Shape<MF>::FA& a,
                                            const typename Shape<MF>::FB& b) {
  __builtin_amdgcn_s_setprio(1);
  if constexpr (MF == 16) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt][s], a[mt][s], acc[mt][nt], 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[s], a[mt][s], acc[mt], 0, 0, 0);
  }
  __builtin_amdgcn_s_setprio(0);
}

template <int MF>
__device__ __forceinline__ f32x4_t chunk_get(const typename Shape<MF>::Acc& acc, int c) {
  if constexpr (MF == 16) {
    return acc[c >> 1][c & 1];
  } else {
    const int mt = c >> 2, i = 4 * (c & 3);
    return f32x4_t{acc[mt][i], acc[mt][i + 1], acc[mt][i + 2], acc[mt][i + 3]};
  }
}
template <int MF>
__device__ __forceinline__ void chunk_set(typename Shape<MF>::Acc& acc, int c, const f32x4_t& v) {
  if constexpr (MF == 16) {
    acc[c >> 1][c & 1] = v;
  } else {
    const int mt = c >> 2, i = 4 * (c & 3);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[mt][i + r] = v[r];
  }
}
template <int MF>
__device__ __forceinline__ void acc_zero(typename Shape<MF>::Acc& acc) {
#pragma unroll
  for (int c = 0; c < 8; ++c) chunk_set<MF>(acc, c, f32x4_t{0.f, 0.f, 0.f, 0.f});
}

template <int EPI, int ACT, int MF, int SCHED>
__global__ __launch_bounds__(kThreads, 2) void gemm_tile_kernel(Args p) {
  using Acc = typename Shape<MF>::Acc;
  using FragA = typename Shape<MF>::FA;
  using FragB = typename Shape<MF>::FB;
  constexpr int kRows = Shape<MF>::kRows, kCpr = Shape<MF>::kCpr;
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];

  const int tid = threadIdx.x;
  const int L = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const bool lag = w >= 4;  // waves 4-7: one barrier interval behind
  const int ks = p.K >> 6;

  // group-M order over all output tiles: 8 row tiles x every column tile per band
  auto tile_coords = [&](int t, int& m0, int& n0) {
    constexpr int GM = 8;
    const int band = GM * p.tiles_n;
    const int first_m = (t / band) * GM;
    const int gsz = min(p.tiles_m - first_m, GM);
    m0 = (first_m + (t % band) % gsz) * 256;
    n0 = ((t % band) / gsz) * 256;
  };

  // ---- fragment reads, swizzle (row >> 1) & 7 (the slot row's low 4 bits are the lane's):
  //   MF 16: row (L & 15) of a 16-row group, logical chunk 4s + L/16 (k-step s of 32)
  //   MF 32: row (L & 31) of a 32-row group, logical chunk 2s + L/32 (k-step s of 16)
  const int cb = (L >> 4) ^ ((L >> 1) & 7);
  const int off0 = (L & 15) * 128 + cb * 16;
  const int off1 = (L & 15) * 128 + (cb ^ 4) * 16;
  auto off32 = [&](int s) { return (L & 31) * 128 + (((2 * s + (L >> 5)) ^ ((L >> 1) & 7)) * 16); };
  auto readA = [&](FragA& a, int q, int buf) {
    const char* base = smem + buf * kBuf + q * kSlot + wr * 64 * 128;
    if constexpr (MF == 16) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        a[mt][0] = *reinterpret_cast<const bf16x8_t*>(base + mt * 2048 + off0);
        a[mt][1] = *reinterpret_cast<const bf16x8_t*>(base + mt * 2048 + off1);
      }
    } else {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int s = 0; s < 4; ++s) a[mt][s] = *reinterpret_cast<const bf16x8_t*>(base + mt * 4096 + off32(s));
    }
  };
  auto readB = [&](FragB& b, int q, int buf) {
    const char* base = smem + buf * kBuf + (2 + q) * kSlot + wc * 32 * 128;
    if constexpr (MF == 16) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        b[nt][0] = *reinterpret_cast<const bf16x8_t*>(base + nt * 2048 + off0);
        b[nt][1] = *reinterpret_cast<const bf16x8_t*>(base + nt * 2048 + off1);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) b[s] = *reinterpret_cast<const bf16x8_t*>(base + off32(s));
    }
  };

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, 0, p.w_bytes, 0x00020000);
  Acc acc00, acc01, acc11, acc10;
  FragA a;
  FragB b0, b1;

  // ---- K-tiles [kb, kb + nk) of the tile at (m0, n0) into the accumulators
  auto mainloop = [&](int m0, int n0, int kb, int nk) {
    // LDS-DMA sources: piece q = 2w + i fills slot rows [8q, 8q+8); lane -> row 8q + L/8,
    // physical chunk L%8 = logical chunk c ^ ((row >> 1) & 7)
    // SCHED 1 addresses through buffer resources: a 32-bit byte offset per (quadrant, piece) and the
    // K-tile step in the scalar offset (half the address VGPRs of 64-bit pointers; the launcher keeps
    // both operands under 2 GB for it).  Rows are clamped either way, so every access is in range.
    const bf16* srcA[2][2];
    const bf16* srcB[2][2];
    unsigned offA[2][2], offB[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rs = (2 * w + i) * 8 + (L >> 3);
      const int c = (L & 7) ^ ((rs >> 1) & 7);
      const int koff = kb * 64 + c * 8;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        int gm = m0 + (rs >> 6) * 128 + q * 64 + (rs & 63);
        gm = gm < p.M ? gm : p.M - 1;
        int gn = n0 + (rs >> 5) * 64 + q * 32 + (rs & 31);
        gn = gn < p.N ? gn : p.N - 1;
        if constexpr (SCHED >= 1) {
          offA[q][i] = (unsigned)(gm * p.lda + koff) * 2u;
          offB[q][i] = (unsigned)(gn * p.ldw + koff) * 2u;
        } else {
          srcA[q][i] = p.A + (size_t)gm * p.lda + koff;
          srcB[q][i] = p.W + (size_t)gn * p.ldw + koff;
        }
      }
    }
    // slot order inside a buffer: 0 A q0, 1 A q1, 2 B q0, 3 B q1
    auto issueA = [&](int q, int kt, int buf) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        char* dst = smem + buf * kBuf + q * kSlot + (2 * w + i) * 1024;
        if constexpr (SCHED >= 1)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_t*)dst, 16, offA[q][i], kt * 128, 0, 0);
        else
          glds16(srcA[q][i] + kt * 64, dst);
      }
    };
    auto issueB = [&](int q, int kt, int buf) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        char* dst = smem + buf * kBuf + (2 + q) * kSlot + (2 * w + i) * 1024;
        if constexpr (SCHED >= 1)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void_t*)dst, 16, offB[q][i], kt * 128, 0, 0);
        else
          glds16(srcB[q][i] + kt * 64, dst);
      }
    };
    acc_zero<MF>(acc00);
    acc_zero<MF>(acc01);
    acc_zero<MF>(acc11);
    acc_zero<MF>(acc10);
    if constexpr (SCHED == 2) {
      // Two-phase schedule: 32 MFMAs per barrier interval instead of 16 (half the barriers per MFMA; the
      // interval's fixed cost -- barrier skew over 8 waves, setprio hand-off, wait -- is what kept the 4-phase
      // schedules at 71-74 % MFMA busy, profiles/pmc_tile_r5.txt).  Per K-tile t (buffer b = t & 1):
      //   L1 reads A q0, B q0, B q1 (16 b128)  refill A q1 of tile t+1 (buffer b^1; read there in L2(t-1))
      //   M1 acc00 = A0 B0, acc01 = A0 B1       (32 MFMAs)
      //   L2 reads A q1 (8 b128)                refill A q0, B q0, B q1 of tile t+2 (buffer b; read in L1(t))
      //   M2 acc10 = A1 B0, acc11 = A1 B1       (32 MFMAs; B q0 / q1 held from L1)
      // Every load segment ends with a counted vmcnt(8) (its own 2 or 6 refills plus the other segment's are
      // the 8 youngest), which retires the batch the NEXT load segment reads -- for the lagging half too,
      // whose load segments coincide with the leading half's MFMA segments.  A refill is issued one segment
      // after the barrier that closes the last read of its slot by either half.  Refills past the last
      // K-tile re-load it (clamped index) into slots nobody reads again, so the counts never change.
      const int klast = nk - 1;
      issueA(0, 0, 0);
      issueB(0, 0, 0);
      issueB(1, 0, 0);
      issueA(1, 0, 0);
      issueA(0, min(1, klast), 1);
      issueB(0, min(1, klast), 1);
      issueB(1, min(1, klast), 1);
      wait_vm<6>();  // tile 0 landed (tile 1's A0 / B0 / B1 are the 6 youngest)
      bar();
      if (lag) bar();
      auto ktile2 = [&](int kt, auto odd_c) {
        constexpr int buf = decltype(odd_c)::value ? 1 : 0;
        // L1
        readA(a, 0, buf);
        readB(b0, 0, buf);
        readB(b1, 1, buf);
        issueA(1, min(kt + 1, klast), buf ^ 1);
        wait_vm<8>();
        wait_lgkm0();
        bar();
        // M1
        mma_cluster<MF>(acc00, a, b0);
        mma_cluster<MF>(acc01, a, b1);
        bar();
        // L2
        readA(a, 1, buf);
        issueA(0, min(kt + 2, klast), buf);
        issueB(0, min(kt + 2, klast), buf);
        issueB(1, min(kt + 2, klast), buf);
        wait_vm<8>();
        wait_lgkm0();
        bar();
        // M2
        mma_cluster<MF>(acc10, a, b0);
        mma_cluster<MF>(acc11, a, b1);
        bar();
      };
      int kt = 0;
      for (; kt < klast; kt += 2) {
        ktile2(kt, std::integral_constant<bool, false>{});
        ktile2(kt + 1, std::integral_constant<bool, true>{});
      }
      if (kt == klast) ktile2(kt, std::integral_constant<bool, false>{});
      wait_vm<0>();  // the clamped re-loads land before the LDS is reused (next segment / stream-K flag)
      if (!lag) bar();
      return;
    }
    if constexpr (SCHED == 1) {
      // Balanced schedule: 8 / 4 / 8 / 4 fragment reads per phase instead of 12 / 4 / 8 / 0.  P4 of
      // K-tile t reads the B quadrant that tile t+1 starts with (its own MFMAs use the other one), so
      // the quadrant order alternates with the tile's parity e (qe = the B held at tile start:
      // 1 on even tiles, 0 on odd):
      //   P1 (0,qe)  A q0        refill B qe of t+2   (its slot was last read in P4 of t-1)
      //   P2 (0,ql)  B ql        refill A q0 of t+2
      //   P3 (1,ql)  A q1        refill B ql of t+2
      //   P4 (1,qe)  B ql of t+1 refill A q1 of t+2
      // Every slot is refilled in the phase after its only read and read 7 phases after the refill
      // (>= 6 needed with the counted vmcnt(8) per phase and the one-interval stagger, see above).
      // The tail needs no variant: the refills of the last two K-tiles re-load the segment's last
      // K-tile (clamped index, valid addresses) into slots nobody reads again, so every phase issues
      // 2 LDS-DMA and one vmcnt(8) count serves all of them; the loop drains before it returns.
      const int klast = nk - 1;
      issueB(1, 0, 0);
      issueA(0, 0, 0);
      issueB(0, 0, 0);
      issueA(1, 0, 0);
      issueB(0, min(1, klast), 1);
      issueA(0, min(1, klast), 1);
      issueB(1, min(1, klast), 1);
      issueA(1, min(1, klast), 1);
      wait_vm<8>();
      bar();
      readB(b1, 1, 0);  // tile 0 starts holding B q1; its slot is refilled in P1(0), after the next barrier
      wait_lgkm0();
      bar();
      if (lag) bar();
      auto ktile2 = [&](int kt, auto odd_c) {
        constexpr bool ODD = decltype(odd_c)::value;
        constexpr int qe = ODD ? 0 : 1, ql = 1 - qe;
        FragB& be = ODD ? b0 : b1;
        FragB& bl = ODD ? b1 : b0;
        Acc& acc0e = ODD ? acc00 : acc01;
        Acc& acc0l = ODD ? acc01 : acc00;
        Acc& acc1e = ODD ? acc10 : acc11;
        Acc& acc1l = ODD ? acc11 : acc10;
        const int buf = kt & 1;
        const int kn = min(kt + 2, klast);
        // P1
        readA(a, 0, buf);
        issueB(qe, kn, buf);
        wait_lgkm0();
        bar();
        mma_cluster<MF>(acc0e, a, be);
        wait_vm<8>();
        bar();
        // P2
        readB(bl, ql, buf);
        issueA(0, kn, buf);
        wait_lgkm0();
        bar();
        mma_cluster<MF>(acc0l, a, bl);
        wait_vm<8>();
        bar();
        // P3
        readA(a, 1, buf);
        issueB(ql, kn, buf);
        wait_lgkm0();
        bar();
        mma_cluster<MF>(acc1l, a, bl);
        wait_vm<8>();
        bar();
        // P4
        if (kt < klast) readB(bl, ql, buf ^ 1);
        issueA(1, kn, buf);
        wait_lgkm0();
        bar();
        mma_cluster<MF>(acc1e, a, be);
        wait_vm<8>();
        bar();
      };
      int kt = 0;
      for (; kt < klast; kt += 2) {
        ktile2(kt, std::integral_constant<bool, false>{});
        ktile2(kt + 1, std::integral_constant<bool, true>{});
      }
      if (kt == klast) ktile2(kt, std::integral_constant<bool, false>{});
      wait_vm<0>();  // the clamped re-loads land before the LDS is reused (next segment / stream-K flag)
      if (!lag) bar();
      return;
    }
    // prologue: tile 0 (all 4 slots) + tile 1 (A q0, B q0, B q1); tile 1's A q1 goes out in P1(0)
    issueA(0, 0, 0);
    issueB(0, 0, 0);
    issueB(1, 0, 0);
    issueA(1, 0, 0);
    if (nk > 1) {
      issueA(0, 1, 1);
      issueB(0, 1, 1);
      issueB(1, 1, 1);
      wait_vm<6>();
    } else {
      wait_vm<0>();
    }
    bar();
    if (lag) bar();

    // one K-tile = 4 phases; STEADY: every refill issued, counted waits
    auto ktile = [&](int kt, auto steady_c) {
      constexpr bool STEADY = decltype(steady_c)::value;
      const int buf = kt & 1;
      // P1: quadrant (0,0)
      readA(a, 0, buf);
      readB(b0, 0, buf);
      if (STEADY || kt + 1 < nk) issueA(1, kt + 1, buf ^ 1);
      wait_lgkm0();
      bar();
      mma_cluster<MF>(acc00, a, b0);
      if (STEADY) wait_vm<8>(); else wait_vm<0>();
      bar();
      // P2: quadrant (0,1)
      readB(b1, 1, buf);
      if (STEADY) issueA(0, kt + 2, buf);
      wait_lgkm0();
      bar();
      mma_cluster<MF>(acc01, a, b1);
      if (STEADY) wait_vm<8>(); else wait_vm<0>();
      bar();
      // P3: quadrant (1,1)
      readA(a, 1, buf);
      if (STEADY) issueB(0, kt + 2, buf);
      wait_lgkm0();
      bar();
      mma_cluster<MF>(acc11, a, b1);
      if (STEADY) wait_vm<8>(); else wait_vm<0>();
      bar();
      // P4: quadrant (1,0)
      if (STEADY) issueB(1, kt + 2, buf);
      bar();
      mma_cluster<MF>(acc10, a, b0);
      if (STEADY) wait_vm<8>(); else wait_vm<0>();
      bar();
    };
    int kt = 0;
    for (; kt + 2 < nk; ++kt) ktile(kt, std::integral_constant<bool, true>{});
    for (; kt < nk; ++kt) ktile(kt, std::integral_constant<bool, false>{});
    if (!lag) bar();
  };

  // ---- epilogue.  Quadrant (qm, qn) chunk c = (row slot rs, i): row m0 + 128 wr + 64 qm + rrow(rs),
  // cols n0 + 64 wc + 32 qn + ccol(i) + 0..3 (chunk map at Shape<>).
  // T21-style widened stores (cdna guide §5.5): one permlane swap per dword pair leaves each lane with 8
  // contiguous columns of its row -> 16-byte stores.
  //   MF 16: a lane holds cols 4g..4g+3 (i 0) and 16+4g.. (i 1), g = L >> 4; v_permlane16_swap trades i-1
  //          data of 16-lane row 0 / 2 for i-0 data of row 1 / 3: g = 0 -> 0..7, 1 -> 16..23, 2 -> 8..15,
  //          3 -> 24..31 of the wave's 32-column block (one store).
  //   MF 32: a lane holds cols 8i + 4h.. (h = L >> 5); v_permlane32_swap of (i 0, i 1) and (i 2, i 3):
  //          h = 0 -> 0..7 and 16..23, h = 1 -> 8..15 and 24..31 (two stores).
  // Partners share the row, so a row guard keeps both lanes of every swap active together.
  auto rrow = [&](int rs) { return MF == 16 ? 16 * rs + (L & 15) : 32 * rs + (L & 31); };
  auto ccol = [&](int i) { return MF == 16 ? 16 * i + 4 * (L >> 4) : 8 * i + 4 * (L >> 5); };
  const bool wide_ok = ((uintptr_t)p.C & 15) == 0 && (p.ldc & 7) == 0;
  auto store_row = [&](bf16* row_base, uint32_t (&d)[kCpr][2]) {
    if constexpr (MF == 16) {
      const int wcol = ((L >> 4) & 1) * 16 + ((L >> 5) & 1) * 8;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto r = __builtin_amdgcn_permlane16_swap(d[0][h], d[1][h], false, false);
        d[0][h] = r[0];
        d[1][h] = r[1];
      }
      *reinterpret_cast<u32x4_t*>(row_base + wcol) = u32x4_t{d[0][0], d[0][1], d[1][0], d[1][1]};
    } else {
      const int wcol = 8 * (L >> 5);
#pragma unroll
      for (int j = 0; j < 4; j += 2)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto r = __builtin_amdgcn_permlane32_swap(d[j][h], d[j + 1][h], false, false);
          d[j][h] = r[0];
          d[j + 1][h] = r[1];
        }
      *reinterpret_cast<u32x4_t*>(row_base + wcol) = u32x4_t{d[0][0], d[0][1], d[1][0], d[1][1]};
      *reinterpret_cast<u32x4_t*>(row_base + wcol + 16) = u32x4_t{d[2][0], d[2][1], d[3][0], d[3][1]};
    }
  };
  auto epilogue = [&](int m0, int n0, int split) {
    const int mrow = m0 + wr * 128;
    if constexpr (EPI == EPI_SILU) {
      bf16* C = (bf16*)p.C;
      const int nb = n0 + wc * 64;  // this wave's 64-column gate/up block: output cols [nb / 2, +32)
      const int obase = nb / 2;
      float bg[kCpr][4], bu[kCpr][4];
#pragma unroll
      for (int i = 0; i < kCpr; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + ccol(i) + r;
          bg[i][r] = (p.bias && n < p.N) ? (float)p.bias[n] : 0.f;
          bu[i][r] = (p.bias && n + 32 < p.N) ? (float)p.bias[n + 32] : 0.f;
        }
      // the wave's 32 output columns of this 64-column gate/up block are whole: 16-byte stores
      const bool wide = wide_ok && 2 * (obase + 32) <= p.N;
      auto emit = [&](const Acc& g, const Acc& u, int qm) {
#pragma unroll
        for (int rs = 0; rs < kRows; ++rs) {
          const int m = mrow + qm * 64 + rrow(rs);
          if (m >= p.M) continue;
          if (wide) {
            uint32_t d[kCpr][2];
#pragma unroll
            for (int i = 0; i < kCpr; ++i) {
              const f32x4_t gv = chunk_get<MF>(g, rs * kCpr + i), uv = chunk_get<MF>(u, rs * kCpr + i);
#pragma unroll
              for (int h = 0; h < 2; ++h)
                d[i][h] = pack_bf16x2(silu_f(gv[2 * h] + bg[i][2 * h]) * (uv[2 * h] + bu[i][2 * h]),
                                      silu_f(gv[2 * h + 1] + bg[i][2 * h + 1]) * (uv[2 * h + 1] + bu[i][2 * h + 1]));
            }
            store_row(C + (size_t)m * p.ldc + obase, d);
            continue;
          }
#pragma unroll
          for (int i = 0; i < kCpr; ++i) {
            const int oc = obase + ccol(i);
            if (2 * oc >= p.N) continue;
            const f32x4_t gv = chunk_get<MF>(g, rs * kCpr + i), uv = chunk_get<MF>(u, rs * kCpr + i);
            bf16x4_t o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = f2bits(silu_f(gv[r] + bg[i][r]) * (uv[r] + bu[i][r]));
            *reinterpret_cast<bf16x4_t*>(C + (size_t)m * p.ldc + oc) = o;
          }
        }
      };
      emit(acc00, acc01, 0);
      emit(acc10, acc11, 1);
    } else {
      float bv[2][kCpr][4];
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int i = 0; i < kCpr; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = n0 + wc * 64 + qn * 32 + ccol(i) + r;
            bv[qn][i][r] = (EPI == EPI_STORE && p.bias && n < p.N) ? (float)p.bias[n] : 0.f;
          }
      auto emit = [&](const Acc& acc, int qm, int qn) {
        const int nbase = n0 + wc * 64 + qn * 32;
        const bool wide = EPI == EPI_STORE && wide_ok && nbase + 32 <= p.N;
#pragma unroll
        for (int rs = 0; rs < kRows; ++rs) {
          const int m = mrow + qm * 64 + rrow(rs);
          if (m >= p.M) continue;
          if constexpr (EPI == EPI_STORE) {
            if (wide) {
              uint32_t d[kCpr][2];
#pragma unroll
              for (int i = 0; i < kCpr; ++i) {
                const f32x4_t v = chunk_get<MF>(acc, rs * kCpr + i);
#pragma unroll
                for (int h = 0; h < 2; ++h)
                  d[i][h] = pack_bf16x2(act_f<ACT>(v[2 * h] + bv[qn][i][2 * h]),
                                        act_f<ACT>(v[2 * h + 1] + bv[qn][i][2 * h + 1]));
              }
              store_row((bf16*)p.C + (size_t)m * p.ldc + nbase, d);
              continue;
            }
          }
#pragma unroll
          for (int i = 0; i < kCpr; ++i) {
            const int n = nbase + ccol(i);
            if (n >= p.N) continue;
            const f32x4_t v = chunk_get<MF>(acc, rs * kCpr + i);
            if constexpr (EPI == EPI_PARTIAL) {
              float* ws = p.slab + ((size_t)split * p.M + m) * p.N + n;
              *reinterpret_cast<f32x4_t*>(ws) = v;
            } else {
              bf16x4_t o;
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = f2bits(act_f<ACT>(v[r] + bv[qn][i][r]));
              *reinterpret_cast<bf16x4_t*>((bf16*)p.C + (size_t)m * p.ldc + n) = o;
            }
          }
        }
      };
      emit(acc00, 0, 0);
      emit(acc01, 0, 1);
      emit(acc11, 1, 1);
      emit(acc10, 1, 0);
    }
  };

  // ---- work: a data-parallel workgroup runs one segment (a whole tile or one K-split of it);
  // a stream-K workgroup runs an equal contiguous share of the remaining tiles' (tile, K-tile)
  // iterations.  A tile split across stream-K workgroups is combined in-launch (cdna guide §5
  // item 2): each part stores its fp32 accumulators to its own slab, drains, one lane releases
  // (agent) and takes a relaxed agent ticket; the part that draws the last ticket acquires,
  // sums every part in workgroup order (bitwise reproducible whichever part arrives last),
  // resets the ticket word and runs the epilogue.
  const bool dp = (int)blockIdx.x < p.dp_tiles;
  const int G = p.sk_grid;
  const int j = dp ? xcd_remap(blockIdx.x, p.dp_tiles) : xcd_remap(blockIdx.x - p.dp_tiles, G);
  const long tot = dp ? 0 : (long)(p.tiles_m * p.tiles_n - p.dp_tiles) * ks;
  auto it_begin = [&](int b) -> long { return (long)b * tot / G; };
  auto owner = [&](long x) -> int { return (int)(((x + 1) * G + tot - 1) / tot) - 1; };
  auto slot_of = [&](int b, int ts) -> int { return 2 * b + (ts == (int)(it_begin(b) / ks) ? 0 : 1); };
  long it = dp ? 0 : it_begin(j);
  const long it1 = dp ? 1 : it_begin(j + 1);
  unsigned* flag = reinterpret_cast<unsigned*>(smem);
  while (it < it1) {
    int tile, kb, ke, split = 0;
    if (dp) {
      split = j % p.ksplit;
      tile = j / p.ksplit;
      kb = split * p.kt_split;
      ke = min(ks, kb + p.kt_split);
      it = 1;
    } else {
      const int ts = (int)(it / ks);
      tile = p.dp_tiles + ts;
      kb = (int)(it % ks);
      ke = (int)min((long)ks, kb + (it1 - it));
      it += ke - kb;
    }
    int m0, n0;
    tile_coords(tile, m0, n0);
    mainloop(m0, n0, kb, ke - kb);
    if (!dp && !(kb == 0 && ke == ks)) {
      const int ts = tile - p.dp_tiles;
      const int first = owner((long)ts * ks), last = owner((long)ts * ks + ks - 1);
      // slab stores write-through (sc1): no L2 write-back fence needed before the ticket
      // (cdna guide §5 item 2, the sc1 form); every wave drains its stores before the barrier
      {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            p.slab + (size_t)slot_of(j, ts) * 65536, 0, 65536 * 4, 0x00020000);
auto slab_store = [&](const Acc& acc, int q) {
#pragma unroll
          for (int c = 0; c < 8; ++c)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, chunk_get<MF>(acc, c)), rs, tid * 16,
                                                   (q * 8 + c) * kThreads * 16, 16);
        };
        slab_store(acc00, 0);
        slab_store(acc01, 1);
        slab_store(acc11, 2);
        slab_store(acc10, 3);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned tk = __hip_atomic_fetch_add(&p.cnt[ts], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tk > (unsigned)(last - first)) report_index_error(ERR_TICKET, tk);  // stale / shared ticket word
        const unsigned is_last = tk == (unsigned)(last - first) ? 1u : 0u;
        if (is_last) {
          __hip_atomic_store(&p.cnt[ts], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag[0] = is_last;
      }
      __syncthreads();
      const bool is_last = flag[0] != 0u;
      __syncthreads();  // every wave has read the flag before the next segment's DMA reuses the LDS
      if (!is_last) continue;
      // fixed-order sum (((s_first + s_first+1) + ...) + s_last) whichever part arrives last (bitwise
      // reproducible for any part count: the running sum is built in part order, this part's own term
      // taken from its registers at its position); 8 loads in flight per quadrant and part
      auto fold = [&](Acc& acc, int q0) {
        f32x4_t s[8];
        for (int c = first; c <= last; ++c) {
          if (c == j) {
            if (c == first) {
#pragma unroll
              for (int i = 0; i < 8; ++i) s[i] = chunk_get<MF>(acc, i);
            } else {
#pragma unroll
              for (int i = 0; i < 8; ++i) s[i] += chunk_get<MF>(acc, i);
            }
            continue;
          }
          const float* src = p.slab + (size_t)slot_of(c, ts) * 65536 + tid * 4;
          f32x4_t t[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = *reinterpret_cast<const f32x4_t*>(src + (q0 + i) * kThreads * 4);
          if (c == first) {
#pragma unroll
            for (int i = 0; i < 8; ++i) s[i] = t[i];
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) s[i] += t[i];
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) chunk_set<MF>(acc, i, s[i]);
      };
      fold(acc00, 0);
      fold(acc01, 8);
      fold(acc11, 16);
      fold(acc10, 24);
    }
    epilogue(m0, n0, split);
  }
}

// Split-K combine: out = epilogue(sum_s ws[s]) — 8 output columns per thread.
// EPI_STORE: out[M, N] = act(sum + bias); EPI_SILU: out[M, N/2] from the interleaved gate/up layout.
template <int EPI, int ACT>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, const bf16* __restrict__ bias,
                                                            bf16* __restrict__ C, int ldc, int M, int N, int S) {
  const int NO = EPI == EPI_SILU ? N / 2 : N;
  const int per_row = NO / 8;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)M * per_row) return;
  const int m = (int)(e / per_row), o = (int)(e % per_row) * 8;
  const size_t plane = (size_t)M * N;
  float v[8];
  if constexpr (EPI == EPI_SILU) {
    const int n = (o / 32) * 64 + (o % 32);  // gate col of output o; up = n + 32
    float g[8], u[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = u[j] = 0.f;
    for (int s = 0; s < S; ++s) {
      const float* r = ws + s * plane + (size_t)m * N + n;
      const f32x4_t g0 = *reinterpret_cast<const f32x4_t*>(r), g1 = *reinterpret_cast<const f32x4_t*>(r + 4);
      const f32x4_t u0 = *reinterpret_cast<const f32x4_t*>(r + 32), u1 = *reinterpret_cast<const f32x4_t*>(r + 36);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g[j] += g0[j]; g[j + 4] += g1[j];
        u[j] += u0[j]; u[j + 4] += u1[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float bg = bias ? (float)bias[n + j] : 0.f, bu = bias ? (float)bias[n + 32 + j] : 0.f;
      v[j] = silu_f(g[j] + bg) * (u[j] + bu);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    for (int s = 0; s < S; ++s) {
      const float* r = ws + s * plane + (size_t)m * N + o;
      const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(r), x1 = *reinterpret_cast<const f32x4_t*>(r + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] += x0[j]; v[j + 4] += x1[j]; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_f<ACT>(v[j] + (bias ? (float)bias[o + j] : 0.f));
  }
  *reinterpret_cast<bf16x8_t*>(C + (size_t)m * ldc + o) = pack8(v);
}

int g_mfma = 16;  // grag_gemm_tile_mfma()
int g_sched = 2;  // grag_gemm_tile_sched(): 2 the two-phase schedule, 32 MFMAs per barrier interval (default:
                  // +0.9-4.1 % over 1 at 7104 rows, bitwise equal, profiles/ab_tile_sched_r6.json); 1 the balanced
                  // 8/4/8/4-read phase schedule (+5-10 % over 0, profiles/ab_tile_sched_r5.json); 0 the 12/4/8/0 one

template <int EPI, int ACT>
int launch(const Args& a, hipStream_t stream) {
  const int nwg = a.dp_tiles + a.sk_grid;
  if (g_mfma == 32) gemm_tile_kernel<EPI, ACT, 32, 0><<<nwg, kThreads, 0, stream>>>(a);
  else if (g_sched == 2 && a.a_bytes > 0 && a.w_bytes > 0) gemm_tile_kernel<EPI, ACT, 16, 2><<<nwg, kThreads, 0, stream>>>(a);
  else if (g_sched == 1 && a.a_bytes > 0 && a.w_bytes > 0) gemm_tile_kernel<EPI, ACT, 16, 1><<<nwg, kThreads, 0, stream>>>(a);
  else gemm_tile_kernel<EPI, ACT, 16, 0><<<nwg, kThreads, 0, stream>>>(a);
  return (int)hipGetLastError();
}

}  // namespace

// MFMA shape of the tile kernel for later launches (16: v_mfma_f32_16x16x32_bf16, the default; 32:
// v_mfma_f32_32x32x16_bf16); any other value only queries.  Returns the previous shape.
GRAG_API int grag_gemm_tile_mfma(int mf) {
  const int prev = g_mfma;
  if (mf == 16 || mf == 32) g_mfma = mf;
  return prev;
}

// Phase schedule of the 16x16x32 tile kernel for later launches (0 or 1, see gemm_tile_kernel's
// mainloop); any other value only queries.  Returns the previous schedule.
GRAG_API int grag_gemm_tile_sched(int sched) {
  const int prev = g_sched;
  if (sched >= 0 && sched <= 2) g_sched = sched;
  return prev;
}

// out = epilogue(sum_s ws[s]) for fp32 split-K planes ws[S][M][N] (also used by gemm_decode.hip).
GRAG_API int grag_splitk_reduce(const void* ws, const void* bias, void* C, int ldc, int M, int N, int S, int epi,
                                int act, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (N % 8 != 0 || ldc % 8 != 0 || (epi == EPI_SILU && N % 64 != 0) || S < 1) return (int)hipErrorInvalidValue;
  const int NO = epi == EPI_SILU ? N / 2 : N;
  const long n8 = (long)M * (NO / 8);
  const int blocks = (int)((n8 + 255) / 256);
#define RED(E, AC) splitk_reduce_kernel<E, AC><<<blocks, 256, 0, stream>>>((const float*)ws, (const bf16*)bias, (bf16*)C, ldc, M, N, S)
  if (epi == EPI_SILU) RED(EPI_SILU, ACT_NONE);
  else if (act == ACT_GELU) RED(EPI_STORE, ACT_GELU);
  else if (act == ACT_GELU_TANH) RED(EPI_STORE, ACT_GELU_TANH);
  else RED(EPI_STORE, ACT_NONE);
#undef RED
  return (int)hipGetLastError();
}

// y = epilogue(x @ w^T).  epi: 0 store (act: 0 none, 1 gelu-erf, 3 gelu-tanh), 1 silu*mul
// (w rows interleaved in 32-row gate/up blocks, out [M, N/2]).
//   ksplit > 1: K split into ksplit parts, fp32 planes into ws (ksplit * M * N floats) and
//               splitk_reduce_kernel applies the epilogue (decode-sized M, few tiles);
//   ksplit == 1, sk_grid > 0: data-parallel rounds of whole tiles, then sk_grid stream-K
//               workgroups share the last (tiles - dp) tiles, dp = (tiles / sk_grid - 1) * sk_grid
//               (all tiles when tiles < sk_grid); ws >= 2 * sk_grid * 65536 floats, cnt >= tiles
//               zero-initialised words (each reset by its tile's last arriver);
//   ksplit == 1, sk_grid < 0: every full round of the device's CUs is data-parallel, dp =
//               (tiles / ncu) * ncu, and |sk_grid| stream-K workgroups share the partial last round
//               (|sk_grid| = ncu: one per CU; fewer for a thin remainder; shares down to a quarter tile);
//   otherwise every tile is one workgroup.
// Requirements (checked): K % 64 == 0, every split >= 2 K-tiles, lda/ldw % 8 == 0,
// N % 8 == 0 (silu: N % 64 == 0), ldc % 8 == 0, 16-B aligned pointers.
namespace {
// compute units of the current device (cached per device; a host query, legal during graph capture)
int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}
}  // namespace

GRAG_API int grag_gemm_tile(const void* A, const void* W, const void* bias, void* C, int lda, int ldw, int ldc,
                            int M, int N, int K, int epi, int act, int ksplit, int sk_grid, void* ws, void* cnt,
                            hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 64 != 0 || K < 128 || lda % 8 != 0 || ldw % 8 != 0 || ldc % 8 != 0 || N % 8 != 0)
    return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU && N % 64 != 0) return (int)hipErrorInvalidValue;
  // epi 2 (EPI_PARTIAL, ksplit > 1 only): leave the fp32 planes in ws for a consumer that reduces
  // them itself (grag_splitk_add_rmsnorm)
  const bool keep = epi == EPI_PARTIAL;
  if (epi != EPI_STORE && epi != EPI_SILU && !keep) return (int)hipErrorInvalidValue;
  if (act != ACT_NONE && act != ACT_GELU && act != ACT_GELU_TANH) return (int)hipErrorInvalidValue;
  if ((epi == EPI_SILU || keep) && act != ACT_NONE) return (int)hipErrorInvalidValue;
  if (keep && (ksplit <= 1 || bias != nullptr)) return (int)hipErrorInvalidValue;
  const int kt = K / 64;
  if (ksplit < 1) ksplit = 1;
  const int kts = (kt + ksplit - 1) / ksplit;
  if (kts < 2 || (ksplit - 1) * kts >= kt) return (int)hipErrorInvalidValue;  // every split non-empty, >= 2 tiles
  if (ksplit > 1 && (kt - (ksplit - 1) * kts) < 2) return (int)hipErrorInvalidValue;
  if (ksplit > 1 && ws == nullptr) return (int)hipErrorInvalidValue;
  Args a;
  a.A = (const bf16*)A;
  a.W = (const bf16*)W;
  a.bias = (const bf16*)bias;
  a.C = C;
  a.slab = (float*)ws;
  a.cnt = (unsigned*)cnt;
  a.lda = lda; a.ldw = ldw; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K;
  {  // SCHED 1's 32-bit offsets: operands of 2 GB or more take schedule 0 (64-bit pointers)
    const long ab = (long)M * lda * 2, wb = (long)N * ldw * 2;
    a.a_bytes = ab < (1L << 31) ? (int)ab : 0;
    a.w_bytes = wb < (1L << 31) ? (int)wb : 0;
  }
  a.tiles_m = (M + 255) / 256;
  a.tiles_n = (N + 255) / 256;
  a.ksplit = ksplit;
  a.kt_split = kts;
  const long tiles = (long)a.tiles_m * a.tiles_n;
  if (tiles * ksplit >= (1L << 30)) return (int)hipErrorInvalidValue;
  a.dp_tiles = (int)(tiles * ksplit);
  a.sk_grid = 0;
  // sk_grid > 0: the last full round and the remainder are streamed (shares >= half a tile);
  // sk_grid < 0: every full round is data-parallel and only the remainder is streamed over |sk_grid|
  // workgroups (shares >= a quarter tile: <= 5 parts per tile, the last arriver folds <= 4 slabs)
  const int skg = sk_grid < 0 ? -sk_grid : sk_grid;
  const int ncu = device_cus();
  if (ksplit == 1 && skg > 0 && tiles % (sk_grid < 0 ? ncu : skg) != 0) {
    if (ws == nullptr || cnt == nullptr) return (int)hipErrorInvalidValue;
    const long rounds = tiles / skg;
    a.dp_tiles = sk_grid < 0 ? (int)((tiles / ncu) * ncu) : rounds >= 1 ? (int)((rounds - 1) * skg) : 0;
    a.sk_grid = skg;
    const long min_share = sk_grid < 0 ? (kt + 3) / 4 : (kt + 1) / 2;
    if ((tiles - a.dp_tiles) * kt < (long)skg * min_share) return (int)hipErrorInvalidValue;
  }
  int err;
  if (ksplit > 1) {
    err = launch<EPI_PARTIAL, ACT_NONE>(a, stream);
    if (err || keep) return err;
    const int NO = epi == EPI_SILU ? N / 2 : N;
    const long n8 = (long)M * (NO / 8);
    const int blocks = (int)((n8 + 255) / 256);
#define RED(E, AC) splitk_reduce_kernel<E, AC><<<blocks, 256, 0, stream>>>((const float*)ws, (const bf16*)bias, (bf16*)C, ldc, M, N, ksplit)
    if (epi == EPI_SILU) RED(EPI_SILU, ACT_NONE);
    else if (act == ACT_GELU) RED(EPI_STORE, ACT_GELU);
    else if (act == ACT_GELU_TANH) RED(EPI_STORE, ACT_GELU_TANH);
    else RED(EPI_STORE, ACT_NONE);
#undef RED
    return (int)hipGetLastError();
  }
  if (epi == EPI_SILU) return launch<EPI_SILU, ACT_NONE>(a, stream);
  if (act == ACT_GELU) return launch<EPI_STORE, ACT_GELU>(a, stream);
  if (act == ACT_GELU_TANH) return launch<EPI_STORE, ACT_GELU_TANH>(a, stream);
  return launch<EPI_STORE, ACT_NONE>(a, stream);
}

GRAG_ERR_UNIT(gemm_tile)
