// Decode-regime MFMA GEMM (SURVEY §2.7 N1c, N1h, N1i, N1j at 32 < M <= 256):
//
//   D[M, N] = A[M, K] · W[N, K]^T        bf16 in, fp32 accumulate
//
// Regime.  At decode batches every weight byte is read once per step and the
// whole A (M x K, <= 1.8 MB) sits in L2, so the kernel is bound by how many W
// bytes each CU keeps in flight (Little's law: 5.5 TB/s over ~3 us of loaded
// HBM latency = ~64 KB per CU).  The 256x256 tile kernel (gemm_tile.hip) keeps
// ~32 KB of W in flight behind one LDS ring shared with A and measured 2.5-2.9
// TB/s on the Qwen2-7B projections (profiles/gemm_tile_ab_v2.jsonl).
//
// Design:
//   * W goes HBM -> VGPRs directly (no LDS): each wave owns 32 W rows (two
//     16-row MFMA tiles) and keeps D+1 K-steps (64 deep) of them in a register
//     ring, D steps in flight.  The loads are inline-asm `global_load_dwordx4 nt`
//     (hidden from hipcc's waitcnt bookkeeping, which would otherwise drain the
//     ring with vmcnt(0) beside the LDS-DMA: cdna guide §5 trap (b)), retired by
//     ONE counted `s_waitcnt vmcnt(N)` per K-step that names the consumed
//     registers ("+v"), so no MFMA can be scheduled above it (guide §5.7 item 1).
//   * A (all M rows, 16*MT padded) arrives per K-step by LDS-DMA into a D+1 deep
//     LDS ring (one 1-KiB wave instruction = 8 rows x 128 B, source-side XOR
//     swizzle -> conflict-free ds_read_b128), fetched once per workgroup and read
//     by all its waves; one raw s_barrier per K-step (the refill goes into the
//     slot every wave finished before that barrier).
//   * The MFMA takes the W fragment as operand A, so each lane ends with 4
//     consecutive output columns of one row (8-byte bf16 / 16-byte fp32 stores).
//   * Work: the N / (16*NTW) wave units (16*NTW W rows each) of every K-range
//     are dealt to `gs` workgroups per K-range in contiguous, balanced runs
//     (floor(g U / gs) .. floor((g+1) U / gs), at most NWV each), XCD-remapped.
//     gs = U / NWV is the plain tiling; a smaller unit count per workgroup lets
//     the grid match the 256 CUs when U / NWV does not (Qwen2-7B gate/up at
//     M > 128: 1184 units = 148 full 8-wave tiles, 58 % of the CUs; dealt as 4-5
//     units to each of 256 five-wave workgroups every CU streams its share).
//     A wave without a unit repeats its neighbour's loads (L2 hits) and stores
//     nothing.  ksplit > 1 writes fp32 partial planes ws[split][M][N];
//     grag_splitk_reduce (in gemm_tile.hip) sums them and applies the epilogue.
//   * Epilogues fused in the kernel: bias + act (none / gelu-erf / gelu-tanh),
//     SiLU(gate)*up for the gate/up weight stored interleaved in 32-row blocks
//     (ops/gemm.py interleave_gate_up): a wave's two n-tiles are then the 16
//     gate rows and the 16 matching up rows, so the product forms in registers.
#include <type_traits>

#include "common.h"

using namespace grag;

GRAG_API int grag_splitk_reduce(const void* ws, const void* bias, void* C, int ldc, int M, int N, int S, int epi,
                                int act, hipStream_t stream);

namespace {

enum { EPI_STORE = 0, EPI_SILU = 1, EPI_PARTIAL = 2 };

// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>): a compile-time loop (register arrays
// indexed by its constant stay in registers)
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(static_cast<F&&>(f));
  }
}
enum { ACT_NONE = 0, ACT_GELU = 1, ACT_GELU_TANH = 3 };

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

// LDS-DMA piece (1 KiB per wave instruction, lane-linear at wave-uniform lds_dst); M0 saved/set/restored in
// one statement; completion tracked only by the caller's counted vmcnt.
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0\n\t"
      "s_nop 2"  // hipcc may hand the address VGPRs to the very next VALU: let the DMA read them first
      : "=&s"(keep)
      : "v"(src), "s"(lds_dst)
      : "memory");
}

// Two 16-B W loads of one row: k [32s + 8 h4, +8) for s = 0, 1 (bytes 16 h4 and 64 + 16 h4 of the 128-B line).
// Two 16-B W loads of one row: k [32s + 8 h4, +8) for s = 0, 1 (bytes 16 h4 and 64 + 16 h4 of the 128-B
// line).  Default cache policy: the two half-line requests of a row share the L2 line (nontemporal loads
// measured 5-20 % slower here: profiles/gemm_decode_ab_v2.jsonl).
// The trailing s_nop: hipcc's hazard pass does not see into the asm, and a VALU write of the address VGPRs
// right after the second load (register reuse across a branch showed it) must not land before the load has
// read them (the same guard as glds16's).
__device__ __forceinline__ void ldw2(bf16x8_t& lo, bf16x8_t& hi, const bf16* p) {
  asm volatile(
      "global_load_dwordx4 %0, %2, off\n\t"
      "global_load_dwordx4 %1, %2, off offset:64\n\t"
      "s_nop 1"
      : "=&v"(lo), "=&v"(hi)
      : "v"(p)
      : "memory");
}
// Retire everything but the N youngest vector-memory ops; the named W registers are read-write here, so
// nothing that consumes them can be scheduled above the wait.
template <int N, int G>
__device__ __forceinline__ void wait_w(bf16x8_t (&w)[G]) {
  if constexpr (G == 4)
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]) : "n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7])
                 : "n"(N)
                 : "memory");
}

// raw barrier that never drains the LDS-DMA in flight; the wave's own ds_reads of the slot the next issue
// refills must be complete before it (hipcc may otherwise sink their lgkmcnt waits below the barrier)
__device__ __forceinline__ void bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr int kDepth = 4;  // K-steps of W and A issued ahead (ring of kDepth + 1 slots)

struct DArgs {
  const bf16* A;
  const bf16* W;
  const bf16* bias;
  void* C;
  int lda, ldw, ldc;
  int M, N, K;
  int units, gs, ksplit, kt_split;  // wave units per K-range, workgroups per K-range
  int msplit;                       // row blocks of 16*MT (adjacent on one XCD: the W lines are shared in L2)
  int packed;                       // W in the unit-packed layout (grag_gemm_decode doc)
  unsigned long long* stamps;       // diagnostics (grag_gemm_decode_stamps): per workgroup {start, end, xcc} or null
  // NRM (grag_gemm_decode_norm): A = RMSNorm(residual + sum of the producer's split-K planes) * nw, formed in the
  // prologue (p.A unused)
  const float* nplanes;  // [nS][M][K] fp32
  int nS;
  const bf16* nres_in;   // [M][K] residual stream before this add (read only)
  bf16* nres_out;        // [M][K] residual stream after it (written by workgroup 0)
  const bf16* nw;        // [K] norm weight
  float neps;
  // NRM = 2 (grag_gemm_decode_scaled): A is the residual stream x; the norm weight rides in the A ring's row
  // 15 (LDS-DMA from `nw`), each A fragment is scaled by it, and the accumulators by 1 / rms(x) (from the
  // producer's per-group sums of squares nss[nG][kNrmRows]) before the epilogue
  const float* nss;
  int nG;
  // RED = 1 (grag_gemm_decode_red, EPI_PARTIAL): the last split to finish a unit group adds the group's
  // columns of all splits' planes into the residual stream rres [M][N] (in place, bf16) and writes the
  // group's sums of squares per row to rss[group][kNrmRows]; rcnt: per-group tickets (zeroed; each last
  // arriver resets its word)
  bf16* rres;
  float* rss;
  unsigned* rcnt;
};

constexpr int kNrmRows = 4;         // NRM: rows of the batch (the reference's --max-num-seqs 4)
constexpr int kNrmLds = 64 * 1024;  // NRM: LDS image of the normalised rows, [M][K + 32] bf16

// NTW 16-row n-tiles per wave (32 or 64 W rows): the A fragment read from LDS feeds NTW MFMAs, so NTW = 4
// halves the LDS read traffic per MFMA (at NTW = 2 it equals the LDS bandwidth at full MFMA rate).
// TQ > 0 (tail split, NWV = 8): a workgroup owns 4 or 5 wave units; waves 0-3 compute one unit each over all
// MT row tiles, and a 5th unit is shared by waves 4-7, TQ = MT / 4 row tiles each.  The CU's 4 SIMDs (two
// waves each) then carry 1.25 units of MFMA work apiece where a 5-wave workgroup put 2 units on one SIMD
// (profiles/pmc_dec_r5.txt: Qwen2-7B gate/up at 176 rows, 4.625 units per CU on 256 CUs; the doubled SIMD
// paced every K-step barrier).  Waves 4-7 load the shared unit's W rows alike (L1 / L2 hits after the first).
// NRM = 1 (MT = 1, TQ = 0, one K-range): the RMSNorm that feeds this projection runs in the prologue -- every
// workgroup sums the producer's split-K planes into the residual row(s), forms the row's RMS and writes the
// normalised rows into an LDS-resident image the whole K loop reads its A fragments from (no A LDS-DMA ring,
// no per-K-step barrier); workgroup 0 also writes the new residual to a second buffer (no other workgroup
// reads what it writes).  Replaces the split-K RMSNorm launch between o_proj and gate/up at 1-4 rows.
template <int EPI, int ACT, int MT, int D, int NWV, int NTW, int TQ = 0, int NRM = 0, int RED = 0>
__global__ __launch_bounds__(64 * NWV, (NWV == 4 && NTW == 2 && (D + 1) * MT * 2 <= 80) ? 2 : 1)
void gemm_dec_kernel(DArgs p) {
  static_assert(TQ == 0 || (NWV == 8 && TQ * 4 == MT), "tail split: 8 waves, MT = 4 TQ");
  static_assert(NRM == 0 || (MT == 1 && TQ == 0), "NRM: one 16-row tile");
  static_assert(RED == 0 || (EPI == EPI_PARTIAL && TQ == 0), "RED: the split-K planes' producer");
  constexpr int NST = D + 1;            // LDS stages = W register slots
  constexpr int ABYTES = MT * 16 * 128;  // one K-step of A
  constexpr int NPC = MT * 2;                  // A pieces (1 KiB = 8 rows x 128 B) per K-step
  constexpr int GA = NRM == 1 ? 0 : (NPC + NWV - 1) / NWV;  // per wave (the last wave may repeat its final piece)
  constexpr int GW = 2 * NTW;                  // W dwordx4 per lane per K-step
  static_assert(NTW == 2 || NTW == 4, "NTW");
  static_assert(NST * ABYTES <= 160 * 1024, "LDS ring exceeds 160 KB");
  constexpr int LDSB = NRM == 1 ? kNrmLds : NST * ABYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDSB];

  const int tid = threadIdx.x;
  const int L = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = L & 15, h4 = L >> 4;
  const unsigned long long t_start = p.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int split = b % p.ksplit;
  const int mb = (b / p.ksplit) % p.msplit, g = b / (p.ksplit * p.msplit);
  const int m0 = mb * 16 * MT;
  const int u0 = (int)((long)g * p.units / p.gs);
  const int cnt = (int)((long)(g + 1) * p.units / p.gs) - u0;
  bool active = w < cnt;                          // wave-uniform
  int q = u0 + min(w, cnt - 1);                   // this wave's unit (an idle wave repeats the last one)
  if constexpr (TQ > 0) {
    if (w >= 4) {
      active = cnt > 4;
      q = u0 + (cnt > 4 ? 4 : min(w - 4, cnt - 1));
    } else {
      active = w < min(cnt, 4);
    }
  }
  const bool tail_wave = TQ > 0 && w >= 4;
  const int ks = p.K >> 6;
  const int kb = split * p.kt_split;
  const int ke = min(ks, kb + p.kt_split);
  const int nsteps = ke - kb;

  // W rows of this wave's n-tiles.  SiLU at NTW = 2: the 16 gate rows of a 16-wide output group and the
  // matching up rows (+32); at NTW = 4 the wave owns one whole 64-row gate/up block (tiles 0,1 gate, 2,3 up).
  int wr[NTW];
  // gate/up units: the SiLU epilogue, or fp32 partials of a weight packed in gate/up units (packed == 2)
  if (NTW == 2 && (EPI == EPI_SILU || p.packed == 2)) {
    wr[0] = (q >> 1) * 64 + (q & 1) * 16;
    wr[1] = wr[0] + 32;
  } else {
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) wr[nt] = 16 * NTW * q + 16 * nt;
  }
  // natural layout: row stride ldw, K-step stride 64 elements; unit-packed: the unit's 16*NTW rows x 64 k
  // of one K-step are one contiguous block (row stride 64), the unit's K-steps follow each other, so a
  // wave streams one contiguous region (DRAM pages are read whole, not 128 B per row per K-step)
  const int kstride = p.packed ? 16 * NTW * 64 : 64;
  const bf16* wp[NTW];
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt)
    wp[nt] = p.packed ? p.W + (size_t)q * ks * kstride + (size_t)kb * kstride + (16 * nt + li) * 64 + 8 * h4
                      : p.W + (size_t)min(wr[nt] + li, p.N - 1) * p.ldw + (size_t)kb * 64 + 8 * h4;

  // A pieces: piece q = w*GA + i covers rows [8q, 8q+8); lane -> row 8q + L/8, physical chunk L%8
  // 32-bit element offsets (not 64-bit pointers): the MT = 16, 5-wave variant needs the registers
  uint32_t ao[GA > 0 ? GA : 1];
  uint32_t adst[GA > 0 ? GA : 1];
  bool agw[GA > 0 ? GA : 1];  // NRM 2: this lane's piece row is row 15, the norm weight's
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int pc = min(w * GA + i, NPC - 1);
    const int row = pc * 8 + (L >> 3);
    const int c = (L & 7) ^ ((row >> 1) & 7);
    agw[i] = NRM == 2 && row == 15;
    ao[i] = agw[i] ? (uint32_t)(kb * 64 + c * 8) : (uint32_t)min(m0 + row, p.M - 1) * p.lda + kb * 64 + c * 8;
    adst[i] = __builtin_amdgcn_readfirstlane(lds0 + pc * 1024);
  }

  bf16x8_t wf[NST][GW];  // [slot][2 nt + s]
  f32x4_t acc[MT][NTW];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // issue K-step `step` into ring slot `slot`; a step past the range (the last D iterations) re-reads
  // L2-resident bytes (A's own rows, one W line) so every iteration issues the same ops and the counted
  // waits stay exact without a branch (a conditional load would make hipcc merge the ring registers through
  // copies that read an asm destination before its data lands)
  auto issue = [&](int step, int slot, bf16x8_t (&wreg)[GW]) {
    const bool live = step < nsteps;
    const int so = live ? step * 64 : 0;
#pragma unroll
    for (int i = 0; i < GA; ++i) glds16((agw[i] ? p.nw : p.A) + (ao[i] + so), adst[i] + slot * ABYTES);
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) ldw2(wreg[2 * nt], wreg[2 * nt + 1], live ? wp[nt] + step * kstride : p.W);
  };

  // A fragment of rows 16 mt + li, logical chunk 4 s + h4 (swizzle depends on li only)
  const int sw = (li >> 1) & 7;
  const int aoff0 = li * 128 + ((h4 ^ sw) << 4);
  const int aoff1 = li * 128 + (((4 + h4) ^ sw) << 4);
  // A fragments are read APF row tiles ahead of their MFMAs into a small register ring, with a scheduling
  // fence between each read group and the MFMA group before it: left alone, hipcc (short of registers at two
  // waves per SIMD) reads one fragment, waits lgkmcnt(0) and issues two MFMAs, exposing the LDS latency
  // before every MFMA pair (measured: the MFMA pipe idle about half the time at M = 192).
  // row tiles [MB, MB + NM) of the staged A against this wave's W fragments into acc[MB .. MB + NM)
  auto compute_n = [&](auto nm_c, auto mb_c, int slot, bf16x8_t (&wreg)[GW]) {
    constexpr int NM = decltype(nm_c)::value;
    constexpr int MB = decltype(mb_c)::value;
    constexpr int APF = NM >= 8 ? 2 : 1;
    const char* As = smem + slot * ABYTES + MB * 2048;
    bf16x8_t af[APF + 1][2];
#pragma unroll
    for (int j = 0; j < APF && j < NM; ++j) {
      af[j][0] = *reinterpret_cast<const bf16x8_t*>(As + j * 2048 + aoff0);
      af[j][1] = *reinterpret_cast<const bf16x8_t*>(As + j * 2048 + aoff1);
    }
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) {
      if (mt + APF < NM) {
        af[(mt + APF) % (APF + 1)][0] = *reinterpret_cast<const bf16x8_t*>(As + (mt + APF) * 2048 + aoff0);
        af[(mt + APF) % (APF + 1)][1] = *reinterpret_cast<const bf16x8_t*>(As + (mt + APF) * 2048 + aoff1);
      }
      __builtin_amdgcn_sched_barrier(0);
      bf16x8_t a0 = af[mt % (APF + 1)][0], a1 = af[mt % (APF + 1)][1];
      if constexpr (NRM == 2) {  // x * norm weight, per element (row 15 of the tile holds the weight)
        const bf16x8_t g0 = *reinterpret_cast<const bf16x8_t*>(As + 15 * 128 + ((h4 ^ 7) << 4));
        const bf16x8_t g1 = *reinterpret_cast<const bf16x8_t*>(As + 15 * 128 + (((4 + h4) ^ 7) << 4));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a0[j] = f2bits(bits2f(a0[j]) * bits2f(g0[j]));
          a1[j] = f2bits(bits2f(a1[j]) * bits2f(g1[j]));
        }
      }
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        acc[MB + mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[2 * nt], a0, acc[MB + mt][nt], 0, 0, 0);
        acc[MB + mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[2 * nt + 1], a1, acc[MB + mt][nt], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // tail split: one body per group of TQ row tiles behind a wave-uniform guard -- the own waves run all four
  // groups, a tail wave the group of its quarter -- so every MFMA appears once in the code and the
  // accumulator of row tile t is acc[t] in both roles (no second, register-hungry copy of the loop)
  const int g_lo = tail_wave ? w - 4 : 0, g_hi = tail_wave ? w - 3 : 4;
  auto compute = [&](int slot, bf16x8_t (&wreg)[GW]) {
    if constexpr (TQ > 0) {
      static_for<4>([&](auto gc) {
        constexpr int G = decltype(gc)::value;
        if (G >= g_lo && G < g_hi) compute_n(std::integral_constant<int, TQ>{}, std::integral_constant<int, G * TQ>{},
                                             slot, wreg);
      });
    } else {
      compute_n(std::integral_constant<int, MT>{}, std::integral_constant<int, 0>{}, slot, wreg);
    }
  };

  // prologue: steps 0 .. D-1 in flight
#pragma unroll
  for (int d = 0; d < D; ++d) issue(d, d, wf[d]);

  // NRM: the A rows, normalised, into the LDS image while the first W steps are in flight.  Same arithmetic
  // as splitk_rmsnorm_kernel (norm.hip): the planes added to the bf16 residual in fp32, the sum rounded to
  // bf16 (the residual stream's precision), the RMS over the rounded row, out = bf16(h * inv * w).
  const int nrp = p.K * 2 + 64;  // image row pitch (bytes): rows start 64 B apart in the bank space
  if constexpr (NRM == 1) {
    __shared__ float nred[NWV][kNrmRows];
    __shared__ float ninv[kNrmRows];
    const int nvec = p.K >> 3;
    const int tot = p.M * nvec;  // (row, 8-column unit) pairs, all rows in one pass
    const size_t plane = (size_t)p.M * p.K;
    const int nthr = 64 * NWV;
    const bool writer = blockIdx.x == 0;  // one workgroup writes the new residual (to its own buffer)
    float ssr[kNrmRows] = {0.f, 0.f, 0.f, 0.f};
    // two units per thread per round, every plane load of both issued before any add: the round costs one
    // L2 round trip, not one per unit
    for (int e0 = tid; e0 < tot; e0 += 2 * nthr) {
      const int e1 = e0 + nthr;
      const bool has1 = e1 < tot;
      const int m0 = e0 / nvec, u0 = e0 - m0 * nvec;
      const int m1 = has1 ? e1 / nvec : m0, u1 = has1 ? e1 - m1 * nvec : u0;
      float a[8], b[8];
      unpack8(reinterpret_cast<const bf16x8_t*>(p.nres_in + (size_t)m0 * p.K)[u0], a);
      unpack8(reinterpret_cast<const bf16x8_t*>(p.nres_in + (size_t)m1 * p.K)[u1], b);
      const float* q0 = p.nplanes + (size_t)m0 * p.K + u0 * 8;
      const float* q1 = p.nplanes + (size_t)m1 * p.K + u1 * 8;
      for (int sp = 0; sp < p.nS; ++sp) {
        const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(q0 + sp * plane);
        const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(q0 + sp * plane + 4);
        const f32x4_t y0 = *reinterpret_cast<const f32x4_t*>(q1 + sp * plane);
        const f32x4_t y1 = *reinterpret_cast<const f32x4_t*>(q1 + sp * plane + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] += x0[j];
          a[j + 4] += x1[j];
          b[j] += y0[j];
          b[j + 4] += y1[j];
        }
      }
      const bf16x8_t ha = pack8(a), hb = pack8(b);
      if (writer) {
        reinterpret_cast<bf16x8_t*>(p.nres_out + (size_t)m0 * p.K)[u0] = ha;
        if (has1) reinterpret_cast<bf16x8_t*>(p.nres_out + (size_t)m1 * p.K)[u1] = hb;
      }
      *reinterpret_cast<bf16x8_t*>(smem + m0 * nrp + u0 * 16) = ha;
      if (has1) *reinterpret_cast<bf16x8_t*>(smem + m1 * nrp + u1 * 16) = hb;
      unpack8(ha, a);
      unpack8(hb, b);
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sa += a[j] * a[j];
        sb += b[j] * b[j];
      }
#pragma unroll
      for (int m = 0; m < kNrmRows; ++m) ssr[m] += (m == m0 ? sa : 0.f) + (has1 && m == m1 ? sb : 0.f);
    }
    const int wv = tid >> 6;
#pragma unroll
    for (int m = 0; m < kNrmRows; ++m) {
      const float t = wave_sum(ssr[m]);
      if ((tid & 63) == 0) nred[wv][m] = t;
    }
    __syncthreads();
    if (tid < p.M) {
      float t = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < NWV; ++w2) t += nred[w2][tid];
      ninv[tid] = rsqrtf(t / (float)p.K + p.neps);
    }
    __syncthreads();
    const bf16x8_t* gw = reinterpret_cast<const bf16x8_t*>(p.nw);
    for (int e = tid; e < tot; e += nthr) {
      const int m = e / nvec, u = e - m * nvec;
      float a[8], g[8];
      char* cell = smem + m * nrp + u * 16;
      unpack8(*reinterpret_cast<const bf16x8_t*>(cell), a);
      unpack8(gw[u], g);
      const float inv = ninv[m];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = a[j] * inv * g[j];
      *reinterpret_cast<bf16x8_t*>(cell) = pack8(a);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the W steps in flight landed too: the loop's waits hold)
    __syncthreads();
  }
  // NRM: A fragments of absolute K-step `step` from the image (rows >= M are zero, never read)
  auto compute_nrm = [&](int step, bf16x8_t (&wreg)[GW]) {
    bf16x8_t a0 = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0}, a1 = a0;
    if (li < p.M) {
      const char* r = smem + li * nrp + ((kb + step) * 64 + 8 * h4) * 2;
      a0 = *reinterpret_cast<const bf16x8_t*>(r);
      a1 = *reinterpret_cast<const bf16x8_t*>(r + 64);
    }
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[2 * nt], a0, acc[0][nt], 0, 0, 0);
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[2 * nt + 1], a1, acc[0][nt], 0, 0, 0);
    }
  };

  // A K-step's LDS slot is read one barrier interval AFTER the wait that retires its LDS-DMA (cdna guide §5
  // "Read a staged buffer one phase AFTER the wait that retires it"): iteration t retires step t + 1 and
  // computes step t.  The round-2 schedule (retire step t, barrier, read step t) is the one that returned
  // wrong results in gemm_w4.hip's 4/8/12-row variants (root cause there, scripts/dev/w4_diag.py); here it
  // had passed every test, by placement.  Steps t + 2 .. t + D - 1 stay in flight across compute(t), as
  // many as before (D is one deeper).
  wait_w<(D - 1) * (GA + GW)>(wf[0]);
  bar();
  for (int t0 = 0; t0 < nsteps; t0 += NST) {
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      wait_w<(D - 2) * (GA + GW)>(wf[(u + 1) % NST]);  // retire step t + 1
      if constexpr (NRM != 1) bar();  // every wave is done with slot (u + D) % NST (= step t - 1's); step t + 1 retired everywhere
      issue(t0 + u + D, (u + D) % NST, wf[(u + D) % NST]);
      if constexpr (NRM == 1) {
        if (t0 + u < nsteps) compute_nrm(t0 + u, wf[u]);
      } else {
        if (t0 + u < nsteps) compute(u, wf[u]);  // uniform: a split's last round may be partial
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing re-reads land before the workgroup retires
  if (p.stamps && tid == 0) {  // diagnostics: 100 MHz constant clock (comparable across CUs / XCDs), main loop end
    unsigned long long* st = p.stamps + 4 * (size_t)blockIdx.x;
    st[0] = t_start;
    st[1] = __builtin_amdgcn_s_memrealtime();
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    st[2] = xcc;
    st[3] = (unsigned long long)b;
  }

  // ---- epilogue: acc[mt][nt][r] = D[W row (wr[nt] + 4 h4 + r)][A row (16 mt + li)]
  if constexpr (NRM == 2) {  // 1 / rms of this lane's row, from the producer's per-group sums of squares
    const int m = m0 + li;
    float rstd = 0.f;
    if (m < p.M) {
      float t = 0.f;
      for (int q = 0; q < p.nG; ++q) t += p.nss[q * kNrmRows + m];  // group order: deterministic
      rstd = rsqrtf(t / (float)p.K + p.neps);
    }
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) acc[0][nt] *= rstd;
  }
  // row tile mt is stored when its group is this wave's (tail split) -- every tile for the own waves
  auto mine = [&](int mt) { return TQ == 0 || (mt >= g_lo * TQ && mt < g_hi * TQ); };
  if (active) {
    constexpr int NM = MT;
    const int mr0 = m0;
    if constexpr (EPI == EPI_SILU) {
      bf16* C = (bf16*)p.C;
      constexpr int NP = NTW / 2;  // gate/up tile pairs: (nt, nt + NP)
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int gr = wr[j] + 4 * h4, ur = wr[j + NP] + 4 * h4;
        if (ur >= p.N) continue;
        const int oc = (gr >> 6) * 32 + (gr & 31);  // gate row 64 q + c  ->  output column 32 q + c
        float bg[4], bu[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bg[r] = p.bias ? (float)p.bias[gr + r] : 0.f;
          bu[r] = p.bias ? (float)p.bias[ur + r] : 0.f;
        }
#pragma unroll
        for (int mt = 0; mt < NM; ++mt) {
          const int m = mr0 + mt * 16 + li;
          if (m >= p.M || !mine(mt)) continue;
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bits(silu_f(acc[mt][j][r] + bg[r]) * (acc[mt][j + NP][r] + bu[r]));
          *reinterpret_cast<bf16x4_t*>(C + (size_t)m * p.ldc + oc) = o;
        }
      }
    } else {
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int n = wr[nt] + 4 * h4;
        if (n >= p.N) continue;
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (EPI == EPI_STORE && p.bias) ? (float)p.bias[n + r] : 0.f;
#pragma unroll
        for (int mt = 0; mt < NM; ++mt) {
          const int m = mr0 + mt * 16 + li;
          if (m >= p.M || !mine(mt)) continue;
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
  if constexpr (RED) {  // the last split of this unit group folds every split's planes into the residual stream
    __shared__ unsigned rlast;
    __shared__ float rred[NWV][kNrmRows];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's plane stores are done
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned tk = __hip_atomic_fetch_add(p.rcnt + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tk >= (unsigned)p.ksplit) report_index_error(ERR_TICKET, tk);  // a stale or shared ticket word
      const unsigned last = tk == (unsigned)(p.ksplit - 1) ? 1u : 0u;
      if (last) {
        __hip_atomic_store(p.rcnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      rlast = last;
    }
    __syncthreads();
    if (rlast == 0u) return;
    const int c0 = u0 * 16 * NTW, nv = cnt * 2 * NTW;  // the group's columns, 8 per vector
    const size_t plane = (size_t)p.M * p.N;
    float ssr[kNrmRows] = {0.f, 0.f, 0.f, 0.f};
    for (int e = tid; e < p.M * nv; e += 64 * NWV) {
      const int m = e / nv, n = c0 + (e - m * nv) * 8;
      bf16x8_t* rp = reinterpret_cast<bf16x8_t*>(p.rres + (size_t)m * p.N + n);
      float a[8];
      unpack8(*rp, a);
      const float* q = (const float*)p.C + (size_t)m * p.N + n;
      for (int sp = 0; sp < p.ksplit; ++sp) {  // split order, as the split-K RMSNorm
        const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(q + sp * plane);
        const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(q + sp * plane + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] += x0[j];
          a[j + 4] += x1[j];
        }
      }
      const bf16x8_t hb = pack8(a);
      *rp = hb;
      unpack8(hb, a);
      float sm = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) sm += a[j] * a[j];
#pragma unroll
      for (int r = 0; r < kNrmRows; ++r) ssr[r] += r == m ? sm : 0.f;
    }
#pragma unroll
    for (int r = 0; r < kNrmRows; ++r) {
      const float t = wave_sum(ssr[r]);
      if ((tid & 63) == 0) rred[w][r] = t;
    }
    __syncthreads();
    if (tid < kNrmRows) {
      float t = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < NWV; ++w2) t += rred[w2][tid];
      p.rss[g * kNrmRows + tid] = t;
    }
  }
}

template <int D, int NWV>
int launch_nrm(const DArgs& a, int epi, int nwg, hipStream_t s) {
  if (epi == EPI_SILU)
    gemm_dec_kernel<EPI_SILU, ACT_NONE, 1, D, NWV, 2, 0, 1><<<nwg, 64 * NWV, 0, s>>>(a);
  else
    gemm_dec_kernel<EPI_STORE, ACT_NONE, 1, D, NWV, 2, 0, 1><<<nwg, 64 * NWV, 0, s>>>(a);
  return (int)hipGetLastError();
}

template <int MT, int D, int NWV, int NTW, int TQ = 0>
int launch_v(const DArgs& a, int epi, int act, int nwg, hipStream_t s) {
#define GO(E, AC) gemm_dec_kernel<E, AC, MT, D, NWV, NTW, TQ><<<nwg, 64 * NWV, 0, s>>>(a)
  if (epi == EPI_PARTIAL) GO(EPI_PARTIAL, ACT_NONE);
  else if (epi == EPI_SILU) GO(EPI_SILU, ACT_NONE);
  else if (act == ACT_GELU) GO(EPI_STORE, ACT_GELU);
  else if (act == ACT_GELU_TANH) GO(EPI_STORE, ACT_GELU_TANH);
  else GO(EPI_STORE, ACT_NONE);
#undef GO
  return (int)hipGetLastError();
}

}  // namespace

// Variants compiled (mt = 16-row tiles of M, nwv = waves per workgroup, ntw = 16-row W tiles per wave;
// depth kDepth): (nwv 4, ntw 2): mt 1, 2, 4, 8, 16;  (nwv 5, ntw 2): mt 1, 2, 4, 8, 12 (mt 1 / 2 also at
// depth 8 and 12: 1-32 rows hold 2-4 KB of A per K-step, so the W ring takes the registers; balanced grids; mt 16 needs
// more than the 256 registers a wave gets at two waves per SIMD);  (nwv 8, ntw 2): mt 12.  ntw = 4 measured no faster than 2 at M = 192 (profiles/gemm_decode_ab_v3.jsonl) and is
// not instantiated.
static unsigned long long* g_dec_stamps = nullptr;
static int g_dec_depth = 0;  // 0: kDepth; 6 / 8: deeper rings where the LDS takes them (A/B, grag_gemm_decode_depth)

// K-steps issued ahead for later launches (A/B of the ring depth): 0 = the default (kDepth = 4); 6 for mt 4 / 8
// and 8 for mt 4 on the 4- and 5-wave grids (the A ring of (depth + 1) x 16 mt x 128 B must fit the LDS);
// 8 or 12 for mt 1 / 2 (>= 12 -> 12).
// Returns the previous setting.
GRAG_API int grag_gemm_decode_depth(int d) {
  const int prev = g_dec_depth;
  g_dec_depth = d;
  return prev;
}

// Diagnostics: while set, every grag_gemm_decode launch writes per workgroup (blockIdx.x) 4 u64 words
// {s_memrealtime at start, at the end of the main loop, XCC id, logical block} to `buf` (grid size x 32 B);
// null turns it off.  Not for graph capture.
GRAG_API void grag_gemm_decode_stamps(void* buf) { g_dec_stamps = (unsigned long long*)buf; }

// tail = 1: the 8-wave tail split (gemm_dec_kernel TQ = mt / 4): at most 5 wave units per workgroup
GRAG_API int grag_gemm_decode_has_t(int mt, int nwv, int ntw, int tail) {
  if (tail) return ntw == 2 && nwv == 8 && (mt == 4 || mt == 8 || mt == 12 || mt == 16);
  if (ntw != 2) return 0;
  if (nwv == 4) return mt == 1 || mt == 2 || mt == 4 || mt == 8 || mt == 16;
  if (nwv == 5) return mt == 1 || mt == 2 || mt == 4 || mt == 8 || mt == 12;
  if (nwv == 8) return mt == 12;
  return 0;
}

GRAG_API int grag_gemm_decode_has(int mt, int nwv, int ntw) { return grag_gemm_decode_has_t(mt, nwv, ntw, 0); }

// y = epilogue(x @ w^T) for M <= 16 * mt rows.  epi 0 store (act 0/1/3), 1 silu*mul (w gate/up interleaved in
// 32-row blocks, out [M, N/2]).  ksplit > 1: fp32 planes into ws (ksplit * M * N floats), then
// grag_splitk_reduce applies the epilogue.  gs = workgroups per K-range over the N / (16 ntw) wave units
// (0: N / (16 ntw nwv), the plain tiling; otherwise ceil(units / gs) <= nwv).  M > 16 mt: the rows go to
// ceil(M / (16 mt)) workgroups per unit run (at most 4).  packed = 1: W in the unit-packed layout
// [N / (16 ntw)][K / 64][16 ntw][64] (ops/gemm.py dec_pack), ldw ignored; packed = 2: the same for an
// interleaved gate/up weight packed in gate/up units (16 gate rows then their 16 up rows; ntw 2).
// Requirements (checked):
// K % 64 == 0, N % (16 * ntw) == 0 (silu: N % 64 == 0), lda/ldw % 8 == 0,
// ldc % 4 == 0, 16-B aligned A/W.
GRAG_API int grag_gemm_decode_t(const void* A, const void* W, const void* bias, void* C, int lda, int ldw, int ldc,
                                int M, int N, int K, int epi, int act, int mt, int nwv, int ntw, int ksplit, int gs,
                                int packed, int tail, void* ws, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  const int msplit = (M + 16 * mt - 1) / (16 * mt);
  if (!grag_gemm_decode_has_t(mt, nwv, ntw, tail) || msplit > 4) return (int)hipErrorInvalidValue;
  if (K % 64 != 0 || K < 64 || N % (16 * ntw) != 0 || lda % 8 != 0 || ldw % 8 != 0 || ldc % 4 != 0)
    return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU && N % 64 != 0) return (int)hipErrorInvalidValue;
  if (packed < 0 || packed > 2 || (packed == 2 && (ntw != 2 || N % 64 != 0))) return (int)hipErrorInvalidValue;
  const int units = N / (16 * ntw);
  if (gs <= 0) {
    if (units % nwv != 0) return (int)hipErrorInvalidValue;
    gs = units / nwv;
  }
  if (gs > units || (units + gs - 1) / gs > (tail ? 5 : nwv)) return (int)hipErrorInvalidValue;
  // epi 2 (EPI_PARTIAL): leave the fp32 planes in ws for a consumer that reduces them itself
  // (grag_splitk_add_rmsnorm: split-K reduce + residual add + RMSNorm in one pass)
  const bool keep = epi == EPI_PARTIAL;
  if (epi != EPI_STORE && epi != EPI_SILU && !keep) return (int)hipErrorInvalidValue;
  if (act != ACT_NONE && act != ACT_GELU && act != ACT_GELU_TANH) return (int)hipErrorInvalidValue;
  if ((epi == EPI_SILU || keep) && act != ACT_NONE) return (int)hipErrorInvalidValue;
  if (keep && bias != nullptr) return (int)hipErrorInvalidValue;
  const int kt = K / 64;
  if (ksplit < 1) ksplit = 1;
  const int kts = (kt + ksplit - 1) / ksplit;
  ksplit = (kt + kts - 1) / kts;  // effective splits (ops/gemm.py dec_ksplit computes the same)
  if ((ksplit > 1 || keep) && ws == nullptr) return (int)hipErrorInvalidValue;
  if (keep && ksplit == 1) return (int)hipErrorInvalidValue;
  DArgs a;
  a.A = (const bf16*)A;
  a.W = (const bf16*)W;
  a.bias = ksplit > 1 ? nullptr : (const bf16*)bias;
  a.C = ksplit > 1 ? ws : C;
  a.lda = lda; a.ldw = ldw; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K;
  a.units = units;
  a.gs = gs;
  a.msplit = msplit;
  a.packed = packed;
  a.stamps = g_dec_stamps;
  a.ksplit = ksplit;
  a.kt_split = kts;
  const int nwg = gs * ksplit * msplit;
  const int e = ksplit > 1 ? EPI_PARTIAL : epi;
  int err;
  if (tail) err = mt == 4 ? launch_v<4, kDepth, 8, 2, 1>(a, e, act, nwg, stream)
                 : mt == 8 ? launch_v<8, kDepth, 8, 2, 2>(a, e, act, nwg, stream)
                 : mt == 12 ? launch_v<12, kDepth, 8, 2, 3>(a, e, act, nwg, stream)
                            : launch_v<16, kDepth, 8, 2, 4>(a, e, act, nwg, stream);
  else if (mt <= 2) {  // 1-32 rows (the reference's 1-4 live sequences): a 2-4 KB A ring, so the W ring can be deep
    const int d = g_dec_depth >= 12 ? 12 : g_dec_depth >= 8 ? 8 : kDepth;
#define SK(MT_, D_) (nwv == 4 ? launch_v<MT_, D_, 4, 2>(a, e, act, nwg, stream) : launch_v<MT_, D_, 5, 2>(a, e, act, nwg, stream))
    err = mt == 1 ? (d == 12 ? SK(1, 12) : d == 8 ? SK(1, 8) : SK(1, kDepth))
                  : (d == 12 ? SK(2, 12) : d == 8 ? SK(2, 8) : SK(2, kDepth));
#undef SK
  } else if (g_dec_depth == 8 && mt == 4 && (nwv == 4 || nwv == 5))
    err = nwv == 4 ? launch_v<4, 8, 4, 2>(a, e, act, nwg, stream) : launch_v<4, 8, 5, 2>(a, e, act, nwg, stream);
  else if (g_dec_depth >= 6 && (mt == 4 || mt == 8) && (nwv == 4 || nwv == 5))
    err = nwv == 4 ? (mt == 4 ? launch_v<4, 6, 4, 2>(a, e, act, nwg, stream) : launch_v<8, 6, 4, 2>(a, e, act, nwg, stream))
                   : (mt == 4 ? launch_v<4, 6, 5, 2>(a, e, act, nwg, stream) : launch_v<8, 6, 5, 2>(a, e, act, nwg, stream));
  else if (nwv == 4) err = mt == 4 ? launch_v<4, kDepth, 4, 2>(a, e, act, nwg, stream)
                     : mt == 8 ? launch_v<8, kDepth, 4, 2>(a, e, act, nwg, stream)
                               : launch_v<16, kDepth, 4, 2>(a, e, act, nwg, stream);
  else if (nwv == 5) err = mt == 4 ? launch_v<4, kDepth, 5, 2>(a, e, act, nwg, stream)
                          : mt == 8 ? launch_v<8, kDepth, 5, 2>(a, e, act, nwg, stream)
                                    : launch_v<12, kDepth, 5, 2>(a, e, act, nwg, stream);
  else err = launch_v<12, kDepth, 8, 2>(a, e, act, nwg, stream);
  if (err || ksplit == 1 || keep) return err;
  return grag_splitk_reduce(ws, bias, C, ldc, M, N, ksplit, epi, act, stream);
}

GRAG_API int grag_gemm_decode(const void* A, const void* W, const void* bias, void* C, int lda, int ldw, int ldc,
                              int M, int N, int K, int epi, int act, int mt, int nwv, int ntw, int ksplit, int gs,
                              int packed, void* ws, hipStream_t stream) {
  return grag_gemm_decode_t(A, W, bias, C, lda, ldw, ldc, M, N, K, epi, act, mt, nwv, ntw, ksplit, gs, packed, 0, ws,
                            stream);
}

// y = epilogue(RMSNorm(res_in + sum_s planes[s]) * nw @ w^T) for M <= 4 rows (NRM kernel): the split-K RMSNorm
// of a decoder layer folded into the projection that consumes it.  planes: the producer's fp32 split-K planes
// [S][M][K] (16-B aligned); res_in [M][K] the residual stream before the add, res_out [M][K] after it
// (written by one workgroup; must not alias res_in); nw [K] the norm weight.  mt must be 1, one K-range
// (ksplit 1), epi 0 (no bias / act) or 1 (silu*mul), K <= 8160; other arguments as grag_gemm_decode_t.
GRAG_API int grag_gemm_decode_norm(const void* planes, int S, const void* res_in, void* res_out, const void* nw,
                                   float eps, const void* W, void* C, int ldw, int ldc, int M, int N, int K,
                                   int epi, int mt, int nwv, int ntw, int gs, int packed, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > kNrmRows || mt != 1 || ntw != 2 || (nwv != 4 && nwv != 5) || S < 1 || !planes || !res_in || !res_out ||
      !nw || res_in == res_out || (epi != EPI_STORE && epi != EPI_SILU))
    return (int)hipErrorInvalidValue;
  if (K % 64 != 0 || K < 64 || M * (K * 2 + 64) > kNrmLds || N % 32 != 0 || ldw % 8 != 0 || ldc % 4 != 0 ||
      (epi == EPI_SILU && N % 64 != 0) || packed < 0 || packed > 2 || (packed == 2 && N % 64 != 0))
    return (int)hipErrorInvalidValue;
  const int units = N / 32;
  if (gs <= 0) {
    if (units % nwv != 0) return (int)hipErrorInvalidValue;
    gs = units / nwv;
  }
  if (gs > units || (units + gs - 1) / gs > nwv) return (int)hipErrorInvalidValue;
  DArgs a{};
  a.A = nullptr;
  a.W = (const bf16*)W;
  a.bias = nullptr;
  a.C = C;
  a.lda = K; a.ldw = ldw; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K;
  a.units = units;
  a.gs = gs;
  a.msplit = 1;
  a.packed = packed;
  a.stamps = nullptr;
  a.ksplit = 1;
  a.kt_split = K / 64;
  a.nplanes = (const float*)planes;
  a.nS = S;
  a.nres_in = (const bf16*)res_in;
  a.nres_out = (bf16*)res_out;
  a.nw = (const bf16*)nw;
  a.neps = eps;
  return nwv == 4 ? launch_nrm<kDepth, 4>(a, epi, gs, stream) : launch_nrm<kDepth, 5>(a, epi, gs, stream);
}

// Producer half of the folded RMSNorm (1-4 rows): the split-K projection (EPI_PARTIAL planes into ws) whose
// last split per unit group adds the group's columns of all planes into `residual` [M][N] in place (bf16,
// the split-K RMSNorm's arithmetic) and writes that group's sums of squares per row to ss [gs][4].
// counters >= gs zeroed uint32 words (self-resetting).  mt 1, ntw 2, nwv 4 or 5, ksplit > 1, no tail.
// Returns the group count through *groups.
GRAG_API int grag_gemm_decode_red(const void* A, const void* W, void* residual, float* ss, unsigned* counters,
                                  int lda, int ldw, int M, int N, int K, int mt, int nwv, int ntw, int ksplit, int gs,
                                  void* ws, int* groups, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > kNrmRows || mt != 1 || ntw != 2 || (nwv != 4 && nwv != 5) || !A || !W || !residual || !ss ||
      !counters || !ws || K % 64 != 0 || K < 64 || N % 32 != 0 || lda % 8 != 0 || ldw % 8 != 0)
    return (int)hipErrorInvalidValue;
  const int units = N / 32;
  if (gs <= 0) {
    if (units % nwv != 0) return (int)hipErrorInvalidValue;
    gs = units / nwv;
  }
  if (gs > units || (units + gs - 1) / gs > nwv || gs > 1024) return (int)hipErrorInvalidValue;
  const int kt = K / 64;
  if (ksplit < 2) return (int)hipErrorInvalidValue;
  const int kts = (kt + ksplit - 1) / ksplit;
  ksplit = (kt + kts - 1) / kts;
  if (ksplit < 2) return (int)hipErrorInvalidValue;
  DArgs a{};
  a.A = (const bf16*)A;
  a.W = (const bf16*)W;
  a.C = ws;
  a.lda = lda; a.ldw = ldw; a.ldc = N;
  a.M = M; a.N = N; a.K = K;
  a.units = units;
  a.gs = gs;
  a.msplit = 1;
  a.packed = 0;
  a.ksplit = ksplit;
  a.kt_split = kts;
  a.rres = (bf16*)residual;
  a.rss = ss;
  a.rcnt = counters;
  if (groups) *groups = gs;
  const int nwg = gs * ksplit;
  if (nwv == 4)
    gemm_dec_kernel<EPI_PARTIAL, ACT_NONE, 1, kDepth, 4, 2, 0, 0, 1><<<nwg, 256, 0, stream>>>(a);
  else
    gemm_dec_kernel<EPI_PARTIAL, ACT_NONE, 1, kDepth, 5, 2, 0, 0, 1><<<nwg, 320, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// Consumer half: y = epilogue((x * nw) @ w^T / rms(x)) for M <= 4 rows, x = the residual stream the producer
// updated, rms from its per-group sums of squares ss [G][4] (mean over K) + eps.  epi 1 (silu*mul, ksplit
// 1) or 2 (fp32 planes into ws for a consumer that reduces them, ksplit > 1).  mt 1, ntw 2, nwv 4 / 5.
GRAG_API int grag_gemm_decode_scaled(const void* A, const void* nw, const float* ss, int G, float eps,
                                     const void* W, void* C, int lda, int ldw, int ldc, int M, int N, int K,
                                     int epi, int mt, int nwv, int ntw, int ksplit, int gs, void* ws,
                                     hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > kNrmRows || mt != 1 || ntw != 2 || (nwv != 4 && nwv != 5) || !A || !nw || !ss || G < 1 ||
      (epi != EPI_SILU && epi != EPI_PARTIAL) || K % 64 != 0 || K < 64 || N % 32 != 0 || lda % 8 != 0 ||
      ldw % 8 != 0 || ldc % 4 != 0 || (epi == EPI_SILU && N % 64 != 0))
    return (int)hipErrorInvalidValue;
  const int units = N / 32;
  if (gs <= 0) {
    if (units % nwv != 0) return (int)hipErrorInvalidValue;
    gs = units / nwv;
  }
  if (gs > units || (units + gs - 1) / gs > nwv) return (int)hipErrorInvalidValue;
  const int kt = K / 64;
  if (ksplit < 1) ksplit = 1;
  const int kts = (kt + ksplit - 1) / ksplit;
  ksplit = (kt + kts - 1) / kts;
  if ((epi == EPI_SILU) != (ksplit == 1) || (ksplit > 1 && !ws)) return (int)hipErrorInvalidValue;
  DArgs a{};
  a.A = (const bf16*)A;
  a.W = (const bf16*)W;
  a.C = ksplit > 1 ? ws : C;
  a.lda = lda; a.ldw = ldw; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K;
  a.units = units;
  a.gs = gs;
  a.msplit = 1;
  a.packed = 0;
  a.ksplit = ksplit;
  a.kt_split = kts;
  a.nw = (const bf16*)nw;
  a.nss = ss;
  a.nG = G;
  a.neps = eps;
  const int nwg = gs * ksplit;
#define SC(E, NW) gemm_dec_kernel<E, ACT_NONE, 1, kDepth, NW, 2, 0, 2, 0><<<nwg, 64 * NW, 0, stream>>>(a)
  if (epi == EPI_SILU) {
    if (nwv == 4) SC(EPI_SILU, 4); else SC(EPI_SILU, 5);
  } else {
    if (nwv == 4) SC(EPI_PARTIAL, 4); else SC(EPI_PARTIAL, 5);
  }
#undef SC
  return (int)hipGetLastError();
}
