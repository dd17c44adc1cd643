// Unified MFMA flash-attention forward for gfx950.
//
// One kernel template serves three ops of SURVEY §2.7:
//   N1f  causal GQA prefill over the paged KV cache (chunked prefill too),
//   N1g  paged decode (q_len = 1) with split-KV ("flash-decoding") + combine,
//   N2c  bidirectional encoder attention over contiguous packed QKV with
//        per-sequence lengths (padding mask).
//
// Work decomposition.  Query rows are GQA-packed: for kv head h of sequence s
// the rows are (position p, group g) flattened as r = p*G + g, so the G query
// heads that share one KV head read every K/V tile once.  A wave owns 16 rows,
// a workgroup NW waves.  Keys stream through LDS in 64-key tiles.
//
// MFMA formulation (cdna_hip_programming.md §B attention, "swapped QK^T"):
//   S^T[key][q] = K · Q^T      A = K tile from LDS (ds_read_b128, XOR-swizzled
//                              rows, T2), B = Q^T held in registers.
//   The accumulator puts all keys of one query row in one lane's registers, so
//   the row max/sum need only 2 cross-lane steps (xor 16, xor 32).
//   O^T[d][q] += V^T · P^T     A = V^T via ds_read_b64_tr_b16 (T10) from a
//                              swizzled V image, B = P^T taken straight from
//                              the S^T accumulators (k-slot permutation chosen
//                              so no lane movement is needed).
// Both products use v_mfma_f32_16x16x32_bf16.  Online softmax runs in the
// log2 domain (exp2).
#include "common.h"

typedef float f32x2_t __attribute__((ext_vector_type(2)));

using namespace grag;

namespace {

constexpr int KT = 64;  // keys per tile
constexpr int kPrefillMaxBlocks = 2048;  // 8-wave prefill: block-table window held in LDS
constexpr float kRescaleLog2 = 8.f;      // 8-wave prefill: deferred-rescale threshold (log2 units)

struct AttnParams {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  bf16* out;
  float* part_o;   // [nsplit, T, Hq, D] (split mode only)
  float* part_ml;  // [nsplit, T, Hq, 2]
  const int32_t* block_tables;
  const int32_t* q_start;  // [nseq+1]
  const int32_t* ctx_len;  // [nseq]
  int q_stride, kv_stride, out_stride;
  int Hq, Hkv, G, BS, bt_stride;
  int tiles_per_seq, num_splits, split_len, total_q;
  float scale_log2;
  int causal;
  int nblocks;  // KV blocks in the cache: the index guard's bound for block-table entries (common.h)
  int xcd_group;  // decode: consecutive sequences of one (kv head, split) run on one XCD (g_decode_xcd)
  // shared-prefix decode (paged_decode_prefix_kernel): the rows of a group share their first pre_len[row]
  // keys (whole KV blocks, one set of block ids), cut into parts of pre_part[row] keys; work item i of the
  // prefix kernel is pre_items[i] = (first row, end row, first key, end key) of one part of one group.
  // null pre_len = no sharing
  const int32_t* pre_len;    // [nseq]
  const int32_t* pre_part;   // [nseq]
  const int32_t* pre_items;  // [n items, 4]
  float* pre_o;              // [pre_planes, T, Hq, D]: the prefix parts' unnormalised O (plane = part index)
  float* pre_ml;             // [pre_planes, T, Hq, 2]: their (m, l)
  int pre_planes;
  // small-batch decode with the RoPE pass folded in (paged_decode_mw_kernel FR): q and the new token's K/V come
  // from the qkv projection's S fp32 split-K planes [S][T][rq_ld] (rq_ld = (Hq + 2 Hkv) D), plus bias and NeoX
  // RoPE at rq_pos[token]; the new K/V is stored to cache slot rq_slot[token] by the sequence's last split
  const float* rq_planes;
  size_t rq_plane;  // elements per plane
  int rq_S, rq_ld;
  const bf16* rq_bias;      // [(Hq + 2 Hkv) D] or null
  const int32_t* rq_pos;    // [T]
  const float* rq_cs;       // [npos, D]: cos | sin
  const int32_t* rq_slot;   // [T]
  int rq_nslots, rq_npos;
};

// grag_attn_decode_xcd(1): decode workgroups remapped so that sequences adjacent in the batch run on the same
// XCD at about the same time (their shared prefix K/V from that XCD's L2).  Off by default: measured
// (scripts/mb_shared_prefix.py, profiles/mb_shared_prefix_r6.json) prefix-sharing rows already read their
// shared blocks mostly from the Infinity Cache in any order (B192 ctx 1792: 122.7 us unshared -> 105.8 us
// shared, adjacent or shuffled alike), and the remap deals whole split columns to XCD halves: B256 with a
// 2048 + 512-key split plan 233 -> 292 us
int g_decode_xcd = 0;

// Chunk (16 B) swizzle for the K image read as row fragments by ds_read_b128.
template <int D>
__device__ __forceinline__ int kswz(int row) {
  if constexpr (D == 128) return row & 15;
  else if constexpr (D == 64) return (row >> 1) & 7;
  else return (row >> 2) & 3;
}
// Chunk (16 B) swizzle for the V image read with ds_read_b64_tr_b16: a 32-lane
// half reads 8 consecutive rows x 4 8-byte units; these XORs spread them over
// all 64 banks (derivation in docs/kernels.md).
template <int D>
__device__ __forceinline__ int vswz(int row) {
  if constexpr (D == 128) return (row & 7) << 1;
  else if constexpr (D == 64) return ((row >> 1) & 3) << 1;
  else return ((row >> 2) & 1) << 1;
}

typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;

// One LDS-DMA wave instruction (global_load_lds_dwordx4): 16 B per lane from
// each lane's `src` into the 1 KiB LDS block at wave-uniform `lds_dst`
// (lane-linear).  Issued from inline asm so hipcc's waitcnt pass does not see
// an LDS write it cannot disambiguate between ring stages (it would put a
// vmcnt(0) in front of every ds_read); completion is tracked only by the
// caller's explicit counted `s_waitcnt vmcnt(N)` (cdna guide §5.7 recipe:
// M0 saved, set, used and restored inside one statement).
template <bool NT = false>
__device__ __forceinline__ void glds16(const void* src, void* lds_dst) {
  const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds_dst;
  const uint32_t lu = __builtin_amdgcn_readfirstlane(lds);
  uint32_t keep;
  if constexpr (NT) {  // non-temporal: once-read streams (decode K/V, MI355X_MICROARCH 'nt-weights')
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(lu)
        : "memory");
  } else {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(lu)
        : "memory");
  }
}

// The same LDS-DMA with the address as a wave-uniform 64-bit base in SGPRs plus a 32-bit per-lane byte
// offset (global_load_lds saddr form): no 64-bit VALU address arithmetic per load.
__device__ __forceinline__ void glds16_s(const void* sbase, uint32_t voff, void* lds_dst) {
  const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds_dst;
  const uint32_t lu = __builtin_amdgcn_readfirstlane(lds);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lu)
      : "memory");
}

template <int D, int NW, bool PAGED>
__global__ __launch_bounds__(64 * NW) void attn_fwd_kernel(AttnParams p) {
  constexpr int CPR = D / 8;      // 16-B chunks per K/V row
  constexpr int RB = 2 * D;       // bytes per K/V row
  constexpr int NC = D / 32;      // k-chunks of the QK^T product
  constexpr int ND = D / 16;      // 16-dim output tiles
  __shared__ __attribute__((aligned(16))) char smem[2 * KT * RB];
  char* k_lds = smem;
  char* v_lds = smem + KT * RB;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h4 = lane >> 4, li = lane & 15;
  const int seq = blockIdx.x / p.tiles_per_seq, tile = blockIdx.x % p.tiles_per_seq;
  const int kvh = blockIdx.y, split = blockIdx.z;
  const int q0 = p.q_start[seq], qlen = p.q_start[seq + 1] - q0;
  const int ctx = p.ctx_len[seq];
  const int G = p.G;
  const int nrows = qlen * G;
  const int row_base = tile * 16 * NW;
  if (row_base >= nrows) return;
  const int my_row = row_base + wave * 16 + li;
  const bool row_valid = my_row < nrows;
  const int pq = row_valid ? my_row / G : 0;
  const int g = row_valid ? my_row % G : 0;

  int kv_lo = split * p.split_len;
  int kv_hi = min(ctx, kv_lo + p.split_len);
  if (p.causal) {
    const int last_row = min(row_base + 16 * NW, nrows) - 1;
    kv_hi = min(kv_hi, ctx - qlen + last_row / G + 1);
  }
  if (kv_lo >= kv_hi && p.num_splits > 1) return;  // combine skips empty splits

  // Q^T fragments: lane holds Q[row li][32c + 8*h4 .. +8]
  bf16x8_t qf[NC];
  {
    const bf16* qp = p.q + (size_t)(q0 + pq) * p.q_stride + (size_t)(kvh * G + g) * D + 8 * h4;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (row_valid) qf[c] = *reinterpret_cast<const bf16x8_t*>(qp + 32 * c);
      else qf[c] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const int key_lim = p.causal ? (ctx - qlen + pq + 1) : ctx;  // keys j < key_lim visible
  // the smallest limit among the wave's valid rows (its first row's): tiles ending at or below it need no mask
  const int wrow0 = min(row_base + __builtin_amdgcn_readfirstlane(wave) * 16, nrows - 1);
  const int wave_lim_min = min(kv_hi, p.causal ? ctx - qlen + wrow0 / G + 1 : ctx);

  float m = -INFINITY, lsum = 0.f;
  f32x4_t o[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) o[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int kt0 = kv_lo; kt0 < kv_hi; kt0 += KT) {
    __syncthreads();  // previous tile fully consumed
    // cooperative K/V tile load: global (16 B/lane) -> swizzled LDS image
    for (int c = threadIdx.x; c < KT * CPR; c += 64 * NW) {
      const int r = c / CPR, ch = c % CPR;
      const int j = kt0 + r;
      bf16x8_t kk = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      bf16x8_t vv = kk;
      if (j < kv_hi) {
        size_t off;
        if constexpr (PAGED) {
          int blk = p.block_tables[(size_t)seq * p.bt_stride + j / p.BS];
          if (!index_ok(blk, p.nblocks, ERR_BLOCK_PREFILL)) blk = 0;
          off = (((size_t)blk * p.Hkv + kvh) * p.BS + (j % p.BS)) * D + ch * 8;
        } else {
          off = (size_t)(q0 + j) * p.kv_stride + (size_t)kvh * D + ch * 8;
        }
        kk = *reinterpret_cast<const bf16x8_t*>(p.k + off);
        vv = *reinterpret_cast<const bf16x8_t*>(p.v + off);
      }
      *reinterpret_cast<bf16x8_t*>(k_lds + r * RB + ((ch ^ kswz<D>(r)) << 4)) = kk;
      *reinterpret_cast<bf16x8_t*>(v_lds + r * RB + ((ch ^ vswz<D>(r)) << 4)) = vv;
    }
    __syncthreads();

    // S^T = K Q^T for 4 key sub-tiles of 16
    f32x4_t s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int row = 16 * t + li;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bf16x8_t a =
            *reinterpret_cast<const bf16x8_t*>(k_lds + row * RB + (((4 * c + h4) ^ kswz<D>(row)) << 4));
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[c], s[t], 0, 0, 0);
      }
    }
    // scale + mask; this lane holds keys kt0 + 16t + 4*h4 + r of query row li.  The mask runs only on
    // tiles that reach the wave's first row's limit (a real wave-uniform branch, see attn_prefill_kernel)
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[t][r] *= p.scale_log2;
    if (kt0 + KT > wave_lim_min) {
      asm volatile("");
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt0 + 16 * t + 4 * h4 + r;
          if (key >= key_lim || key >= kv_hi) s[t][r] = -INFINITY;
        }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[t][r]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m, tmax);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f(m - m_use);
    m = m_new;
    lsum *= alpha;
#pragma unroll
    for (int n = 0; n < ND; ++n) o[n] *= alpha;
    float pr[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pr[t][r] = exp2f(s[t][r] - m_use);
        lsum += pr[t][r];
      }

    // O^T += V^T P^T over two 32-key chunks
    const int tq = li >> 2, tp = li & 3;  // tr-read: this lane addresses row tq, unit tp
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      bf16x8_t bp;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bp[r] = f2bits(pr[2 * cc][r]);
        bp[4 + r] = f2bits(pr[2 * cc + 1][r]);
      }
      const int r0 = 32 * cc + 4 * h4 + tq;  // row of first block
      const int r1 = r0 + 16;                // row of second block
#pragma unroll
      for (int n = 0; n < ND; ++n) {
        const int unit = 4 * n + tp;  // 8-byte unit within the row
        const int b0 = r0 * RB + ((unit ^ (vswz<D>(r0) << 1)) << 3);
        const int b1 = r1 * RB + ((unit ^ (vswz<D>(r1) << 1)) << 3);
        const bf16x4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b0));
        const bf16x4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b1));
        const bf16x8_t a = bf16x8_t{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bp, o[n], 0, 0, 0);
      }
    }
  }

  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (!row_valid) return;
  const int tok = q0 + pq, head = kvh * G + g;
  if (p.num_splits > 1) {
    float* po = p.part_o + (((size_t)split * p.total_q + tok) * p.Hq + head) * D;
#pragma unroll
    for (int n = 0; n < ND; ++n)
      *reinterpret_cast<float4*>(po + 16 * n + 4 * h4) = make_float4(o[n][0], o[n][1], o[n][2], o[n][3]);
    if (h4 == 0) {
      float* pm = p.part_ml + (((size_t)split * p.total_q + tok) * p.Hq + head) * 2;
      pm[0] = m;
      pm[1] = lsum;
    }
  } else {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16* op = p.out + (size_t)tok * p.out_stride + (size_t)head * D;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      bf16x4_t w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = f2bits(o[n][r] * inv);
      *reinterpret_cast<bf16x4_t*>(op + 16 * n + 4 * h4) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// Paged prefill, 8-wave variant (nw code 5): more query rows per K/V tile and
// K/V streamed by LDS-DMA into a 2-stage ring.
//
// The 4-wave kernel above stages 64 GQA rows per 32 KiB K/V tile through
// registers, so every tile costs a full global->LDS round trip per 64 rows
// and the load latency sits in front of the MFMAs.  Here a workgroup is 8
// waves x RPW row groups of 16 = 256 rows (36 positions x 7 heads at GQA 7):
//   * K and V tiles arrive by global_load_lds_dwordx4 (1 KiB per wave
//     instruction, lane-linear LDS destination, XOR swizzle applied to the
//     per-lane SOURCE chunk — rule 21), tile t+1 issued right after the
//     barrier that opens tile t, so its flight overlaps tile t's MFMAs;
//   * one barrier per tile: s_waitcnt vmcnt(0) (own pieces of tile t landed)
//     then the barrier (everyone's pieces landed AND everyone finished tile
//     t-1, whose stage the next issue overwrites);
//   * every K fragment (ds_read_b128) and V^T fragment (ds_read_b64_tr_b16) a
//     wave reads feeds RPW MFMAs (one per row group), halving LDS reads per
//     FLOP against the 4-wave kernel;
//   * the workgroup's block-table window sits in LDS, so no dependent global
//     load precedes the DMA of a tile;
//   * causal: a row group skips the tiles wholly above its diagonal (wave-
//     uniform test), and the heaviest (latest) q tiles are dispatched first.
// The math (swapped QK^T, exp2 online softmax, P^T straight from the S^T
// accumulators) is the 4-wave kernel's.
//
// NS = ring stages: 2 issues tile t+1 after the barrier that opens tile t and
// waits vmcnt(0) at the next tile (one barrier per tile, all 8 waves in step);
// 3 runs the staggered ping-pong schedule described at its loop (two barrier
// intervals per tile, waves 4-7 one interval behind).  Barriers are raw
// s_barrier: __syncthreads() would drain the younger tile with a vmcnt(0).
template <int D, int RPW, int NS, int NW = 8>
__global__ __launch_bounds__(64 * NW) void attn_prefill_kernel(AttnParams p) {
  static_assert(NS == 2 || NW == 8, "the staggered schedule pairs waves w and w + 4 on one SIMD");
  constexpr int RB = 2 * D;            // bytes per K/V row
  constexpr int CPR = D / 8;           // 16-B chunks per row
  constexpr int NC = D / 32;
  constexpr int ND = D / 16;
  constexpr int TILE = KT * RB;        // bytes per K (or V) tile
  constexpr int NP = TILE / 1024;      // LDS-DMA pieces per tile per tensor
  constexpr int PPW = NP / NW;         // pieces per wave per tensor
  constexpr int RPP = 1024 / RB;       // rows per piece
  constexpr int ROWS = 16 * RPW * NW;  // GQA rows per workgroup
  constexpr int BS = 16;               // KV block size (launcher falls back to the 4-wave kernel otherwise)
  constexpr int MAXB = kPrefillMaxBlocks;  // block-table window in LDS (32 K keys)
  static_assert(PPW >= 1 && PPW * NW == NP, "piece split");
  static_assert(NS == 2 || NS == 3, "ring stages");
  __shared__ __attribute__((aligned(16))) char smem[NS * 2 * TILE + MAXB * 4];
  int* bt_lds = reinterpret_cast<int*>(smem + NS * 2 * TILE);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h4 = lane >> 4, li = lane & 15;
  const int tiles = p.tiles_per_seq;
  const int seq = blockIdx.x / tiles;
  const int tile = tiles - 1 - (int)(blockIdx.x % tiles);
  const int kvh = blockIdx.y;
  const int q0 = p.q_start[seq], qlen = p.q_start[seq + 1] - q0;
  const int ctx = p.ctx_len[seq];
  const int G = p.G;
  const int nrows = qlen * G;
  const int row_base = tile * ROWS;
  if (row_base >= nrows) return;
  const int last_row = min(row_base + ROWS, nrows) - 1;
  const int kv_hi = p.causal ? min(ctx, ctx - qlen + last_row / G + 1) : ctx;

  // the whole block-table window goes to LDS once: the per-tile DMA addresses then come from
  // ds_reads (lgkmcnt) — a global/flat read there would need a vmcnt wait that drains the K/V
  // pieces in flight.  The launcher guarantees bt_stride <= MAXB.
  const int nb = (kv_hi + BS - 1) / BS;
  const int32_t* bt = p.block_tables + (size_t)seq * p.bt_stride;
  for (int i = threadIdx.x; i < nb; i += 64 * NW) {
    int b = bt[i];
    if (!index_ok(b, p.nblocks, ERR_BLOCK_PREFILL)) b = 0;  // reported; block 0 read instead of faulting
    bt_lds[i] = b;
  }

  bf16x8_t qf[RPW][NC];
  int key_lim[RPW];  // this lane's row limit
  bool valid[RPW];
  int pq[RPW], gq[RPW];
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int grow = row_base + (wave * RPW + j) * 16;
    const int my_row = grow + li;
    valid[j] = my_row < nrows;
    pq[j] = valid[j] ? my_row / G : 0;
    gq[j] = valid[j] ? my_row % G : 0;
    key_lim[j] = p.causal ? ctx - qlen + pq[j] + 1 : ctx;
    const bf16* qp = p.q + (size_t)(q0 + pq[j]) * p.q_stride + (size_t)(kvh * G + gq[j]) * D + 8 * h4;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (valid[j]) qf[j][c] = *reinterpret_cast<const bf16x8_t*>(qp + 32 * c);
      else qf[j][c] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  // Q fragments and the block-table window landed (a compiler-visible wait: without it hipcc's
  // waitcnt pass cannot prove the Q loads retired on the loop back-edge and puts a vmcnt(0) in
  // front of the first MFMA of every tile, which also drains the K/V DMA issued for the next tile)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  __syncthreads();  // block-table window visible
  // smallest key limit over the wave's rows (its first row), wave-uniform:
  // tiles ending below it need no mask
  const int wrow0 = row_base + __builtin_amdgcn_readfirstlane(wave) * RPW * 16;
  const int wave_lim_min = min(kv_hi, p.causal ? ctx - qlen + min(wrow0, nrows - 1) / G + 1 : ctx);

  const int lrow = lane / CPR, lch = lane % CPR;
  // A wave's PPW pieces are PPW * RPP consecutive keys inside one KV block (tiles start on block
  // boundaries), so the block lookup and the base address are wave-uniform (SGPRs) and each lane adds a
  // 32-bit byte offset.  Keys past the context end re-read its last key (finite V for the masked keys,
  // as a per-key clamp would): the wave's block is clamped to the last valid one and so is the slot.
  static_assert(BS % (PPW * RPP) == 0 && KT % BS == 0, "a wave's DMA rows sit in one KV block");
  const int last_blk = (kv_hi - 1) / BS, last_slot = (kv_hi - 1) % BS;
  const int wrow = __builtin_amdgcn_readfirstlane(wave) * PPW * RPP;
  auto issue = [&](int kt0, int stage) {
    char* kdst = smem + stage * 2 * TILE;
    char* vdst = kdst + TILE;
    const int blk = __builtin_amdgcn_readfirstlane(bt_lds[min((kt0 + wrow) / BS, last_blk)]);
    const size_t base = ((size_t)blk * p.Hkv + kvh) * BS * D;
    const bf16* kb = p.k + base;
    const bf16* vb = p.v + base;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = wave * PPW + i;
      const int row = piece * RPP + lrow;
      const int slot = kt0 + row < kv_hi ? row % BS : last_slot;
      glds16_s(kb, (uint32_t)(slot * D + ((lch ^ kswz<D>(row)) << 3)) * 2u, kdst + piece * 1024);
      glds16_s(vb, (uint32_t)(slot * D + ((lch ^ vswz<D>(row)) << 3)) * 2u, vdst + piece * 1024);
    }
  };

  float m[RPW], lsum[RPW];
  f32x4_t o[RPW][ND];
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    m[j] = -INFINITY;
    lsum[j] = 0.f;
#pragma unroll
    for (int n = 0; n < ND; ++n) o[j][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  const int ntiles = (kv_hi + KT - 1) / KT;
  bf16x8_t bp[RPW][2];
  // phase A: S^T for tile t from the K image at k_lds, softmax -> P^T fragments bp (rescales O)
  auto phaseA = [&](const int kt0, const char* k_lds) {
    // S^T = K Q^T: every K fragment read once, used by all RPW row groups
    f32x4_t s[RPW][4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int row = 16 * tt + li;
      bf16x8_t a[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c)
        a[c] = *reinterpret_cast<const bf16x8_t*>(k_lds + row * RB + (((4 * c + h4) ^ kswz<D>(row)) << 4));
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        s[j][tt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < NC; ++c) s[j][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], qf[j][c], s[j][tt], 0, 0, 0);
      }
    }
    // masking is needed only on tiles that reach the wave's diagonal / the context end.  The empty
    // volatile asm keeps this a real wave-uniform branch: without it hipcc if-converted the selects
    // into ~100 compares / cndmasks per tile on EVERY tile (the prefill loop was VALU-bound)
    if (kt0 + KT > wave_lim_min) {
      asm volatile("");
#pragma unroll
      for (int j = 0; j < RPW; ++j)
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kt0 + 16 * tt + 4 * h4 + r;
            s[j][tt][r] = (key >= key_lim[j] || key >= kv_hi) ? -INFINITY : s[j][tt][r];
          }
    }
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      // raw scores: the softmax scale (log2 domain) is folded into the exponent's FMA, and the
      // row max is taken before scaling (the scale is positive)
      float tmax = -INFINITY;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) tmax = __builtin_fmaxf(tmax, s[j][tt][r]);
      tmax = __builtin_fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = __builtin_fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      // deferred rescale (cdna guide §5.5 T13): the running max m (scaled units) moves only when a
      // row's tile max passes it by more than kRescaleLog2, so p = 2^(s c - m) stays <= 2^8 in fp32 and
      // the O / l rescale runs on the few tiles where some row of the wave moved (wave-uniform branch;
      // every lane then takes its exact new max, so O and l always see the same factor)
      const float m_cand = __builtin_fmaxf(m[j], tmax * p.scale_log2);
      if (__any(m_cand > m[j] + kRescaleLog2)) {
        const float m_use = m_cand == -INFINITY ? 0.f : m_cand;
        const float alpha = __builtin_amdgcn_exp2f(m[j] - m_use);
        m[j] = m_cand;
        lsum[j] *= alpha;
#pragma unroll
        for (int n = 0; n < ND; ++n) o[j][n] *= alpha;
      }
      const float nm = m[j] == -INFINITY ? 0.f : -m[j];
      // exponent arguments and the row-sum adds as packed f32 pairs (v_pk_fma_f32 / v_pk_add_f32: one issue
      // per two lanes' worth of work -- the softmax VALU, not the MFMA pipe, paces this loop)
      const f32x2_t sc2 = {p.scale_log2, p.scale_log2}, nm2 = {nm, nm};
      f32x2_t ls2 = {0.f, 0.f};
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int rp = 0; rp < 2; ++rp) {
          const f32x2_t x0 = __builtin_elementwise_fma(f32x2_t{s[j][2 * cc][2 * rp], s[j][2 * cc][2 * rp + 1]}, sc2, nm2);
          const f32x2_t x1 =
              __builtin_elementwise_fma(f32x2_t{s[j][2 * cc + 1][2 * rp], s[j][2 * cc + 1][2 * rp + 1]}, sc2, nm2);
          const f32x2_t p0 = {__builtin_amdgcn_exp2f(x0[0]), __builtin_amdgcn_exp2f(x0[1])};
          const f32x2_t p1 = {__builtin_amdgcn_exp2f(x1[0]), __builtin_amdgcn_exp2f(x1[1])};
          ls2 += p0 + p1;
          bp[j][cc][2 * rp] = f2bits(p0[0]);
          bp[j][cc][2 * rp + 1] = f2bits(p0[1]);
          bp[j][cc][4 + 2 * rp] = f2bits(p1[0]);
          bp[j][cc][4 + 2 * rp + 1] = f2bits(p1[1]);
        }
      lsum[j] += ls2[0] + ls2[1];
    }
  };
  // phase B: O^T += V^T P^T from the V image at v_lds
  auto phaseB = [&](const char* v_lds) {
    // O^T += V^T P^T: every V^T fragment read once, used by all RPW row groups
    const int tq = li >> 2, tp = li & 3;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int r0 = 32 * cc + 4 * h4 + tq;
      const int r1 = r0 + 16;
      bf16x8_t a[ND];
#pragma unroll
      for (int n = 0; n < ND; ++n) {
        const int unit = 4 * n + tp;
        const int b0 = r0 * RB + ((unit ^ (vswz<D>(r0) << 1)) << 3);
        const int b1 = r1 * RB + ((unit ^ (vswz<D>(r1) << 1)) << 3);
        const bf16x4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b0));
        const bf16x4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b1));
        a[n] = bf16x8_t{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      }
#pragma unroll
      for (int n = 0; n < ND; ++n)
#pragma unroll
        for (int j = 0; j < RPW; ++j) o[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[n], bp[j][cc], o[j][n], 0, 0, 0);
    }
  };
  auto bar = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  issue(0, 0);
  if constexpr (NS == 2) {
    for (int t = 0; t < ntiles; ++t) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      if (t + 1 < ntiles) issue((t + 1) * KT, (t + 1) & 1);
      const char* k_lds = smem + (t & 1) * 2 * TILE;
      phaseA(t * KT, k_lds);
      phaseB(k_lds + TILE);
    }
  } else {
    // Staggered ping-pong over a 3-stage ring (cdna guide "Two waves per SIMD"): waves 4-7 run one
    // barrier interval behind waves 0-3, and every tile is two intervals, A (QK^T MFMAs + softmax VALU)
    // then B (PV MFMAs), so on each SIMD one wave's softmax overlaps its partner's MFMAs instead of
    // both waves stalling the matrix core together.  Leading waves: barrier 2t opens A(t), 2t+1 opens
    // B(t); lagging waves: 2t+1 and 2t+2.  Tile t+2 is issued after the barrier that opens B(t) into the
    // stage of tile t-1, whose last reader (the lagging B(t-1)) ended at that barrier.  RAW: a leading
    // wave retires tile t (vmcnt(2 PPW): t+1 stays in flight) before barrier 2t; a lagging wave retires
    // everything it issued (vmcnt(0)) before the barrier opening its B, which precedes every first read
    // of those tiles (the leading A of tile t+1 at barrier 2t+2).
    const bool lag = wave >= NW / 2;
    if (ntiles > 1) issue(KT, 1);
    if (lag) {
      if (ntiles > 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPW) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();  // barrier 0: the leading A(0) reads tile 0
    }
    int stage = 0;  // t % 3
    for (int t = 0; t < ntiles; ++t) {
      if (!lag) {
        if (t + 1 < ntiles)
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPW) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      bar();
      const char* k_lds = smem + stage * 2 * TILE;
      phaseA(t * KT, k_lds);
      if (lag) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      if (t + 2 < ntiles) issue((t + 2) * KT, stage == 0 ? 2 : stage - 1);
      phaseB(k_lds + TILE);
      stage = stage == 2 ? 0 : stage + 1;
    }
    if (!lag) bar();  // the lagging waves' last B
  }

#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    float l = lsum[j];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (!valid[j]) continue;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* op = p.out + (size_t)(q0 + pq[j]) * p.out_stride + (size_t)(kvh * G + gq[j]) * D;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      bf16x4_t w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = f2bits(o[j][n][r] * inv);
      *reinterpret_cast<bf16x4_t*>(op + 16 * n + 4 * h4) = w;
    }
  }
}

// Prefix parts (planes) of decode row `seq` whose first `pre` keys a shared prefix covers; a part length or
// count out of range is reported and gives 0 (the caller then attends to all keys itself).
__device__ __forceinline__ int prefix_planes(const AttnParams& p, int seq, int pre) {
  const int part = p.pre_part[seq];
  if (part <= 0) {
    report_index_error(ERR_PREFIX_GROUP, part);
    return 0;
  }
  const int nv = (pre + part - 1) / part;
  return index_ok(nv, p.pre_planes + 1, ERR_PREFIX_GROUP) ? nv : 0;
}

// Keys [0, pre) of decode row `seq` that a shared-prefix part covers (paged_decode_prefix_kernel); 0 without
// sharing.  A value outside [0, ctx) is reported and treated as 0: the row then attends to all its keys
// itself and merges nothing, which is still the exact result.
__device__ __forceinline__ int prefix_of(const AttnParams& p, int seq, int ctx) {
  if (p.pre_len == nullptr) return 0;
  const int pre = p.pre_len[seq];
  if (pre == 0 || !index_ok(pre, ctx, ERR_PREFIX_GROUP)) return 0;
  return prefix_planes(p, seq, pre) > 0 ? pre : 0;
}

// Merge the prefix parts of (tok, head) into a decode wave's running state (m, l, O) -- lane (li, h4) holds
// O[16 n + 4 h4 + r], the layout the prefix kernel wrote its parts in.  m stays the reference of l and O.
template <int D>
__device__ __forceinline__ void merge_prefix(const AttnParams& p, int tok, int head, int pre, int h4, float& m,
                                             float& l, f32x4_t (&o)[D / 16]) {
  constexpr int ND = D / 16;
  const int nv = prefix_planes(p, tok, pre);
  float M = m;
  for (int s = 0; s < nv; ++s) M = fmaxf(M, p.pre_ml[(((size_t)s * p.total_q + tok) * p.Hq + head) * 2]);
  if (M == -INFINITY) return;
  const float a = exp2f(m - M);
  l *= a;
#pragma unroll
  for (int n = 0; n < ND; ++n) o[n] *= a;
  for (int s = 0; s < nv; ++s) {
    const size_t base = ((size_t)s * p.total_q + tok) * p.Hq + head;
    const float w = exp2f(p.pre_ml[base * 2] - M);
    l += p.pre_ml[base * 2 + 1] * w;
    const float* po = p.pre_o + base * D + 4 * h4;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const float4 v = *reinterpret_cast<const float4*>(po + 16 * n);
      o[n] += f32x4_t{v.x, v.y, v.z, v.w} * w;
    }
  }
  m = M;
}

// ---------------------------------------------------------------------------
// Decode (q_len == 1) specialisation: one wave per (sequence, kv head, split).
// The GQA group's G <= 16 query heads are the 16 MFMA columns.  K/V tiles are
// fetched by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave instruction,
// destination lane-linear, so the XOR swizzle of the K and V images is applied
// to the per-lane SOURCE address — cdna guide §5.4 rule 21) into a 2-stage
// ring; the block-table entry of every 4..16-key group is wave-uniform and
// comes through the scalar cache, so no vector load sits between two tiles.
// Tile t+1 is issued before tile t is computed and retired with a counted
// vmcnt, keeping 32 KiB per wave in flight under the MFMA/softmax work.
//
// NS > 2 stages (round 4): NS - 1 tiles stay in flight while one is computed.
// The ring is what bounds the bytes in flight per CU: with 32-key tiles a
// 2-stage ring (32 KiB per wave, 5 waves per CU) keeps 5 x 16 KiB = 80 KiB
// in flight, a 4-stage ring (64 KiB per wave, 2 waves per CU) 2 x 48 KiB =
// 96 KiB, and 512 resident waves divide the (sequence x kv-head) grid of
// power-of-two batches into whole rounds (2 048 / 4 096 waves at 512 / 1024
// live sequences) where 1 280 resident waves leave a 0.2-0.6 partial round.
template <int D, int TK, int NS = 2, bool NT = false>
__global__ __launch_bounds__(64) void paged_decode_kernel(AttnParams p) {
  static_assert(TK == 32 || TK == 64, "keys per tile");
  static_assert(NS >= 2 && NS <= 4, "ring stages");
  constexpr int NT16 = TK / 16, NCC = TK / 32;
  constexpr int RB = 2 * D;
  constexpr int CPR = D / 8;
  constexpr int NC = D / 32;
  constexpr int ND = D / 16;
  constexpr int TILE = TK * RB;      // bytes per K (or V) tile
  constexpr int NI = TILE / 1024;    // LDS-DMA instructions per tile per tensor
  constexpr int RPI = 1024 / RB;     // rows per instruction
  static_assert((NS - 1) * 2 * NI <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[NS * 2 * TILE];

  const int lane = threadIdx.x;
  const int h4 = lane >> 4, li = lane & 15;
  int seq = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z;
  if (p.xcd_group) {  // logical ids dealt to one XCD are contiguous, sequence index fastest (common.h xcd_remap)
    const int nseq = gridDim.x;
    const int lg = xcd_remap(blockIdx.x + nseq * (blockIdx.y + gridDim.y * blockIdx.z),
                             nseq * gridDim.y * gridDim.z);
    seq = lg % nseq;
    kvh = (lg / nseq) % gridDim.y;
    split = lg / (nseq * gridDim.y);
  }
  const int ctx = p.ctx_len[seq];
  const int pre = prefix_of(p, seq, ctx);  // keys a shared-prefix part already covered (0: none)
  const int kv_lo = pre + split * p.split_len;
  const int kv_hi = min(ctx, kv_lo + p.split_len);
  if (kv_lo >= kv_hi) return;
  const int G = p.G;
  const bool row_valid = li < G;
  const int tok = p.q_start[seq];
  bf16x8_t qf[NC];
  {
    const bf16* qp = p.q + (size_t)tok * p.q_stride + (size_t)(kvh * G + (row_valid ? li : 0)) * D + 8 * h4;
#pragma unroll
    for (int c = 0; c < NC; ++c) qf[c] = *reinterpret_cast<const bf16x8_t*>(qp + 32 * c);
  }
  const int32_t* bt = p.block_tables + (size_t)seq * p.bt_stride;
  const int lrow = lane / CPR, lch = lane % CPR;
  // Block ids of a 64-block window live one per lane; readlane with a
  // wave-uniform index hands them to the scalar unit, so no vector load ever
  // sits between two LDS-DMA issues (a vector load there costs a vmcnt(0)
  // drain of the whole pipeline).
  // A 64-key tile never straddles a window (64 blocks x BS keys, BS % 16 == 0),
  // so the window is refreshed at most once per tile, outside the unrolled
  // issue loop (once per split for split_len <= 64*BS).
  const int nblk_seq = (ctx + p.BS - 1) / p.BS;
  int win = (kv_lo / p.BS) >> 6;
  int bvec = bt[min((win << 6) + lane, nblk_seq - 1)];
  if (!index_ok(bvec, p.nblocks, ERR_BLOCK_DECODE)) bvec = 0;
  // Retire the Q and block-id loads with a wait hipcc understands, so its
  // scoreboard is empty when the asm-issued LDS-DMA pipeline starts (else it
  // re-waits vmcnt(0) for them inside every iteration).
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll
  for (int c = 0; c < NC; ++c) asm volatile("" : "+v"(qf[c]));
  asm volatile("" : "+v"(bvec));

  auto issue = [&](int kt0, int stage) {
    char* kdst = smem + stage * 2 * TILE;
    char* vdst = kdst + TILE;
    const int w = (kt0 / p.BS) >> 6;
    if (w != win) {
      win = w;
      bvec = bt[min((w << 6) + lane, nblk_seq - 1)];
      if (!index_ok(bvec, p.nblocks, ERR_BLOCK_DECODE)) bvec = 0;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int key0 = min(kt0 + i * RPI, ctx - 1);        // wave-uniform
      const int blk = __builtin_amdgcn_readlane(bvec, (key0 / p.BS) & 63);
      const int row = i * RPI + lrow;
      const int key = min(kt0 + row, ctx - 1);
      const size_t off = (((size_t)blk * p.Hkv + kvh) * p.BS + (key % p.BS)) * D;
      const bf16* ks = p.k + off + ((lch ^ kswz<D>(row)) << 3);
      const bf16* vs = p.v + off + ((lch ^ vswz<D>(row)) << 3);
      glds16<NT>(ks, kdst + i * 1024);
      glds16<NT>(vs, vdst + i * 1024);
    }
  };

  float m = -INFINITY, lsum = 0.f;
  f32x4_t o[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) o[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int ntiles = (kv_hi - kv_lo + TK - 1) / TK;
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < ntiles) issue(kv_lo + t * TK, t);
  for (int t = 0; t < ntiles; ++t) {
    const int stage = t % NS;
    const int kt0 = kv_lo + t * TK;
    if (t + NS - 1 < ntiles) issue(kt0 + (NS - 1) * TK, (t + NS - 1) % NS);
    // retire tile t: the tiles issued after it may stay in flight (counted, in issue order)
    const int after = min(NS - 1, ntiles - 1 - t);
    if (after >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * 2 * NI) : "memory");
    else if (after == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * 2 * NI) : "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const char* k_lds = smem + stage * 2 * TILE;
    const char* v_lds = k_lds + TILE;
    f32x4_t s[NT16];
#pragma unroll
    for (int tt = 0; tt < NT16; ++tt) {
      s[tt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int row = 16 * tt + li;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bf16x8_t a =
            *reinterpret_cast<const bf16x8_t*>(k_lds + row * RB + (((4 * c + h4) ^ kswz<D>(row)) << 4));
        s[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[c], s[tt], 0, 0, 0);
      }
    }
    // raw-score max, scale folded into the exponent's FMA; deferred rescale as in the prefill kernel:
    // O (held in accumulator registers) is touched only on tiles where some row's max moved by more
    // than kRescaleLog2
    float tmax = -INFINITY;
    if (kt0 + TK > kv_hi) {  // the context's last tile only; a real branch (see attn_prefill_kernel)
      asm volatile("");
#pragma unroll
      for (int tt = 0; tt < NT16; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt0 + 16 * tt + 4 * h4 + r;
          s[tt][r] = key >= kv_hi ? -INFINITY : s[tt][r];
        }
    }
#pragma unroll
    for (int tt = 0; tt < NT16; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[tt][r]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_cand = fmaxf(m, tmax * p.scale_log2);
    if (__any(m_cand > m + kRescaleLog2)) {
      const float m_use = m_cand == -INFINITY ? 0.f : m_cand;
      const float alpha = exp2f(m - m_use);
      m = m_cand;
      lsum *= alpha;
#pragma unroll
      for (int n = 0; n < ND; ++n) o[n] *= alpha;
    }
    const float nm = m == -INFINITY ? 0.f : -m;
    float pr[NT16][4];
#pragma unroll
    for (int tt = 0; tt < NT16; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pr[tt][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[tt][r], p.scale_log2, nm));
        lsum += pr[tt][r];
      }
    const int tq = li >> 2, tp = li & 3;
#pragma unroll
    for (int cc = 0; cc < NCC; ++cc) {
      bf16x8_t bp;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bp[r] = f2bits(pr[2 * cc][r]);
        bp[4 + r] = f2bits(pr[2 * cc + 1][r]);
      }
      const int r0 = 32 * cc + 4 * h4 + tq;
      const int r1 = r0 + 16;
#pragma unroll
      for (int n = 0; n < ND; ++n) {
        const int unit = 4 * n + tp;
        const int b0 = r0 * RB + ((unit ^ (vswz<D>(r0) << 1)) << 3);
        const int b1 = r1 * RB + ((unit ^ (vswz<D>(r1) << 1)) << 3);
        const bf16x4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b0));
        const bf16x4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b1));
        const bf16x8_t a = bf16x8_t{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bp, o[n], 0, 0, 0);
      }
    }
    // every LDS read of this stage has been consumed before the next issue
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (!row_valid) return;
  const int head = kvh * G + li;
  if (p.num_splits > 1) {
    float* po = p.part_o + (((size_t)split * p.total_q + tok) * p.Hq + head) * D;
#pragma unroll
    for (int n = 0; n < ND; ++n)
      *reinterpret_cast<float4*>(po + 16 * n + 4 * h4) = make_float4(o[n][0], o[n][1], o[n][2], o[n][3]);
    if (h4 == 0) {
      float* pm = p.part_ml + (((size_t)split * p.total_q + tok) * p.Hq + head) * 2;
      pm[0] = m;
      pm[1] = lsum;
    }
  } else {
    if (pre > 0) merge_prefix<D>(p, tok, head, pre, h4, m, lsum, o);
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16* op = p.out + (size_t)tok * p.out_stride + (size_t)head * D;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      bf16x4_t w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = f2bits(o[n][r] * inv);
      *reinterpret_cast<bf16x4_t*>(op + 16 * n + 4 * h4) = w;
    }
  }
}

// Combine split-KV partials of decode (q_len == 1 per sequence: token == seq), and the shared-prefix parts
// of a sequence whose first keys paged_decode_prefix_kernel covered.
template <int D>
__global__ __launch_bounds__(D) void attn_combine_kernel(AttnParams p) {
  const int tok = blockIdx.x, head = blockIdx.y, d = threadIdx.x;
  const int ctx = p.ctx_len[tok];
  const int pre = prefix_of(p, tok, ctx);
  int nvalid = (ctx - pre + p.split_len - 1) / p.split_len;
  nvalid = max(1, min(nvalid, p.num_splits));
  const int npre = pre > 0 ? prefix_planes(p, tok, pre) : 0;
  float M = -INFINITY;
  for (int s = 0; s < nvalid; ++s)
    M = fmaxf(M, p.part_ml[(((size_t)s * p.total_q + tok) * p.Hq + head) * 2]);
  for (int s = 0; s < npre; ++s)
    M = fmaxf(M, p.pre_ml[(((size_t)s * p.total_q + tok) * p.Hq + head) * 2]);
  const float Mu = M == -INFINITY ? 0.f : M;
  float L = 0.f, acc = 0.f;
  for (int s = 0; s < nvalid; ++s) {
    const size_t base = ((size_t)s * p.total_q + tok) * p.Hq + head;
    const float w = exp2f(p.part_ml[base * 2] - Mu);
    L += p.part_ml[base * 2 + 1] * w;
    acc += p.part_o[base * D + d] * w;
  }
  for (int s = 0; s < npre; ++s) {
    const size_t base = ((size_t)s * p.total_q + tok) * p.Hq + head;
    const float w = exp2f(p.pre_ml[base * 2] - Mu);
    L += p.pre_ml[base * 2 + 1] * w;
    acc += p.pre_o[base * D + d] * w;
  }
  p.out[(size_t)tok * p.out_stride + (size_t)head * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
}

// ---------------------------------------------------------------------------
// Shared-prefix ("cascade") decode.  Sequences that share a cached prompt prefix -- ingest's summary /
// title / keyword calls over one chunk, an agent job's calls over the same documents -- hold the SAME KV
// block ids for it, and the per-sequence decode kernel above would read those blocks once per sequence.
// Here the batch's rows are grouped (engine: adjacent rows with a common leading run of block ids) and:
//   1. paged_decode_prefix_kernel: one wave per (group, kv head, prefix part) reads the group's prefix K/V
//      ONCE and computes every member's G query heads against it: the rows (member, head) are the MFMA
//      columns, RG row groups of 16 per wave (RG = 2 covers 4 members at GQA 7), each K / V^T fragment read
//      from LDS feeding RG MFMAs.  It writes per-part (m, l, O) to the prefix planes.
//   2. the per-sequence decode kernel runs over each row's own keys [pre_len, ctx) only and merges the
//      prefix planes into its state before normalising (one part), or the combine pass merges them with
//      the split parts.
// The math is the decode kernel's (swapped QK^T, exp2 online softmax in the log2 domain, deferred rescale);
// K/V go through the same 2-stage LDS-DMA ring of 32-key tiles.
template <int D, int RG>
__global__ __launch_bounds__(64) void paged_decode_prefix_kernel(AttnParams p) {
  constexpr int TK = 32, NS = 2;
  constexpr int NT16 = TK / 16;
  constexpr int RB = 2 * D;
  constexpr int CPR = D / 8;
  constexpr int NC = D / 32;
  constexpr int ND = D / 16;
  constexpr int TILE = TK * RB;
  constexpr int NI = TILE / 1024;
  constexpr int RPI = 1024 / RB;
  __shared__ __attribute__((aligned(16))) char smem[NS * 2 * TILE];

  const int lane = threadIdx.x;
  const int h4 = lane >> 4, li = lane & 15;
  const int item = blockIdx.x, kvh = blockIdx.y;
  const int4 it = reinterpret_cast<const int4*>(p.pre_items)[item];
  const int r0 = it.x, r1 = it.y, kv_lo = it.z, kv_hi = it.w;
  if (r1 - r0 < 2) return;  // padding item (or a lone row: the per-sequence kernel covers it)
  if (!index_ok(r0, p.total_q, ERR_PREFIX_GROUP) || !index_ok(r1, p.total_q + 1, ERR_PREFIX_GROUP)) return;
  const int nmem = r1 - r0;
  const int P = p.pre_len[r0];
  const int part = p.pre_part[r0];
  if (P <= 0 || !index_ok(P, p.ctx_len[r0], ERR_PREFIX_GROUP) || part <= 0) return;
  if (kv_lo < 0 || kv_lo >= kv_hi || kv_hi > P || kv_lo % part != 0 || kv_hi - kv_lo > part) {
    report_index_error(ERR_PREFIX_GROUP, kv_lo);
    return;
  }
  const int split = kv_lo / part;  // the plane this part writes
  if (!index_ok(split, p.pre_planes, ERR_PREFIX_GROUP)) return;
  const int G = p.G;

  // column li of row group j is the pair (member, head) = divmod(16 j + li, G)
  bf16x8_t qf[RG][NC];
  int tok[RG], head[RG];
  bool valid[RG];
#pragma unroll
  for (int j = 0; j < RG; ++j) {
    const int row = 16 * j + li;
    const int mem = row / G;
    valid[j] = mem < nmem;
    tok[j] = p.q_start[r0 + (valid[j] ? mem : 0)];
    head[j] = kvh * G + (valid[j] ? row % G : 0);
    if (valid[j] && h4 == 0 && kvh == 0 && split == 0 && row % G == 0 &&
        (p.pre_len[r0 + mem] != P || p.pre_part[r0 + mem] != part))
      report_index_error(ERR_PREFIX_GROUP, r0 + mem);  // a member whose merge would read other planes
    const bf16* qp = p.q + (size_t)tok[j] * p.q_stride + (size_t)head[j] * D + 8 * h4;
#pragma unroll
    for (int c = 0; c < NC; ++c) qf[j][c] = *reinterpret_cast<const bf16x8_t*>(qp + 32 * c);
  }
  const int32_t* bt = p.block_tables + (size_t)r0 * p.bt_stride;  // the leader's ids cover the prefix
  const int lrow = lane / CPR, lch = lane % CPR;
  const int nblk = (P + p.BS - 1) / p.BS;
  int win = (kv_lo / p.BS) >> 6;
  int bvec = bt[min((win << 6) + lane, nblk - 1)];
  if (!index_ok(bvec, p.nblocks, ERR_BLOCK_DECODE)) bvec = 0;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): Q and block ids retired before the counted DMA pipeline
#pragma unroll
  for (int j = 0; j < RG; ++j)
#pragma unroll
    for (int c = 0; c < NC; ++c) asm volatile("" : "+v"(qf[j][c]));
  asm volatile("" : "+v"(bvec));

  auto issue = [&](int kt0, int stage) {
    char* kdst = smem + stage * 2 * TILE;
    char* vdst = kdst + TILE;
    const int w = (kt0 / p.BS) >> 6;
    if (w != win) {
      win = w;
      bvec = bt[min((w << 6) + lane, nblk - 1)];
      if (!index_ok(bvec, p.nblocks, ERR_BLOCK_DECODE)) bvec = 0;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int key0 = min(kt0 + i * RPI, P - 1);
      const int blk = __builtin_amdgcn_readlane(bvec, (key0 / p.BS) & 63);
      const int row = i * RPI + lrow;
      const int key = min(kt0 + row, P - 1);
      const size_t off = (((size_t)blk * p.Hkv + kvh) * p.BS + (key % p.BS)) * D;
      glds16(p.k + off + ((lch ^ kswz<D>(row)) << 3), kdst + i * 1024);
      glds16(p.v + off + ((lch ^ vswz<D>(row)) << 3), vdst + i * 1024);
    }
  };

  float m[RG], lsum[RG];
  f32x4_t o[RG][ND];
#pragma unroll
  for (int j = 0; j < RG; ++j) {
    m[j] = -INFINITY;
    lsum[j] = 0.f;
#pragma unroll
    for (int n = 0; n < ND; ++n) o[j][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  const int ntiles = (kv_hi - kv_lo + TK - 1) / TK;
  issue(kv_lo, 0);
  for (int t = 0; t < ntiles; ++t) {
    const int stage = t & 1;
    const int kt0 = kv_lo + t * TK;
    if (t + 1 < ntiles) {
      issue(kt0 + TK, stage ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");  // tile t landed, t + 1 in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const char* k_lds = smem + stage * 2 * TILE;
    const char* v_lds = k_lds + TILE;
    f32x4_t s[RG][NT16];
#pragma unroll
    for (int tt = 0; tt < NT16; ++tt) {
#pragma unroll
      for (int j = 0; j < RG; ++j) s[j][tt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int row = 16 * tt + li;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bf16x8_t a =
            *reinterpret_cast<const bf16x8_t*>(k_lds + row * RB + (((4 * c + h4) ^ kswz<D>(row)) << 4));
#pragma unroll
        for (int j = 0; j < RG; ++j) s[j][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[j][c], s[j][tt], 0, 0, 0);
      }
    }
    if (kt0 + TK > kv_hi) {  // the part's last tile only
      asm volatile("");
#pragma unroll
      for (int j = 0; j < RG; ++j)
#pragma unroll
        for (int tt = 0; tt < NT16; ++tt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kt0 + 16 * tt + 4 * h4 + r;
            s[j][tt][r] = key >= kv_hi ? -INFINITY : s[j][tt][r];
          }
    }
    bf16x8_t bp[RG];
#pragma unroll
    for (int j = 0; j < RG; ++j) {
      float tmax = -INFINITY;
#pragma unroll
      for (int tt = 0; tt < NT16; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[j][tt][r]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float m_cand = fmaxf(m[j], tmax * p.scale_log2);
      if (__any(m_cand > m[j] + kRescaleLog2)) {
        const float m_use = m_cand == -INFINITY ? 0.f : m_cand;
        const float alpha = exp2f(m[j] - m_use);
        m[j] = m_cand;
        lsum[j] *= alpha;
#pragma unroll
        for (int n = 0; n < ND; ++n) o[j][n] *= alpha;
      }
      const float nm = m[j] == -INFINITY ? 0.f : -m[j];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j][0][r], p.scale_log2, nm));
        const float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j][1][r], p.scale_log2, nm));
        lsum[j] += p0 + p1;
        bp[j][r] = f2bits(p0);
        bp[j][4 + r] = f2bits(p1);
      }
    }
    const int tq = li >> 2, tp = li & 3;
    const int rr0 = 4 * h4 + tq, rr1 = rr0 + 16;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int unit = 4 * n + tp;
      const int b0 = rr0 * RB + ((unit ^ (vswz<D>(rr0) << 1)) << 3);
      const int b1 = rr1 * RB + ((unit ^ (vswz<D>(rr1) << 1)) << 3);
      const bf16x4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b0));
      const bf16x4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b1));
      const bf16x8_t a = bf16x8_t{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
      for (int j = 0; j < RG; ++j) o[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bp[j], o[j][n], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's LDS reads done before its refill
  }
#pragma unroll
  for (int j = 0; j < RG; ++j) {
    float l = lsum[j];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (!valid[j]) continue;
    const size_t base = ((size_t)split * p.total_q + tok[j]) * p.Hq + head[j];
    float* po = p.pre_o + base * D;
#pragma unroll
    for (int n = 0; n < ND; ++n)
      *reinterpret_cast<float4*>(po + 16 * n + 4 * h4) = make_float4(o[j][n][0], o[j][n][1], o[j][n][2], o[j][n][3]);
    if (h4 == 0) {
      p.pre_ml[base * 2] = m[j];
      p.pre_ml[base * 2 + 1] = l;
    }
  }
}

// ---------------------------------------------------------------------------
// Small-batch decode (the reference's own regime: 1-16 live sequences, contexts up to 11.7K; vLLM
// --max-num-seqs 4).  paged_decode_kernel puts ONE wave on a (sequence, kv head, split) and merges the
// splits in a second launch: at B = 1 the grid is 4 kv heads x splits, each wave walks its tiles one
// round trip at a time, and the combine pass re-reads every split's partial -- 15 / 25 / 38-49 us per
// layer at 1K / 4K / 11.6K keys for 2 / 8 / 24 MB of K/V (profiles/attn_sweep_r5.json).  Here:
//   * NW waves share one (sequence, kv head, split) and take its 32-key tiles round robin, each wave with
//     its own 2-stage LDS-DMA ring (the single-wave kernel's body), so a split keeps NW tiles in flight and
//     the split count -- the number of partials to merge -- drops NW-fold for the same parallelism;
//   * the waves' (m, l, O) merge in LDS (the rings' space, after a barrier);
//   * the splits of one (sequence, kv head) merge IN this launch: each workgroup writes its partial, takes
//     an agent-scope ticket (release fence first, as gemm_stream.hip's split tiles), and the last arriver
//     (acquire) reads the others' partials and writes the output; it resets its counter, so the launch
//     replays inside hipGraphs without a memset.  No second kernel, no partial round trip for the others.
//
// FR (the RoPE pass folded in, ops/attention.py paged_decode_mw_rope): the workgroup forms its G q heads from
// the qkv projection's split-K planes (sum in plane order, bias, NeoX RoPE: the values qkv_rope_kernel<true>
// stores) cooperatively -- one thread per 4-dim rotary pair, all planes' loads in flight together, while the
// first K / V tile's DMA is in flight -- and stages them in LDS past the rings.  The new token's key never goes
// through the cache in this launch: the sequence's last split stops its tile loop one key short, its workgroup
// also forms the new K / V (stored to the token's cache slot for the next steps, and staged in LDS), and wave 0
// folds that key into its (m, l, O) after the loop.  One launch (and the q round trip) fewer per layer.
template <int D>
constexpr int mw_rope_lds() { return 16 * D * 2 + D * 2 + D * 4; }  // q [16][D] bf16, new K [D] bf16, new V [D] f32

// token t's qkv projection at column col, 4 dims: the split-K planes summed in plane order and rounded to bf16,
// the bias added and rounded again (elementwise.hip qkv_rope_kernel<true> load8)
__device__ __forceinline__ f32x4_t rq_load4(const AttnParams& p, int t, int col) {
  f32x4_t x = plane_sum4(p.rq_planes + (size_t)t * p.rq_ld + col, p.rq_plane, p.rq_S);
#pragma unroll
  for (int r = 0; r < 4; ++r) x[r] = bits2f(f2bits(x[r]));
  if (p.rq_bias) {
    const bf16x4_t b = *reinterpret_cast<const bf16x4_t*>(p.rq_bias + col);
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = bits2f(f2bits(x[r] + bits2f(b[r])));
  }
  return x;
}

template <int D, int NW, bool FR>
__global__ __launch_bounds__(64 * NW) void paged_decode_mw_kernel(AttnParams p, unsigned* counters) {
  constexpr int TK = 32, NS = 2;
  constexpr int NT16 = TK / 16, NCC = TK / 32;
  constexpr int RB = 2 * D;
  constexpr int CPR = D / 8;
  constexpr int NC = D / 32;
  constexpr int ND = D / 16;
  constexpr int TILE = TK * RB;      // bytes per K (or V) tile
  constexpr int NI = TILE / 1024;    // LDS-DMA instructions per tile per tensor
  constexpr int RPI = 1024 / RB;     // rows per instruction
  static_assert((NS - 1) * 2 * NI <= 63, "vmcnt range");
  static_assert((NW * 16 * D + NW * 32 + 1) * 4 <= NW * NS * 2 * TILE, "merge scratch fits in the rings");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h4 = lane >> 4, li = lane & 15;
  const int seq = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z;
  const int ctx = p.ctx_len[seq];
  const int kv_lo = split * p.split_len;
  const int kv_hi = min(ctx, kv_lo + p.split_len);
  if (kv_lo >= kv_hi) return;  // (workgroup-uniform) past this sequence's last split: no ticket either
  const int G = p.G;
  const int tok = p.q_start[seq];
  const int nvalid = min(p.num_splits, (ctx + p.split_len - 1) / p.split_len);
  // FR: the last split's tiles stop before the new token's key (folded in from registers after the loop)
  const bool newkey = FR && split == nvalid - 1;
  const int kv_end = newkey ? kv_hi - 1 : kv_hi;
  bf16x8_t qf[NC];
  int pos = 0, slot = -1;
  if constexpr (FR) {  // q (and the new K / V) are formed once the first K / V tile is in flight (below)
    pos = p.rq_pos[tok];
    if (newkey) slot = p.rq_slot[tok];
  } else {
    const bf16* qp = p.q + (size_t)tok * p.q_stride + (size_t)(kvh * G + (li < G ? li : 0)) * D + 8 * h4;
#pragma unroll
    for (int c = 0; c < NC; ++c) qf[c] = *reinterpret_cast<const bf16x8_t*>(qp + 32 * c);
  }
  const int32_t* bt = p.block_tables + (size_t)seq * p.bt_stride;
  const int lrow = lane / CPR, lch = lane % CPR;
  const int nblk_seq = (ctx + p.BS - 1) / p.BS;
  int win = ((kv_lo + w * TK) / p.BS) >> 6;
  int bvec = bt[min((win << 6) + lane, nblk_seq - 1)];
  if (!index_ok(bvec, p.nblocks, ERR_BLOCK_DECODE)) bvec = 0;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): Q and block ids retired before the counted DMA pipeline
#pragma unroll
  for (int c = 0; c < NC; ++c) asm volatile("" : "+v"(qf[c]));
  asm volatile("" : "+v"(bvec));

  char* ring = smem + w * NS * 2 * TILE;
  auto issue = [&](int kt0, int stage) {
    char* kdst = ring + stage * 2 * TILE;
    char* vdst = kdst + TILE;
    const int wn = (kt0 / p.BS) >> 6;
    if (wn != win) {
      win = wn;
      bvec = bt[min((wn << 6) + lane, nblk_seq - 1)];
      if (!index_ok(bvec, p.nblocks, ERR_BLOCK_DECODE)) bvec = 0;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int key0 = min(kt0 + i * RPI, kv_end - 1);
      const int blk = __builtin_amdgcn_readlane(bvec, (key0 / p.BS) & 63);
      const int row = i * RPI + lrow;
      const int key = min(kt0 + row, kv_end - 1);
      const size_t off = (((size_t)blk * p.Hkv + kvh) * p.BS + (key % p.BS)) * D;
      glds16(p.k + off + ((lch ^ kswz<D>(row)) << 3), kdst + i * 1024);
      glds16(p.v + off + ((lch ^ vswz<D>(row)) << 3), vdst + i * 1024);
    }
  };

  float m = -INFINITY, lsum = 0.f;
  f32x4_t o[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) o[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int ntot = (kv_end - kv_lo + TK - 1) / TK;
  const int nmine = w < ntot ? (ntot - w + NW - 1) / NW : 0;  // this wave's tiles: w, w + NW, ...
  if (nmine > 0) issue(kv_lo + w * TK, 0);
  // FR staging past the rings (mw_rope_lds): q [16][D] bf16, the new K [D] bf16 and V [D] fp32
  bf16* q_st = reinterpret_cast<bf16*>(smem + NW * NS * 2 * TILE);
  bf16* k_st = q_st + 16 * D;
  float* v_st = reinterpret_cast<float*>(k_st + D);
  if constexpr (FR) {
    // the planes' loads overlap the first tile's DMA and retire here (the RoPE math consumes them), before the
    // loop's counted vmcnt
    if (!index_ok(pos, p.rq_npos, ERR_ROPE_POS)) pos = 0;
    if (slot >= 0 && !index_ok(slot, p.rq_nslots, ERR_KV_SLOT)) slot = -1;
    const float* cs = p.rq_cs + (size_t)pos * D;
    constexpr int HU = D / 8;  // rotary units (dims i0..i0+3 with i0 + D/2..) per head
    const int nq = G * HU, nk = newkey ? HU : 0, nv = newkey ? D / 4 : 0;
    const size_t cache_off = slot >= 0 ? (((size_t)(slot / p.BS) * p.Hkv + kvh) * p.BS + slot % p.BS) * D : 0;
    for (int u = threadIdx.x; u < nq + nk + nv; u += 64 * NW) {
      if (u < nq + nk) {
        const bool isk = u >= nq;
        const int i0 = ((isk ? u - nq : u) % HU) * 4;
        const int col = (isk ? p.Hq + kvh : kvh * G + u / HU) * D;
        const f32x4_t x1 = rq_load4(p, tok, col + i0), x2 = rq_load4(p, tok, col + i0 + D / 2);
        const f32x4_t cv = *reinterpret_cast<const f32x4_t*>(cs + i0);
        const f32x4_t sv = *reinterpret_cast<const f32x4_t*>(cs + D / 2 + i0);
        bf16x4_t r1, r2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          r1[r] = f2bits(x1[r] * cv[r] - x2[r] * sv[r]);
          r2[r] = f2bits(x2[r] * cv[r] + x1[r] * sv[r]);
        }
        bf16* dst = isk ? k_st : q_st + (u / HU) * D;
        *reinterpret_cast<bf16x4_t*>(dst + i0) = r1;
        *reinterpret_cast<bf16x4_t*>(dst + i0 + D / 2) = r2;
        if (isk && slot >= 0) {
          bf16* kd = const_cast<bf16*>(p.k) + cache_off;
          *reinterpret_cast<bf16x4_t*>(kd + i0) = r1;
          *reinterpret_cast<bf16x4_t*>(kd + i0 + D / 2) = r2;
        }
      } else {
        const int i0 = (u - nq - nk) * 4;
        const f32x4_t x = rq_load4(p, tok, (p.Hq + p.Hkv + kvh) * D + i0);
        *reinterpret_cast<f32x4_t*>(v_st + i0) = x;
        if (slot >= 0)
          *reinterpret_cast<bf16x4_t*>(const_cast<bf16*>(p.v) + cache_off + i0) =
              bf16x4_t{f2bits(x[0]), f2bits(x[1]), f2bits(x[2]), f2bits(x[3])};
      }
    }
    __syncthreads();
    const bf16* qr = q_st + (li < G ? li : 0) * D + 8 * h4;
#pragma unroll
    for (int c = 0; c < NC; ++c) qf[c] = *reinterpret_cast<const bf16x8_t*>(qr + 32 * c);
  }
  for (int t = 0; t < nmine; ++t) {
    const int stage = t & 1;
    const int kt0 = kv_lo + (w + t * NW) * TK;
    if (t + 1 < nmine) {
      issue(kt0 + NW * TK, stage ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");  // tile t landed, t + 1 in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const char* k_lds = ring + stage * 2 * TILE;
    const char* v_lds = k_lds + TILE;
    f32x4_t sc[NT16];
#pragma unroll
    for (int tt = 0; tt < NT16; ++tt) {
      sc[tt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int row = 16 * tt + li;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bf16x8_t a =
            *reinterpret_cast<const bf16x8_t*>(k_lds + row * RB + (((4 * c + h4) ^ kswz<D>(row)) << 4));
        sc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[c], sc[tt], 0, 0, 0);
      }
    }
    float tmax = -INFINITY;
    if (kt0 + TK > kv_end) {  // the context's last tile only; a real branch (see attn_prefill_kernel)
      asm volatile("");
#pragma unroll
      for (int tt = 0; tt < NT16; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt0 + 16 * tt + 4 * h4 + r;
          sc[tt][r] = key >= kv_end ? -INFINITY : sc[tt][r];
        }
    }
#pragma unroll
    for (int tt = 0; tt < NT16; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, sc[tt][r]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_cand = fmaxf(m, tmax * p.scale_log2);
    if (__any(m_cand > m + kRescaleLog2)) {
      const float m_use = m_cand == -INFINITY ? 0.f : m_cand;
      const float alpha = exp2f(m - m_use);
      m = m_cand;
      lsum *= alpha;
#pragma unroll
      for (int n = 0; n < ND; ++n) o[n] *= alpha;
    }
    const float nm = m == -INFINITY ? 0.f : -m;
    float pr[NT16][4];
#pragma unroll
    for (int tt = 0; tt < NT16; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pr[tt][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[tt][r], p.scale_log2, nm));
        lsum += pr[tt][r];
      }
    const int tq = li >> 2, tp = li & 3;
#pragma unroll
    for (int cc = 0; cc < NCC; ++cc) {
      bf16x8_t bp;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bp[r] = f2bits(pr[2 * cc][r]);
        bp[4 + r] = f2bits(pr[2 * cc + 1][r]);
      }
      const int r0 = 32 * cc + 4 * h4 + tq;
      const int r1 = r0 + 16;
#pragma unroll
      for (int n = 0; n < ND; ++n) {
        const int unit = 4 * n + tp;
        const int b0 = r0 * RB + ((unit ^ (vswz<D>(r0) << 1)) << 3);
        const int b1 = r1 * RB + ((unit ^ (vswz<D>(r1) << 1)) << 3);
        const bf16x4_t a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b0));
        const bf16x4_t a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(v_lds + b1));
        const bf16x8_t a = bf16x8_t{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bp, o[n], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's LDS reads done before its refill
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);

  if constexpr (FR) {
    if (newkey && w == 0) {  // (wave-uniform) the new token's key: one more online-softmax key, from the staging
      bf16x8_t kf[NC];
      float vn[ND][4];
#pragma unroll
      for (int c = 0; c < NC; ++c) kf[c] = *reinterpret_cast<const bf16x8_t*>(k_st + 32 * c + 8 * h4);
#pragma unroll
      for (int n = 0; n < ND; ++n) {
        const f32x4_t x = *reinterpret_cast<const f32x4_t*>(v_st + 16 * n + 4 * h4);
#pragma unroll
        for (int r = 0; r < 4; ++r) vn[n][r] = bits2f(f2bits(x[r]));
      }
      float dot = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) dot = __builtin_fmaf(bits2f(qf[c][j]), bits2f(kf[c][j]), dot);
      dot += __shfl_xor(dot, 16, 64);
      dot += __shfl_xor(dot, 32, 64);
      const float s = dot * p.scale_log2;
      const float mn = fmaxf(m, s);
      const float alpha = exp2f(m - mn), beta = exp2f(s - mn);
      m = mn;
      lsum = lsum * alpha + beta;
#pragma unroll
      for (int n = 0; n < ND; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[n][r] = __builtin_fmaf(beta, vn[n][r], o[n][r] * alpha);
    }
  }

  // ---- the waves' states merge in LDS (the rings are free once every wave passed the barrier)
  __syncthreads();
  float* so = reinterpret_cast<float*>(smem);  // [NW][16 rows][D]: lane (li, h4) holds O[row li][16 n + 4 h4 + r]
  float* sml = so + NW * 16 * D;               // [NW][16][2]: (m, l)
  unsigned* flag = reinterpret_cast<unsigned*>(sml + NW * 32);
#pragma unroll
  for (int n = 0; n < ND; ++n)
    *reinterpret_cast<f32x4_t*>(so + (w * 16 + li) * D + 16 * n + 4 * h4) = o[n];
  if (h4 == 0) {
    sml[(w * 16 + li) * 2] = m;
    sml[(w * 16 + li) * 2 + 1] = lsum;
  }
  __syncthreads();
  const bool single = nvalid <= 1;
  for (int idx = threadIdx.x; idx < G * D; idx += 64 * NW) {
    const int row = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int wv = 0; wv < NW; ++wv) M = fmaxf(M, sml[(wv * 16 + row) * 2]);
    float L = 0.f, acc = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) {
        const float wt = exp2f(sml[(wv * 16 + row) * 2] - M);
        L += sml[(wv * 16 + row) * 2 + 1] * wt;
        acc += so[(wv * 16 + row) * D + d] * wt;
      }
    }
    const int head = kvh * G + row;
    if (single) {
      p.out[(size_t)tok * p.out_stride + (size_t)head * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
    } else {
      const size_t base = ((size_t)split * p.total_q + tok) * p.Hq + head;
      p.part_o[base * D + d] = acc;
      if (d == 0) {
        p.part_ml[base * 2] = M;
        p.part_ml[base * 2 + 1] = L;
      }
    }
  }
  if (single) return;

  // ---- the splits of this (sequence, kv head) merge in the last arriving workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned* cnt = counters + (size_t)seq * p.Hkv + kvh;
    const unsigned tk = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk >= (unsigned)nvalid) report_index_error(ERR_TICKET, tk);  // a stale or shared ticket word
    const unsigned last = tk == (unsigned)(nvalid - 1) ? 1u : 0u;
    if (last) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    flag[0] = last;
  }
  __syncthreads();
  if (flag[0] == 0u) return;
  // last arriver: every split's (m, l) of the G rows staged in LDS in one parallel pass, the per-split
  // weights formed once per row, then ONE pass over the partial O vectors (independent loads per thread)
  float* wm = reinterpret_cast<float*>(smem);  // [nvalid][16]: m, then the split's weight
  float* wl = wm + nvalid * 16;                // [nvalid][16]: l
  float* rowL = wl + nvalid * 16;              // [16]
  for (int e = threadIdx.x; e < nvalid * 16; e += 64 * NW) {
    const int sp = e >> 4, row = e & 15;
    float mv = -INFINITY, lv = 0.f;
    if (row < G) {
      const size_t base = (((size_t)sp * p.total_q + tok) * p.Hq + kvh * G + row) * 2;
      mv = p.part_ml[base];
      lv = p.part_ml[base + 1];
    }
    wm[e] = mv;
    wl[e] = lv;
  }
  __syncthreads();
  if (threadIdx.x < 16) {
    const int row = threadIdx.x;
    float M = -INFINITY;
    for (int sp = 0; sp < nvalid; ++sp) M = fmaxf(M, wm[sp * 16 + row]);
    const float Mu = M == -INFINITY ? 0.f : M;
    float L = 0.f;
    for (int sp = 0; sp < nvalid; ++sp) {
      const float wt = exp2f(wm[sp * 16 + row] - Mu);
      wm[sp * 16 + row] = wt;
      L += wl[sp * 16 + row] * wt;
    }
    rowL[row] = L;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < G * D; idx += 64 * NW) {
    const int row = idx / D, d = idx % D;
    const int head = kvh * G + row;
    const float* po = p.part_o + ((size_t)tok * p.Hq + head) * D + d;
    const size_t sstride = (size_t)p.total_q * p.Hq * D;
    float acc = 0.f;
#pragma unroll 8
    for (int sp = 0; sp < nvalid; ++sp) acc += po[sp * sstride] * wm[sp * 16 + row];
    const float L = rowL[row];
    p.out[(size_t)tok * p.out_stride + (size_t)head * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
  }
}

template <int D, int NW, bool FR = false>
int launch_decode_mw(const AttnParams& prm, int nseq, unsigned* counters, hipStream_t stream) {
  constexpr int lds = NW * 2 * 2 * 32 * 2 * D + (FR ? mw_rope_lds<D>() : 0);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)paged_decode_mw_kernel<D, NW, FR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        lds);
    attr_set = true;
  }
  paged_decode_mw_kernel<D, NW, FR><<<dim3(nseq, prm.Hkv, prm.num_splits), 64 * NW, lds, stream>>>(prm, counters);
  return (int)hipGetLastError();
}

template <int D, int NW, bool PAGED>
int launch(const AttnParams& prm, int nseq, hipStream_t stream) {
  dim3 grid(nseq * prm.tiles_per_seq, prm.Hkv, prm.num_splits);
  attn_fwd_kernel<D, NW, PAGED><<<grid, 64 * NW, 0, stream>>>(prm);
  int err = (int)hipGetLastError();
  if (err) return err;
  if (prm.num_splits > 1) {
    dim3 g2(prm.total_q, prm.Hq);
    attn_combine_kernel<D><<<g2, D, 0, stream>>>(prm);
    err = (int)hipGetLastError();
  }
  return err;
}

template <int D>
int launch_decode(const AttnParams& prm_in, int nseq, int tk, int ns, bool nt, hipStream_t stream) {
  AttnParams prm = prm_in;
  prm.xcd_group = g_decode_xcd;
  dim3 grid(nseq, prm.Hkv, prm.num_splits);
  if (nt && tk == 32 && ns == 3)
    paged_decode_kernel<D, 32, 3, true><<<grid, 64, 0, stream>>>(prm);
  else if (nt && tk == 32)
    paged_decode_kernel<D, 32, 2, true><<<grid, 64, 0, stream>>>(prm);
  else if (tk == 32 && ns == 4)
    paged_decode_kernel<D, 32, 4><<<grid, 64, 0, stream>>>(prm);
  else if (tk == 32 && ns == 3)
    paged_decode_kernel<D, 32, 3><<<grid, 64, 0, stream>>>(prm);
  else if (tk == 32)
    paged_decode_kernel<D, 32, 2><<<grid, 64, 0, stream>>>(prm);
  else
    paged_decode_kernel<D, 64, 2><<<grid, 64, 0, stream>>>(prm);
  int err = (int)hipGetLastError();
  if (err) return err;
  if (prm.num_splits > 1) {
    dim3 g2(prm.total_q, prm.Hq);
    attn_combine_kernel<D><<<g2, D, 0, stream>>>(prm);
    err = (int)hipGetLastError();
  }
  return err;
}

template <int D>
int launch_decode_prefix(const AttnParams& prm, int n_items, int rg, hipStream_t stream) {
  dim3 grid(n_items, prm.Hkv);
  if (rg == 4)
    paged_decode_prefix_kernel<D, 4><<<grid, 64, 0, stream>>>(prm);
  else
    paged_decode_prefix_kernel<D, 2><<<grid, 64, 0, stream>>>(prm);
  return (int)hipGetLastError();
}

template <int D>
int launch_prefill(const AttnParams& prm, int nseq, int nw, hipStream_t stream) {
  dim3 grid(nseq * prm.tiles_per_seq, prm.Hkv, 1);
  if (nw == 6)
    attn_prefill_kernel<D, 2, 3><<<grid, 512, 0, stream>>>(prm);
  else
    attn_prefill_kernel<D, 2, 2><<<grid, 512, 0, stream>>>(prm);
  return (int)hipGetLastError();
}

template <int D>
int dispatch_nw(const AttnParams& prm, int nseq, int nw, bool paged, hipStream_t stream) {
  // nw == 1 / 3 with q_len == 1: LDS-DMA pipelined decode kernel with 64- / 32-key
  // tiles (32-key tiles halve the LDS ring so more single-wave workgroups share a
  // CU); nw == 2: the generic kernel with one wave per workgroup (A/B reference)
  // nw == 7 / 8: 32-key tiles in a 4- / 3-stage ring; nw == 11 / 12: 3 / 8 with non-temporal K/V loads
  if (paged && (nw == 1 || nw == 3 || nw == 7 || nw == 8 || nw == 11 || nw == 12) && prm.tiles_per_seq == 1 &&
      prm.G <= 16 && prm.BS % 16 == 0)
    return launch_decode<D>(prm, nseq, nw == 1 ? 64 : 32, nw == 7 ? 4 : (nw == 8 || nw == 12) ? 3 : 2,
                            nw >= 11, stream);
  if (nw == 5 || nw == 6) {  // LDS-DMA prefill: 8 waves, 2-stage (5) / staggered 3-stage (6) ring
    if constexpr (D == 128 || D == 64) {
      if (paged && prm.num_splits == 1 && prm.BS == 16 && prm.bt_stride <= kPrefillMaxBlocks)
        return launch_prefill<D>(prm, nseq, nw, stream);
    }
    return (int)hipErrorInvalidValue;
  }
  if (nw == 3 || nw == 7 || nw == 8 || nw == 11 || nw == 12) nw = 1;
  if (nw == 2) nw = 1;
  if (paged) {
    return nw == 1 ? launch<D, 1, true>(prm, nseq, stream) : launch<D, 4, true>(prm, nseq, stream);
  }
  return nw == 1 ? launch<D, 1, false>(prm, nseq, stream) : launch<D, 4, false>(prm, nseq, stream);
}

}  // namespace

// Paged attention (prefill / decode).  q: [T, Hq, D] token-major rows of
// stride q_stride; caches [blocks, Hkv, BS, D]; out [T, Hq*D] (stride
// out_stride).  max_q_len bounds the per-sequence q length (tiles are implicit
// so the launch is graph-capturable).  num_splits > 1 (decode only) needs
// workspaces part_o [num_splits, T, Hq, D] f32 and part_ml [num_splits, T, Hq, 2].
GRAG_API int grag_paged_attention(const void* q, int q_stride, const void* k_cache,
                                  const void* v_cache, void* out, int out_stride,
                                  const int32_t* block_tables, int bt_stride,
                                  const int32_t* q_start, const int32_t* ctx_len, int nseq,
                                  int total_q, int max_q_len, int Hq, int Hkv, int D, int BS,
                                  float scale, int causal, int num_splits, int split_len,
                                  float* part_o, float* part_ml, int nw, int nblocks, hipStream_t stream) {
  if (nseq <= 0) return 0;
  if (Hq % Hkv != 0 || BS <= 0 || nw < 1 || (nw > 8 && nw != 11 && nw != 12)) return (int)hipErrorInvalidValue;
  if ((nw == 5 || nw == 6) && num_splits > 1) return (int)hipErrorInvalidValue;
  if (num_splits > 1 && (max_q_len != 1 || !part_o || !part_ml || split_len % KT != 0))
    return (int)hipErrorInvalidValue;
  AttnParams prm{};
  prm.q = (const bf16*)q;
  prm.k = (const bf16*)k_cache;
  prm.v = (const bf16*)v_cache;
  prm.out = (bf16*)out;
  prm.part_o = part_o;
  prm.part_ml = part_ml;
  prm.block_tables = block_tables;
  prm.q_start = q_start;
  prm.ctx_len = ctx_len;
  prm.q_stride = q_stride;
  prm.kv_stride = 0;
  prm.out_stride = out_stride;
  prm.Hq = Hq;
  prm.Hkv = Hkv;
  prm.G = Hq / Hkv;
  prm.BS = BS;
  prm.bt_stride = bt_stride;
  // 8-wave prefill needs KV blocks of 16 and a block table that fits its LDS window; otherwise
  // the 4-wave kernel (same math) takes the launch
  if (nw >= 5 && !(BS == 16 && bt_stride <= kPrefillMaxBlocks && (D == 128 || D == 64))) nw = 4;
  const int rows_per_wg = nw >= 5 ? 256 : 16 * (nw == 2 ? 1 : nw);  // nw 5/6: 256 GQA rows per workgroup
  prm.tiles_per_seq = (max_q_len * prm.G + rows_per_wg - 1) / rows_per_wg;
  if (nw == 1 && max_q_len != 1) return (int)hipErrorInvalidValue;
  prm.num_splits = num_splits < 1 ? 1 : num_splits;
  prm.split_len = prm.num_splits > 1 ? split_len : (1 << 30);
  prm.total_q = total_q;
  prm.scale_log2 = scale * 1.4426950408889634f;
  prm.causal = causal;
  prm.nblocks = nblocks;
  switch (D) {
    case 128: return dispatch_nw<128>(prm, nseq, nw, true, stream);
    case 64: return dispatch_nw<64>(prm, nseq, nw, true, stream);
    case 32: return dispatch_nw<32>(prm, nseq, nw, true, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

// Shared-prefix decode (q_len == 1): paged_decode_prefix_kernel over the groups' common prefixes, then the
// per-sequence decode kernel (nw 1 / 3 / 7 / 8 / 11 / 12 as grag_paged_attention) over each row's own keys
// [pre_len, ctx), merging the prefix parts.  pre_len [nseq]: keys the row's group shares (0 = none);
// pre_part [nseq]: the group's part length (keys); items [n_items, 4]: (first row, end row, first key, end key)
// of one part of one group -- rows of a group are adjacent and share their first pre_len block-table entries,
// a part [k0, k1) starts at a multiple of the part length and writes plane k0 / part; items spanning < 2 rows
// are padding.  pre_o / pre_ml: [pre_planes, total_q, Hq, D | 2] f32.  rg = 2 or 4 row groups of 16
// (member, head) pairs per wave: a group has at most 16 * rg / G members.
GRAG_API int grag_paged_decode_cascade(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                       void* out, int out_stride, const int32_t* block_tables, int bt_stride,
                                       const int32_t* q_start, const int32_t* ctx_len, int nseq, int total_q,
                                       int Hq, int Hkv, int D, int BS, float scale, int num_splits, int split_len,
                                       float* part_o, float* part_ml, int nw, int nblocks, const int32_t* pre_len,
                                       const int32_t* pre_part, const int32_t* items, int n_items, int pre_planes,
                                       float* pre_o, float* pre_ml, int rg, hipStream_t stream) {
  if (nseq <= 0) return 0;
  if (Hq % Hkv != 0 || Hq / Hkv > 16 || BS <= 0 || BS % 16 != 0 || (D != 64 && D != 128)) return (int)hipErrorInvalidValue;
  if (!(nw == 1 || nw == 3 || nw == 7 || nw == 8 || nw == 11 || nw == 12)) return (int)hipErrorInvalidValue;
  if (num_splits < 1) num_splits = 1;
  if (num_splits > 1 && (!part_o || !part_ml || split_len % KT != 0)) return (int)hipErrorInvalidValue;
  if (!pre_len || !pre_part || !items || !pre_o || !pre_ml || n_items < 0 || pre_planes < 1 ||
      (reinterpret_cast<uintptr_t>(items) & 15) || (rg != 2 && rg != 4) || 2 * (Hq / Hkv) > 16 * rg)
    return (int)hipErrorInvalidValue;
  AttnParams prm{};
  prm.q = (const bf16*)q;
  prm.k = (const bf16*)k_cache;
  prm.v = (const bf16*)v_cache;
  prm.out = (bf16*)out;
  prm.part_o = part_o;
  prm.part_ml = part_ml;
  prm.block_tables = block_tables;
  prm.q_start = q_start;
  prm.ctx_len = ctx_len;
  prm.q_stride = q_stride;
  prm.out_stride = out_stride;
  prm.Hq = Hq;
  prm.Hkv = Hkv;
  prm.G = Hq / Hkv;
  prm.BS = BS;
  prm.bt_stride = bt_stride;
  prm.tiles_per_seq = 1;
  prm.num_splits = num_splits;
  prm.split_len = num_splits > 1 ? split_len : (1 << 30);
  prm.total_q = total_q;
  prm.scale_log2 = scale * 1.4426950408889634f;
  prm.causal = 1;
  prm.nblocks = nblocks;
  prm.pre_len = pre_len;
  prm.pre_part = pre_part;
  prm.pre_items = items;
  prm.pre_o = pre_o;
  prm.pre_ml = pre_ml;
  prm.pre_planes = pre_planes;
  int err = 0;
  if (n_items > 0)
    err = D == 128 ? launch_decode_prefix<128>(prm, n_items, rg, stream)
                   : launch_decode_prefix<64>(prm, n_items, rg, stream);
  if (err) return err;
  const int tk = nw == 1 ? 64 : 32, ns = nw == 7 ? 4 : (nw == 8 || nw == 12) ? 3 : 2;
  return D == 128 ? launch_decode<128>(prm, nseq, tk, ns, nw >= 11, stream)
                  : launch_decode<64>(prm, nseq, tk, ns, nw >= 11, stream);
}

// Decode workgroup placement for later launches (1: sequences adjacent in the batch on one XCD, 0: the
// dispatcher's round robin); any other value only queries.  Returns the previous setting.
GRAG_API int grag_attn_decode_xcd(int on) {
  const int prev = g_decode_xcd;
  if (on == 0 || on == 1) g_decode_xcd = on;
  return prev;
}

// Small-batch decode (paged_decode_mw_kernel): nw = 2 or 4 waves per (sequence, kv head, split), the splits
// merged in the same launch by the last arriving workgroup.  counters: >= nseq * Hkv zero-initialised
// uint32 words (each reset by its last arriver); num_splits > 1 needs part_o / part_ml as
// grag_paged_attention.  head_dim 64 / 128, G <= 16, BS % 16 == 0, split_len % 32 == 0.
GRAG_API int grag_paged_decode_mw(const void* q, int q_stride, const void* k_cache, const void* v_cache, void* out,
                                  int out_stride, const int32_t* block_tables, int bt_stride, const int32_t* q_start,
                                  const int32_t* ctx_len, int nseq, int total_q, int Hq, int Hkv, int D, int BS,
                                  float scale, int num_splits, int split_len, float* part_o, float* part_ml,
                                  unsigned* counters, int nw, int nblocks, hipStream_t stream) {
  if (nseq <= 0) return 0;
  if (Hq % Hkv != 0 || Hq / Hkv > 16 || BS <= 0 || BS % 16 != 0 || (nw != 2 && nw != 4) || (D != 64 && D != 128))
    return (int)hipErrorInvalidValue;
  if (num_splits < 1) num_splits = 1;
  if (num_splits > 1 && (!part_o || !part_ml || !counters || split_len <= 0 || split_len % 32 != 0))
    return (int)hipErrorInvalidValue;
  if ((num_splits * 32 + 16) * 4 > nw * 2 * 2 * 32 * 2 * D) return (int)hipErrorInvalidValue;  // merge scratch
  AttnParams prm{};
  prm.q = (const bf16*)q;
  prm.k = (const bf16*)k_cache;
  prm.v = (const bf16*)v_cache;
  prm.out = (bf16*)out;
  prm.part_o = part_o;
  prm.part_ml = part_ml;
  prm.block_tables = block_tables;
  prm.q_start = q_start;
  prm.ctx_len = ctx_len;
  prm.q_stride = q_stride;
  prm.out_stride = out_stride;
  prm.Hq = Hq;
  prm.Hkv = Hkv;
  prm.G = Hq / Hkv;
  prm.BS = BS;
  prm.bt_stride = bt_stride;
  prm.tiles_per_seq = 1;
  prm.num_splits = num_splits;
  prm.split_len = num_splits > 1 ? split_len : (1 << 30);
  prm.total_q = total_q;
  prm.scale_log2 = scale * 1.4426950408889634f;
  prm.causal = 1;
  prm.nblocks = nblocks;
  if (D == 128) return nw == 4 ? launch_decode_mw<128, 4>(prm, nseq, counters, stream)
                               : launch_decode_mw<128, 2>(prm, nseq, counters, stream);
  return nw == 4 ? launch_decode_mw<64, 4>(prm, nseq, counters, stream)
                 : launch_decode_mw<64, 2>(prm, nseq, counters, stream);
}

// The same with the RoPE pass folded in (paged_decode_mw_kernel FR): instead of q, the qkv projection's S fp32
// split-K planes [S][total_q][(Hq + 2 Hkv) D] with its bias (or null), the positions / cos|sin table of
// grag_qkv_rope_kvstore_planes and the new tokens' cache slots; one query token per sequence (decode).  The
// new K / V land in the cache as grag_qkv_rope_kvstore_planes would store them.
GRAG_API int grag_paged_decode_mw_rope(const float* planes, int S, const void* bias, const int32_t* positions,
                                       const float* cos_sin, const int32_t* slot_mapping, const void* k_cache,
                                       const void* v_cache, void* out, int out_stride, const int32_t* block_tables,
                                       int bt_stride, const int32_t* q_start, const int32_t* ctx_len, int nseq,
                                       int total_q, int Hq, int Hkv, int D, int BS, float scale, int num_splits,
                                       int split_len, float* part_o, float* part_ml, unsigned* counters, int nw,
                                       int nblocks, int nslots, int npos, hipStream_t stream) {
  if (nseq <= 0) return 0;
  if (Hq % Hkv != 0 || Hq / Hkv > 16 || BS <= 0 || BS % 16 != 0 || (nw != 2 && nw != 4) || (D != 64 && D != 128))
    return (int)hipErrorInvalidValue;
  if (!planes || S < 1 || !positions || !cos_sin || !slot_mapping || npos < 1 || total_q < nseq)
    return (int)hipErrorInvalidValue;
  if (num_splits < 1) num_splits = 1;
  if (num_splits > 1 && (!part_o || !part_ml || !counters || split_len <= 0 || split_len % 32 != 0))
    return (int)hipErrorInvalidValue;
  if ((num_splits * 32 + 16) * 4 > nw * 2 * 2 * 32 * 2 * D) return (int)hipErrorInvalidValue;  // merge scratch
  AttnParams prm{};
  prm.k = (const bf16*)k_cache;
  prm.v = (const bf16*)v_cache;
  prm.out = (bf16*)out;
  prm.part_o = part_o;
  prm.part_ml = part_ml;
  prm.block_tables = block_tables;
  prm.q_start = q_start;
  prm.ctx_len = ctx_len;
  prm.out_stride = out_stride;
  prm.Hq = Hq;
  prm.Hkv = Hkv;
  prm.G = Hq / Hkv;
  prm.BS = BS;
  prm.bt_stride = bt_stride;
  prm.tiles_per_seq = 1;
  prm.num_splits = num_splits;
  prm.split_len = num_splits > 1 ? split_len : (1 << 30);
  prm.total_q = total_q;
  prm.scale_log2 = scale * 1.4426950408889634f;
  prm.causal = 1;
  prm.nblocks = nblocks;
  prm.rq_planes = planes;
  prm.rq_ld = (Hq + 2 * Hkv) * D;
  prm.rq_plane = (size_t)total_q * prm.rq_ld;
  prm.rq_S = S;
  prm.rq_bias = (const bf16*)bias;
  prm.rq_pos = positions;
  prm.rq_cs = cos_sin;
  prm.rq_slot = slot_mapping;
  prm.rq_nslots = nslots;
  prm.rq_npos = npos;
  if (D == 128) return nw == 4 ? launch_decode_mw<128, 4, true>(prm, nseq, counters, stream)
                               : launch_decode_mw<128, 2, true>(prm, nseq, counters, stream);
  return nw == 4 ? launch_decode_mw<64, 4, true>(prm, nseq, counters, stream)
                 : launch_decode_mw<64, 2, true>(prm, nseq, counters, stream);
}

// Contiguous (varlen) self-attention over packed QKV rows, e.g. encoder
// layers: q/k/v point at the first element of each tensor inside the packed
// row (row stride qkv_stride); seq_start [nseq+1] gives token offsets.
GRAG_API int grag_varlen_attention(const void* q, const void* k, const void* v, int qkv_stride,
                                   void* out, int out_stride, const int32_t* seq_start,
                                   const int32_t* seq_len, int nseq, int max_len, int H, int Hkv,
                                   int D, float scale, int causal, hipStream_t stream) {
  if (nseq <= 0) return 0;
  if (H % Hkv != 0) return (int)hipErrorInvalidValue;
  AttnParams prm{};
  prm.q = (const bf16*)q;
  prm.k = (const bf16*)k;
  prm.v = (const bf16*)v;
  prm.out = (bf16*)out;
  prm.q_start = seq_start;
  prm.ctx_len = seq_len;
  prm.q_stride = qkv_stride;
  prm.kv_stride = qkv_stride;
  prm.out_stride = out_stride;
  prm.Hq = H;
  prm.Hkv = Hkv;
  prm.G = H / Hkv;
  prm.BS = 1;
  prm.tiles_per_seq = (max_len * prm.G + 63) / 64;
  prm.num_splits = 1;
  prm.split_len = 1 << 30;
  prm.scale_log2 = scale * 1.4426950408889634f;
  prm.causal = causal;
  switch (D) {
    case 128: return dispatch_nw<128>(prm, nseq, 4, false, stream);
    case 64: return dispatch_nw<64>(prm, nseq, 4, false, stream);
    case 32: return dispatch_nw<32>(prm, nseq, 4, false, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

GRAG_ERR_UNIT(attention)
