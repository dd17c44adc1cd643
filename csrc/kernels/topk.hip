// Fused cosine-score + metadata-filter + top-k for the GPU vector index
// (SURVEY §2.7 N3a/N3b/N3c/N3e).
//
// Vectors are stored L2-normalised in bf16, so cosine == dot product.
// S^T[row][q] = X · Q^T on v_mfma_f32_16x16x32_bf16: A = 16 database rows read
// straight from HBM (16 B per lane; each row is read exactly once per launch),
// B = Q^T from an XOR-swizzled LDS image shared by the workgroup's 8 waves.
// A 16-row tile of 1024-d vectors is 32 KB of HBM traffic against 32*NQT MFMAs,
// so the kernel stays HBM-bound and the per-lane top-k upkeep hides under the
// loads.
//
// Top-k: every lane keeps a sorted register list (KMAX) for each of its query
// columns — a lane sees rows 4*(lane>>4)+r of each tile for query lane&15.
// At the end the four lanes of a query merge with two bitonic xor-shuffle
// rounds (top-K of two sorted lists = elementwise max against the reversed
// partner list, then a half-cleaner network), so each wave emits one list per
// query.  The host merges the per-wave partial lists (tiny) with topk.
//
// Filters (N3c): up to 4 predicates over dictionary-encoded int32 columns
// (op 1: col == val, op 2: (col & val) != 0 for multi-valued bitset columns)
// plus an optional allow-bitmap, evaluated per row inside the scan.
//
// Two modes:
//   flat : blockIdx.x = row chunk, blockIdx.y = query tile (NQT*16 queries)
//   work : blockIdx.x = work item {row range, NQT*16 query ids} (IVF probes:
//          rows of one inverted list scanned for the queries that probe it)
#include "common.h"

using namespace grag;

namespace {

constexpr int NWAVES = 8;

struct TopkParams {
  const bf16* X;
  int64_t n_rows;
  int d;
  const bf16* Q;
  int nq;
  int k;
  const int32_t* fcol[4];
  int32_t fval[4];
  int32_t fop[4];
  int nfilt;
  const uint32_t* bitmap;
  const int64_t* row_ids;
  int64_t row_begin, row_end, rows_per_wg;
  int nchunks;
  const int64_t* work_rows;  // [nwork][2]
  const int32_t* work_q;     // [nwork][NQT*16]
  // per-query equality predicate (graph traversal: one query per (edge,
  // value) pair): row passes for query q iff qcols[q_colsel[q]][row] == q_val[q]
  // (q_colsel[q] < 0 disables it for that query)
  const int32_t* qcols[8];
  const int32_t* q_colsel;
  const int32_t* q_val;
  float* out_s;
  int64_t* out_i;
};

template <int K>
__device__ __forceinline__ void list_insert(float (&v)[K], uint32_t (&id)[K], float x, uint32_t xi) {
  if (x > v[K - 1]) {
#pragma unroll
    for (int i = K - 1; i > 0; --i) {
      const bool up = x > v[i - 1];
      const bool here = x > v[i];
      id[i] = up ? id[i - 1] : (here ? xi : id[i]);
      v[i] = up ? v[i - 1] : (here ? x : v[i]);
    }
    if (x > v[0]) {
      v[0] = x;
      id[0] = xi;
    }
  }
}

template <int K>
__device__ __forceinline__ void list_merge_xor(float (&v)[K], uint32_t (&id)[K], int mask) {
  float w[K];
  uint32_t wi[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    w[i] = __shfl_xor(v[K - 1 - i], mask, 64);
    wi[i] = (uint32_t)__shfl_xor((int)id[K - 1 - i], mask, 64);
  }
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const bool take = w[i] > v[i];
    v[i] = take ? w[i] : v[i];
    id[i] = take ? wi[i] : id[i];
  }
  // bitonic half-cleaners -> descending order
#pragma unroll
  for (int j = K / 2; j > 0; j >>= 1) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
      if ((i & j) == 0) {
        const bool sw = v[i] < v[i + j];
        const float a = v[i], b = v[i + j];
        const uint32_t ia = id[i], ib = id[i + j];
        v[i] = sw ? b : a;
        v[i + j] = sw ? a : b;
        id[i] = sw ? ib : ia;
        id[i + j] = sw ? ia : ib;
      }
    }
  }
}

__device__ __forceinline__ bool row_passes(const TopkParams& p, int64_t row) {
  if (p.bitmap && !((p.bitmap[row >> 5] >> (row & 31)) & 1u)) return false;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    if (f < p.nfilt) {
      const int32_t c = p.fcol[f][row];
      if (p.fop[f] == 1 && c != p.fval[f]) return false;
      if (p.fop[f] == 2 && (c & p.fval[f]) == 0) return false;
    }
  }
  return true;
}

template <int NQT, int KMAX>
__global__ __launch_bounds__(64 * NWAVES) void score_topk_kernel(TopkParams p) {
  constexpr int NQ = NQT * 16;
  extern __shared__ __attribute__((aligned(16))) char qlds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h4 = lane >> 4, li = lane & 15;
  const int d = p.d;
  const int RB = 2 * d;   // bytes per query row in LDS
  const int CPR = d / 8;  // 16-B chunks per row
  // XOR swizzle within aligned blocks of SWZ + 1 chunks: SWZ + 1 = the largest power of two (<= 16) dividing
  // CPR, so (ch ^ m) stays inside the row for every d % 32 == 0 (d = 32 / 64 / 96 rows have 4 / 8 / 12
  // chunks: a plain 15-mask would write past the row and past the tile)
  const int SWZ = min(16, CPR & -CPR) - 1;

  int64_t r0, r1;
  int64_t slot_base;
  if (p.work_rows) {
    r0 = p.work_rows[2 * blockIdx.x];
    r1 = p.work_rows[2 * blockIdx.x + 1];
    slot_base = (int64_t)blockIdx.x * NQ;
  } else {
    r0 = p.row_begin + (int64_t)blockIdx.x * p.rows_per_wg;
    r1 = r0 + p.rows_per_wg;
    if (r1 > p.row_end) r1 = p.row_end;
    slot_base = ((int64_t)blockIdx.y * p.nchunks + blockIdx.x) * NQ;
  }

  // stage the query tile: row qq, chunk ch -> qq*RB + ((ch ^ (qq & SWZ)) << 4)
  for (int c = threadIdx.x; c < NQ * CPR; c += 64 * NWAVES) {
    const int qq = c / CPR, ch = c % CPR;
    int qidx;
    if (p.work_rows) qidx = p.work_q[(int64_t)blockIdx.x * NQ + qq];
    else qidx = blockIdx.y * NQ + qq;
    bf16x8_t val = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    if (qidx >= 0 && qidx < p.nq) val = *reinterpret_cast<const bf16x8_t*>(p.Q + (int64_t)qidx * d + ch * 8);
    *reinterpret_cast<bf16x8_t*>(qlds + qq * RB + ((ch ^ (qq & SWZ)) << 4)) = val;
  }
  __syncthreads();

  // per-lane per-query predicate (column selector, value)
  int qsel[NQT], qv[NQT];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    qsel[qt] = -1;
    qv[qt] = 0;
    if (p.q_colsel) {
      const int qq = qt * 16 + li;
      const int qidx = p.work_rows ? p.work_q[(int64_t)blockIdx.x * NQ + qq] : (int)blockIdx.y * NQ + qq;
      if (qidx >= 0 && qidx < p.nq) {
        qsel[qt] = p.q_colsel[qidx];
        qv[qt] = p.q_val[qidx];
      }
    }
  }

  float ls[NQT][KMAX];
  uint32_t lid[NQT][KMAX];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      ls[qt][i] = -INFINITY;
      lid[qt][i] = 0xFFFFFFFFu;
    }

  const int nc = d / 32;
  for (int64_t t0 = r0 + wave * 16; t0 < r1; t0 += 16 * NWAVES) {
    int64_t lrow = t0 + li;
    if (lrow >= r1) lrow = r1 - 1;
    const bf16* xp = p.X + lrow * d + 8 * h4;
    f32x4_t acc[NQT];
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) acc[qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nc; c += 4) {
      bf16x8_t a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (c + u < nc) a[u] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(xp + 32 * (c + u)));
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (c + u < nc) {
#pragma unroll
          for (int qt = 0; qt < NQT; ++qt) {
            const int qq = qt * 16 + li;
            const int ch = 4 * (c + u) + h4;
            const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(qlds + qq * RB + ((ch ^ (qq & SWZ)) << 4));
            acc[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b, acc[qt], 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = t0 + 4 * h4 + r;
      const bool ok = row < r1 && row_passes(p, row);
      const uint32_t off = (uint32_t)(row - r0);
#pragma unroll
      for (int qt = 0; qt < NQT; ++qt) {
        bool okq = ok;
        if (qsel[qt] >= 0 && okq) okq = p.qcols[qsel[qt]][row] == qv[qt];
        list_insert<KMAX>(ls[qt], lid[qt], okq ? acc[qt][r] : -INFINITY, off);
      }
    }
  }

#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    list_merge_xor<KMAX>(ls[qt], lid[qt], 16);
    list_merge_xor<KMAX>(ls[qt], lid[qt], 32);
  }
  if (h4 != 0) return;
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    const int64_t slot = ((slot_base + qt * 16 + li) * NWAVES + wave) * p.k;
    for (int i = 0; i < p.k; ++i) {
      const bool valid = ls[qt][i] != -INFINITY && lid[qt][i] != 0xFFFFFFFFu;
      const int64_t row = r0 + (int64_t)lid[qt][i];
      p.out_s[slot + i] = ls[qt][i];
      p.out_i[slot + i] = valid ? (p.row_ids ? p.row_ids[row] : row) : -1;
    }
  }
}

template <int NQT, int KMAX>
int launch_topk(const TopkParams& prm, dim3 grid, hipStream_t stream) {
  const size_t lds = (size_t)NQT * 16 * prm.d * 2;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)score_topk_kernel<NQT, KMAX>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  score_topk_kernel<NQT, KMAX><<<grid, 64 * NWAVES, lds, stream>>>(prm);
  return (int)hipGetLastError();
}

int dispatch(const TopkParams& prm, int nqt, int kmax, dim3 grid, hipStream_t stream) {
  if (kmax == 16) {
    if (nqt == 1) return launch_topk<1, 16>(prm, grid, stream);
    if (nqt == 2) return launch_topk<2, 16>(prm, grid, stream);
    if (nqt == 4) return launch_topk<4, 16>(prm, grid, stream);
  } else if (kmax == 32) {
    if (nqt == 1) return launch_topk<1, 32>(prm, grid, stream);
    if (nqt == 2) return launch_topk<2, 32>(prm, grid, stream);
  }
  return (int)hipErrorInvalidValue;
}

void fill_qfilters(TopkParams& prm, const int32_t* const* qcols, int nqcols, const int32_t* q_colsel,
                   const int32_t* q_val) {
  for (int i = 0; i < 8; ++i) prm.qcols[i] = (qcols && i < nqcols) ? qcols[i] : nullptr;
  prm.q_colsel = q_colsel;
  prm.q_val = q_val;
}

void fill_filters(TopkParams& prm, const int32_t* const* fcols, const int32_t* fvals,
                  const int32_t* fops, int nfilt) {
  prm.nfilt = nfilt;
  for (int i = 0; i < 4; ++i) {
    prm.fcol[i] = i < nfilt ? fcols[i] : nullptr;
    prm.fval[i] = i < nfilt ? fvals[i] : 0;
    prm.fop[i] = i < nfilt ? fops[i] : 0;
  }
}

}  // namespace

GRAG_API int grag_topk_num_waves() { return NWAVES; }

// Flat scan.  Output slots: [nqtiles][nchunks][nqt*16][NWAVES][k].
GRAG_API int grag_score_topk_flat(const void* X, int64_t row_begin, int64_t row_end,
                                  int64_t rows_per_wg, int d, const void* Q, int nq, int k,
                                  int nqt, int kmax, const int32_t* const* fcols,
                                  const int32_t* fvals, const int32_t* fops, int nfilt,
                                  const uint32_t* bitmap, const int64_t* row_ids,
                                  const int32_t* const* qcols, int nqcols, const int32_t* q_colsel,
                                  const int32_t* q_val, float* out_s, int64_t* out_i,
                                  hipStream_t stream) {
  if (nq <= 0 || row_end <= row_begin) return 0;
  if (nqcols > 8) return (int)hipErrorInvalidValue;
  if (d % 32 != 0 || k > kmax || nfilt > 4 || rows_per_wg <= 0) return (int)hipErrorInvalidValue;
  TopkParams prm{};
  prm.X = (const bf16*)X;
  prm.n_rows = row_end;
  prm.d = d;
  prm.Q = (const bf16*)Q;
  prm.nq = nq;
  prm.k = k;
  fill_filters(prm, fcols, fvals, fops, nfilt);
  prm.bitmap = bitmap;
  prm.row_ids = row_ids;
  prm.row_begin = row_begin;
  prm.row_end = row_end;
  prm.rows_per_wg = rows_per_wg;
  prm.nchunks = (int)((row_end - row_begin + rows_per_wg - 1) / rows_per_wg);
  fill_qfilters(prm, qcols, nqcols, q_colsel, q_val);
  prm.out_s = out_s;
  prm.out_i = out_i;
  const int nqtiles = (nq + nqt * 16 - 1) / (nqt * 16);
  return dispatch(prm, nqt, kmax, dim3(prm.nchunks, nqtiles), stream);
}

// Work-item scan (IVF).  Output slots: [nwork][nqt*16][NWAVES][k].
GRAG_API int grag_score_topk_work(const void* X, int d, const void* Q, int nq, int k, int nqt,
                                  int kmax, const int64_t* work_rows, const int32_t* work_q,
                                  int nwork, const int32_t* const* fcols, const int32_t* fvals,
                                  const int32_t* fops, int nfilt, const uint32_t* bitmap,
                                  const int64_t* row_ids, const int32_t* const* qcols, int nqcols,
                                  const int32_t* q_colsel, const int32_t* q_val, float* out_s,
                                  int64_t* out_i, hipStream_t stream) {
  if (nwork <= 0) return 0;
  if (nqcols > 8) return (int)hipErrorInvalidValue;
  if (d % 32 != 0 || k > kmax || nfilt > 4) return (int)hipErrorInvalidValue;
  TopkParams prm{};
  prm.X = (const bf16*)X;
  prm.d = d;
  prm.Q = (const bf16*)Q;
  prm.nq = nq;
  prm.k = k;
  fill_filters(prm, fcols, fvals, fops, nfilt);
  prm.bitmap = bitmap;
  prm.row_ids = row_ids;
  prm.work_rows = work_rows;
  prm.work_q = work_q;
  fill_qfilters(prm, qcols, nqcols, q_colsel, q_val);
  prm.out_s = out_s;
  prm.out_i = out_i;
  return dispatch(prm, nqt, kmax, dim3(nwork), stream);
}
