// IVF search glue on the GPU:
//
//   ivf_plan_kernel   one workgroup turns the coarse probe lists [nq, nprobe] into
//                     score_topk_work items: (query, list) pairs sorted by list in
//                     LDS (bitonic), each list's queries packed 16 per item, the
//                     item's row range read from the list offsets.  Items past the
//                     real count are written empty ([0, 0) rows, no queries), so the
//                     scan launches with the static upper bound nq * nprobe and no
//                     host ever reads the count.
//   topk_merge_kernel one workgroup per query merges that query's partial top-k
//                     lists (per-wave lists of the scan kernels, plus any extra list
//                     such as the flat scan of an IVF table's append region) into
//                     the final top-k: per-wave k rounds of wave argmax over an
//                     LDS image of the candidates, then the same over the 4 wave
//                     winners' lists — no torch.topk, no host sync.
//   bitmap_update     set / clear live-row bits (deletes, upserts) with atomics,
//                     replacing a host round trip of the whole bitmap.
#include "common.h"

using namespace grag;

namespace {

constexpr int kPlanThreads = 256;  // one wave per SIMD: fits beside a resident GEMM workgroup
constexpr int kMaxPairs = 16384;  // nq * nprobe handled by one plan workgroup

__global__ __launch_bounds__(kPlanThreads) void ivf_plan_kernel(const int64_t* __restrict__ lists, int nq, int nprobe,
                                                                const int64_t* __restrict__ offsets, int nlist,
                                                                int64_t* __restrict__ work_rows,
                                                                int32_t* __restrict__ work_q,
                                                                int32_t* __restrict__ cand) {
  // dynamic LDS sized to the plan (a 256-pair plan takes 6 KB, so it co-resides with the
  // 128-KB GEMM workgroups of the engine stream instead of waiting for a free CU)
  extern __shared__ __attribute__((aligned(16))) char plan_lds[];
  int* scan = reinterpret_cast<int*>(plan_lds);
  unsigned long long* key = reinterpret_cast<unsigned long long*>(plan_lds + kPlanThreads * sizeof(int));
  const int P = nq * nprobe;
  int np2 = 1;
  while (np2 < P) np2 <<= 1;
  const int tid = threadIdx.x;
  for (int i = tid; i < np2; i += kPlanThreads) {
    unsigned long long kv = ~0ull;
    if (i < P) {
      int64_t l = lists[i];
      l = (l < 0 || l >= nlist) ? (int64_t)nlist : l;  // -1 (fewer lists than nprobe): empty sentinel list
      kv = ((unsigned long long)l << 20) | (unsigned)i;
    }
    key[i] = kv;
  }
  __syncthreads();
  // bitonic sort (ascending)
  for (int sz = 2; sz <= np2; sz <<= 1) {
    for (int st = sz >> 1; st > 0; st >>= 1) {
      for (int i = tid; i < np2; i += kPlanThreads) {
        const int j = i ^ st;
        if (j > i) {
          const bool up = (i & sz) == 0;
          const unsigned long long a = key[i], b = key[j];
          if ((a > b) == up) {
            key[i] = b;
            key[j] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // each thread owns a contiguous chunk; group start = last position whose list differs
  // from its predecessor; rank = position - group start; an item starts at rank % 16 == 0
  const int E = (P + kPlanThreads - 1) / kPlanThreads;
  const int c0 = min(P, tid * E), c1 = min(P, c0 + E);
  auto list_at = [&](int i) -> long long { return (long long)(key[i] >> 20); };
  // pass 1: last group start inside the chunk (or -1), and count of item starts
  int last_start = -1, nitems = 0;
  {
    int gs = -1;
    for (int i = c0; i < c1; ++i) {
      if (i == 0 || list_at(i) != list_at(i - 1)) gs = i;
      last_start = gs;
    }
  }
  // prefix-max of group starts across chunks (a chunk without a start inherits the previous)
  scan[tid] = last_start;
  __syncthreads();
  for (int o = 1; o < kPlanThreads; o <<= 1) {
    const int v = tid >= o ? scan[tid - o] : -1;
    __syncthreads();
    scan[tid] = max(scan[tid], v);
    __syncthreads();
  }
  const int carry_start = tid > 0 ? scan[tid - 1] : -1;
  __syncthreads();
  {
    int gs = carry_start;
    for (int i = c0; i < c1; ++i) {
      if (i == 0 || list_at(i) != list_at(i - 1)) gs = i;
      if (((i - gs) & 15) == 0) ++nitems;
    }
  }
  // exclusive prefix sum of item starts
  scan[tid] = nitems;
  __syncthreads();
  for (int o = 1; o < kPlanThreads; o <<= 1) {
    const int v = tid >= o ? scan[tid - o] : 0;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  int item = (tid > 0 ? scan[tid - 1] : 0) - 1;
  const int W = scan[kPlanThreads - 1];
  // every slot of every item starts empty (items are shared by adjacent threads' chunks, so
  // this pass is separated from the slot writes by a barrier)
  for (int e = tid; e < P * 16; e += kPlanThreads) work_q[e] = -1;
  __syncthreads();
  {
    int gs = carry_start;
    for (int i = c0; i < c1; ++i) {
      const long long l = list_at(i);
      if (i == 0 || l != list_at(i - 1)) gs = i;
      const int rank = i - gs;
      if ((rank & 15) == 0) {
        ++item;
        const bool real = l < nlist;
        work_rows[2 * item] = real ? offsets[l] : 0;
        work_rows[2 * item + 1] = real ? offsets[l + 1] : 0;
      }
      const int pair = (int)(key[i] & 0xFFFFF);
      work_q[item * 16 + (rank & 15)] = l < nlist ? pair / nprobe : -1;
      cand[pair] = item * 16 + (rank & 15);
    }
  }
  // items [W, P): empty
  for (int it = W + tid; it < P; it += kPlanThreads) {
    work_rows[2 * it] = 0;
    work_rows[2 * it + 1] = 0;
  }
}

// Candidates of query q: rows r_j of the partial arrays (each row = L entries):
//   cand != nullptr : r_j = cand[q * cnt + j]
//   else (affine)   : r_j = (q / G) * A + (q % G) + j * B
// plus an optional extra list ex_s/ex_i [nq][L2].  Output [nq][k], ids -1 where empty.
constexpr int kMergeThreads = 256;
constexpr int kMergeCap = 16384;

__device__ __forceinline__ void wave_argmax(float& v, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
}

__global__ __launch_bounds__(kMergeThreads) void topk_merge_kernel(const float* __restrict__ ps,
                                                                   const int64_t* __restrict__ pi, int L,
                                                                   const int32_t* __restrict__ cand, int cnt, int G,
                                                                   int A, int B, const float* __restrict__ ex_s,
                                                                   const int64_t* __restrict__ ex_i, int L2, int k,
                                                                   float* __restrict__ out_s,
                                                                   int64_t* __restrict__ out_i) {
  // dynamic LDS: C candidate scores (sized per launch: small merges co-reside with GEMM workgroups)
  extern __shared__ __attribute__((aligned(16))) char merge_lds[];
  int64_t* wi = reinterpret_cast<int64_t*>(merge_lds);
  float* ws = reinterpret_cast<float*>(merge_lds + 4 * 32 * sizeof(int64_t));
  float* cs = ws + 4 * 32;
  const int q = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = cnt * L + L2;
  auto id_at = [&](int e) -> int64_t {
    if (e < cnt * L) {
      const int j = e / L, t = e % L;
      const int64_t r = cand ? (int64_t)cand[(int64_t)q * cnt + j] : (int64_t)(q / G) * A + (q % G) + (int64_t)j * B;
      return pi[r * L + t];
    }
    return ex_i[(int64_t)q * L2 + (e - cnt * L)];
  };
  for (int e = tid; e < C; e += kMergeThreads) {
    float s;
    int64_t id;
    if (e < cnt * L) {
      const int j = e / L, t = e % L;
      const int64_t r = cand ? (int64_t)cand[(int64_t)q * cnt + j] : (int64_t)(q / G) * A + (q % G) + (int64_t)j * B;
      s = ps[r * L + t];
      id = pi[r * L + t];
    } else {
      const int t = e - cnt * L;
      s = ex_s[(int64_t)q * L2 + t];
      id = ex_i[(int64_t)q * L2 + t];
    }
    cs[e] = id < 0 ? -INFINITY : s;  // ids are re-read only for the winners
  }
  __syncthreads();
  // each wave: top-k of its quarter of the candidates
  const int per = (C + 3) / 4;
  const int b0 = wave * per, b1 = min(C, b0 + per);
  for (int r = 0; r < k; ++r) {
    float v = -INFINITY;
    int idx = 0x7fffffff;
    for (int e = b0 + lane; e < b1; e += 64) {
      if (cs[e] > v || (cs[e] == v && e < idx)) {
        v = cs[e];
        idx = e;
      }
    }
    wave_argmax(v, idx);
    if (lane == 0) {
      ws[wave * 32 + r] = v;
      wi[wave * 32 + r] = (idx != 0x7fffffff && v != -INFINITY) ? id_at(idx) : -1;
      if (idx != 0x7fffffff) cs[idx] = -INFINITY;
    }
    __syncthreads();  // the removal is visible to the next round's scan (block-wide: waves share cs[])
  }
  // wave 0 merges the 4 sorted lists of k
  if (wave == 0) {
    for (int r = 0; r < k; ++r) {
      float v = -INFINITY;
      int idx = 0x7fffffff;
      if (lane < 4 * k) {
        const int w = lane / k, t = lane % k;
        v = ws[w * 32 + t];
        idx = lane;
        if (wi[w * 32 + t] < 0) v = -INFINITY;
      }
      wave_argmax(v, idx);
      if (lane == 0) {
        const bool ok = idx != 0x7fffffff && v != -INFINITY;
        out_s[(int64_t)q * k + r] = ok ? v : -INFINITY;
        out_i[(int64_t)q * k + r] = ok ? wi[(idx / k) * 32 + idx % k] : -1;
        if (ok) ws[(idx / k) * 32 + idx % k] = -INFINITY;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
  }
}

__global__ void bitmap_update_kernel(uint32_t* __restrict__ bm, const int64_t* __restrict__ rows, int n, int alive) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  if (r < 0) return;
  const uint32_t bit = 1u << (r & 31);
  if (alive) atomicOr(bm + (r >> 5), bit);
  else atomicAnd(bm + (r >> 5), ~bit);
}

}  // namespace

// work_rows [nq*nprobe][2] int64, work_q [nq*nprobe][16] int32, cand [nq][nprobe] int32
GRAG_API int grag_ivf_plan(const int64_t* lists, int nq, int nprobe, const int64_t* offsets, int nlist,
                           int64_t* work_rows, int32_t* work_q, int32_t* cand, hipStream_t stream) {
  if (nq <= 0 || nprobe <= 0) return 0;
  if ((long)nq * nprobe > kMaxPairs || nlist >= (1 << 30)) return (int)hipErrorInvalidValue;
  int np2 = 1;
  while (np2 < nq * nprobe) np2 <<= 1;
  const size_t lds = kPlanThreads * sizeof(int) + (size_t)np2 * sizeof(unsigned long long);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)ivf_plan_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  ivf_plan_kernel<<<1, kPlanThreads, lds, stream>>>(lists, nq, nprobe, offsets, nlist, work_rows, work_q, cand);
  return (int)hipGetLastError();
}

GRAG_API int grag_ivf_plan_max_pairs() { return kMaxPairs; }

GRAG_API int grag_topk_merge(const float* ps, const int64_t* pi, int L, const int32_t* cand, int cnt, int G, int A,
                             int B, const float* ex_s, const int64_t* ex_i, int L2, int nq, int k, float* out_s,
                             int64_t* out_i, hipStream_t stream) {
  if (nq <= 0) return 0;
  if (k < 1 || k > 32 || L < 0 || L2 < 0 || (long)cnt * L + L2 > kMergeCap || 4 * k > 64 * 2)
    return (int)hipErrorInvalidValue;
  if (4 * k > 64) return (int)hipErrorInvalidValue;  // wave-0 merge holds 4 lists of k in one wave
  const size_t lds = 4 * 32 * (sizeof(int64_t) + sizeof(float)) + ((size_t)cnt * L + L2) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)topk_merge_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  topk_merge_kernel<<<nq, kMergeThreads, lds, stream>>>(ps, pi, L, cand, cnt, G, A, B, ex_s, ex_i, L2, k, out_s,
                                                        out_i);
  return (int)hipGetLastError();
}

GRAG_API int grag_topk_merge_cap() { return kMergeCap; }

GRAG_API int grag_bitmap_update(void* bitmap, const int64_t* rows, int n, int alive, hipStream_t stream) {
  if (n <= 0) return 0;
  bitmap_update_kernel<<<(n + 255) / 256, 256, 0, stream>>>((uint32_t*)bitmap, rows, n, alive);
  return (int)hipGetLastError();
}
