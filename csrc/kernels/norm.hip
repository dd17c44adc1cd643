// Normalisation kernels: fused residual-add + RMSNorm (Qwen2, N1b),
// fused bias + residual + LayerNorm (BERT-family encoders, N2d),
// fused word/pos/type embedding gather + LayerNorm (N2a) and the plain
// token-embedding gather used by the decoder (N1a).
//
// Design: one 256-thread block per row, the row held in registers as 16-B
// bf16x8 vectors (Guideline 13), fp32 statistics, one LDS round trip per
// reduction.  These ops are HBM-bound; at H=3584 a row is 7 KB read + 7 KB
// written (+7 KB residual each way when fused), which is why the residual add
// is folded in instead of being a separate pass.
#include "common.h"
#include <string.h>

using namespace grag;

namespace {

constexpr int kThreads = 256;

template <int VPT>
__global__ __launch_bounds__(kThreads) void rmsnorm_kernel(
    const bf16* __restrict__ x, bf16* __restrict__ residual, const bf16* __restrict__ w,
    bf16* __restrict__ out, int H, float eps) {
  __shared__ float red[kThreads / 64];
  const int row = blockIdx.x;
  const int nvec = H >> 3;
  const bf16x8_t* xr = reinterpret_cast<const bf16x8_t*>(x + (size_t)row * H);
  bf16x8_t* rr = residual ? reinterpret_cast<bf16x8_t*>(residual + (size_t)row * H) : nullptr;
  float v[VPT][8];
  float ss = 0.f;
  // gamma is loaded before the reduction, so its latency overlaps the row loads instead of following the
  // block sum (at decode batches of 1-16 rows these kernels are latency chains, not bandwidth)
  const bf16x8_t* wr = reinterpret_cast<const bf16x8_t*>(w);
  bf16x8_t gv[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) gv[i] = wr[idx];
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
      float a[8];
      unpack8(xr[idx], a);
      if (rr) {
        float b[8];
        unpack8(rr[idx], b);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += b[j];
        // the residual stream is kept in bf16, so normalise the rounded sum
        bf16x8_t s = pack8(a);
        rr[idx] = s;
        unpack8(s, a);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = a[j];
        ss += a[j] * a[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
  bf16x8_t* orow = reinterpret_cast<bf16x8_t*>(out + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
      float g[8], o[8];
      unpack8(gv[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * g[j];
      orow[idx] = pack8(o);
    }
  }
}

// Split-K reduce fused into the decoder's block boundary: h = sum_s ws[s] (fp32
// planes a split-K projection left behind, ops/linear.py linear_deferred),
// residual += h (rounded to bf16, the residual stream's precision), out =
// RMSNorm(residual) * w.  Replaces splitk_reduce (fp32 planes -> bf16 h) +
// rmsnorm (h + residual): one launch and one bf16 round trip of h fewer per
// o_proj / down_proj at decode batches, and h is never rounded before the add.
constexpr int kFewRows = 16;
template <int VPT>
__global__ __launch_bounds__(kThreads) void splitk_rmsnorm_kernel(
    const float* __restrict__ ws, int S, size_t plane, bf16* __restrict__ residual,
    const bf16* __restrict__ w, bf16* __restrict__ out, int H, float eps) {
  __shared__ float red[kThreads / 64];
  const int row = blockIdx.x;
  const int nvec = H >> 3;
  const float* hr = ws + (size_t)row * H;
  bf16x8_t* rr = reinterpret_cast<bf16x8_t*>(residual + (size_t)row * H);
  float v[VPT][8];
  float ss = 0.f;
  const bf16x8_t* wr = reinterpret_cast<const bf16x8_t*>(w);
  bf16x8_t gv[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) gv[i] = wr[idx];
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
      float a[8];
      unpack8(rr[idx], a);
      if (gridDim.x <= kFewRows) {
        // a few rows (small-batch decode): latency-bound, every plane's loads in flight together (common.h
        // plane_acc4; residual first, then plane order, as the loop below)
        f32x4_t a0 = f32x4_t{a[0], a[1], a[2], a[3]}, a1 = f32x4_t{a[4], a[5], a[6], a[7]};
        plane_acc4(a0, hr + idx * 8, plane, S);
        plane_acc4(a1, hr + idx * 8 + 4, plane, S);
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[j] = a0[j]; a[j + 4] = a1[j]; }
      } else {  // many rows: bandwidth-bound, no wasted plane reads (the branch-free pass: 9.3 -> 12.8 us at B176)
#pragma unroll 4
        for (int sp = 0; sp < S; ++sp) {
          const float* q = hr + sp * plane + idx * 8;
          const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(q), x1 = *reinterpret_cast<const f32x4_t*>(q + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { a[j] += x0[j]; a[j + 4] += x1[j]; }
        }
      }
      bf16x8_t sum = pack8(a);
      rr[idx] = sum;
      unpack8(sum, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = a[j];
        ss += a[j] * a[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
  bf16x8_t* orow = reinterpret_cast<bf16x8_t*>(out + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
      float g[8], o[8];
      unpack8(gv[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * g[j];
      orow[idx] = pack8(o);
    }
  }
}

// y = LN(x [+ bias] [+ residual]) * gamma + beta.
// WRITEBACK (pre-LN decoders, GPT-2): the bf16-rounded sum x + bias + residual
// is stored back into `residual` (the residual stream) before it is
// normalised, so a pre-LN block boundary is one pass over the row:
// residual += h + b ; y = LN(residual).
template <int VPT, bool WRITEBACK>
__global__ __launch_bounds__(kThreads) void layernorm_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ bias, bf16* __restrict__ residual,
    const bf16* __restrict__ gamma, const bf16* __restrict__ beta, bf16* __restrict__ out, int H,
    float eps) {
  __shared__ float red[kThreads / 64];
  const int row = blockIdx.x;
  const int nvec = H >> 3;
  const bf16x8_t* xr = reinterpret_cast<const bf16x8_t*>(x + (size_t)row * H);
  bf16x8_t* rr = residual ? reinterpret_cast<bf16x8_t*>(residual + (size_t)row * H) : nullptr;
  const bf16x8_t* br = bias ? reinterpret_cast<const bf16x8_t*>(bias) : nullptr;
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    if (idx < nvec) {
      unpack8(xr[idx], v[i]);
      if (br) {
        float b[8];
        unpack8(br[idx], b);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += b[j];
      }
      if (rr) {
        float b[8];
        unpack8(rr[idx], b);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += b[j];
        if (WRITEBACK) {  // the stream is bf16: normalise the rounded sum
          const bf16x8_t sum = pack8(v[i]);
          rr[idx] = sum;
          unpack8(sum, v[i]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = block_sum(s, red) / (float)H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        s2 += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum(s2, red) / (float)H + eps);
  const bf16x8_t* gr = reinterpret_cast<const bf16x8_t*>(gamma);
  const bf16x8_t* er = reinterpret_cast<const bf16x8_t*>(beta);
  bf16x8_t* orow = reinterpret_cast<bf16x8_t*>(out + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
      float g[8], b[8], o[8];
      unpack8(gr[idx], g);
      unpack8(er[idx], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * inv * g[j] + b[j];
      orow[idx] = pack8(o);
    }
  }
}

// BERT embeddings: LN(word[id] + pos[p] + type[tt]) — one block per token.
template <int VPT>
__global__ __launch_bounds__(kThreads) void bert_embed_ln_kernel(
    const int32_t* __restrict__ ids, const int32_t* __restrict__ pos_ids,
    const int32_t* __restrict__ type_ids, const bf16* __restrict__ word,
    const bf16* __restrict__ pos, const bf16* __restrict__ type, const bf16* __restrict__ gamma,
    const bf16* __restrict__ beta, bf16* __restrict__ out, int H, int V, int P, float eps) {
  __shared__ float red[kThreads / 64];
  const int t = blockIdx.x;
  const int nvec = H >> 3;
  int tid = ids[t], pid = pos_ids[t];
  if (!index_ok(tid, V, ERR_BERT_TOKEN)) tid = 0;  // (workgroup-uniform) reported; row 0 read instead
  if (!index_ok(pid, P, ERR_BERT_TOKEN)) pid = 0;
  const bf16x8_t* wr = reinterpret_cast<const bf16x8_t*>(word + (size_t)tid * H);
  const bf16x8_t* pr = reinterpret_cast<const bf16x8_t*>(pos + (size_t)pid * H);
  const bf16x8_t* tr =
      reinterpret_cast<const bf16x8_t*>(type + (size_t)(type_ids ? type_ids[t] : 0) * H);
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    if (idx < nvec) {
      float a[8], b[8], c[8];
      unpack8(wr[idx], a);
      unpack8(pr[idx], b);
      unpack8(tr[idx], c);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = a[j] + b[j] + c[j];
        s += v[i][j];
      }
    }
  }
  const float mean = block_sum(s, red) / (float)H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        s2 += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum(s2, red) / (float)H + eps);
  const bf16x8_t* gr = reinterpret_cast<const bf16x8_t*>(gamma);
  const bf16x8_t* er = reinterpret_cast<const bf16x8_t*>(beta);
  bf16x8_t* orow = reinterpret_cast<bf16x8_t*>(out + (size_t)t * H);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
      float g[8], b[8], o[8];
      unpack8(gr[idx], g);
      unpack8(er[idx], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * inv * g[j] + b[j];
      orow[idx] = pack8(o);
    }
  }
}

// out[t] = table[ids[t]] — 16 B per lane, grid-stride over (token, vec).
__global__ __launch_bounds__(kThreads) void embed_gather_kernel(const int32_t* __restrict__ ids,
                                                                const bf16* __restrict__ table,
                                                                bf16* __restrict__ out, int T,
                                                                int H, int V) {
  const int nvec = H >> 3;
  const size_t total = (size_t)T * nvec;
  for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < total;
       i += (size_t)gridDim.x * kThreads) {
    const int t = (int)(i / nvec), v = (int)(i % nvec);
    int id = ids[t];
    if (!index_ok(id, V, ERR_EMBED_TOKEN)) id = 0;  // reported (ops/_lib.py raises at the next sync)
    reinterpret_cast<bf16x8_t*>(out + (size_t)t * H)[v] =
        reinterpret_cast<const bf16x8_t*>(table + (size_t)id * H)[v];
  }
}

int vpt_for(int H) {
  const int nvec = H / 8;
  if (nvec <= kThreads) return 1;
  if (nvec <= 2 * kThreads) return 2;
  if (nvec <= 4 * kThreads) return 4;
  return 8;
}

}  // namespace

GRAG_API int grag_rmsnorm(const void* x, void* residual, const void* w, void* out, int T, int H,
                          float eps, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8 != 0 || H > 8 * 8 * kThreads) return (int)hipErrorInvalidValue;
  const bf16* xp = (const bf16*)x;
  bf16* rp = (bf16*)residual;
  switch (vpt_for(H)) {
    case 1: rmsnorm_kernel<1><<<T, kThreads, 0, stream>>>(xp, rp, (const bf16*)w, (bf16*)out, H, eps); break;
    case 2: rmsnorm_kernel<2><<<T, kThreads, 0, stream>>>(xp, rp, (const bf16*)w, (bf16*)out, H, eps); break;
    case 4: rmsnorm_kernel<4><<<T, kThreads, 0, stream>>>(xp, rp, (const bf16*)w, (bf16*)out, H, eps); break;
    default: rmsnorm_kernel<8><<<T, kThreads, 0, stream>>>(xp, rp, (const bf16*)w, (bf16*)out, H, eps); break;
  }
  return (int)hipGetLastError();
}

// residual += sum_s ws[s] ; out = RMSNorm(residual) * w   (ws: S fp32 planes [T][H], 16-B aligned)
// Small batches (1-16 rows, the reference's 1-4 live sequences): splitk_rmsnorm_kernel gives a row ONE
// workgroup, which then reads all S planes of the row alone (7-9 x 14 KB at Qwen2-7B: 5.6 us at B = 1).
// Here a row is cut into 64-unit chunks (8 columns per unit), one 64-thread workgroup each: every chunk sums
// its planes into the residual (bf16, as the one-block kernel) and its share of sum(h^2); the chunk sums go
// to part_ss and an agent-scope ticket per row names the last arriving chunk (release / acquire fences as
// gemm_stream.hip), which adds the chunk sums in chunk order and normalises the whole row.  The ticket resets
// itself, so the launch replays inside hipGraphs.
__global__ __launch_bounds__(64) void splitk_rmsnorm_small_kernel(
    const float* __restrict__ ws, int S, size_t plane, bf16* __restrict__ residual, const bf16* __restrict__ w,
    bf16* __restrict__ out, int H, float eps, float* __restrict__ part_ss, unsigned* __restrict__ counters) {
  const int row = blockIdx.x, c = blockIdx.y, nch = gridDim.y;
  const int nvec = H >> 3;
  const int u = c * 64 + threadIdx.x;
  const float* hr = ws + (size_t)row * H;
  bf16x8_t* rr = reinterpret_cast<bf16x8_t*>(residual + (size_t)row * H);
  float ss = 0.f;
  if (u < nvec) {
    float a[8];
    unpack8(rr[u], a);
#pragma unroll 8
    for (int sp = 0; sp < S; ++sp) {
      const float* q = hr + sp * plane + u * 8;
      const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(q), x1 = *reinterpret_cast<const f32x4_t*>(q + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { a[j] += x0[j]; a[j + 4] += x1[j]; }
    }
    const bf16x8_t sum = pack8(a);
    rr[u] = sum;
    unpack8(sum, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  __shared__ unsigned last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's residual store landed before the release
  __syncthreads();
  if (threadIdx.x == 0) {
    part_ss[(size_t)row * nch + c] = ss;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned tk = __hip_atomic_fetch_add(&counters[row], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk >= (unsigned)nch) report_index_error(ERR_TICKET, tk);  // stale / shared ticket word
    last = tk == (unsigned)(nch - 1) ? 1u : 0u;
    if (last) {
      __hip_atomic_store(&counters[row], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  float tot = 0.f;
  for (int k = 0; k < nch; ++k) tot += part_ss[(size_t)row * nch + k];  // chunk order: deterministic
  const float inv = rsqrtf(tot / (float)H + eps);
  const bf16x8_t* wr = reinterpret_cast<const bf16x8_t*>(w);
  bf16x8_t* orow = reinterpret_cast<bf16x8_t*>(out + (size_t)row * H);
  for (int v = threadIdx.x; v < nvec; v += 64) {
    float a[8], g[8];
    unpack8(rr[v], a);
    unpack8(wr[v], g);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = a[j] * inv * g[j];
    orow[v] = pack8(a);
  }
}

// Small-batch form of grag_splitk_add_rmsnorm (T <= 64 rows): part_ss >= T * ceil(H / 512) floats of scratch,
// counters >= T zero-initialised uint32 words (each reset by its last arriver).
GRAG_API int grag_splitk_add_rmsnorm_small(const void* ws, int S, void* residual, const void* w, void* out, int T,
                                           int H, float eps, float* part_ss, unsigned* counters,
                                           hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8 != 0 || S < 1 || ws == nullptr || residual == nullptr || !part_ss || !counters || T > 64)
    return (int)hipErrorInvalidValue;
  const int nch = (H / 8 + 63) / 64;
  splitk_rmsnorm_small_kernel<<<dim3(T, nch), 64, 0, stream>>>((const float*)ws, S, (size_t)T * H, (bf16*)residual,
                                                              (const bf16*)w, (bf16*)out, H, eps, part_ss, counters);
  return (int)hipGetLastError();
}

GRAG_API int grag_splitk_add_rmsnorm(const void* ws, int S, void* residual, const void* w, void* out, int T,
                                     int H, float eps, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8 != 0 || H > 8 * 8 * kThreads || S < 1 || ws == nullptr || residual == nullptr)
    return (int)hipErrorInvalidValue;
  const size_t plane = (size_t)T * H;
  const float* wp = (const float*)ws;
  bf16* rp = (bf16*)residual;
#define SRN(V) splitk_rmsnorm_kernel<V><<<T, kThreads, 0, stream>>>(wp, S, plane, rp, (const bf16*)w, (bf16*)out, H, eps)
  switch (vpt_for(H)) {
    case 1: SRN(1); break;
    case 2: SRN(2); break;
    case 4: SRN(4); break;
    default: SRN(8); break;
  }
#undef SRN
  return (int)hipGetLastError();
}

template <bool WB>
static int launch_layernorm(const void* x, const void* bias, void* residual, const void* gamma,
                            const void* beta, void* out, int T, int H, float eps,
                            hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8 != 0 || H > 8 * 8 * kThreads) return (int)hipErrorInvalidValue;
  auto args = [&](auto kern) {
    kern<<<T, kThreads, 0, stream>>>((const bf16*)x, (const bf16*)bias, (bf16*)residual,
                                     (const bf16*)gamma, (const bf16*)beta, (bf16*)out, H, eps);
  };
  switch (vpt_for(H)) {
    case 1: args(layernorm_kernel<1, WB>); break;
    case 2: args(layernorm_kernel<2, WB>); break;
    case 4: args(layernorm_kernel<4, WB>); break;
    default: args(layernorm_kernel<8, WB>); break;
  }
  return (int)hipGetLastError();
}

GRAG_API int grag_layernorm(const void* x, const void* bias, const void* residual,
                            const void* gamma, const void* beta, void* out, int T, int H,
                            float eps, hipStream_t stream) {
  return launch_layernorm<false>(x, bias, const_cast<void*>(residual), gamma, beta, out, T, H, eps,
                                 stream);
}

// Pre-LN block boundary: residual += x (+ bias), out = LN(residual).
GRAG_API int grag_add_layernorm(const void* x, const void* bias, void* residual,
                                const void* gamma, const void* beta, void* out, int T, int H,
                                float eps, hipStream_t stream) {
  if (residual == nullptr) return (int)hipErrorInvalidValue;
  return launch_layernorm<true>(x, bias, residual, gamma, beta, out, T, H, eps, stream);
}

GRAG_API int grag_bert_embed_ln(const int32_t* ids, const int32_t* pos_ids,
                                const int32_t* type_ids, const void* word, const void* pos,
                                const void* type, const void* gamma, const void* beta, void* out,
                                int T, int H, int V, int P, float eps, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8 != 0 || H > 8 * 8 * kThreads) return (int)hipErrorInvalidValue;
  auto args = [&](auto kern) {
    kern<<<T, kThreads, 0, stream>>>(ids, pos_ids, type_ids, (const bf16*)word, (const bf16*)pos,
                                     (const bf16*)type, (const bf16*)gamma, (const bf16*)beta,
                                     (bf16*)out, H, V, P, eps);
  };
  switch (vpt_for(H)) {
    case 1: args(bert_embed_ln_kernel<1>); break;
    case 2: args(bert_embed_ln_kernel<2>); break;
    case 4: args(bert_embed_ln_kernel<4>); break;
    default: args(bert_embed_ln_kernel<8>); break;
  }
  return (int)hipGetLastError();
}

GRAG_API int grag_embed_gather(const int32_t* ids, const void* table, void* out, int T, int H, int V,
                               hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8 != 0) return (int)hipErrorInvalidValue;
  const size_t total = (size_t)T * (H / 8);
  int grid = (int)((total + kThreads - 1) / kThreads);
  if (grid > 4096) grid = 4096;
  embed_gather_kernel<<<grid, kThreads, 0, stream>>>(ids, (const bf16*)table, (bf16*)out, T, H, V);
  return (int)hipGetLastError();
}

GRAG_ERR_UNIT(norm)

// The index guard's error block (common.h): pinned, device-mapped, coherent host memory, so a kernel's
// report is visible to the host without a copy.  Returns the host address (nullptr when no device);
// *dev_out receives the device address every unit's grag_err_bind_* takes.
GRAG_API void* grag_err_alloc(void** dev_out) {
  void* h = nullptr;
  if (hipHostMalloc(&h, 256, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  memset(h, 0, 256);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) d = h;
  *dev_out = d;
  return h;
}
