// Fused token sampler: one workgroup per sequence row.
//
//   x_i = logit_i, repetition penalty on tokens already seen (prompt + output,
//         HF/vLLM rule: x>0 ? x/pen : x*pen), then x_i /= temperature
//   greedy (temperature <= 0): argmax
//   else: exact top-k and top-p (nucleus) thresholds by 4-round radix select
//         over the order-preserving uint32 image of x (8 bits per round, LDS
//         histograms of counts or probability mass), then Gumbel-max sampling
//         over the kept tokens: argmax(x_i + G_i), G_i = -log(-log u_i).
//   The sampled token's bit is set in the per-row seen bitmap so the next
//   step's penalty needs no host round trip; the per-row RNG counter is
//   advanced on device, so the whole sampler is hipGraph-capturable.
#include "common.h"

using namespace grag;

namespace {

constexpr int kThreads = 1024;

__device__ __forceinline__ uint32_t fkey(float x) {
  const uint32_t b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
__device__ __forceinline__ float load_logit(const T* p, int i) {
  if constexpr (sizeof(T) == 4) return p[i];
  else return (float)p[i];
}

struct Ctl {
  float temp, top_p, pen;
  int top_k;
  const uint32_t* seen;
};

template <typename T>
__device__ __forceinline__ float adj(const T* row, int i, const Ctl& c) {
  float x = load_logit(row, i);
  if (c.pen != 1.f && c.seen && ((c.seen[i >> 5] >> (i & 31)) & 1u)) x = x > 0.f ? x / c.pen : x * c.pen;
  return c.temp > 0.f ? x / c.temp : x;
}

// block argmax of (value, index) — ties break to the lower index
__device__ __forceinline__ void block_argmax(float& v, int& idx, float* rv, int* ri) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
  __syncthreads();
  if (lane == 0) {
    rv[wid] = v;
    ri[wid] = idx;
  }
  __syncthreads();
  v = rv[0];
  idx = ri[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
    if (rv[w] > v || (rv[w] == v && ri[w] < idx)) {
      v = rv[w];
      idx = ri[w];
    }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void sample_kernel(
    const T* __restrict__ logits, int ld, int V, const float* __restrict__ temperature,
    const float* __restrict__ top_p, const int32_t* __restrict__ top_k,
    const float* __restrict__ penalty, uint32_t* __restrict__ seen, int seen_words,
    int64_t* __restrict__ rng_counter, uint64_t seed, const int32_t* __restrict__ slots,
    int32_t* __restrict__ out_tok) {
  __shared__ float red[kThreads / 64];
  __shared__ int redi[kThreads / 64];
  __shared__ float hist[256];
  __shared__ uint32_t sh_u32[2];
  __shared__ float sh_f[2];
  const int row = blockIdx.x;
  // per-sequence state lives in persistent slots; `slots` maps batch row -> slot
  const int sl = slots ? slots[row] : row;
  const T* lr = logits + (size_t)row * ld;
  Ctl c;
  c.temp = temperature ? temperature[sl] : 1.f;
  c.top_p = top_p ? top_p[sl] : 1.f;
  c.top_k = top_k ? top_k[sl] : 0;
  c.pen = penalty ? penalty[sl] : 1.f;
  c.seen = seen ? seen + (size_t)sl * seen_words : nullptr;

  // pass 1: max / argmax
  float mx = -INFINITY;
  int mi = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += kThreads) {
    const float x = adj(lr, i, c);
    if (x > mx) {
      mx = x;
      mi = i;
    }
  }
  block_argmax(mx, mi, red, redi);
  int token = mi;

  if (c.temp > 0.f && mx != -INFINITY) {
    uint32_t thr = 0u;  // keep keys >= thr
    // top-k threshold by count
    if (c.top_k > 0 && c.top_k < V) {
      uint32_t prefix = 0u, pmask = 0u;
      int need = c.top_k;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += kThreads) hist[b] = 0.f;
        __syncthreads();
        for (int i = threadIdx.x; i < V; i += kThreads) {
          const uint32_t kk = fkey(adj(lr, i, c));
          if ((kk & pmask) == prefix) atomicAdd(&hist[(kk >> shift) & 255u], 1.f);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          float acc = 0.f;
          int b = 255;
          for (; b > 0; --b) {
            if (acc + hist[b] >= (float)need) break;
            acc += hist[b];
          }
          sh_u32[0] = (uint32_t)b;
          sh_f[0] = acc;
        }
        __syncthreads();
        need -= (int)sh_f[0];
        prefix |= sh_u32[0] << shift;
        pmask |= 255u << shift;
        __syncthreads();
      }
      thr = prefix;
    }
    // softmax mass of the kept set
    float z = 0.f;
    for (int i = threadIdx.x; i < V; i += kThreads) {
      const float x = adj(lr, i, c);
      if (fkey(x) >= thr) z += __expf(x - mx);
    }
    z = block_sum(z, red);
    // top-p threshold by probability mass within the kept set
    if (c.top_p < 1.f) {
      uint32_t prefix = 0u, pmask = 0u;
      float need = c.top_p * z;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += kThreads) hist[b] = 0.f;
        __syncthreads();
        for (int i = threadIdx.x; i < V; i += kThreads) {
          const float x = adj(lr, i, c);
          const uint32_t kk = fkey(x);
          if (kk >= thr && (kk & pmask) == prefix) atomicAdd(&hist[(kk >> shift) & 255u], __expf(x - mx));
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          float acc = 0.f;
          int b = 255;
          for (; b > 0; --b) {
            if (acc + hist[b] >= need) break;
            acc += hist[b];
          }
          sh_u32[0] = (uint32_t)b;
          sh_f[0] = acc;
        }
        __syncthreads();
        need -= sh_f[0];
        prefix |= sh_u32[0] << shift;
        pmask |= 255u << shift;
        __syncthreads();
      }
      thr = prefix > thr ? prefix : thr;
    }
    // Gumbel-max over kept tokens
    const uint64_t ctr = rng_counter ? (uint64_t)rng_counter[sl] : 0ull;
    const uint64_t base = mix64(seed ^ mix64(ctr * 0x100000001B3ull + (uint64_t)sl));
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < V; i += kThreads) {
      const float x = adj(lr, i, c);
      if (fkey(x) >= thr) {
        const uint64_t h = mix64(base + (uint64_t)i);
        const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
        const float y = x - __logf(-__logf(u));
        if (y > best) {
          best = y;
          bi = i;
        }
      }
    }
    block_argmax(best, bi, red, redi);
    if (bi != 0x7fffffff) token = bi;
  }
  if (threadIdx.x == 0) {
    if (token < 0 || token >= V) token = 0;
    out_tok[row] = token;
    if (c.seen) atomicOr(seen + (size_t)sl * seen_words + (token >> 5), 1u << (token & 31));
    if (rng_counter) rng_counter[sl] += 1;
  }
}

// Set seen bits for prompt tokens: tokens [n] with slot index rows[n].
__global__ void mark_seen_kernel(const int32_t* __restrict__ tokens, const int32_t* __restrict__ rows,
                                 int n, uint32_t* __restrict__ seen, int seen_words, int V) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = tokens[i];
  if (t < 0 || t >= V) return;
  atomicOr(seen + (size_t)rows[i] * seen_words + (t >> 5), 1u << (t & 31));
}

}  // namespace

// dtype: 0 = fp32 logits, 1 = bf16 logits
GRAG_API int grag_sample(const void* logits, int dtype, int ld, int B, int V,
                         const float* temperature, const float* top_p, const int32_t* top_k,
                         const float* penalty, uint32_t* seen, int seen_words,
                         int64_t* rng_counter, uint64_t seed, const int32_t* slots,
                         int32_t* out_tok, hipStream_t stream) {
  if (B <= 0) return 0;
  if (dtype == 0)
    sample_kernel<float><<<B, kThreads, 0, stream>>>((const float*)logits, ld, V, temperature, top_p,
                                                     top_k, penalty, seen, seen_words, rng_counter,
                                                     seed, slots, out_tok);
  else
    sample_kernel<bf16><<<B, kThreads, 0, stream>>>((const bf16*)logits, ld, V, temperature, top_p,
                                                    top_k, penalty, seen, seen_words, rng_counter,
                                                    seed, slots, out_tok);
  return (int)hipGetLastError();
}

GRAG_API int grag_mark_seen(const int32_t* tokens, const int32_t* rows, int n, uint32_t* seen,
                            int seen_words, int V, hipStream_t stream) {
  if (n <= 0) return 0;
  mark_seen_kernel<<<(n + 255) / 256, 256, 0, stream>>>(tokens, rows, n, seen, seen_words, V);
  return (int)hipGetLastError();
}
