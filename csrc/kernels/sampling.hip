// Fused token sampler: one 1024-thread workgroup per row.
//
//   x_i = logit_i, repetition penalty on tokens already seen (prompt + output,
//         HF/vLLM rule: x>0 ? x/pen : x*pen), then x_i /= temperature
//   greedy (temperature <= 0): argmax
//   else: exact top-k and top-p (nucleus) thresholds by 4-round radix select
//         over the order-preserving uint32 image of x (8 bits per round, LDS
//         histograms of counts or of probability mass, bin search by one
//         wave-level suffix scan), then Gumbel-max sampling over the kept
//         tokens: argmax(x_i + G_i), G_i = -log(-log u_i) from a counter-based
//         hash (seed, per-slot step counter, token).
// Every pass is vectorised 8 tokens per lane (one 16-B bf16 load, one seen-
// bitmap word per 8 tokens); the first pass computes max and the softmax
// normaliser together (online rescaling), so a top-p draw is 6 streaming
// passes over the row (L2/MALL-resident: 300 KB per row at V=152064).
// The sampled token's bit is set in the slot's seen bitmap and the slot's RNG
// counter advances on device, so the whole sampler is hipGraph-capturable.
#include "common.h"

using namespace grag;

namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;

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

struct Ctl {
  float inv_temp, pen;
  bool greedy;
  const uint32_t* seen;
};

// Load 8 adjusted logits starting at i (i % 8 == 0, i + 8 <= V).
template <typename T>
__device__ __forceinline__ void load8(const T* row, int i, const Ctl& c, float* x) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(row + i);
    const float4 b = *reinterpret_cast<const float4*>(row + i + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
    unpack8(*reinterpret_cast<const bf16x8_t*>(row + i), x);
  }
  if (c.pen != 1.f && c.seen) {
    const uint32_t w = c.seen[i >> 5] >> (i & 31);
    if (w & 0xFFu) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if ((w >> j) & 1u) x[j] = x[j] > 0.f ? x[j] / c.pen : x[j] * c.pen;
    }
  }
  if (!c.greedy) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] *= c.inv_temp;
  }
}

template <typename T>
__device__ __forceinline__ float load1(const T* row, int i, const Ctl& c) {
  float x = (float)row[i];
  if (c.pen != 1.f && c.seen && ((c.seen[i >> 5] >> (i & 31)) & 1u)) x = x > 0.f ? x / c.pen : x * c.pen;
  return c.greedy ? x : x * c.inv_temp;
}

// Apply fn(index, value) to every adjusted logit of the row.
template <typename T, typename F>
__device__ __forceinline__ void for_each(const T* row, int V, const Ctl& c, F&& fn) {
  const int V8 = V & ~7;
  for (int i = threadIdx.x * 8; i < V8; i += kThreads * 8) {
    float x[8];
    load8(row, i, c, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) fn(i + j, x[j]);
  }
  for (int i = V8 + threadIdx.x; i < V; i += kThreads) fn(i, load1(row, i, c));
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
#pragma unroll
  for (int w = 1; w < kWaves; ++w)
    if (rv[w] > v || (rv[w] == v && ri[w] < idx)) {
      v = rv[w];
      idx = ri[w];
    }
}

// Wave 0 finds the highest bin b whose inclusive suffix sum (bins b..255)
// reaches `need`; writes b and the sum of bins strictly above b.
__device__ __forceinline__ void find_bin(const float* hist, float need, uint32_t* out_b, float* out_above) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  // lane owns bins 255-4*lane .. 252-4*lane (descending)
  float h[4], own = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = hist[255 - 4 * lane - j];
    own += h[j];
  }
  float incl = own;  // inclusive prefix over lanes (descending bin order)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const float excl = incl - own;
  const bool mine = excl < need && incl >= need;
  const unsigned long long ball = __ballot(mine);
  int owner = ball ? __ffsll((long long)ball) - 1 : 63;
  if (lane == owner) {
    float acc = excl;
    int b = 255 - 4 * lane;
    int j = 0;
    for (; j < 3; ++j) {
      if (acc + h[j] >= need) break;
      acc += h[j];
    }
    b -= j;
    if (!ball) {  // rounding: take the lowest bin
      b = 0;
      acc = incl - hist[0];
    }
    *out_b = (uint32_t)b;
    *out_above = acc;
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void sample_kernel(
    const T* __restrict__ logits, int ld, int V, const float* __restrict__ temperature,
    const float* __restrict__ top_p, const int32_t* __restrict__ top_k,
    const float* __restrict__ penalty, uint32_t* __restrict__ seen, int seen_words,
    int64_t* __restrict__ rng_counter, uint64_t seed, const int32_t* __restrict__ slots,
    int32_t* __restrict__ out_tok) {
  __shared__ float red[kWaves];
  __shared__ int redi[kWaves];
  __shared__ float hist[256];
  __shared__ uint32_t sh_b;
  __shared__ float sh_above;
  const int row = blockIdx.x;
  // per-sequence state lives in persistent slots; `slots` maps batch row -> slot
  const int sl = slots ? slots[row] : row;
  const T* lr = logits + (size_t)row * ld;
  const float temp = temperature ? temperature[sl] : 1.f;
  const float tp = top_p ? top_p[sl] : 1.f;
  const int tk = top_k ? top_k[sl] : 0;
  Ctl c;
  c.greedy = !(temp > 0.f);
  c.inv_temp = c.greedy ? 1.f : 1.f / temp;
  c.pen = penalty ? penalty[sl] : 1.f;
  c.seen = seen ? seen + (size_t)sl * seen_words : nullptr;

  // pass 1: argmax + online softmax normaliser
  float mx = -INFINITY, z = 0.f;
  int mi = 0x7fffffff;
  for_each(lr, V, c, [&](int i, float x) {
    if (x > mx) {
      z = z * __expf(mx - x) + 1.f;
      mx = x;
      mi = i;
    } else if (x > -INFINITY) {
      z += __expf(x - mx);
    }
  });
  // combine (max, z) across the block
  float bm = mx;
  int bi = mi;
  block_argmax(bm, bi, red, redi);
  z = mx == -INFINITY ? 0.f : z * __expf(mx - bm);
  z = block_sum(z, red);
  mx = bm;
  int token = bi;

  if (!c.greedy && mx != -INFINITY) {
    uint32_t thr = 0u;  // keep keys >= thr
    if (tk > 0 && tk < V) {  // top-k by count
      uint32_t prefix = 0u, pmask = 0u;
      float need = (float)tk;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += kThreads) hist[b] = 0.f;
        __syncthreads();
        for_each(lr, V, c, [&](int, float x) {
          const uint32_t kk = fkey(x);
          if ((kk & pmask) == prefix) atomicAdd(&hist[(kk >> shift) & 255u], 1.f);
        });
        __syncthreads();
        find_bin(hist, need, &sh_b, &sh_above);
        __syncthreads();
        need -= sh_above;
        prefix |= sh_b << shift;
        pmask |= 255u << shift;
      }
      thr = prefix;
      // normaliser restricted to the top-k set
      float zk = 0.f;
      for_each(lr, V, c, [&](int, float x) {
        if (fkey(x) >= thr) zk += __expf(x - mx);
      });
      z = block_sum(zk, red);
    }
    if (tp < 1.f) {  // top-p by probability mass within the kept set
      uint32_t prefix = 0u, pmask = 0u;
      float need = tp * z;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += kThreads) hist[b] = 0.f;
        __syncthreads();
        for_each(lr, V, c, [&](int, float x) {
          const uint32_t kk = fkey(x);
          if (kk >= thr && (kk & pmask) == prefix) atomicAdd(&hist[(kk >> shift) & 255u], __expf(x - mx));
        });
        __syncthreads();
        find_bin(hist, need, &sh_b, &sh_above);
        __syncthreads();
        need -= sh_above;
        prefix |= sh_b << shift;
        pmask |= 255u << shift;
      }
      thr = prefix > thr ? prefix : thr;
    }
    // Gumbel-max over kept tokens
    const uint64_t ctr = rng_counter ? (uint64_t)rng_counter[sl] : 0ull;
    const uint64_t base = mix64(seed ^ mix64(ctr * 0x100000001B3ull + (uint64_t)sl));
    float best = -INFINITY;
    int bidx = 0x7fffffff;
    for_each(lr, V, c, [&](int i, float x) {
      if (fkey(x) >= thr) {
        const uint64_t h = mix64(base + (uint64_t)i);
        const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
        const float y = x - __logf(-__logf(u));
        if (y > best) {
          best = y;
          bidx = i;
        }
      }
    });
    block_argmax(best, bidx, red, redi);
    if (bidx != 0x7fffffff) token = bidx;
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

// dtype: 0 = fp32 logits, 1 = bf16 logits.  ld must be a multiple of 8.
GRAG_API int grag_sample(const void* logits, int dtype, int ld, int B, int V,
                         const float* temperature, const float* top_p, const int32_t* top_k,
                         const float* penalty, uint32_t* seen, int seen_words,
                         int64_t* rng_counter, uint64_t seed, const int32_t* slots,
                         int32_t* out_tok, hipStream_t stream) {
  if (B <= 0) return 0;
  if (ld % 8 != 0) return (int)hipErrorInvalidValue;
  if (dtype == 0)
    sample_kernel<float><<<B, kThreads, 0, stream>>>((const float*)logits, ld, V, temperature, top_p, top_k,
                                                     penalty, seen, seen_words, rng_counter, seed, slots, out_tok);
  else
    sample_kernel<bf16><<<B, kThreads, 0, stream>>>((const bf16*)logits, ld, V, temperature, top_p, top_k,
                                                    penalty, seen, seen_words, rng_counter, seed, slots, out_tok);
  return (int)hipGetLastError();
}

GRAG_API int grag_mark_seen(const int32_t* tokens, const int32_t* rows, int n, uint32_t* seen,
                            int seen_words, int V, hipStream_t stream) {
  if (n <= 0) return 0;
  mark_seen_kernel<<<(n + 255) / 256, 256, 0, stream>>>(tokens, rows, n, seen, seen_words, V);
  return (int)hipGetLastError();
}
