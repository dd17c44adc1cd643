// Fused token sampler, multi-workgroup form.
//
//   x_i = logit_i, repetition penalty on tokens already seen (prompt + output,
//         HF/vLLM rule: x>0 ? x/pen : x*pen), then x_i /= temperature
//   greedy (temperature <= 0): argmax
//   else: top-k (by count) then top-p (nucleus, by probability mass inside
//         the top-k set) thresholds by radix select, then Gumbel-max sampling
//         over the kept tokens: argmax(x_i + G_i), G_i = -log(-log u_i) from a
//         counter-based hash (seed, per-slot step counter, slot, token).
//
// Every row is split into S segments and every pass runs on B x S
// workgroups (~8K tokens each), so the whole chip works on the batch; the
// previous one-workgroup-per-row kernel kept only B CUs busy and took
// ~300 us at B = 64 over Qwen's 152K vocabulary.  Fixed launch chain, so the
// sampler is captured in the decode hipGraph:
//   max     per-segment max / argmax of the adjusted logits
//   round r (r = 0..7): every workgroup folds the S partial histograms of
//           round r-1 into the row's radix state (all workgroups of a row
//           compute the same thing; segment 0 publishes it for the next
//           launch), then histograms its own segment for round r.  Rounds 0-3
//           select the top-k threshold (counts), rounds 4-7 the top-p
//           threshold (mass exp(x - M) restricted to the top-k set, whose total
//           is the renormaliser).  Inactive rounds (top_k = 0, top_p = 1) only
//           forward the state.
//   gumbel  final threshold, per-segment Gumbel argmax over the kept tokens
//   final   per-row combine, seen-bitmap update, RNG counter advance.
// Radix keys are the fixed-point image of (M - x) (qkey), so a row's relevant
// logits spread over the bins (the raw float bits put a whole row into one bin
// of the first round).  The first digit (4 bits, every token of the row takes
// part) is histogrammed in registers + a wave butterfly; the three 8-bit
// digits after it see only the tokens of the selected bin (LDS atomics).
// Measured (scripts/microbench.py, B=64, V=152064, top-p, in a hipGraph):
// one-workgroup-per-row kernel 298 us -> this chain ~60-110 us.
#include "common.h"

using namespace grag;

namespace {

constexpr int kT = 256;   // threads per workgroup
constexpr int kNB = 256;  // bins per radix round
constexpr int kRounds = 8;
constexpr int kMaxS = 32;  // max segments per row

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Complemented fixed point (27 fractional bits) of d = M - x clamped to
// [0, 32]: larger key = more probable.  Resolution 2^-27 logit units is finer
// than the fp32 ulp of the logits; tokens with d > 32 (p < 1e-13 of the top
// token) share key 0.
__device__ __forceinline__ uint32_t qkey(float x, float M) {
  const float d = fminf(fmaxf(M - x, 0.f), 32.f) * 134217728.f;  // 2^27
  return d >= 4294967295.f ? 0u : ~(uint32_t)d;
}

struct Params {
  const void* logits;
  int ld, B, V, S, seglen;
  const float* temperature;
  const float* top_p;
  const int32_t* top_k;
  const float* penalty;
  uint32_t* seen;
  int seen_words;
  int64_t* rng_counter;
  uint64_t seed;
  const int32_t* slots;
  int32_t* out_tok;
  // workspace
  float* seg_max;    // [B][S]
  int32_t* seg_arg;  // [B][S]
  float* gval;       // [B][S]
  int32_t* gidx;     // [B][S]
  float* hist;       // [2][B][S][kNB]
  uint32_t* state;   // [2][B][4]: prefix, pmask, thr_k, need (float bits)
  // vocab-parallel (TP) form: this call sees columns [v0, v0 + V) of a Vg-token vocabulary;
  // gmax / ghist (when set) are the group-wide row max / previous-round histogram the host
  // reduced over the TP group between launches (grag_sample_tp)
  int v0, Vg;
  const float* gmax;  // [B]
  const float* ghist; // [B][kNB]
};

struct Row {
  int sl;
  float inv_temp, pen, top_p;
  int top_k;
  bool greedy;
  uint32_t* seen;
};

__device__ __forceinline__ Row row_params(const Params& p, int row) {
  Row r;
  r.sl = p.slots ? p.slots[row] : row;
  const float temp = p.temperature ? p.temperature[r.sl] : 1.f;
  r.greedy = !(temp > 0.f);
  r.inv_temp = r.greedy ? 1.f : 1.f / temp;
  r.pen = p.penalty ? p.penalty[r.sl] : 1.f;
  r.top_p = p.top_p ? p.top_p[r.sl] : 1.f;
  r.top_k = p.top_k ? p.top_k[r.sl] : 0;
  r.seen = p.seen ? p.seen + (size_t)r.sl * p.seen_words : nullptr;
  return r;
}

// Apply fn(index, adjusted value) to every logit of [lo, hi): 8 per lane per
// step from one 16-B (bf16) or two 16-B (fp32) loads + one seen-bitmap word.
template <typename T, typename F>
__device__ __forceinline__ void for_seg(const T* row, int lo, int hi, const Row& c, F&& fn, int v0 = 0) {
  // i: local column (loads), i + v0: global token id (seen bitmap, RNG stream, tie order); v0 % 8 == 0
  const int hi8 = lo + ((hi - lo) & ~7);
  const bool pen = c.pen != 1.f && c.seen;
  for (int i = lo + threadIdx.x * 8; i < hi8; i += kT * 8) {
    float x[8];
    if constexpr (sizeof(T) == 4) {
      const float4 a = *reinterpret_cast<const float4*>(row + i);
      const float4 b = *reinterpret_cast<const float4*>(row + i + 4);
      x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    } else {
      unpack8(*reinterpret_cast<const bf16x8_t*>(row + i), x);
    }
    const int g = i + v0;
    const uint32_t w = pen ? (c.seen[g >> 5] >> (g & 31)) & 0xFFu : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = x[j];
      if ((w >> j) & 1u) v = v > 0.f ? v / c.pen : v * c.pen;
      fn(g + j, c.greedy ? v : v * c.inv_temp);
    }
  }
  for (int i = hi8 + threadIdx.x; i < hi; i += kT) {
    const int g = i + v0;
    float v = (float)row[i];
    if (pen && ((c.seen[g >> 5] >> (g & 31)) & 1u)) v = v > 0.f ? v / c.pen : v * c.pen;
    fn(g, c.greedy ? v : v * c.inv_temp);
  }
}

// (value, index) max, ties to the lower index
__device__ __forceinline__ void better(float& v, int& i, float ov, int oi) {
  if (ov > v || (ov == v && oi < i)) {
    v = ov;
    i = oi;
  }
}

__device__ __forceinline__ void block_argmax(float& v, int& idx, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) better(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
  __syncthreads();
  if (lane == 0) {
    sv[wid] = v;
    si[wid] = idx;
  }
  __syncthreads();
  v = sv[0];
  idx = si[0];
#pragma unroll
  for (int w = 1; w < kT / 64; ++w) better(v, idx, sv[w], si[w]);
}

// row max from the S partial maxima (every thread gets it)
__device__ __forceinline__ float row_max(const Params& p, int row, float* sv) {
  if (p.gmax) return p.gmax[row];  // TP: the group-wide max (uniform branch)
  float m = -INFINITY;
  for (int s = threadIdx.x; s < p.S; s += kT) m = fmaxf(m, p.seg_max[row * p.S + s]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sv[threadIdx.x >> 6] = m;
  __syncthreads();
  m = sv[0];
#pragma unroll
  for (int w = 1; w < kT / 64; ++w) m = fmaxf(m, sv[w]);
  return m;
}

// Wave 0: highest bin b whose inclusive suffix sum (bins b..255) reaches
// `need`; writes b and the sum strictly above b.
__device__ __forceinline__ void find_bin(const float* hist, float need, uint32_t* out_b, float* out_above) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  float h[4], own = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = hist[255 - 4 * lane - j];
    own += h[j];
  }
  float incl = own;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const float excl = incl - own;
  const bool mine = excl < need && incl >= need;
  const unsigned long long ball = __ballot(mine);
  const int owner = ball ? __ffsll((long long)ball) - 1 : 63;
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

struct RState {
  uint32_t prefix, pmask, thr_k;
  float need;
};

__device__ __forceinline__ bool round_active(int r, const Row& c, int Vg) {
  return r < 4 ? (c.top_k > 0 && c.top_k < Vg) : (c.top_p < 1.f);
}
// Digit plan of a 4-round radix select: a 4-bit first digit (16 bins: every
// token of the row takes part, so it is histogrammed in registers, not with
// LDS atomics), then three 8-bit digits (only tokens inside the selected bin
// take part) -> 28 key bits (2^-23 logit units).
__device__ __forceinline__ int round_shift(int r) { return (r & 3) == 0 ? 28 : 28 - 8 * (r & 3); }
__device__ __forceinline__ uint32_t round_mask(int r) { return (r & 3) == 0 ? 15u : 255u; }

// Row state published by launch j (state after the round launch j-1 ran);
// j < 0: the initial state.
__device__ __forceinline__ RState load_state(const Params& p, int row, int j, const Row& c) {
  RState st;
  if (j < 0) {
    st.prefix = 0u;
    st.pmask = 0u;
    st.thr_k = 0u;
    st.need = (float)c.top_k;
    return st;
  }
  const uint32_t* s = p.state + ((size_t)(j & 1) * p.B + row) * 4;
  st.prefix = s[0];
  st.pmask = s[1];
  st.thr_k = s[2];
  st.need = __uint_as_float(s[3]);
  return st;
}

// Fold round r (histogrammed by launch j) into the row state (-> state after
// round r).  Every workgroup of the row does this identically.
__device__ void fold_round(const Params& p, int row, int r, int j, const Row& c, RState& st, float* lds_hist,
                           uint32_t* sh_b, float* sh_f) {
  if (r < 0) return;
  if (round_active(r, c, p.Vg)) {
    if (p.ghist) {  // TP: the histogram already summed over segments and ranks
      for (int b = threadIdx.x; b < kNB; b += kT) lds_hist[b] = p.ghist[(size_t)row * kNB + b];
    } else {
      const float* src = p.hist + ((size_t)(j & 1) * p.B + row) * p.S * kNB;
      for (int b = threadIdx.x; b < kNB; b += kT) {
        // all kMaxS partial loads issued back to back (clamped index, masked
        // add: no per-load branch), summed in a fixed order -> deterministic
        float v[kMaxS];
#pragma unroll
        for (int g = 0; g < kMaxS; ++g) v[g] = src[min(g, p.S - 1) * kNB + b];
        float s = 0.f;
#pragma unroll
        for (int g = 0; g < kMaxS; ++g) s += g < p.S ? v[g] : 0.f;
        lds_hist[b] = s;
      }
    }
    __syncthreads();
    if (r == 4) {  // first top-p round: its histogram holds the whole kept mass
      float tot = 0.f;
      for (int b = threadIdx.x; b < kNB; b += kT) tot += lds_hist[b];
      tot = wave_sum(tot);
      if ((threadIdx.x & 63) == 0) sh_f[1 + (threadIdx.x >> 6)] = tot;
      __syncthreads();
      tot = 0.f;
#pragma unroll
      for (int w = 0; w < kT / 64; ++w) tot += sh_f[1 + w];
      st.need = c.top_p * tot;
    }
    find_bin(lds_hist, st.need, sh_b, sh_f);
    __syncthreads();
    st.need -= sh_f[0];
    st.prefix |= sh_b[0] << round_shift(r);
    st.pmask |= round_mask(r) << round_shift(r);
    __syncthreads();
  }
  if (r == 3) {  // top-k threshold complete (0 = keep all); top-p starts fresh inside it
    st.thr_k = round_active(3, c, p.Vg) ? st.prefix : 0u;
    st.prefix = 0u;
    st.pmask = 0u;
  }
}

// ---------------------------------------------------------------- kernels
template <typename T>
__global__ __launch_bounds__(kT) void samp_max_kernel(Params p) {
  __shared__ float sv[kT / 64];
  __shared__ int si[kT / 64];
  const int row = blockIdx.x, seg = blockIdx.y;
  const Row c = row_params(p, row);
  const T* lr = (const T*)p.logits + (size_t)row * p.ld;
  const int lo = seg * p.seglen, hi = min(p.V, lo + p.seglen);
  float m = -INFINITY;
  int mi = 0x7fffffff;
  for_seg(lr, lo, hi, c, [&](int i, float x) { better(m, mi, x, i); }, p.v0);
  block_argmax(m, mi, sv, si);
  if (threadIdx.x == 0) {
    p.seg_max[row * p.S + seg] = m;
    p.seg_arg[row * p.S + seg] = mi;
  }
}

// Launch j runs round r: fold the previous launch's round r_prev (segment 0
// publishes the resulting state), then histogram round r over its segment.
template <typename T>
__global__ __launch_bounds__(kT) void samp_round_kernel(Params p, int r, int r_prev, int j) {
  __shared__ float hist[kNB];
  __shared__ float sv[kT / 64];
  __shared__ uint32_t sh_b[1];
  __shared__ float sh_f[1 + kT / 64];
  const int row = blockIdx.x, seg = blockIdx.y;
  const Row c = row_params(p, row);
  if (c.greedy) return;
  const float M = row_max(p, row, sv);
  RState st = load_state(p, row, j - 1 >= 1 ? j - 1 : -1, c);
  if (r_prev >= 0) {
    fold_round(p, row, r_prev, j - 1, c, st, hist, sh_b, sh_f);
    if (seg == 0 && threadIdx.x == 0) {
      uint32_t* s = p.state + ((size_t)(j & 1) * p.B + row) * 4;
      s[0] = st.prefix;
      s[1] = st.pmask;
      s[2] = st.thr_k;
      s[3] = __float_as_uint(st.need);
    }
  }
  if (!round_active(r, c, p.Vg)) return;
  __syncthreads();
  for (int b = threadIdx.x; b < kNB; b += kT) hist[b] = 0.f;
  __syncthreads();
  const T* lr = (const T*)p.logits + (size_t)row * p.ld;
  const int lo = seg * p.seglen, hi = min(p.V, lo + p.seglen);
  const int shift = round_shift(r);
  const bool mass = r >= 4;
  const uint32_t prefix = st.prefix, pmask = st.pmask, thr_k = st.thr_k;
  if ((r & 3) == 0) {
    // dense first digit: 16 register bins per lane (static indices, masked
    // adds), a wave butterfly, then one LDS add per bin per wave
    float acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    for_seg(lr, lo, hi, c, [&](int, float x) {
      const uint32_t k = qkey(x, M);
      const float w = k >= thr_k ? (mass ? __expf(x - M) : 1.f) : 0.f;
      const uint32_t b = k >> 28;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] += b == (uint32_t)q ? w : 0.f;
    }, p.v0);
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = wave_sum(acc[q]);
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) atomicAdd(&hist[q], acc[q]);
    }
  } else {
    // sparse digits: only tokens inside the selected bin; run-length
    // pre-aggregation of consecutive tokens falling into the same bin
    uint32_t cb = 0xFFFFFFFFu;
    float cv = 0.f;
    for_seg(lr, lo, hi, c, [&](int, float x) {
      const uint32_t k = qkey(x, M);
      if (k >= thr_k && (k & pmask) == prefix) {
        const uint32_t b = (k >> shift) & 255u;
        const float w = mass ? __expf(x - M) : 1.f;
        if (b == cb) {
          cv += w;
        } else {
          if (cb != 0xFFFFFFFFu) atomicAdd(&hist[cb], cv);
          cb = b;
          cv = w;
        }
      }
    }, p.v0);
    if (cb != 0xFFFFFFFFu) atomicAdd(&hist[cb], cv);
  }
  __syncthreads();
  float* dst = p.hist + (((size_t)(j & 1) * p.B + row) * p.S + seg) * kNB;
  for (int b = threadIdx.x; b < kNB; b += kT) dst[b] = hist[b];
}

// After J round launches (the last ran round r_last, -1 if none).
template <typename T>
__global__ __launch_bounds__(kT) void samp_gumbel_kernel(Params p, int r_last, int J) {
  __shared__ float hist[kNB];
  __shared__ float sv[kT / 64];
  __shared__ int si[kT / 64];
  __shared__ uint32_t sh_b[1];
  __shared__ float sh_f[1 + kT / 64];
  const int row = blockIdx.x, seg = blockIdx.y;
  const Row c = row_params(p, row);
  if (c.greedy) return;
  const float M = row_max(p, row, sv);
  RState st = load_state(p, row, J - 1 >= 1 ? J - 1 : -1, c);
  fold_round(p, row, r_last, J - 1, c, st, hist, sh_b, sh_f);
  const uint32_t thr = (r_last >= 4 && round_active(r_last, c, p.Vg)) ? st.prefix : st.thr_k;
  const uint64_t ctr = p.rng_counter ? (uint64_t)p.rng_counter[c.sl] : 0ull;
  const uint64_t base = mix64(p.seed ^ mix64(ctr * 0x100000001B3ull + (uint64_t)c.sl));
  const T* lr = (const T*)p.logits + (size_t)row * p.ld;
  const int lo = seg * p.seglen, hi = min(p.V, lo + p.seglen);
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for_seg(lr, lo, hi, c, [&](int i, float x) {
    if (qkey(x, M) >= thr) {
      const uint64_t h = mix64(base + (uint64_t)i);
      const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
      better(best, bidx, x - __logf(-__logf(u)), i);
    }
  }, p.v0);
  block_argmax(best, bidx, sv, si);
  if (threadIdx.x == 0) {
    p.gval[row * p.S + seg] = best;
    p.gidx[row * p.S + seg] = bidx;
  }
}

__global__ __launch_bounds__(64) void samp_final_kernel(Params p) {
  const int row = blockIdx.x;
  const Row c = row_params(p, row);
  float v = -INFINITY;
  int idx = 0x7fffffff;
  const float* vals = c.greedy ? p.seg_max : p.gval;
  const int32_t* ids = c.greedy ? p.seg_arg : p.gidx;
  for (int s = threadIdx.x; s < p.S; s += 64) better(v, idx, vals[row * p.S + s], ids[row * p.S + s]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) better(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
  if (threadIdx.x == 0) {
    int token = idx;
    if (token < 0 || token >= p.V) token = 0;
    p.out_tok[row] = token;
    if (c.seen) atomicOr(c.seen + (token >> 5), 1u << (token & 31));
    if (p.rng_counter) p.rng_counter[c.sl] += 1;
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

// rounds: bit 0 = top-k rounds (0-3) needed by some row, bit 1 = top-p rounds
// (4-7); the caller knows which sampling features the batch uses, so unused
// rounds are not launched at all.
template <typename T>
int launch_all(const Params& p, int rounds, hipStream_t stream) {
  const dim3 grid(p.B, p.S);
  samp_max_kernel<T><<<grid, kT, 0, stream>>>(p);
  int r_prev = -1, j = 0;
  for (int r = 0; r < kRounds; ++r) {
    if (!((rounds >> (r / 4)) & 1)) continue;
    samp_round_kernel<T><<<grid, kT, 0, stream>>>(p, r, r_prev, j);
    r_prev = r;
    ++j;
  }
  samp_gumbel_kernel<T><<<grid, kT, 0, stream>>>(p, r_prev, j);
  samp_final_kernel<<<p.B, 64, 0, stream>>>(p);
  return (int)hipGetLastError();
}


// ---------------------------------------------------------------- vocab-parallel (TP) stages
// Per-row best (value, global index) over the S segment partials -> pair[row] = {value, index}
// (the index is exact in fp32: vocabularies are < 2^24).
__global__ __launch_bounds__(64) void samp_pair_kernel(const float* vals, const int32_t* ids, int S, float* pair) {
  const int row = blockIdx.x;
  float v = -INFINITY;
  int idx = 0x7fffffff;
  for (int s = threadIdx.x; s < S; s += 64) better(v, idx, vals[row * S + s], ids[row * S + s]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) better(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
  if (threadIdx.x == 0) {
    pair[2 * row] = v;
    pair[2 * row + 1] = (float)idx;
  }
}

// Segment partial histograms of launch j -> one [B][kNB] row histogram (fixed summation order).
__global__ __launch_bounds__(kNB) void samp_hist_reduce_kernel(const float* hist, int B, int S, int j, float* out) {
  const int row = blockIdx.x, b = threadIdx.x;
  const float* src = hist + ((size_t)(j & 1) * B + row) * S * kNB;
  float acc = 0.f;
  for (int g = 0; g < S; ++g) acc += src[g * kNB + b];
  out[(size_t)row * kNB + b] = acc;
}

// Group-wide max from the all-gathered pairs [W][B][2] -> gmax[B].
__global__ void samp_gmax_kernel(const float* pairs, int W, int B, float* gmax) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  float m = -INFINITY;
  for (int w = 0; w < W; ++w) m = fmaxf(m, pairs[((size_t)w * B + row) * 2]);
  gmax[row] = m;
}

// Final: best (value, index) over the W ranks' pairs (greedy rows: the max pairs, sampled rows: the
// Gumbel pairs), then the same token / seen bit / RNG counter update on every rank.
__global__ void samp_final_tp_kernel(Params p, const float* max_pairs, const float* gum_pairs, int W) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= p.B) return;
  const Row c = row_params(p, row);
  const float* src = c.greedy ? max_pairs : gum_pairs;
  float v = -INFINITY;
  int idx = 0x7fffffff;
  for (int w = 0; w < W; ++w) better(v, idx, src[((size_t)w * p.B + row) * 2], (int)src[((size_t)w * p.B + row) * 2 + 1]);
  int token = idx;
  if (token < 0 || token >= p.Vg) token = 0;
  p.out_tok[row] = token;
  if (c.seen) atomicOr(c.seen + (token >> 5), 1u << (token & 31));
  if (p.rng_counter) p.rng_counter[c.sl] += 1;
}

}  // namespace

// Segments per row (~8K tokens per workgroup) and the workspace (floats) a
// B-row call needs.
GRAG_API int grag_sample_segments(int V) {
  const int S = (V + 8191) / 8192;
  return S < 1 ? 1 : (S > kMaxS ? kMaxS : S);
}
GRAG_API long grag_sample_ws_floats(int B, int V) {
  const long S = grag_sample_segments(V);
  return (long)B * S * (4 + 2 * kNB) + 2L * B * 4 + 64;
}

// dtype: 0 = fp32 logits, 1 = bf16 logits.  ld must be a multiple of 8.
// ws: >= grag_sample_ws_floats(B, V) floats of device scratch.  rounds: bit 0
// if any row may use top-k, bit 1 if any row may use top-p < 1.
GRAG_API int grag_sample(const void* logits, int dtype, int ld, int B, int V, const float* temperature,
                         const float* top_p, const int32_t* top_k, const float* penalty, uint32_t* seen,
                         int seen_words, int64_t* rng_counter, uint64_t seed, const int32_t* slots, int32_t* out_tok,
                         float* ws, int rounds, hipStream_t stream) {
  if (B <= 0) return 0;
  if (ld % 8 != 0 || ws == nullptr) return (int)hipErrorInvalidValue;
  Params p{};
  p.logits = logits;
  p.ld = ld;
  p.B = B;
  p.V = V;
  p.S = grag_sample_segments(V);
  p.seglen = ((V + p.S - 1) / p.S + 7) & ~7;
  p.temperature = temperature;
  p.top_p = top_p;
  p.top_k = top_k;
  p.penalty = penalty;
  p.seen = seen;
  p.seen_words = seen_words;
  p.rng_counter = rng_counter;
  p.seed = seed;
  p.slots = slots;
  p.out_tok = out_tok;
  const size_t BS = (size_t)B * p.S;
  p.seg_max = ws;
  p.seg_arg = reinterpret_cast<int32_t*>(ws + BS);
  p.gval = ws + 2 * BS;
  p.gidx = reinterpret_cast<int32_t*>(ws + 3 * BS);
  p.hist = ws + 4 * BS;
  p.state = reinterpret_cast<uint32_t*>(ws + 4 * BS + 2 * BS * kNB);
  p.v0 = 0;
  p.Vg = V;
  return dtype == 0 ? launch_all<float>(p, rounds, stream) : launch_all<bf16>(p, rounds, stream);
}

GRAG_API int grag_mark_seen(const int32_t* tokens, const int32_t* rows, int n, uint32_t* seen,
                            int seen_words, int V, hipStream_t stream) {
  if (n <= 0) return 0;
  mark_seen_kernel<<<(n + 255) / 256, 256, 0, stream>>>(tokens, rows, n, seen, seen_words, V);
  return (int)hipGetLastError();
}

// Vocab-parallel sampler, one stage per call (the host runs the TP collectives between stages;
// every stage is a fixed launch sequence, so the whole chain is captured in the decode graph):
//   stage 0: segment max/argmax of this rank's columns -> pair_out [B][2]
//            (host: all-gather -> pairs_max [W][B][2]; gmax computed here from it by stage 1's
//            first call with r_prev < 0)
//   stage 1: radix round r (fold of round r_prev from ghist) -> hist_out [B][kNB] (host: SUM all-reduce
//            in place, it is the next stage's ghist)
//   stage 2: Gumbel argmax over the kept tokens (fold of r_last from ghist) -> pair_out
//            (host: all-gather -> pairs_gum [W][B][2])
//   stage 3: final token from pairs_max / pairs_gum, seen bit, RNG counter
// logits: [B, ld] holding this rank's V columns = global tokens [v0, v0 + V); Vg = global vocab.
// ws: grag_sample_ws_floats(B, V) floats; gmax [B] and ghist [B][256] are caller buffers.
GRAG_API int grag_sample_tp(int stage, const void* logits, int dtype, int ld, int B, int V, int v0, int Vg,
                            const float* temperature, const float* top_p, const int32_t* top_k,
                            const float* penalty, uint32_t* seen, int seen_words, int64_t* rng_counter,
                            uint64_t seed, const int32_t* slots, int32_t* out_tok, float* ws, int r, int r_prev,
                            int j, float* gmax, float* ghist, float* pair_out, const float* pairs_max,
                            const float* pairs_gum, int W, hipStream_t stream) {
  if (B <= 0) return 0;
  if (ld % 8 != 0 || ws == nullptr || (v0 & 7) != 0 || V < 0) return (int)hipErrorInvalidValue;
  Params p{};
  p.logits = logits;
  p.ld = ld;
  p.B = B;
  p.V = V;
  p.S = grag_sample_segments(V);
  p.seglen = ((V + p.S - 1) / p.S + 7) & ~7;
  p.temperature = temperature;
  p.top_p = top_p;
  p.top_k = top_k;
  p.penalty = penalty;
  p.seen = seen;
  p.seen_words = seen_words;
  p.rng_counter = rng_counter;
  p.seed = seed;
  p.slots = slots;
  p.out_tok = out_tok;
  const size_t BS = (size_t)B * p.S;
  p.seg_max = ws;
  p.seg_arg = reinterpret_cast<int32_t*>(ws + BS);
  p.gval = ws + 2 * BS;
  p.gidx = reinterpret_cast<int32_t*>(ws + 3 * BS);
  p.hist = ws + 4 * BS;
  p.state = reinterpret_cast<uint32_t*>(ws + 4 * BS + 2 * BS * kNB);
  p.v0 = v0;
  p.Vg = Vg;
  const dim3 grid(B, p.S);
  const bool f32 = dtype == 0;
  switch (stage) {
    case 0:
      if (f32) samp_max_kernel<float><<<grid, kT, 0, stream>>>(p);
      else samp_max_kernel<bf16><<<grid, kT, 0, stream>>>(p);
      samp_pair_kernel<<<B, 64, 0, stream>>>(p.seg_max, p.seg_arg, p.S, pair_out);
      break;
    case 1:
      if (r_prev < 0) samp_gmax_kernel<<<(B + 255) / 256, 256, 0, stream>>>(pairs_max, W, B, gmax);
      p.gmax = gmax;
      p.ghist = r_prev >= 0 ? ghist : nullptr;
      if (f32) samp_round_kernel<float><<<grid, kT, 0, stream>>>(p, r, r_prev, j);
      else samp_round_kernel<bf16><<<grid, kT, 0, stream>>>(p, r, r_prev, j);
      samp_hist_reduce_kernel<<<B, kNB, 0, stream>>>(p.hist, B, p.S, j, ghist);
      break;
    case 2:
      if (r_prev < 0) samp_gmax_kernel<<<(B + 255) / 256, 256, 0, stream>>>(pairs_max, W, B, gmax);
      p.gmax = gmax;
      p.ghist = r_prev >= 0 ? ghist : nullptr;
      if (f32) samp_gumbel_kernel<float><<<grid, kT, 0, stream>>>(p, r_prev, j);
      else samp_gumbel_kernel<bf16><<<grid, kT, 0, stream>>>(p, r_prev, j);
      samp_pair_kernel<<<B, 64, 0, stream>>>(p.gval, p.gidx, p.S, pair_out);
      break;
    case 3:
      samp_final_tp_kernel<<<(B + 63) / 64, 64, 0, stream>>>(p, pairs_max, pairs_gum, W);
      break;
    default:
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
