// Fused elementwise kernels:
//   * qkv_bias_rope_kvstore  (N1c epilogue + N1d + N1e): QKV bias add, NeoX
//     rotary embedding on q/k, q written token-major for attention, k/v
//     scattered straight into the paged KV cache [blocks, Hkv, BS, D].
//   * silu_mul (N1i epilogue), gelu_bias (N2d FFN1 epilogue), bias_add.
//   * pool_l2norm (N2e): masked-mean or CLS pooling + L2 normalisation,
//     writing fp32 (index staging) and optionally bf16.
// All HBM-bound; every access is 16 B per lane.
#include "common.h"

using namespace grag;

namespace {
constexpr int kThreads = 256;

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
}
// GPT-2 "gelu_new": 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))),
// tanh(u) = 1 - 2 / (1 + exp(2u)) (saturates correctly at +-inf)
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * u));
  return 0.5f * x * (1.f + t);
}

// One block per token (few tokens: gridDim.y blocks of 64 threads per token share its units, so a decode step
// of 1-32 sequences spreads the row over several CUs).  Work units (16 B each):
//   [0, (Hq+Hkv)*D/16)           rotary units: 8 pairs (i..i+7, i+D/2..i+D/2+7)
//   [.., + Hkv*D/8)              v copy units
// PL: the projection arrives as S fp32 split-K planes [S][T][ld] (ops/gemm.py SplitKPartial): the reduce is
// folded in here (sum in plane order, rounded to bf16 exactly as grag_splitk_reduce would store it).
template <bool PL>
__global__ __launch_bounds__(kThreads) void qkv_rope_kernel(
    const bf16* __restrict__ qkv, int ld, const bf16* __restrict__ bias,
    const int32_t* __restrict__ positions, const float* __restrict__ cos_sin,
    const int32_t* __restrict__ slot_mapping, bf16* __restrict__ q_out, bf16* __restrict__ k_cache,
    bf16* __restrict__ v_cache, int Hq, int Hkv, int D, int BS, const float* __restrict__ planes, int S,
    size_t plane, int nslots, int npos) {
  const int t = blockIdx.x;
  const float* prow = PL ? planes + (size_t)t * ld : nullptr;
  // 8 consecutive projection outputs of this token as bf16-rounded floats
  auto load8 = [&](int col, float* x) {
    if constexpr (PL) {
      // (common.h plane_sum4: up to 8 planes' loads in flight at once; sums stay in plane order)
      const f32x4_t a = plane_sum4(prow + col, plane, S), b = plane_sum4(prow + col + 4, plane, S);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = bits2f(f2bits(a[j]));
        x[j + 4] = bits2f(f2bits(b[j]));
      }
    } else {
      unpack8(*reinterpret_cast<const bf16x8_t*>(qkv + (size_t)t * ld + col), x);
    }
  };
  const int half = D >> 1;
  const int upp = half >> 3;  // rotary units per head
  const int n_rot = (Hq + Hkv) * upp;
  const int n_v = Hkv * (D >> 3);
  int pos = positions[t];
  int slot = slot_mapping ? slot_mapping[t] : -1;
  // index inputs checked (common.h index guard): a bad position reads row 0 of the table, a bad slot skips
  // the K/V store; either is reported and raised on the host at its next sync
  if (cos_sin && !index_ok(pos, npos, ERR_ROPE_POS)) pos = 0;
  if (slot >= 0 && !index_ok(slot, nslots, ERR_KV_SLOT)) slot = -1;
  // cos_sin == nullptr: no rotary (absolute-position decoders, GPT-2) — the
  // kernel is then the fused bias add + q split + paged K/V store
  const float* cs = cos_sin ? cos_sin + (size_t)pos * D : nullptr;
  const int blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;
  for (int u = blockIdx.y * blockDim.x + threadIdx.x; u < n_rot + n_v; u += gridDim.y * blockDim.x) {
    if (u < n_rot) {
      const int head = u / upp;  // 0..Hq-1 are q heads, then k heads
      const int i0 = (u % upp) * 8;
      const int col = head * D + i0;
      float x1[8], x2[8];
      load8(col, x1);
      load8(col + half, x2);
      if (bias) {
        float b1[8], b2[8];
        unpack8(*reinterpret_cast<const bf16x8_t*>(bias + col), b1);
        unpack8(*reinterpret_cast<const bf16x8_t*>(bias + col + half), b2);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // match the unfused path: bias add rounds to bf16 before rotary
          x1[j] = bits2f(f2bits(x1[j] + b1[j]));
          x2[j] = bits2f(f2bits(x2[j] + b2[j]));
        }
      }
      float o1[8], o2[8];
      if (cs) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float c = cs[i0 + j], s = cs[half + i0 + j];
          o1[j] = x1[j] * c - x2[j] * s;
          o2[j] = x2[j] * c + x1[j] * s;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o1[j] = x1[j];
          o2[j] = x2[j];
        }
      }
      if (head < Hq) {
        bf16* qo = q_out + ((size_t)t * Hq + head) * D + i0;
        *reinterpret_cast<bf16x8_t*>(qo) = pack8(o1);
        *reinterpret_cast<bf16x8_t*>(qo + half) = pack8(o2);
      } else if (slot >= 0) {
        const int kh = head - Hq;
        bf16* ko = k_cache + (((size_t)blk * Hkv + kh) * BS + off) * D + i0;
        *reinterpret_cast<bf16x8_t*>(ko) = pack8(o1);
        *reinterpret_cast<bf16x8_t*>(ko + half) = pack8(o2);
      }
    } else if (slot >= 0) {
      const int vu = u - n_rot;
      const int vh = vu / (D >> 3);
      const int i0 = (vu % (D >> 3)) * 8;
      const int col = (Hq + Hkv + vh) * D + i0;
      bf16x8_t v;
      if (bias || PL) {
        float a[8];
        load8(col, a);
        if (bias) {
          float b[8];
          unpack8(*reinterpret_cast<const bf16x8_t*>(bias + col), b);
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] += b[j];
        }
        v = pack8(a);
      } else {
        v = *reinterpret_cast<const bf16x8_t*>(qkv + (size_t)t * ld + col);
      }
      *reinterpret_cast<bf16x8_t*>(v_cache + (((size_t)blk * Hkv + vh) * BS + off) * D + i0) = v;
    }
  }
}

// out[t, i] = silu(gu[t, i]) * gu[t, I + i]
// grid (ceil(I/8 / 256), ceil(T / kSiluRows)): a thread owns one 16-B column
// vector and walks kSiluRows token rows (unrolled, so 8 row loads are in
// flight per thread); 32-bit indexing only (the grid-stride form spent most of
// its issue slots on 64-bit div/mod).
constexpr int kSiluRows = 8;
__global__ __launch_bounds__(kThreads) void silu_mul_kernel(const bf16* __restrict__ gu,
                                                            bf16* __restrict__ out, int T, int I, int rows) {
  const int nvec = I >> 3;
  const int v = blockIdx.x * kThreads + threadIdx.x;
  if (v >= nvec) return;
  const int t0 = blockIdx.y * rows;
  const int t1 = min(T, t0 + rows);
  const bf16x8_t* src = reinterpret_cast<const bf16x8_t*>(gu) + (size_t)t0 * 2 * nvec + v;
  bf16x8_t* dst = reinterpret_cast<bf16x8_t*>(out) + (size_t)t0 * nvec + v;
#pragma unroll 4
  for (int t = t0; t < t1; ++t) {
    float g[8], u[8], o[8];
    unpack8(src[0], g);
    unpack8(src[nvec], u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] * __builtin_amdgcn_rcpf(1.f + __expf(-g[j])) * u[j];
    dst[0] = pack8(o);
    src += 2 * nvec;
    dst += nvec;
  }
}

// y = act(x + b); act 0 = identity, 1 = gelu(erf), 2 = silu, 3 = gelu(tanh).  In place allowed.
__global__ __launch_bounds__(kThreads) void bias_act_kernel(const bf16* __restrict__ x,
                                                            const bf16* __restrict__ b,
                                                            bf16* __restrict__ y, int T, int N,
                                                            int act) {
  const int nvec = N >> 3;
  const size_t total = (size_t)T * nvec;
  for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < total;
       i += (size_t)gridDim.x * kThreads) {
    const int v = (int)(i % nvec);
    float a[8], c[8];
    unpack8(reinterpret_cast<const bf16x8_t*>(x)[i], a);
    if (b) {
      unpack8(reinterpret_cast<const bf16x8_t*>(b)[v], c);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += c[j];
    }
    if (act == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = gelu_erf(a[j]);
    } else if (act == 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = silu(a[j]);
    } else if (act == 3) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = gelu_tanh(a[j]);
    }
    reinterpret_cast<bf16x8_t*>(y)[i] = pack8(a);
  }
}

// Pool sequences of token-major hidden rows: sequence b starts at row
// starts[b] (packed varlen layout) or b*S when starts is null (padded layout),
// with lengths[b] valid tokens.  mode 0 = masked mean, 1 = CLS (token 0).
// Writes L2-normalised fp32 [B, H] and optionally bf16 [B, H].
__global__ __launch_bounds__(kThreads) void pool_l2norm_kernel(
    const bf16* __restrict__ hidden, const int32_t* __restrict__ starts,
    const int32_t* __restrict__ lengths, float* __restrict__ outf, bf16* __restrict__ outb, int S,
    int H, int mode, int normalize) {
  __shared__ float red[kThreads / 64];
  const int b = blockIdx.x;
  const int len = lengths[b] > 0 ? lengths[b] : 1;
  const int nvec = H >> 3;
  const bf16* base = hidden + (size_t)(starts ? starts[b] : b * S) * H;
  // each thread owns up to 2 vectors of the output row (H <= 4096)
  float acc[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  const int ntok = mode == 1 ? 1 : len;
  for (int t = 0; t < ntok; ++t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = threadIdx.x + i * kThreads;
      if (idx < nvec) {
        float a[8];
        unpack8(reinterpret_cast<const bf16x8_t*>(base + (size_t)t * H)[idx], a);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] += a[j];
      }
    }
  }
  float ss = 0.f;
  const float scale = 1.f / (float)ntok;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[i][j] *= scale;
        ss += acc[i][j] * acc[i][j];
      }
    }
  }
  ss = block_sum(ss, red);
  const float inv = normalize ? 1.f / fmaxf(sqrtf(ss), 1e-12f) : 1.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + i * kThreads;
    if (idx < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = acc[i][j] * inv;
      if (outf) {
        float4* of = reinterpret_cast<float4*>(outf + (size_t)b * H + idx * 8);
        of[0] = make_float4(o[0], o[1], o[2], o[3]);
        of[1] = make_float4(o[4], o[5], o[6], o[7]);
      }
      if (outb) reinterpret_cast<bf16x8_t*>(outb + (size_t)b * H)[idx] = pack8(o);
    }
  }
}

int grid_for(size_t total) {
  size_t g = (total + kThreads - 1) / kThreads;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

// Blocks of qkv_rope_kernel: rope_block(T) threads per block.  Under 32 tokens one 64-thread block per 64
// units of each token; at decode batches of 32-511 tokens one 128-thread block per 128 units (a block per
// token left CUs idle and kept too few plane loads in flight: 9.9 -> 7.9 us at 176 tokens); at prefill
// sizes one 256-thread block per token (the split grid measured slower there: 35 vs 21 us per call).
static int rope_block(int T) { return T < 32 ? 64 : T < 512 ? 128 : kThreads; }
static dim3 rope_grid(int T, int Hq, int Hkv, int D) {
  if (T >= 512) return dim3(T, 1);
  const int units = (Hq + Hkv) * (D / 16) + Hkv * (D / 8);
  const int b = rope_block(T);
  return dim3(T, (units + b - 1) / b);
}

GRAG_API int grag_qkv_rope_kvstore(const void* qkv, int ld, const void* bias,
                                   const int32_t* positions, const float* cos_sin,
                                   const int32_t* slot_mapping, void* q_out, void* k_cache,
                                   void* v_cache, int T, int Hq, int Hkv, int D, int BS, int nslots,
                                   int npos, hipStream_t stream) {
  if (T <= 0) return 0;
  if (D % 16 != 0 || ld % 8 != 0) return (int)hipErrorInvalidValue;
  const dim3 g = rope_grid(T, Hq, Hkv, D);
  qkv_rope_kernel<false><<<g, rope_block(T), 0, stream>>>((const bf16*)qkv, ld, (const bf16*)bias, positions,
                                                     cos_sin, slot_mapping, (bf16*)q_out,
                                                     (bf16*)k_cache, (bf16*)v_cache, Hq, Hkv, D, BS, nullptr, 1, 0,
                                                     nslots, npos);
  return (int)hipGetLastError();
}

// Same from the S fp32 split-K planes [S][T][N] of the projection (N = (Hq + 2 Hkv) D): the split-K reduce of
// a deferred qkv projection (ops/gemm.py SplitKPartial) folded into this pass.
GRAG_API int grag_qkv_rope_kvstore_planes(const float* planes, int S, int N, const void* bias,
                                          const int32_t* positions, const float* cos_sin,
                                          const int32_t* slot_mapping, void* q_out, void* k_cache,
                                          void* v_cache, int T, int Hq, int Hkv, int D, int BS, int nslots,
                                          int npos, hipStream_t stream) {
  if (T <= 0) return 0;
  if (D % 16 != 0 || N % 8 != 0 || S < 1 || N != (Hq + 2 * Hkv) * D) return (int)hipErrorInvalidValue;
  const dim3 g = rope_grid(T, Hq, Hkv, D);
  qkv_rope_kernel<true><<<g, rope_block(T), 0, stream>>>(nullptr, N, (const bf16*)bias, positions, cos_sin,
                                                    slot_mapping, (bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache,
                                                    Hq, Hkv, D, BS, planes, S, (size_t)T * N, nslots, npos);
  return (int)hipGetLastError();
}

GRAG_API int grag_silu_mul(const void* gu, void* out, int T, int I, hipStream_t stream) {
  if (T <= 0) return 0;
  if (I % 8 != 0) return (int)hipErrorInvalidValue;
  // decode-sized T: one row per thread so the grid still fills 256 CUs
  // (T = 192, I = 18944: 240 blocks with 8 rows, 1920 with 1)
  const int rows = T >= 2048 ? kSiluRows : 1;
  dim3 grid((I / 8 + kThreads - 1) / kThreads, (T + rows - 1) / rows);
  silu_mul_kernel<<<grid, kThreads, 0, stream>>>((const bf16*)gu, (bf16*)out, T, I, rows);
  return (int)hipGetLastError();
}

GRAG_API int grag_bias_act(const void* x, const void* b, void* y, int T, int N, int act,
                           hipStream_t stream) {
  if (T <= 0) return 0;
  if (N % 8 != 0) return (int)hipErrorInvalidValue;
  bias_act_kernel<<<grid_for((size_t)T * N / 8), kThreads, 0, stream>>>(
      (const bf16*)x, (const bf16*)b, (bf16*)y, T, N, act);
  return (int)hipGetLastError();
}

GRAG_API int grag_pool_l2norm(const void* hidden, const int32_t* starts, const int32_t* lengths,
                              float* outf, void* outb, int B, int S, int H, int mode, int normalize,
                              hipStream_t stream) {
  if (B <= 0) return 0;
  if (H % 8 != 0 || H > 16 * kThreads) return (int)hipErrorInvalidValue;
  pool_l2norm_kernel<<<B, kThreads, 0, stream>>>((const bf16*)hidden, starts, lengths, outf,
                                                 (bf16*)outb, S, H, mode, normalize);
  return (int)hipGetLastError();
}

GRAG_ERR_UNIT(elementwise)
