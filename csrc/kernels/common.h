// Common device helpers for the gfx950 (CDNA4 / MI355X) kernel library.
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 storage is clang's __bf16; conversions go through plain casts so
//     hipcc emits v_cvt_pk_bf16_f32 (NaN-preserving, RNE) — see
//     MI355X_MICROARCH.md "Correctness boundaries".
//   * wave = 64 lanes; block sizes are multiples of 64.
//   * every global load of bf16 data is vectorised to 16 B/lane (bf16x8).
//   * exported entry points are extern "C", take raw device pointers plus the
//     caller's hipStream_t (PyTorch's current stream), and return hipError_t
//     so the Python side can raise loudly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GRAG_API extern "C" __attribute__((visibility("default")))

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

typedef __bf16 bf16;

namespace grag {

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

__device__ __forceinline__ float bits2f(short s) {
  return __uint_as_float(((uint32_t)(uint16_t)s) << 16);
}
__device__ __forceinline__ short f2bits(float f) {
  bf16 b = (bf16)f;
  return __builtin_bit_cast(short, b);
}

// a += four consecutive floats of each of S fp32 split-K planes (plane stride `plane` elements), in plane order.
// For S <= 16 the planes are walked in one fully unrolled, branch-free pass of 2, 4, 8, 12 or 16 (indices past S re-read
// plane 0 and add zero: fma(1, y, x) rounds as x + y), so every plane's load can be in flight together -- a
// runtime-count loop under "#pragma unroll" runs its remainder iterations one plane per memory round trip.
template <int MAXS>
__device__ __forceinline__ void plane_acc4_fixed(f32x4_t& a, const float* p, size_t plane, int S) {
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    const bool on = s < S;
    const f32x4_t v = *reinterpret_cast<const f32x4_t*>(p + (on ? s : 0) * plane);
    const float m = on ? 1.f : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] = __builtin_fmaf(m, v[r], a[r]);
  }
}
__device__ __forceinline__ void plane_acc4(f32x4_t& a, const float* p, size_t plane, int S) {
  if (S <= 2) {  // (the pass length: the first of 2, 4, 8, 12, 16 >= S)
    plane_acc4_fixed<2>(a, p, plane, S);
  } else if (S <= 4) {
    plane_acc4_fixed<4>(a, p, plane, S);
  } else if (S <= 8) {
    plane_acc4_fixed<8>(a, p, plane, S);
  } else if (S <= 12) {
    plane_acc4_fixed<12>(a, p, plane, S);
  } else if (S <= 16) {
    plane_acc4_fixed<16>(a, p, plane, S);
  } else {
    for (int s = 0; s < S; ++s) a += *reinterpret_cast<const f32x4_t*>(p + s * plane);
  }
}
// the plane sum alone (from -0, the additive identity of every float, so the bits are the plain sum's)
__device__ __forceinline__ f32x4_t plane_sum4(const float* p, size_t plane, int S) {
  f32x4_t a = f32x4_t{-0.f, -0.f, -0.f, -0.f};
  plane_acc4(a, p, plane, S);
  return a;
}

// Unpack a 16-byte bf16x8 vector into 8 floats.
__device__ __forceinline__ void unpack8(const bf16x8_t& v, float* f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bits2f(v[i]);
}
__device__ __forceinline__ bf16x8_t pack8(const float* f) {
  bf16x8_t v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = f2bits(f[i]);
  return v;
}

// ---- wave / block reductions (wave64) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum; `red` must hold >= blockDim.x/64 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks that the dispatcher deals to one XCD
// (orig % 8 equal) get a contiguous range of logical tile ids so neighbouring
// tiles share that XCD's L2.  Speed-only; correctness never depends on it.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

// ---- device-side index guard --------------------------------------------------------------------
// Kernels whose addresses come from index INPUTS (token ids, KV slot ids, block-table entries, row ids,
// cross-workgroup tickets) check them.  An out-of-range index skips its access and records (code, value)
// in a small host-mapped error block instead of faulting the device: an illegal address poisons every
// stream of the process and names no kernel, a recorded code names the kernel and the bad value, and the
// host raises on it at its next sync point (ops/_lib.py check_device_errors).  The block pointer is one
// per translation unit (no relocatable device code here), bound once at library load by
// grag_err_bind_<unit>; it is read with plain (scalar) loads and written only with vector atomics.
enum : unsigned {
  ERR_EMBED_TOKEN = 1u << 0,   // decoder embedding gather: token id >= vocab
  ERR_KV_SLOT = 1u << 1,       // RoPE + KV store: slot id >= KV slots
  ERR_ROPE_POS = 1u << 2,      // RoPE: position >= cos/sin table rows
  ERR_BLOCK_PREFILL = 1u << 3, // prefill attention: block-table entry >= KV blocks
  ERR_BLOCK_DECODE = 1u << 4,  // decode attention: block-table entry >= KV blocks
  ERR_TICKET = 1u << 5,        // a split-merge / stream-K ticket past its part count (shared or stale word)
  ERR_SAMPLER_SLOT = 1u << 6,  // sampler / seen-bit row >= sampler slots
  ERR_TOPK_ROW = 1u << 7,      // top-k merge / IVF scan: candidate row or list range out of range
  ERR_BERT_TOKEN = 1u << 8,    // encoder embedding: token / position id out of range
  ERR_PREFIX_GROUP = 1u << 9,  // shared-prefix decode: group row range or prefix length out of range
};

static __device__ unsigned* g_err_block = nullptr;  // [0] codes (OR), [1] last bad value, [2] count, [3] code of [1]

// The block is pinned host memory mapped into the device address space: plain (non-RMW) system-scope
// stores only -- they travel as posted writes on any host link, where read-modify-write atomics to host
// memory would need link atomics.  Two reporters racing may lose one code bit or count: this is a
// diagnostic that something went wrong and where, not a tally.
__device__ __noinline__ void report_index_error(unsigned code, unsigned value) {
  unsigned* e = g_err_block;
  if (e == nullptr) return;
  const unsigned prev = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(e, prev | code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(e + 1, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned cnt = __hip_atomic_load(e + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(e + 2, cnt + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(e + 3, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// true when 0 <= v < n; otherwise reports (code, v) and returns false
__device__ __forceinline__ bool index_ok(long v, long n, unsigned code) {
  if (__builtin_expect(v >= 0 && v < n, 1)) return true;
  report_index_error(code, (unsigned)v);
  return false;
}

}  // namespace grag

// exported per translation unit: bind this unit's error-block pointer (host-mapped memory)
#define GRAG_ERR_UNIT(unit)                                                                 \
  GRAG_API int grag_err_bind_##unit(void* p) {                                              \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(grag::g_err_block), &p, sizeof(p), 0,          \
                                  hipMemcpyHostToDevice);                                   \
  }
