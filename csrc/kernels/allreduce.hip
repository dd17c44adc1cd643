// One-shot all-reduce over IPC-mapped peer buffers (the TP
// all-reduce of Qwen2 o_proj / down_proj at decode is latency-bound — 7 KB per
// sequence row — so instead of a ring (one xGMI link per direction, 2(W-1)
// dependent hops) every rank reads all W-1 peers' copies directly, which
// drives all 7 xGMI links of an MI355X at once and costs one signal round).
//
// Per rank, one uncached (fine-grained, system-coherent) region, exported with
// hipIpcGetMemHandle and opened by every peer:
//     [ flags: kMaxBlocks x kMaxRanks uint32 | pad | data: 2 slots x slot_bytes ]
// Block b of every rank owns the same element range R_b, so no grid-wide
// barrier is needed:
//   1. read+bump this block's private epoch counter e (regular device memory;
//      identical on all ranks because every call launches the same grid);
//   2. copy x[R_b] into my data slot (e & 1), fence (system scope);
//   3. signal: store e into peer p's flags[b][rank] for every peer (release);
//   4. wait until my flags[b][p] >= e for every peer (acquire; bounded spin —
//      on timeout set *err and return, so a lost peer can never hang the GPU);
//   5. out[R_b] = sum_r slot_r[R_b] in rank order (fp32 accumulate), so every
//      rank produces bit-identical results.
// Double buffering by epoch parity makes step 2 of call k+2 safe: a peer only
// signals call k+1 after its kernel k (which read slot k & 1) has finished.
// The peer pointers are a by-value kernel argument, so the launch is
// hipGraph-capturable; in-place (out == x) is allowed.
//
// The same protocol serves the TP sampler's small exchanges (SURVEY §2.8 C2:
// per-rank (max, id) pairs, 256-bin histograms, Gumbel winners): OP_SUM_F32
// sums fp32 vectors (rank order, bit-identical on every rank) and OP_GATHER
// concatenates every rank's bytes (out = [W][n]).  All three ops of one
// communicator share its epochs, so they may be mixed in any order as long as
// every rank issues the same sequence — the engine's lockstep TP decode does,
// and a decode graph then holds no RCCL call at all.
#include "common.h"

#include <cstring>

using namespace grag;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;
constexpr int kThreads = 512;

struct Peers {
  const bf16* data[kMaxRanks];
  unsigned* flags[kMaxRanks];
};

enum { OP_SUM_BF16 = 0, OP_SUM_F32 = 1, OP_GATHER = 2 };
typedef float f32x4v_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x4v_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_release_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned ld_acquire_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// n8: 16-byte vectors per rank (8 bf16 / 4 fp32 / 16 raw bytes); slot_elems in bf16 units.
template <int W, int OP>
__global__ __launch_bounds__(kThreads) void ar_oneshot_kernel(Peers peers, int rank, const bf16* __restrict__ x,
                                                              bf16* out, long n8, long slot_elems,
                                                              unsigned* __restrict__ epochs, unsigned* err,
                                                              long spin_max) {
  __shared__ unsigned s_epoch;
  __shared__ int s_fail;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) {
    s_epoch = epochs[b] + 1u;
    epochs[b] = s_epoch;
    s_fail = 0;
  }
  __syncthreads();
  const unsigned ep = s_epoch;
  const long off = (long)(ep & 1u) * slot_elems;
  // block b's range of 16-B vectors
  const long per = (n8 + gridDim.x - 1) / gridDim.x;
  const long v0 = (long)b * per, v1 = min(n8, v0 + per);
  bf16x8_t* mine = reinterpret_cast<bf16x8_t*>(const_cast<bf16*>(peers.data[rank]) + off);
  const bf16x8_t* xv = reinterpret_cast<const bf16x8_t*>(x);
  for (long i = v0 + threadIdx.x; i < v1; i += kThreads) mine[i] = xv[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < W && threadIdx.x != rank)
    st_release_sys(&peers.flags[threadIdx.x][b * kMaxRanks + rank], ep);
  if (threadIdx.x < W && threadIdx.x != rank) {
    // bounded by WALL time, not iterations: `spin_max` = s_memrealtime ticks (100 MHz) a block waits for a
    // peer before giving up with the error word set (an iteration count was unbounded in practice: a system-
    // scope acquire load per iteration on an oversubscribed device made 1 << 24 iterations minutes long)
    const unsigned* f = &peers.flags[rank][b * kMaxRanks + threadIdx.x];
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime() + (unsigned long long)spin_max;
    unsigned it = 0;
    while (ld_acquire_sys(f) < ep) {
      if ((++it & 63u) == 0 && __builtin_amdgcn_s_memrealtime() > t_end) {
        atomicOr(err, 1u);
        s_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (s_fail) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: peers' slot data, not stale L1 lines
  if constexpr (OP == OP_SUM_BF16) {
    bf16x8_t* ov = reinterpret_cast<bf16x8_t*>(out);
    for (long i = v0 + threadIdx.x; i < v1; i += kThreads) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < W; ++r) {
        float v[8];
        unpack8(reinterpret_cast<const bf16x8_t*>(peers.data[r] + off)[i], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
      ov[i] = pack8(acc);
    }
  } else if constexpr (OP == OP_SUM_F32) {
    f32x4v_t* ov = reinterpret_cast<f32x4v_t*>(out);
    for (long i = v0 + threadIdx.x; i < v1; i += kThreads) {
      f32x4v_t acc = reinterpret_cast<const f32x4v_t*>(peers.data[0] + off)[i];
#pragma unroll
      for (int r = 1; r < W; ++r) acc += reinterpret_cast<const f32x4v_t*>(peers.data[r] + off)[i];
      ov[i] = acc;
    }
  } else {  // OP_GATHER: out[r][i] = rank r's vector i
    u32x4v_t* ov = reinterpret_cast<u32x4v_t*>(out);
    for (long i = v0 + threadIdx.x; i < v1; i += kThreads) {
#pragma unroll
      for (int r = 0; r < W; ++r) ov[r * n8 + i] = reinterpret_cast<const u32x4v_t*>(peers.data[r] + off)[i];
    }
  }
}

}  // namespace

// Region layout helpers (host): data offset (bytes) and total size for a slot size.
GRAG_API long grag_ar_data_offset() { return (long)kMaxBlocks * kMaxRanks * sizeof(unsigned) + 256; }
GRAG_API long grag_ar_region_bytes(long slot_bytes) { return grag_ar_data_offset() + 2 * slot_bytes; }

// Allocate a zeroed uncached (fine-grained) region that peers can map.
GRAG_API int grag_ar_alloc(long bytes, void** ptr) {
  hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*ptr, 0, (size_t)bytes);
}
GRAG_API int grag_ar_free(void* ptr) { return (int)hipFree(ptr); }

GRAG_API int grag_ar_get_handle(void* ptr, void* handle_out /* 64 bytes */) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e == hipSuccess) std::memcpy(handle_out, &h, sizeof(h));
  return (int)e;
}
GRAG_API int grag_ar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

GRAG_API int grag_ar_open_handle(const void* handle /* 64 bytes */, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}
GRAG_API int grag_ar_close_handle(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

namespace {
template <int OP>
int launch_oneshot(void* const* regions, int W, int rank, const void* x, void* out, long n16, long slot_bytes,
                   void* epochs, void* err, int grid, long spin_max, hipStream_t stream);
}  // namespace

// regions: host array of W region base pointers (own + opened peers), rank order.
// n: elements (bf16, multiple of 8, <= slot_bytes / 2); grid: fixed per communicator (<= kMaxBlocks).
GRAG_API int grag_ar_oneshot(void* const* regions, int W, int rank, const void* x, void* out, long n,
                             long slot_bytes, void* epochs, void* err, int grid, long spin_max,
                             hipStream_t stream) {
  if (n % 8 != 0 || n * 2 > slot_bytes) return (int)hipErrorInvalidValue;
  return launch_oneshot<OP_SUM_BF16>(regions, W, rank, x, out, n / 8, slot_bytes, epochs, err, grid, spin_max, stream);
}

// op 1: fp32 sum of `nbytes` per rank (out may alias x); op 2: gather, out = W x nbytes (rank order, no alias).
// nbytes: multiple of 16, <= slot_bytes.  Same communicator (regions / epochs / grid) as grag_ar_oneshot.
GRAG_API int grag_ar_oneshot_op(void* const* regions, int W, int rank, int op, const void* x, void* out, long nbytes,
                                long slot_bytes, void* epochs, void* err, int grid, long spin_max,
                                hipStream_t stream) {
  if (nbytes % 16 != 0 || nbytes > slot_bytes || nbytes < 0) return (int)hipErrorInvalidValue;
  if (op == OP_SUM_F32)
    return launch_oneshot<OP_SUM_F32>(regions, W, rank, x, out, nbytes / 16, slot_bytes, epochs, err, grid, spin_max,
                                      stream);
  if (op == OP_GATHER)
    return launch_oneshot<OP_GATHER>(regions, W, rank, x, out, nbytes / 16, slot_bytes, epochs, err, grid, spin_max,
                                     stream);
  return (int)hipErrorInvalidValue;
}

namespace {
template <int OP>
int launch_oneshot(void* const* regions, int W, int rank, const void* x, void* out, long n16, long slot_bytes,
                   void* epochs, void* err, int grid, long spin_max, hipStream_t stream) {
  if (W < 1 || W > kMaxRanks || rank < 0 || rank >= W || grid < 1 || grid > kMaxBlocks) return (int)hipErrorInvalidValue;
  Peers p{};
  const long doff = grag_ar_data_offset();
  for (int r = 0; r < W; ++r) {
    p.flags[r] = reinterpret_cast<unsigned*>(regions[r]);
    p.data[r] = reinterpret_cast<const bf16*>(reinterpret_cast<char*>(regions[r]) + doff);
  }
  const long n8 = n16, slot_elems = slot_bytes / 2;
  auto go = [&](auto kern) {
    kern<<<grid, kThreads, 0, stream>>>(p, rank, (const bf16*)x, (bf16*)out, n8, slot_elems, (unsigned*)epochs,
                                        (unsigned*)err, spin_max);
  };
  switch (W) {
    case 1: go(ar_oneshot_kernel<1, OP>); break;
    case 2: go(ar_oneshot_kernel<2, OP>); break;
    case 3: go(ar_oneshot_kernel<3, OP>); break;
    case 4: go(ar_oneshot_kernel<4, OP>); break;
    case 5: go(ar_oneshot_kernel<5, OP>); break;
    case 6: go(ar_oneshot_kernel<6, OP>); break;
    case 7: go(ar_oneshot_kernel<7, OP>); break;
    default: go(ar_oneshot_kernel<8, OP>); break;
  }
  return (int)hipGetLastError();
}
}  // namespace
