// Shared helpers for the libabc_hip C-ABI (gfx950 / CDNA4 only).
//
// Conventions of every exported entry point (see include/abc_hip.h):
//   * all pointers are device pointers owned by the caller (torch tensors);
//   * the last argument is the hipStream_t the work is enqueued on (async);
//   * the return value is 0 on success, <0 on failure; abc_last_error()
//     returns a thread-local message for the failing call;
//   * no allocation, no synchronisation, no host<->device copies inside a
//     call (graph-capturable), except where a function's comment says so.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cmath>

namespace abc {

enum Status : int {
  kOk = 0,
  kInvalidArg = -1,
  kHipError = -2,
  kUnsupported = -3,
};

void set_error(const char* fmt, ...);

// Launch-shape tuning knobs (environment variables, tools/ sweeps and the
// knob tests only; none changes a result bit except the two routing
// experiments marked below).  The table is read from the
// environment ONCE per process (capi.hip) and again only by
// abc_tuning_reload(), so no launch path calls getenv.
enum Knob : int {
  kKnobKdeMfmaSplit = 0,  // ABC_KDE_MFMA_SPLIT
  kKnobKdeMfmaIb,         // ABC_KDE_MFMA_IB
  kKnobKdeMfmaPipe,       // ABC_KDE_MFMA_PIPE
  kKnobKdeMfmaLds2,       // ABC_KDE_MFMA_LDS2
  kKnobKdeMfmaSmajor,     // ABC_KDE_MFMA_SMAJOR
  kKnobKdeTier,           // ABC_KDE_TIER
  kKnobLzIb,              // ABC_LZ_IB
  kKnobLzTpb,             // ABC_LZ_TPB
  kKnobKnnRows,           // ABC_KNN_ROWS
  // routing experiments of the MFMA KDE pass (tools/kde_offsets.py): these
  // two DO move rows between the folded pass and its refine, i.e. change
  // bits within the derived bound (kde_mfma.hip, "refine")
  kKnobKdeParentShift,    // ABC_KDE_PARENT_SHIFT
  kKnobKdeParentWin,      // ABC_KDE_PARENT_WIN
  kKnobProposeGroup,      // ABC_PROPOSE_GROUP (1 four lanes per proposal, 0 one)
  kKnobCount
};
// the knob's integer value, or dflt when the variable is unset
int tuning_knob(Knob k, int dflt);

#define ABC_REQUIRE(cond, ...)              \
  do {                                      \
    if (!(cond)) {                          \
      ::abc::set_error(__VA_ARGS__);        \
      return ::abc::kInvalidArg;            \
    }                                       \
  } while (0)

#define ABC_LAUNCH_CHECK(what)                                              \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) {                                                 \
      ::abc::set_error("%s: %s", what, hipGetErrorString(e_));              \
      return ::abc::kHipError;                                              \
    }                                                                       \
  } while (0)

#define ABC_HIP(call)                                                       \
  do {                                                                      \
    hipError_t e_ = (call);                                                 \
    if (e_ != hipSuccess) {                                                 \
      ::abc::set_error("%s: %s", #call, hipGetErrorString(e_));             \
      return ::abc::kHipError;                                              \
    }                                                                       \
  } while (0)

constexpr int kWave = 64;

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) {
  return (a + b - 1) / b;
}

// grid size for a grid-stride streaming kernel (Guideline 11: cap ~2048)
inline unsigned stream_grid(int64_t n, int block, int cap = 4096) {
  int64_t g = ceil_div(n, block);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<unsigned>(g);
}

// Resolve one kernel of a translation unit on the current device, which
// loads that unit's code object (the per-unit abc::preload_* hooks).
template <typename F>
inline int preload_kernel(F* f) {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(f)) == hipSuccess ? 0 : 1;
}
int preload_propose();
int preload_kde();
int preload_kde_mfma();
int preload_distance();
int preload_select();
int preload_stochastic();
int preload_local();
int preload_local_pdf32();
int preload_sort();
int preload_local_mfma();

// ---- wave / block reductions (64-lane waves) -------------------------------
template <typename T>
__device__ inline T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ inline T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

// Block sum with a fixed reduction tree (deterministic for a fixed blockDim).
template <typename T, int BLOCK>
__device__ inline T block_sum(T v, T* lds /* >= BLOCK/64 */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  T r = 0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < BLOCK / 64; ++i) r += lds[i];
    lds[0] = r;
  }
  __syncthreads();
  r = lds[0];
  __syncthreads();
  return r;
}

// Block-wide reduction then ONE device atomic per block.  Per-wave atomics
// on a single address serialise (~100 per microsecond chip-wide): the
// one-pass max / sum kernels spent 20-40 us in them at n = 1e5.  Every
// thread of the block must call these (they hold a barrier).
template <int BLOCK>
__device__ inline void block_atomic_max_u64(unsigned long long* addr,
                                            unsigned long long v) {
  __shared__ unsigned long long red[BLOCK / 64];
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 1; i < BLOCK / 64; ++i) v = red[i] > v ? red[i] : v;
    if (v) atomicMax(addr, v);
  }
}
template <int BLOCK>
__device__ inline void block_atomic_min_u64(unsigned long long* addr,
                                            unsigned long long v) {
  __shared__ unsigned long long red[BLOCK / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 1; i < BLOCK / 64; ++i) v = red[i] < v ? red[i] : v;
    if (v != ~0ull) atomicMin(addr, v);
  }
}
template <int BLOCK>
__device__ inline void block_atomic_add_u64(unsigned long long* addr,
                                            unsigned long long v) {
  __shared__ unsigned long long red[BLOCK / 64];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 1; i < BLOCK / 64; ++i) v += red[i];
    if (v) atomicAdd(addr, v);
  }
}

// Order-preserving map of an IEEE double to uint64 (total order, -0 < +0).
__device__ inline uint64_t f64_key(double x) {
  uint64_t b = __double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ inline double key_f64(uint64_t k) {
  uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double(b);
}

}  // namespace abc
