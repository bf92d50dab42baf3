// Key/value radix sort of the spatial index (spatial.hpp): Hilbert keys of
// the particles (or of the evaluation points) with their int32 indices, in
// place of cKDTree's build (local_transition.py:82-83).  Round 6: this
// repo's own stable LSD radix sort (8-bit digits) replaces the rocPRIM
// (hipcub::DeviceRadixSort) call of rounds 3-5, so no library kernel runs on
// the LocalTransition path.
//
// One pass per 8-bit digit, three kernels each:
//   * rs_hist: per block of kRsTile keys the digit histogram (LDS atomics),
//     written digit-major: cnt[digit][block];
//   * rs_scan: one block, the exclusive prefix of cnt in that order -- the
//     first output slot of (digit, block);
//   * rs_scatter: the block re-reads its keys in order, kRsBlock at a time,
//     and ranks each key among the equal digits before it: within a wave by
//     an 8-ballot match of the digit, across the block's 4 waves and the
//     earlier rounds by LDS counters.  Equal digits keep their input order,
//     so the sort is stable (the same permutation as the library's).
#include <cstdint>

#include "common.hpp"

namespace abc {
namespace {

constexpr int kRsBlock = 256;               // threads (4 waves)
constexpr int kRsRounds = 8;                // rounds of kRsBlock keys
constexpr int kRsTile = kRsBlock * kRsRounds;  // keys per block
constexpr int kRsBins = 256;

__global__ __launch_bounds__(kRsBlock) void rs_hist_kernel(
    const uint64_t* __restrict__ keys, int64_t n, int shift, unsigned dmask,
    int* __restrict__ cnt, int nb) {
  __shared__ int h[kRsBins];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRsTile;
  for (int r = 0; r < kRsRounds; ++r) {
    const int64_t i = base + r * kRsBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & dmask], 1);
  }
  __syncthreads();
  cnt[static_cast<int64_t>(threadIdx.x) * nb + blockIdx.x] = h[threadIdx.x];
}

// exclusive prefix of cnt[0 .. m) in place (one block of 1024 threads)
__global__ __launch_bounds__(1024) void rs_scan_kernel(int* __restrict__ cnt,
                                                       int64_t m) {
  __shared__ int part[1024];
  const int64_t per = (m + 1023) / 1024;
  const int64_t lo = threadIdx.x * per;
  const int64_t hi = lo + per < m ? lo + per : m;
  int s = 0;
  for (int64_t k = lo; k < hi; ++k) s += cnt[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int64_t k = lo; k < hi; ++k) {
    const int c = cnt[k];
    cnt[k] = run;
    run += c;
  }
}

__global__ __launch_bounds__(kRsBlock) void rs_scatter_kernel(
    const uint64_t* __restrict__ kin, const int32_t* __restrict__ vin, int64_t n,
    int shift, unsigned dmask, const int* __restrict__ off, int nb,
    uint64_t* __restrict__ kout,
    int32_t* __restrict__ vout) {
  __shared__ int run[kRsBins];   // keys of each digit placed by earlier rounds
  __shared__ int wc[4][kRsBins];  // this round's count per (wave, digit)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  run[threadIdx.x] = off[static_cast<int64_t>(threadIdx.x) * nb + blockIdx.x];
  const uint64_t lt = (1ull << lane) - 1ull;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRsTile;
  for (int r = 0; r < kRsRounds; ++r) {
#pragma unroll
    for (int w = 0; w < 4; ++w) wc[w][threadIdx.x] = 0;
    __syncthreads();
    const int64_t i = base + r * kRsBlock + threadIdx.x;
    const bool live = i < n;
    const uint64_t k = live ? kin[i] : 0;
    const int dig = static_cast<int>((k >> shift) & dmask);
    // lanes of this wave holding the same digit
    uint64_t peers = __ballot(live);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t m = __ballot(live && ((dig >> b) & 1));
      peers &= ((dig >> b) & 1) ? m : ~m;
    }
    const int below = __popcll(peers & lt);
    if (live && below == 0) wc[wid][dig] = __popcll(peers);
    __syncthreads();
    if (live) {
      int pos = run[dig] + below;
      for (int w = 0; w < wid; ++w) pos += wc[w][dig];
      kout[pos] = k;
      vout[pos] = vin[i];
    }
    __syncthreads();
    run[threadIdx.x] += wc[0][threadIdx.x] + wc[1][threadIdx.x] +
                        wc[2][threadIdx.x] + wc[3][threadIdx.x];
  }
}

int rs_blocks(int64_t n) { return static_cast<int>(ceil_div(n > 0 ? n : 1, kRsTile)); }

}  // namespace

// scratch: the digit counts, then one key and one value buffer (ping-pong)
size_t sort_pairs_temp_bytes(int64_t n) {
  const size_t m = static_cast<size_t>(n > 0 ? n : 1);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  return al(static_cast<size_t>(kRsBins) * rs_blocks(n) * 4) + al(m * 8) + al(m * 4);
}

// Sorts (keys_in, vals_in) by the low end_bit bits of the keys into
// (keys_out, vals_out); keys_in / vals_in serve as ping-pong buffers.
hipError_t sort_pairs(void* temp, size_t temp_bytes, uint64_t* keys_in,
                      uint64_t* keys_out, int32_t* vals_in, int32_t* vals_out,
                      int64_t n, int end_bit, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (temp_bytes < sort_pairs_temp_bytes(n) || end_bit < 1 || end_bit > 64)
    return hipErrorInvalidValue;
  const int nb = rs_blocks(n);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  char* q = static_cast<char*>(temp);
  int* cnt = reinterpret_cast<int*>(q);
  q += al(static_cast<size_t>(kRsBins) * nb * 4);
  uint64_t* tk = reinterpret_cast<uint64_t*>(q);
  q += al(static_cast<size_t>(n) * 8);
  int32_t* tv = reinterpret_cast<int32_t*>(q);
  const int passes = (end_bit + 7) / 8;
  uint64_t* sk = keys_in;
  int32_t* sv = vals_in;
  for (int p = 0; p < passes; ++p) {
    uint64_t* dk;
    int32_t* dv;
    if (p == passes - 1) {
      dk = keys_out;
      dv = vals_out;
    } else if (sk == tk) {
      dk = keys_in;
      dv = vals_in;
    } else {
      dk = tk;
      dv = tv;
    }
    // the last digit keeps only the bits below end_bit
    const int nbits = end_bit - 8 * p < 8 ? end_bit - 8 * p : 8;
    const unsigned dmask = (1u << nbits) - 1u;
    hipLaunchKernelGGL(rs_hist_kernel, dim3(nb), dim3(kRsBlock), 0, st, sk, n, 8 * p,
                       dmask, cnt, nb);
    hipLaunchKernelGGL(rs_scan_kernel, dim3(1), dim3(1024), 0, st, cnt,
                       static_cast<int64_t>(kRsBins) * nb);
    hipLaunchKernelGGL(rs_scatter_kernel, dim3(nb), dim3(kRsBlock), 0, st, sk, sv, n,
                       8 * p, dmask, cnt, nb, dk, dv);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    sk = dk;
    sv = dv;
  }
  return hipSuccess;
}

}  // namespace abc

extern "C" {
// The spatial index's key sort as an entry point of its own (the tests pin
// it against numpy's stable argsort; cKDTree's build, local_transition.py:
// 82-83, is what the index replaces).  keys / vals are overwritten.
size_t abc_radix_sort_workspace_bytes(int64_t n) {
  return abc::sort_pairs_temp_bytes(n);
}
int abc_radix_sort_pairs_u64(uint64_t* keys, int32_t* vals, int64_t n, int end_bit,
                             uint64_t* keys_out, int32_t* vals_out, void* ws,
                             size_t ws_bytes, hipStream_t st) {
  ABC_REQUIRE(n >= 0 && end_bit >= 1 && end_bit <= 64, "radix_sort: bad arguments");
  if (n == 0) return abc::kOk;
  ABC_REQUIRE(keys && vals && keys_out && vals_out && ws, "radix_sort: null pointer");
  ABC_REQUIRE(ws_bytes >= abc::sort_pairs_temp_bytes(n), "radix_sort: workspace too small");
  ABC_HIP(abc::sort_pairs(ws, ws_bytes, keys, keys_out, vals, vals_out, n, end_bit, st));
  return abc::kOk;
}
}  // extern "C"

namespace abc {
// Loads this translation unit's code object up front (abc_preload).
int preload_sort() { return preload_kernel(rs_scatter_kernel); }
}  // namespace abc
