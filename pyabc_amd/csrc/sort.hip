// Key/value radix sort of the spatial index (spatial.hpp): Hilbert keys of
// the particles (or of the evaluation points) with their int32 indices, in
// place of cKDTree's build (local_transition.py:82-83).  Round 6: this
// repo's own stable LSD radix sort (8-bit digits) replaces the rocPRIM
// (hipcub::DeviceRadixSort) call of rounds 3-5, so no library kernel runs on
// the LocalTransition path.
//
// One pass per 8-bit digit, three kernels each:
//   * rs_hist: per block of rounds * kRsBlock keys the digit histogram (LDS atomics),
//     written digit-major: cnt[digit][block];
//   * rs_scan: one block per digit, the exclusive prefix of cnt[digit][.]
//     over the blocks in place, and the digit's total (the first form ran
//     the whole digit-major prefix on one block: 31 us per pass at 2e5 keys,
//     two thirds of the sort);
//   * rs_scatter: the digits' bases (an exclusive scan of the 256 totals in
//     LDS) plus the block's prefix give the first output slot of (digit,
//     block); the block re-reads its keys in order, kRsBlock at a time,
//     and ranks each key among the equal digits before it: within a wave by
//     an 8-ballot match of the digit, across the block's 4 waves and the
//     earlier rounds by LDS counters.  Equal digits keep their input order,
//     so the sort is stable (the same permutation as the library's).
#include <cstdint>

#include "common.hpp"

namespace abc {
namespace {

constexpr int kRsBlock = 256;               // threads (4 waves)
// rounds of kRsBlock keys per block: 8 from 2^19 keys, else 2 (a 2e5-key
// sort had 98 blocks of 8 rounds for 256 CUs: 11 -> 8 us per scatter pass,
// 0.17 -> 0.14 ms per sort; at 1e6 keys 2 rounds made the per-digit scans
// 4x longer: 0.25 -> 0.35 ms)
inline int rs_rounds(int64_t n) { return n >= (int64_t{1} << 19) ? 8 : 2; }
constexpr int kRsBins = 256;
static_assert(kRsBins == kRsBlock, "one thread per digit");

__global__ __launch_bounds__(kRsBlock) void rs_hist_kernel(
    const uint64_t* __restrict__ keys, int64_t n, int rounds, int shift,
    unsigned dmask, int* __restrict__ cnt, int nb) {
  __shared__ int h[kRsBins];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = static_cast<int64_t>(blockIdx.x) * rounds * kRsBlock;
  for (int r = 0; r < rounds; ++r) {
    const int64_t i = base + r * kRsBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & dmask], 1);
  }
  __syncthreads();
  cnt[static_cast<int64_t>(threadIdx.x) * nb + blockIdx.x] = h[threadIdx.x];
}

// block-wide exclusive scan of one int per thread (kRsBlock threads)
__device__ inline int rs_block_excl(int v, int* part, int& total) {
  const int t = threadIdx.x;
  part[t] = v;
  __syncthreads();
  for (int o = 1; o < kRsBlock; o <<= 1) {  // Hillis-Steele inclusive scan
    const int a = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += a;
    __syncthreads();
  }
  total = part[kRsBlock - 1];
  const int r = part[t] - v;
  __syncthreads();
  return r;
}

// per digit (one block each): cnt[digit][0 .. nb) -> its exclusive prefix
// in place; tot[digit] = the digit's count
__global__ __launch_bounds__(kRsBlock) void rs_scan_kernel(int* __restrict__ cnt,
                                                           int nb,
                                                           int* __restrict__ tot) {
  __shared__ int part[kRsBlock];
  int* c = cnt + static_cast<int64_t>(blockIdx.x) * nb;
  int carry = 0;
  for (int base = 0; base < nb; base += kRsBlock) {
    const int i = base + threadIdx.x;
    const int v = i < nb ? c[i] : 0;
    int t;
    const int e = rs_block_excl(v, part, t);
    if (i < nb) c[i] = carry + e;
    carry += t;
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

__global__ __launch_bounds__(kRsBlock) void rs_scatter_kernel(
    const uint64_t* __restrict__ kin, const int32_t* __restrict__ vin, int64_t n,
    int rounds, int shift, unsigned dmask, const int* __restrict__ off, int nb,
    const int* __restrict__ tot, uint64_t* __restrict__ kout,
    int32_t* __restrict__ vout) {
  __shared__ int run[kRsBins];   // keys of each digit placed by earlier rounds
  __shared__ int wc[4][kRsBins];  // this round's count per (wave, digit)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int all;
  const int dbase = rs_block_excl(tot[threadIdx.x], &wc[0][0], all);
  run[threadIdx.x] =
      dbase + off[static_cast<int64_t>(threadIdx.x) * nb + blockIdx.x];
  const uint64_t lt = (1ull << lane) - 1ull;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * rounds * kRsBlock;
  for (int r = 0; r < rounds; ++r) {
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

int rs_blocks(int64_t n) {
  return static_cast<int>(ceil_div(n > 0 ? n : 1, int64_t{rs_rounds(n)} * kRsBlock));
}

}  // namespace

// scratch: the digit counts, the digit totals, then one key and one value
// buffer (ping-pong)
size_t sort_pairs_temp_bytes(int64_t n) {
  const size_t m = static_cast<size_t>(n > 0 ? n : 1);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  return al(static_cast<size_t>(kRsBins) * rs_blocks(n) * 4) + al(kRsBins * 4) +
         al(m * 8) + al(m * 4);
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
  const int rounds = rs_rounds(n);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  char* q = static_cast<char*>(temp);
  int* cnt = reinterpret_cast<int*>(q);
  q += al(static_cast<size_t>(kRsBins) * nb * 4);
  int* tot = reinterpret_cast<int*>(q);
  q += al(kRsBins * 4);
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
    hipLaunchKernelGGL(rs_hist_kernel, dim3(nb), dim3(kRsBlock), 0, st, sk, n, rounds,
                       8 * p, dmask, cnt, nb);
    hipLaunchKernelGGL(rs_scan_kernel, dim3(kRsBins), dim3(kRsBlock), 0, st, cnt, nb,
                       tot);
    hipLaunchKernelGGL(rs_scatter_kernel, dim3(nb), dim3(kRsBlock), 0, st, sk, sv, n,
                       rounds, 8 * p, dmask, cnt, nb, tot, dk, dv);
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
