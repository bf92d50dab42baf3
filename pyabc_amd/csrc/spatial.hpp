// Spatial index of a particle population for the LocalTransition kNN
// (cKDTree(X).query(X, k + 1), local_transition.py:82-83).
//
// The population is put in Hilbert order (d coordinates quantised to
// b = min(21, 63 / d) bits each on the population's bounding box, Skilling's
// transpose form of the Hilbert index, keys radix-sorted with their indices)
// and cut into tiles of 64 consecutive particles.  Hilbert order has no
// jumps, so a tile's box is tighter than under Morton order: a numpy count at
// C4's shape (N = 2e5, d = 6, k = 50, 4 rows per wave) needs 238 instead of
// 377 tiles per wave at the final thresholds.  A tile carries the bounding box of its fp32 centred
// coordinates (x - X[0], the same rounding the kNN filter computes with).
// The kNN skips a tile for a query row when the box distance, computed with
// the filter's own rounded operations (rounding is monotone), is not below
// the row's filter threshold: no candidate in the tile could pass the
// filter, so the neighbour sets are those of the full scan.  (The same
// bound does not pay for the density pass: in 6-D the k = 50 local kernels
// are as wide as the population -- a numpy simulation of C4 needs 97.6 % of
// the tiles per row at a 2^-40 loss bound)
#pragma once

#include "common.hpp"

namespace abc {

constexpr int kTile = 64;  // particles per tile (one per lane)

size_t sort_pairs_temp_bytes(int64_t n);
// this repo's stable LSD radix sort (sort.hip); keys_in / vals_in are
// overwritten (ping-pong buffers)
hipError_t sort_pairs(void* temp, size_t temp_bytes, uint64_t* keys_in,
                      uint64_t* keys_out, int32_t* vals_in, int32_t* vals_out,
                      int64_t n, int end_bit, hipStream_t st);

__host__ __device__ inline int morton_bits(int d) {
  const int b = 63 / d;
  return b < 21 ? b : 21;
}

namespace {  // kernels: internal linkage in every including unit

// Quantisation frame: per dimension the extent of (x - X[0]) over the
// population as ordered fp64 keys, min in [q], max in [8 + q].
template <int D>
__global__ __launch_bounds__(256) void sp_extent_kernel(
    const double* __restrict__ X, int64_t N,
    unsigned long long* __restrict__ ext) {
  __shared__ unsigned long long red[2 * D][4];
  uint64_t mn[D], mx[D];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    mn[q] = ~0ull;
    mx[q] = 0ull;
  }
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < N;
       i += static_cast<int64_t>(gridDim.x) * 256) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const uint64_t k = f64_key(X[i * D + q] - X[q]);
      mn[q] = k < mn[q] ? k : mn[q];
      mx[q] = k > mx[q] ? k : mx[q];
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < D; ++q) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t a = __shfl_xor(mn[q], o, 64), b = __shfl_xor(mx[q], o, 64);
      mn[q] = a < mn[q] ? a : mn[q];
      mx[q] = b > mx[q] ? b : mx[q];
    }
    if (lane == 0) {
      red[q][wid] = mn[q];
      red[D + q][wid] = mx[q];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * D) {
    const int c = threadIdx.x;
    unsigned long long v = red[c][0];
#pragma unroll
    for (int w = 1; w < 4; ++w)
      v = c < D ? (red[c][w] < v ? red[c][w] : v) : (red[c][w] > v ? red[c][w] : v);
    if (c < D)
      atomicMin(ext + c, v);
    else
      atomicMax(ext + 8 + (c - D), v);
  }
}

// Hilbert key of the points P[n][D] in the frame of X (clamped to the grid):
// J. Skilling, "Programming the Hilbert curve" (AIP Conf. Proc. 707, 2004),
// AxesToTranspose, then the transposed index interleaved into one key.
template <int D>
__global__ __launch_bounds__(256) void sp_key_kernel(
    const double* __restrict__ P, int64_t n, const double* __restrict__ X,
    const unsigned long long* __restrict__ ext, uint64_t* __restrict__ keys,
    int32_t* __restrict__ vals) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  constexpr int B = 63 / D < 21 ? 63 / D : 21;
  const double cells = static_cast<double>((1u << B) - 1);
  uint64_t c[D];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const double lo = key_f64(ext[q]), hi = key_f64(ext[8 + q]);
    const double span = hi - lo;
    double v = span > 0.0 ? (P[i * D + q] - X[q] - lo) * (cells / span) : 0.0;
    v = v > 0.0 ? (v < cells ? v : cells) : 0.0;  // NaN -> 0
    c[q] = static_cast<uint64_t>(v);
  }
  constexpr uint64_t M = 1ull << (B - 1);
  for (uint64_t Q = M; Q > 1; Q >>= 1) {  // inverse undo
    const uint64_t P1 = Q - 1;
#pragma unroll
    for (int q = 0; q < D; ++q) {
      if (c[q] & Q) {
        c[0] ^= P1;
      } else {
        const uint64_t t = (c[0] ^ c[q]) & P1;
        c[0] ^= t;
        c[q] ^= t;
      }
    }
  }
#pragma unroll
  for (int q = 1; q < D; ++q) c[q] ^= c[q - 1];  // Gray encode
  uint64_t tg = 0;
  for (uint64_t Q = M; Q > 1; Q >>= 1)
    if (c[D - 1] & Q) tg ^= Q - 1;
#pragma unroll
  for (int q = 0; q < D; ++q) c[q] ^= tg;
  uint64_t key = 0;
#pragma unroll
  for (int b = B - 1; b >= 0; --b)
#pragma unroll
    for (int q = 0; q < D; ++q) key = (key << 1) | ((c[q] >> b) & 1u);
  keys[i] = key;
  vals[i] = static_cast<int32_t>(i);
}

// Order-preserving-within-block compaction of the sorted positions whose
// original index lies in [rlo, rhi) (the rank's row share).  Blocks append
// in arbitrary order; the passes' results do not depend on the row order.
__global__ __launch_bounds__(256) void sp_rows_in_range_kernel(
    const int32_t* __restrict__ perm, int64_t N, int64_t rlo, int64_t rhi,
    int32_t* __restrict__ out, int* __restrict__ count) {
  __shared__ int wcnt[4];
  __shared__ int base;
  const int64_t s = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const bool in = s < N && perm[s] >= rlo && perm[s] < rhi;
  const uint64_t m = __ballot(in);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) wcnt[wid] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0)
    base = atomicAdd(count, wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3]);
  __syncthreads();
  int off = base;
  for (int w = 0; w < wid; ++w) off += wcnt[w];
  if (in) out[off + __popcll(m & ((1ull << lane) - 1ull))] = static_cast<int32_t>(s);
}

// Squared distance lower bound of a point to a box with the fp32 operations
// of the passes (gap per dimension, fma chain): monotone in the gap.
template <int D>
__device__ inline float box_dist2(const float (&x)[D], const float* __restrict__ lo,
                                  const float* __restrict__ hi) {
  float s = 0.0f;
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const float g = fmaxf(fmaxf(lo[q] - x[q], x[q] - hi[q]), 0.0f);
    s = __builtin_fmaf(g, g, s);
  }
  return s;
}

inline size_t al256(size_t b) { return (b + 255) / 256 * 256; }
// Workspace of the spatial index (spatial.hpp) over n points padded to
// whole tiles: header (ext keys, counters) | keys_in[n] | keys_out[n] |
// vals_in[n] | perm[T*64] | tbox[T][2][8] | sort temp.
struct SpatialWs {
  unsigned long long* ext;  // [16]: per-dim min keys, then max keys
  int* count;
  uint64_t* keys_in;
  uint64_t* keys_out;
  int32_t* vals_in;
  int32_t* perm;
  float* tbox;
  void* temp;
  size_t temp_bytes;
  int T;
};

inline size_t spatial_ws_bytes(int64_t n) {
  const int64_t T = ceil_div(n > 0 ? n : 1, kTile);
  return 256 + 2 * al256(static_cast<size_t>(n) * 8) + al256(static_cast<size_t>(n) * 4) +
         al256(static_cast<size_t>(T) * kTile * 4) + al256(static_cast<size_t>(T) * 2 * 8 * 4) +
         al256(sort_pairs_temp_bytes(n));
}

inline SpatialWs spatial_ws(void* ws, int64_t n) {
  SpatialWs v;
  char* q = static_cast<char*>(ws);
  v.T = static_cast<int>(ceil_div(n > 0 ? n : 1, kTile));
  v.ext = reinterpret_cast<unsigned long long*>(q);
  v.count = reinterpret_cast<int*>(q + 128);
  q += 256;
  v.keys_in = reinterpret_cast<uint64_t*>(q);
  q += al256(static_cast<size_t>(n) * 8);
  v.keys_out = reinterpret_cast<uint64_t*>(q);
  q += al256(static_cast<size_t>(n) * 8);
  v.vals_in = reinterpret_cast<int32_t*>(q);
  q += al256(static_cast<size_t>(n) * 4);
  v.perm = reinterpret_cast<int32_t*>(q);
  q += al256(static_cast<size_t>(v.T) * kTile * 4);
  v.tbox = reinterpret_cast<float*>(q);
  q += al256(static_cast<size_t>(v.T) * 2 * 8 * 4);
  v.temp = q;
  v.temp_bytes = al256(sort_pairs_temp_bytes(n));
  return v;
}

// Hilbert order of X (spatial.hpp): ext, keys, sort -> keys_out / perm (the
// padding positions of the last tile map to particle 0).
template <int D>
int spatial_sort_population(const double* X, int64_t N, SpatialWs& v,
                                   hipStream_t st) {
  ABC_HIP(hipMemsetAsync(v.ext, 0xff, 64, st));
  ABC_HIP(hipMemsetAsync(v.ext + 8, 0, 64 + 8, st));
  hipLaunchKernelGGL((sp_extent_kernel<D>), dim3(stream_grid(N, 256, 64)), dim3(256),
                     0, st, X, N, v.ext);
  hipLaunchKernelGGL((sp_key_kernel<D>), dim3(ceil_div(N, 256)), dim3(256), 0, st,
                     X, N, X, v.ext, v.keys_in, v.vals_in);
  ABC_HIP(sort_pairs(v.temp, v.temp_bytes, v.keys_in, v.keys_out, v.vals_in, v.perm,
                     N, morton_bits(D) * D, st));
  const int64_t pad = static_cast<int64_t>(v.T) * kTile - N;
  if (pad > 0) ABC_HIP(hipMemsetAsync(v.perm + N, 0, pad * 4, st));
  return kOk;
}


}  // namespace
}  // namespace abc
