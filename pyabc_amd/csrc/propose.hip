// Proposal generation: MultivariateNormalTransition.rvs + prior support.
//
// Reference semantics (pyabc/transition/multivariatenormal.py:87-95 and
// pyabc/smc.py:602-645, numpy legacy RandomState):
//   cdf = cumsum(w); cdf /= cdf[-1]            (sequential fp64)
//   idx = cdf.searchsorted(u, side='right')    (u = random_sample())
//   theta = X[idx] + z @ A,  A = sqrt(s)[:,None] * V  from svd(cov)
//   valid iff prior.pdf(theta) > 0; for RV('uniform', lo, scale) scipy tests
//   0 <= (theta - lo) / scale <= 1 in fp64 (random_variables.py:425-452).
// The CDF is built by ONE lane in sequential order so that it is bit-identical
// to numpy's; the resampled indices are then bit-exact for injected u.
// Production proposals draw u and z from Philox4x32-10 inside the kernel
// (no u/z round trip through HBM); the parity entry point takes them as
// inputs.  Out-of-support draws are not evaluations: an order-preserving
// compaction assigns proposal ids to in-support draws only.
#include "common.hpp"
#include "philox.hpp"

namespace abc {

// ---------------------------------------------------------------------------
// Exact sequential fp64 cumsum, evaluated in parallel.
//
// numpy's cumsum is the chain c_k = fl(c_{k-1} + w_k).  While c stays in one
// binade [2^e, 2^(e+1)) every double there is an integer multiple of
// u = 2^(e-52), so with C = c/u (an integer < 2^53) and v = w * 2^(52-e)
// (exact scaling) the rounded sum is fl(c + w) = u * (C + floor(v) +
// [frac(v) > 1/2]) -- except when frac(v) == 1/2 (a tie, resolved by the
// parity of the result) or when the sum leaves the binade.  So a block turns
// each 8192-element tile into INTEGER increments, prefix-sums them exactly
// (int64), and writes every c_k up to the first element that ties or leaves
// the binade; that element is evaluated with the real fp64 add, the grid is
// re-derived from the new c, and the tile continues.  Breaks happen about
// once per binade crossing (~60 for any N), so the result is bit-identical to
// the sequential chain at tile-scan cost.
constexpr int kScanThreads = 1024;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__global__ __launch_bounds__(kScanThreads) void cdf_scan_kernel(
    const double* __restrict__ w, int64_t n, double* __restrict__ cdf) {
  __shared__ long long wsum[kScanThreads / 64];
  __shared__ int first_bad;
  __shared__ double sh_c;
  __shared__ int sh_s;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double c = 0.0;  // running value (uniform)
  for (int64_t base = 0; base < n; base += kScanTile) {
    double wv[kScanItems];
#pragma unroll
    for (int q = 0; q < kScanItems; ++q) {
      const int64_t i = base + static_cast<int64_t>(tid) * kScanItems + q;
      wv[q] = i < n ? w[i] : 0.0;
    }
    const int tile_n = static_cast<int>(n - base < kScanTile ? n - base : kScanTile);
    int s = 0;  // first unprocessed element of the tile (uniform)
    while (s < tile_n) {
      // grid of the current binade
      int ex;
      const double mant = frexp(c, &ex);  // c = mant * 2^ex, mant in [0.5,1)
      (void)mant;
      const bool exact_mode = c >= 0x1p-1000;
      const int e = ex - 1;
      const long long C = exact_mode ? static_cast<long long>(ldexp(c, 52 - e)) : 0;
      long long dl[kScanItems];
      bool bad[kScanItems];
      long long tsum = 0;
#pragma unroll
      for (int q = 0; q < kScanItems; ++q) {
        const int k = tid * kScanItems + q;
        long long dq = 0;
        bool b = false;
        if (k >= s && k < tile_n) {
          if (!exact_mode || wv[q] < 0.0) {
            b = (c != 0.0) || (wv[q] != 0.0);
          } else {
            const double v = ldexp(wv[q], 52 - e);
            if (!(v < 0x1p62)) {
              b = true;
            } else {
              const double fl = floor(v);
              const double fr = v - fl;
              dq = static_cast<long long>(fl) + (fr > 0.5 ? 1 : 0);
              b = (fr == 0.5);
            }
          }
        }
        tsum += dq;
        dl[q] = tsum;  // inclusive within the thread
        bad[q] = b;
      }
      // block exclusive scan of the thread totals
      long long incl = tsum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const long long t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      if (lane == 63) wsum[wid] = incl;
      if (tid == 0) first_bad = 1 << 30;
      __syncthreads();
      long long woff = 0;
      for (int q = 0; q < wid; ++q) woff += wsum[q];
      const long long excl = woff + incl - tsum;
      // binade exit: C + prefix must stay below 2^53 (with one unit margin)
      int my_bad = 1 << 30;
#pragma unroll
      for (int q = 0; q < kScanItems; ++q) {
        const int k = tid * kScanItems + q;
        if (k >= s && k < tile_n) {
          const long long Ck = C + excl + dl[q];
          if (bad[q] || (exact_mode && Ck + 1 >= (1ll << 53))) {
            my_bad = k;
            break;
          }
        }
      }
      if (my_bad < (1 << 30)) atomicMin(&first_bad, my_bad);
      __syncthreads();
      const int b = first_bad;
      // write every element before the first break
#pragma unroll
      for (int q = 0; q < kScanItems; ++q) {
        const int k = tid * kScanItems + q;
        if (k >= s && k < tile_n && k < b) {
          const long long Ck = C + excl + dl[q];
          cdf[base + k] = ldexp(static_cast<double>(Ck), e - 52);
        }
      }
      // the breaking element: the real fp64 add, by its owner
      if (b < tile_n && b / kScanItems == tid) {
        const int q0 = b - tid * kScanItems;
        double prev = c;
        double wb = 0.0;
        long long dprev = 0;
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) {
          if (q == q0) wb = wv[q];
          if (q == q0 - 1) dprev = dl[q];
        }
        if (b > s) prev = ldexp(static_cast<double>(C + excl + dprev), e - 52);
        const double cb = (base + b == 0) ? wb : prev + wb;
        cdf[base + b] = cb;
        sh_c = cb;
        sh_s = b + 1;
      }
      __syncthreads();
      if (b < tile_n) {
        c = sh_c;
        s = sh_s;
      } else {
        // value at the end of the tile = C + total
        long long total = 0;
        for (int q = 0; q < kScanThreads / 64; ++q) total += wsum[q];
        if (exact_mode) c = ldexp(static_cast<double>(C + total), e - 52);
        s = tile_n;
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(256) void cdf_normalize_kernel(double* __restrict__ cdf,
                                                            int64_t n) {
  const double last = cdf[n - 1];
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    cdf[i] = cdf[i] / last;
}

// first index i with cdf[i] > u (numpy searchsorted side='right')
__device__ inline int64_t search_right(const double* __restrict__ cdf, int64_t n,
                                       double u) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cdf[mid] <= u)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

template <int D>
__device__ inline void perturb_one(const double* __restrict__ X, int64_t N,
                                   int d, const double* __restrict__ cdf,
                                   double u, const double (&z)[D],
                                   const double* __restrict__ A,
                                   const double* __restrict__ lo,
                                   const double* __restrict__ scale,
                                   double* __restrict__ theta_row,
                                   int64_t* idx_out, uint8_t* sup_out) {
  int64_t idx = search_right(cdf, N, u);
  const int64_t idx_c = idx < N ? idx : N - 1;  // numpy would raise; u<1 always
  bool ok = true;
#pragma unroll
  for (int l = 0; l < D; ++l) {
    if (l < d) {
      double p = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k)
        if (k < d) p = fma(z[k], A[k * d + l], p);
      const double th = X[idx_c * d + l] + p;
      theta_row[l] = th;
      if (lo) {
        const double x = (th - lo[l]) / scale[l];
        ok = ok && (x >= 0.0) && (x <= 1.0);
      }
    }
  }
  *idx_out = idx;
  *sup_out = ok ? 1 : 0;
}

template <int D>
__global__ __launch_bounds__(256) void resample_perturb_kernel(
    const double* __restrict__ X, int64_t N, int d,
    const double* __restrict__ cdf, const double* __restrict__ u,
    const double* __restrict__ z, const double* __restrict__ A,
    const double* __restrict__ lo, const double* __restrict__ scale,
    int64_t B, double* __restrict__ theta, int64_t* __restrict__ idx,
    uint8_t* __restrict__ sup) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double zz[D];
#pragma unroll
  for (int k = 0; k < D; ++k) zz[k] = k < d ? z[b * d + k] : 0.0;
  perturb_one<D>(X, N, d, cdf, u[b], zz, A, lo, scale, theta + b * d, idx + b,
                 sup + b);
}

// Production proposals: u from stream (2*sid), z from stream (2*sid+1).
//   u[b]   = philox_uniform(seed, 2*sid,   offset + b)
//   z[b,k] = philox_normal (seed, 2*sid+1, (offset + b) * d + k)
template <int D>
__global__ __launch_bounds__(256) void propose_philox_kernel(
    const double* __restrict__ X, int64_t N, int d,
    const double* __restrict__ cdf, const double* __restrict__ A,
    const double* __restrict__ lo, const double* __restrict__ scale,
    uint64_t seed, uint64_t sid, uint64_t offset, int64_t B,
    double* __restrict__ theta, int64_t* __restrict__ idx,
    uint8_t* __restrict__ sup) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t ui = offset + static_cast<uint64_t>(b);
  const u32x4 ub = philox_block(seed, 2 * sid, ui >> 1);
  const double u = (ui & 1) ? u53(ub.z, ub.w) : u53(ub.x, ub.y);
  double zz[D];
  const uint64_t zi0 = ui * static_cast<uint64_t>(d);
#pragma unroll
  for (int k = 0; k < D; ++k) {
    if (k < d) {
      const uint64_t zi = zi0 + k;
      double c0, c1;
      box_muller(philox_block(seed, 2 * sid + 1, zi >> 1), c0, c1);
      zz[k] = (zi & 1) ? c1 : c0;
    } else {
      zz[k] = 0.0;
    }
  }
  perturb_one<D>(X, N, d, cdf, u, zz, A, lo, scale, theta + b * d, idx + b,
                 sup + b);
}

// prior sampling at t=0: theta = lo + scale * U  (scipy uniform.rvs)
__global__ __launch_bounds__(256) void prior_uniform_kernel(
    const double* __restrict__ lo, const double* __restrict__ scale, int d,
    uint64_t seed, uint64_t sid, uint64_t offset, int64_t B,
    double* __restrict__ theta) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= B * d) return;
  const int k = static_cast<int>(i % d);
  const uint64_t ui = offset * d + static_cast<uint64_t>(i);
  const u32x4 ub = philox_block(seed, sid, ui >> 1);
  const double u = (ui & 1) ? u53(ub.z, ub.w) : u53(ub.x, ub.y);
  theta[i] = lo[k] + scale[k] * u;
}

// ---------------------------------------------------------------------------
// RNG fills (for tests and for callers that need raw streams)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void philox_uniform_kernel(uint64_t seed,
                                                             uint64_t sid,
                                                             uint64_t offset,
                                                             int64_t n,
                                                             double* __restrict__ u) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ui = offset + static_cast<uint64_t>(i);
  const u32x4 b = philox_block(seed, sid, ui >> 1);
  u[i] = (ui & 1) ? u53(b.z, b.w) : u53(b.x, b.y);
}

__global__ __launch_bounds__(256) void philox_normal_kernel(uint64_t seed,
                                                            uint64_t sid,
                                                            uint64_t offset,
                                                            int64_t n,
                                                            double* __restrict__ z) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t zi = offset + static_cast<uint64_t>(i);
  double c0, c1;
  box_muller(philox_block(seed, sid, zi >> 1), c0, c1);
  z[i] = (zi & 1) ? c1 : c0;
}

// ---------------------------------------------------------------------------
// order-preserving stream compaction of u8 flags -> int64 positions
// ---------------------------------------------------------------------------
constexpr int kCompactBlock = 256;
constexpr int kCompactItems = 16;  // per thread
constexpr int kCompactTile = kCompactBlock * kCompactItems;

__global__ __launch_bounds__(kCompactBlock) void compact_count_kernel(
    const uint8_t* __restrict__ flags, int64_t n, int64_t* __restrict__ counts) {
  __shared__ int64_t red[4];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kCompactTile;
  int64_t c = 0;
  for (int k = 0; k < kCompactItems; ++k) {
    const int64_t i = base + k * kCompactBlock + threadIdx.x;
    if (i < n) c += flags[i] != 0;
  }
  c = block_sum<int64_t, kCompactBlock>(c, red);
  if (threadIdx.x == 0) counts[blockIdx.x] = c;
}

// exclusive scan of the per-tile counts by one block; writes the total
__global__ __launch_bounds__(1024) void compact_scan_kernel(int64_t* __restrict__ counts,
                                                            int64_t ntiles,
                                                            int64_t* __restrict__ total) {
  __shared__ int64_t s[1024];
  int64_t carry = 0;
  for (int64_t base = 0; base < ntiles; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < ntiles ? counts[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int64_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < ntiles) counts[i] = carry + s[threadIdx.x] - v;
    const int64_t tot = s[1023];
    __syncthreads();
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(kCompactBlock) void compact_scatter_kernel(
    const uint8_t* __restrict__ flags, int64_t n,
    const int64_t* __restrict__ offsets, int64_t* __restrict__ out) {
  __shared__ int wsum[4];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kCompactTile;
  int64_t run = offsets[blockIdx.x];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int k = 0; k < kCompactItems; ++k) {
    const int64_t i = base + k * kCompactBlock + threadIdx.x;
    const bool f = i < n && flags[i] != 0;
    const uint64_t m = __ballot(f);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wid] = __popcll(m);
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wid; ++w) woff += wsum[w];
    if (f) out[run + woff + before] = i;
    run += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
}

// gather rows: out[i, :] = src[idx[i], :]   (int64 idx, fp64 rows of width w)
__global__ __launch_bounds__(256) void gather_rows_kernel(
    const double* __restrict__ src, int64_t width, const int64_t* __restrict__ idx,
    int64_t n, double* __restrict__ out) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n * width) return;
  const int64_t i = t / width, k = t % width;
  out[t] = src[idx[i] * width + k];
}

// ---------------------------------------------------------------------------
static int check_dim(int d) {
  return d >= 1 && d <= 32;
}

#define DISPATCH_D(d, MACRO) \
  if ((d) <= 1) { MACRO(1) } \
  else if ((d) <= 2) { MACRO(2) } \
  else if ((d) <= 4) { MACRO(4) } \
  else if ((d) <= 8) { MACRO(8) } \
  else if ((d) <= 16) { MACRO(16) } \
  else if ((d) <= 24) { MACRO(24) } \
  else { MACRO(32) }

}  // namespace abc

using namespace abc;

extern "C" {

int abc_resample_cdf_f64(const double* w, int64_t n, double* cdf,
                         hipStream_t st) {
  ABC_REQUIRE(n > 0 && w && cdf, "resample_cdf: need n > 0 and buffers");
  hipLaunchKernelGGL(cdf_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, w,
                     n, cdf);
  ABC_LAUNCH_CHECK("cdf_scan_kernel");
  hipLaunchKernelGGL(cdf_normalize_kernel, dim3(stream_grid(n, 256, 1024)),
                     dim3(256), 0, st, cdf, n);
  ABC_LAUNCH_CHECK("cdf_normalize_kernel");
  return kOk;
}

int abc_resample_perturb_f64(const double* X, int64_t N, int d,
                             const double* cdf, const double* u,
                             const double* z, const double* A,
                             const double* lo, const double* scale, int64_t B,
                             double* theta, int64_t* idx, uint8_t* in_support,
                             hipStream_t st) {
  ABC_REQUIRE(check_dim(d), "resample_perturb: unsupported d=%d", d);
  ABC_REQUIRE(N > 0 && B >= 0, "resample_perturb: bad sizes");
  if (B == 0) return kOk;
  ABC_REQUIRE(X && cdf && u && z && A && theta && idx && in_support,
              "resample_perturb: null pointer");
  ABC_REQUIRE((lo == nullptr) == (scale == nullptr),
              "resample_perturb: lo and scale must both be given or NULL");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
#define L(DD)                                                                \
  hipLaunchKernelGGL((resample_perturb_kernel<DD>), dim3(g), dim3(256), 0, st, \
                     X, N, d, cdf, u, z, A, lo, scale, B, theta, idx,         \
                     in_support);
  DISPATCH_D(d, L)
#undef L
  ABC_LAUNCH_CHECK("resample_perturb_kernel");
  return kOk;
}

int abc_propose_philox_f64(const double* X, int64_t N, int d,
                           const double* cdf, const double* A,
                           const double* lo, const double* scale,
                           uint64_t seed, uint64_t sid, uint64_t offset,
                           int64_t B, double* theta, int64_t* idx,
                           uint8_t* in_support, hipStream_t st) {
  ABC_REQUIRE(check_dim(d), "propose: unsupported d=%d", d);
  ABC_REQUIRE(N > 0 && B >= 0, "propose: bad sizes");
  if (B == 0) return kOk;
  ABC_REQUIRE(X && cdf && A && theta && idx && in_support,
              "propose: null pointer");
  ABC_REQUIRE((lo == nullptr) == (scale == nullptr),
              "propose: lo and scale must both be given or NULL");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
#define L(DD)                                                              \
  hipLaunchKernelGGL((propose_philox_kernel<DD>), dim3(g), dim3(256), 0, st, \
                     X, N, d, cdf, A, lo, scale, seed, sid, offset, B, theta, \
                     idx, in_support);
  DISPATCH_D(d, L)
#undef L
  ABC_LAUNCH_CHECK("propose_philox_kernel");
  return kOk;
}

int abc_prior_uniform_f64(const double* lo, const double* scale, int d,
                          uint64_t seed, uint64_t sid, uint64_t offset,
                          int64_t B, double* theta, hipStream_t st) {
  ABC_REQUIRE(d >= 1 && B >= 0, "prior_uniform: bad sizes");
  if (B == 0) return kOk;
  hipLaunchKernelGGL(prior_uniform_kernel, dim3(ceil_div(B * d, 256)),
                     dim3(256), 0, st, lo, scale, d, seed, sid, offset, B,
                     theta);
  ABC_LAUNCH_CHECK("prior_uniform_kernel");
  return kOk;
}

int abc_philox_uniform_f64(uint64_t seed, uint64_t sid, uint64_t offset,
                           int64_t n, double* u, hipStream_t st) {
  ABC_REQUIRE(n >= 0, "philox_uniform: n < 0");
  if (n == 0) return kOk;
  hipLaunchKernelGGL(philox_uniform_kernel, dim3(ceil_div(n, 256)), dim3(256),
                     0, st, seed, sid, offset, n, u);
  ABC_LAUNCH_CHECK("philox_uniform_kernel");
  return kOk;
}

int abc_philox_normal_f64(uint64_t seed, uint64_t sid, uint64_t offset,
                          int64_t n, double* z, hipStream_t st) {
  ABC_REQUIRE(n >= 0, "philox_normal: n < 0");
  if (n == 0) return kOk;
  hipLaunchKernelGGL(philox_normal_kernel, dim3(ceil_div(n, 256)), dim3(256),
                     0, st, seed, sid, offset, n, z);
  ABC_LAUNCH_CHECK("philox_normal_kernel");
  return kOk;
}

size_t abc_compact_workspace_bytes(int64_t n) {
  return static_cast<size_t>(ceil_div(n > 0 ? n : 1, kCompactTile)) * 8 + 64;
}

int abc_compact_flags(const uint8_t* flags, int64_t n, int64_t* out_idx,
                      int64_t* out_count, void* ws, size_t ws_bytes,
                      hipStream_t st) {
  ABC_REQUIRE(n >= 0, "compact: n < 0");
  if (n == 0) {
    ABC_HIP(hipMemsetAsync(out_count, 0, 8, st));
    return kOk;
  }
  const int64_t tiles = ceil_div(n, kCompactTile);
  ABC_REQUIRE(ws_bytes >= static_cast<size_t>(tiles) * 8,
              "compact: workspace too small");
  int64_t* counts = static_cast<int64_t*>(ws);
  hipLaunchKernelGGL(compact_count_kernel, dim3(tiles), dim3(kCompactBlock), 0,
                     st, flags, n, counts);
  ABC_LAUNCH_CHECK("compact_count_kernel");
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, st, counts,
                     tiles, out_count);
  ABC_LAUNCH_CHECK("compact_scan_kernel");
  hipLaunchKernelGGL(compact_scatter_kernel, dim3(tiles), dim3(kCompactBlock),
                     0, st, flags, n, counts, out_idx);
  ABC_LAUNCH_CHECK("compact_scatter_kernel");
  return kOk;
}

int abc_gather_rows_f64(const double* src, int64_t width, const int64_t* idx,
                        int64_t n, double* out, hipStream_t st) {
  ABC_REQUIRE(width > 0 && n >= 0, "gather_rows: bad sizes");
  if (n == 0) return kOk;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(ceil_div(n * width, 256)),
                     dim3(256), 0, st, src, width, idx, n, out);
  ABC_LAUNCH_CHECK("gather_rows_kernel");
  return kOk;
}

}  // extern "C"
