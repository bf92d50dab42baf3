// Pieces of the LocalTransition passes shared by local.hip (kNN, covariances,
// fp64 density, proposals) and local_mfma.hip (the fp32 density on the
// f32 matrix cores): per-particle constants, the exact quadratic form, the
// centred fp32 evaluation points, the finalize and the exact fixup.
// Internal linkage: each translation unit keeps its own copy.
#pragma once

#include "common.hpp"

namespace abc {
namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// per-previous-particle constants: lc_n = log(w_n / sqrt((2 pi)^d det_n)),
// the global offset L = max_n lc_n (ordered-key atomic max), and the
// symmetric quadratic-form coefficients of inv_n packed row by row:
// (A_aa, A_ab + A_ba for b > a), d(d+1)/2 per particle.
__device__ inline void local_pack_coef(const double* __restrict__ invs, int64_t n,
                                       int d, double* __restrict__ coef) {
  const double* A = invs + n * d * d;
  double* c = coef + n * (d * (d + 1) / 2);
  int t = 0;
  for (int a = 0; a < d; ++a) {
    c[t++] = A[a * d + a];
    for (int b = a + 1; b < d; ++b) c[t++] = A[a * d + b] + A[b * d + a];
  }
}

__global__ __launch_bounds__(256) void local_const_kernel(
    const double* __restrict__ w, const double* __restrict__ dets,
    const double* __restrict__ invs, int64_t N, int d,
    double* __restrict__ lc, double* __restrict__ coef,
    unsigned long long* __restrict__ lc_max_key) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  uint64_t key = 0;
  if (n < N) {
    const double norm = sqrt(pow(2.0 * 3.141592653589793, d) * dets[n]);
    const double v = w[n] > 0.0 ? log(w[n] / norm) : -INFINITY;
    lc[n] = v;
    if (v == v) key = f64_key(v);
    if (coef) local_pack_coef(invs, n, d, coef);
  }
  block_atomic_max_u64<256>(lc_max_key, static_cast<unsigned long long>(key));
}

// the z-form pass needs the packed coefficients only for its fixup rows:
// built after the main pass, and only when some row needs them
__global__ __launch_bounds__(256) void local_coef_kernel(
    const double* __restrict__ invs, int64_t N, int d, double* __restrict__ coef,
    const int* __restrict__ n_fix) {
  if (*n_fix == 0) return;
  const int64_t n = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (n < N) local_pack_coef(invs, n, d, coef);
}

// q = (theta - X_n)^T inv_n (theta - X_n) from the packed symmetric form
// (d(d+1)/2 + d FMAs instead of d^2 + d)
template <int D>
__device__ inline double local_qform(const double (&dl)[D],
                                     const double* __restrict__ c) {
  double q = 0.0;
  int t = 0;
#pragma unroll
  for (int a = 0; a < D; ++a) {
    double r = c[t++] * dl[a];
#pragma unroll
    for (int b = a + 1; b < D; ++b) r = fma(c[t++], dl[b], r);
    q = fma(dl[a], r, q);
  }
  return q;
}

template <int D>
__global__ __launch_bounds__(256) void local_pts32_kernel(const double* __restrict__ pts,
                                                          int64_t M,
                                                          const double* __restrict__ X,
                                                          float* __restrict__ pts32,
                                                          float* __restrict__ pts32lo) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= M) return;
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const double c = pts[i * D + q] - X[q];
    const float h = static_cast<float>(c);
    pts32[i * D + q] = h;
    pts32lo[i * D + q] = static_cast<float>(c - static_cast<double>(h));
  }
}

__global__ __launch_bounds__(256) void local_pdf_final_kernel(
    const double* __restrict__ part, int64_t M, int split,
    const unsigned long long* __restrict__ lc_max_key,
    const double* __restrict__ logsumw, double* __restrict__ out,
    int* __restrict__ n_fix, int* __restrict__ fix_rows, double thresh) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= M) return;
  double S = 0.0;
  for (int s = 0; s < split; ++s) S += part[s * M + i];
  if (S >= thresh) {
    out[i] = key_f64(*lc_max_key) + log(S) - *logsumw;
  } else {  // the fixed offset underflowed: exact two-pass evaluation
    fix_rows[atomicAdd(n_fix, 1)] = static_cast<int>(i);
    out[i] = -INFINITY;
  }
}

// exact max-then-sum for rows whose fixed-offset sum underflowed
template <int D>
__global__ __launch_bounds__(256) void local_pdf_fixup_kernel(
    const double* __restrict__ pts, const double* __restrict__ X,
    const double* __restrict__ coef, const double* __restrict__ lc, int64_t N,
    const double* __restrict__ logsumw, const int* __restrict__ n_fix,
    const int* __restrict__ fix_rows, double* __restrict__ out) {
  constexpr int NC = D * (D + 1) / 2;
  __shared__ double red[4];
  const int count = *n_fix;
  for (int f = blockIdx.x; f < count; f += gridDim.x) {
    const int64_t i = fix_rows[f];
    double th[D];
#pragma unroll
    for (int q = 0; q < D; ++q) th[q] = pts[i * D + q];
    double m = -INFINITY;
    for (int64_t n = threadIdx.x; n < N; n += 256) {
      double dl[D];
#pragma unroll
      for (int q = 0; q < D; ++q) dl[q] = th[q] - X[n * D + q];
      m = fmax(m, fma(-0.5, local_qform<D>(dl, coef + n * NC), lc[n]));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    __syncthreads();
    double sum = 0.0;
    if (m > -INFINITY)
      for (int64_t n = threadIdx.x; n < N; n += 256) {
        double dl[D];
#pragma unroll
        for (int q = 0; q < D; ++q) dl[q] = th[q] - X[n * D + q];
        sum += exp(fma(-0.5, local_qform<D>(dl, coef + n * NC), lc[n]) - m);
      }
    sum = block_sum<double, 256>(sum, red);
    if (threadIdx.x == 0)
      out[i] = (m > -INFINITY ? m + log(sum) : -INFINITY) - *logsumw;
    __syncthreads();
  }
}

// log(sum w) in two fixed-order stages: `nb` blocks sum contiguous ranges
// into part[0 .. nb) (eight loads in flight per thread), one wave adds the
// nb partials in order -- the same bits run to run.  (One 1024-thread block
// took 89 us at N = 2e5, latency bound; 0.29 ms with 256 threads.)
__global__ __launch_bounds__(256) void local_sumw_part_kernel(const double* __restrict__ w,
                                                              int64_t N,
                                                              double* __restrict__ part) {
  __shared__ double red[4];
  const int64_t chunk = ceil_div(N, static_cast<int64_t>(gridDim.x));
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * chunk;
  int64_t hi = lo + chunk;
  if (hi > N) hi = N;
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += 8 * 256) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = i0 + u * 256;
      if (i < hi) s[u] += w[i];
    }
  }
  const double t = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  const double b = block_sum<double, 256>(t, red);
  if (threadIdx.x == 0) part[blockIdx.x] = b;
}
__global__ void local_sumw_final_kernel(const double* __restrict__ part, int nb,
                                        double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[b];
  *out = log(s);
}
// launch both (part: >= nb doubles of scratch that is free until the main
// pass; nb = the pass's split, >= 1)
inline void local_sumw(const double* w, int64_t N, int nb, double* part, double* out,
                       hipStream_t st) {
  hipLaunchKernelGGL(local_sumw_part_kernel, dim3(nb), dim3(256), 0, st, w, N, part);
  hipLaunchKernelGGL(local_sumw_final_kernel, dim3(1), dim3(64), 0, st, part, nb, out);
}

// The n-range is cut into a fixed number of chunks that depends on N only,
// so a row's log-sum-exp does not depend on M or on how rows are shared
// between ranks (multi-GPU results equal single-GPU results bit for bit).
inline void local_plan(int64_t /*M*/, int64_t N, int& split, int64_t& nchunk) {
  int64_t sp = 64;
  if (sp > N) sp = N;
  if (sp < 1) sp = 1;
  split = static_cast<int>(sp);
  nchunk = ceil_div(N, sp);
}

}  // namespace
}  // namespace abc
