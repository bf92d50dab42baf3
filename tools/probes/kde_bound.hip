// Derived accuracy bound of the folded MFMA KDE pass, evaluated on EVERY row
// (test infrastructure, built into tools/probes/libabc_probe.so beside the
// issue probe; never part of libabc_hip.so).  The fp64 restatement of
// tests/kde_bound.py:row_stats ("Accuracy of the folded
// accumulation"), one thread per row against the whole population, so the
// full-size tests can assert the bound on all 1e6 rows instead of a sample:
//
//   e_ij   = lw2_j - |y_i - y_j|^2                     (fp64, log2 units)
//   hi_ij  = 2 y1_i.y1_j + aH_j + bH_i,  y1 = g rint(y / g),
//            aH_j = G rint((lw2_j - |y_j|^2) / G),
//            bH_i = G rint((-|y_i|^2 - m_i) / G),  G = g^2
//   lo_ij  = (e_ij - m_i) - hi_ij
//   p_ij   = 2^e_ij / sum_j 2^e_ij
//   bound_i = ln2 (1.5 KL sum_j p_ij ulp32(|hi_ij| + |lo_ij|) + D G 2^-12)
//             + 2^-23 + 6 2^-24
//
// plus log2 S_i'' (the row sum relative to its offset m_i) and the term-share
// entropy H_i (bits).  P is the packed direct population [npad][D + 1]
// (y_j, lw2_j; kde_mfma.hip), Y the whitened rows [M][D] (WhitenedRows.Y),
// off the per-row offsets m_i.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace {

constexpr int kTJ = 64;  // population rows staged in LDS per step

__device__ inline double ulp32(double x) {
  if (!(x > 0x1p-126)) return 0x1p-149;
  return ldexp(1.0, ilogb(x) - 23);
}

template <int D>
__global__ __launch_bounds__(256) void bound_kernel(
    const double* __restrict__ P, int64_t n, const double* __restrict__ Y,
    const double* __restrict__ off, int64_t M, double g, int KL,
    double* __restrict__ bound, double* __restrict__ log2s,
    double* __restrict__ ent) {
  __shared__ double sy[kTJ][D];
  __shared__ double sy1[kTJ][D];
  __shared__ double sc[kTJ][3];  // lw2, |y|^2, aH
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool live = i < M;
  const double G = g * g;
  double y[D], y1[D];
  double n2 = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    y[k] = live ? Y[i * D + k] : 0.0;
    y1[k] = g * rint(y[k] / g);
    n2 = fma(y[k], y[k], n2);
  }
  const double m = live && off ? off[i] : 0.0;
  const double bH = G * rint((-n2 - m) / G);
  double mx = -INFINITY, s = 0.0, su = 0.0, se = 0.0;
  for (int64_t j0 = 0; j0 < n; j0 += kTJ) {
    __syncthreads();
    for (int t = threadIdx.x; t < kTJ * (D + 1); t += blockDim.x) {
      const int jj = t / (D + 1), k = t % (D + 1);
      const int64_t j = j0 + jj;
      const double v = j < n ? P[j * (D + 1) + k] : 0.0;
      if (k < D) {
        sy[jj][k] = v;
        sy1[jj][k] = g * rint(v / g);
      } else {
        sc[jj][0] = j < n ? v : -INFINITY;
      }
    }
    __syncthreads();
    if (threadIdx.x < kTJ) {
      double q = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) q = fma(sy[threadIdx.x][k], sy[threadIdx.x][k], q);
      sc[threadIdx.x][1] = q;
      sc[threadIdx.x][2] = G * rint((sc[threadIdx.x][0] - q) / G);
    }
    __syncthreads();
    const int nj = n - j0 < kTJ ? static_cast<int>(n - j0) : kTJ;
    for (int jj = 0; jj < nj; ++jj) {
      double dot = 0.0, d1 = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        dot = fma(y[k], sy[jj][k], dot);
        d1 = fma(y1[k], sy1[jj][k], d1);
      }
      const double e = sc[jj][0] - (n2 + sc[jj][1] - 2.0 * dot);
      const double ee = e - m;
      const double hi = 2.0 * d1 + sc[jj][2] + bH;
      const double lo = ee - hi;
      const double u = ulp32(fabs(hi) + fabs(lo));
      if (ee > mx) {
        const double sc0 = exp2(mx - ee);
        s *= sc0;
        su *= sc0;
        se *= sc0;
        mx = ee;
      }
      const double t = exp2(ee - mx);
      s += t;
      su = fma(t, u, su);
      se = fma(t, ee, se);
    }
  }
  if (!live) return;
  const double ls = mx + log2(s);
  bound[i] = 0.6931471805599453 * (1.5 * KL * (su / s) + D * G * 0x1p-12) +
             0x1p-23 + 6.0 * 0x1p-24;
  log2s[i] = ls;
  ent[i] = ls - se / s;
}

}  // namespace

extern "C" {

// bound / log2 S'' / entropy of M rows (device pointers, fp64); 0 on success
int abc_probe_kde_bound(const double* P, int64_t n, int D, const double* Y,
                        const double* off, int64_t M, double g, int KL,
                        double* bound, double* log2s, double* ent,
                        hipStream_t st) {
  if (M <= 0) return 0;
  const dim3 grid(static_cast<unsigned>((M + 255) / 256)), block(256);
  switch (D) {
#define CASE(DD)                                                              \
  case DD:                                                                    \
    hipLaunchKernelGGL(bound_kernel<DD>, grid, block, 0, st, P, n, Y, off, M, \
                       g, KL, bound, log2s, ent);                             \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16) CASE(20)
    CASE(24)
#undef CASE
    default:
      return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
