// Batched summary-statistic distances, acceptance, and the synthetic batch
// simulators used by the benchmark configurations.
//
// PNormDistance.__call__ (pyabc/distance/distance.py:76-102):
//   d = pow( sum_{key in x_0 order} pow(|(f*w)[key] * (x[key] - x0[key])|, p), 1/p )
//   p = inf: max_key |(f*w) (x - x0)|
// UniformAcceptor (pyabc/acceptor/acceptor.py:235-244): accept iff d <= eps.
//
// Layout: statistics are STAT-MAJOR, stats_T[S][ld] with one column per
// proposal, so lane b reads x[s, b] for s = 0..S-1 with fully coalesced rows;
// the sum over keys is sequential in key order per lane (as the reference's
// Python sum).  Powers p = 1, 2 use t, t*t and sqrt (the reference's glibc
// pow(s, .5) differs from sqrt by at most 1 ulp, for ~1e-3 of all s); the
// kernel flags every particle whose distance lies within 4 ulp of eps (16 for
// a general p) -- the guard band, where that ulp could flip the decision --
// and the engine re-decides the flagged particles on the host with libm pow
// (engine.redecide_guard_band), so accept masks equal the reference's.
#include "common.hpp"
#include "philox.hpp"

namespace abc {

__device__ inline double ulp_of(double x) {
  const double a = fabs(x);
  return nextafter(a, INFINITY) - a;
}

template <int PMODE>  // 1: p=1, 2: p=2, 0: general p, 3: p=inf
__global__ __launch_bounds__(256) void pnorm_kernel(
    const double* __restrict__ stats_T, int64_t ld,
    const double* __restrict__ x0, const double* __restrict__ fw, int64_t B,
    int S, double p, double eps, double* __restrict__ d_out,
    uint8_t* __restrict__ accept, uint8_t* __restrict__ guard) {
#pragma clang fp contract(off)  // t*t then +, separately rounded (ref. pow, sum)
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double acc = 0.0;
  for (int s = 0; s < S; ++s) {
    const double t = fabs(fw[s] * (stats_T[static_cast<int64_t>(s) * ld + b] - x0[s]));
    if (PMODE == 1)
      acc += t;
    else if (PMODE == 2)
      acc += t * t;
    else if (PMODE == 3)
      acc = fmax(acc, t);
    else
      acc += pow(t, p);
  }
  double d;
  if (PMODE == 1 || PMODE == 3)
    d = acc;
  else if (PMODE == 2)
    d = sqrt(acc);
  else
    d = pow(acc, 1.0 / p);
  d_out[b] = d;
  if (accept) accept[b] = d <= eps ? 1 : 0;
  // band: sqrt vs libm pow(s, .5) differ by <= 1 ulp; a general p adds
  // device-pow vs libm-pow error in every term and in the root
  if (guard)
    guard[b] = fabs(d - eps) <= (PMODE == 0 ? 16.0 : 4.0) * ulp_of(eps) ? 1 : 0;
}

// y[s, b] = sum_k A[s, k] theta[b, k] + c[s] + sigma * z(b, s)
// z(b, s) = fast normal (offset + b) * S + s: block i / 4, member i % 4 of
// box_muller4_f32 (philox.hpp) -- the fp64 Box-Muller of the proposal
// streams cost 70 % of this kernel's time, for noise whose precision no
// statistic resolves
__global__ __launch_bounds__(256) void sim_linear_gaussian_kernel(
    const double* __restrict__ theta, int64_t B, int d,
    const double* __restrict__ A, const double* __restrict__ c, int S,
    double sigma, uint64_t seed, uint64_t sid, uint64_t offset,
    double* __restrict__ out_T, int64_t ld) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double th[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) th[k] = k < d ? theta[b * d + k] : 0.0;
  const uint64_t base = (offset + static_cast<uint64_t>(b)) * static_cast<uint64_t>(S);
  float z4[4] = {0.f, 0.f, 0.f, 0.f};
  uint64_t have = ~0ull;
  for (int s = 0; s < S; ++s) {
    double acc = c ? c[s] : 0.0;
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (k < d) acc = fma(A[s * d + k], th[k], acc);
    const uint64_t zi = base + s;
    if ((zi >> 2) != have) {
      box_muller4_f32(philox_block(seed, sid, zi >> 2), z4);
      have = zi >> 2;
    }
    const double z = static_cast<double>(z4[zi & 3]);
    out_T[static_cast<int64_t>(s) * ld + b] = fma(sigma, z, acc);
  }
}

// Fused simulation + distance for rounds whose statistics nobody keeps
// (no recorded statistics, no stored population statistics): the column
// y[., b] of sim_linear_gaussian_kernel is formed stat by stat in registers
// -- the same fma sequence and the same Philox / Box-Muller noise -- and fed
// straight into pnorm_kernel's key-ordered chain, so distances, accept and
// guard flags are bit-identical to the two-kernel path while the 8 S bytes
// per evaluation are neither written nor read back (test_sim_pnorm_fused).
// Round 6: DMAX-sized theta rows (the 32-entry array held 64 VGPRs at any
// d) and, when they fit (LDS_A), the model matrix A and c staged in LDS
// once per block -- read as broadcast LDS loads instead of one scalar load
// per element and statistic.  Same products, same order: the same bits.
template <int PMODE, int DMAX, bool LDS_A>
__global__ __launch_bounds__(256) void sim_lg_pnorm_kernel(
    const double* __restrict__ theta, int64_t B, int d,
    const double* __restrict__ Ag, const double* __restrict__ cg, int S,
    double sigma, uint64_t seed, uint64_t sid, uint64_t offset,
    const double* __restrict__ x0, const double* __restrict__ fw, double p,
    double eps, double* __restrict__ d_out, uint8_t* __restrict__ accept,
    uint8_t* __restrict__ guard, double* __restrict__ out_T, int64_t ld) {
#pragma clang fp contract(off)  // as pnorm_kernel; the fmas are explicit
  extern __shared__ double smem[];
  const double* __restrict__ A = Ag;
  const double* __restrict__ c = cg;
  if constexpr (LDS_A) {
    for (int i = threadIdx.x; i < S * d; i += blockDim.x) smem[i] = Ag[i];
    if (cg)
      for (int i = threadIdx.x; i < S; i += blockDim.x) smem[S * d + i] = cg[i];
    __syncthreads();
    A = smem;
    c = cg ? smem + S * d : nullptr;
  }
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double th[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) th[k] = k < d ? theta[b * d + k] : 0.0;
  const uint64_t base = (offset + static_cast<uint64_t>(b)) * static_cast<uint64_t>(S);
  float z4[4] = {0.f, 0.f, 0.f, 0.f};
  uint64_t have = ~0ull;
  double acc2 = 0.0;
  for (int s = 0; s < S; ++s) {
    double acc = c ? c[s] : 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k)
      if (k < d) acc = fma(A[s * d + k], th[k], acc);
    const uint64_t zi = base + s;
    if ((zi >> 2) != have) {
      box_muller4_f32(philox_block(seed, sid, zi >> 2), z4);
      have = zi >> 2;
    }
    const double y = fma(sigma, static_cast<double>(z4[zi & 3]), acc);
    if (out_T) out_T[static_cast<int64_t>(s) * ld + b] = y;  // kept statistics
    const double t = fabs(fw[s] * (y - x0[s]));
    if (PMODE == 1)
      acc2 += t;
    else if (PMODE == 2)
      acc2 += t * t;
    else if (PMODE == 3)
      acc2 = fmax(acc2, t);
    else
      acc2 += pow(t, p);
  }
  double dist;
  if (PMODE == 1 || PMODE == 3)
    dist = acc2;
  else if (PMODE == 2)
    dist = sqrt(acc2);
  else
    dist = pow(acc2, 1.0 / p);
  d_out[b] = dist;
  if (accept) accept[b] = dist <= eps ? 1 : 0;
  if (guard)
    guard[b] = fabs(dist - eps) <= (PMODE == 0 ? 16.0 : 4.0) * ulp_of(eps) ? 1 : 0;
}

// quickstart model (doc/examples/parameter_inference.ipynb cell 2):
// y = mean + 0.5 * N(0,1), one statistic
__global__ __launch_bounds__(256) void sim_gaussian_mean_kernel(
    const double* __restrict__ theta, int64_t B, double sigma, uint64_t seed,
    uint64_t sid, uint64_t offset, double* __restrict__ out) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t zi = offset + static_cast<uint64_t>(b);
  double z0, z1;
  box_muller(philox_block(seed, sid, zi >> 1), z0, z1);
  out[b] = theta[b] + sigma * ((zi & 1) ? z1 : z0);
}

}  // namespace abc

using namespace abc;

extern "C" {

int abc_pnorm_distance_f64(const double* stats_T, int64_t ld, const double* x0,
                           const double* fw, int64_t B, int S, double p,
                           double eps, double* d_out, uint8_t* accept,
                           uint8_t* guard, hipStream_t st) {
  ABC_REQUIRE(B >= 0 && S >= 0 && ld >= B, "pnorm: bad sizes");
  ABC_REQUIRE(p >= 1.0, "pnorm: It must be p >= 1");
  if (B == 0) return kOk;
  ABC_REQUIRE(stats_T && x0 && fw && d_out, "pnorm: null pointer");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
  if (std::isinf(p))
    hipLaunchKernelGGL(pnorm_kernel<3>, dim3(g), dim3(256), 0, st, stats_T, ld,
                       x0, fw, B, S, p, eps, d_out, accept, guard);
  else if (p == 1.0)
    hipLaunchKernelGGL(pnorm_kernel<1>, dim3(g), dim3(256), 0, st, stats_T, ld,
                       x0, fw, B, S, p, eps, d_out, accept, guard);
  else if (p == 2.0)
    hipLaunchKernelGGL(pnorm_kernel<2>, dim3(g), dim3(256), 0, st, stats_T, ld,
                       x0, fw, B, S, p, eps, d_out, accept, guard);
  else
    hipLaunchKernelGGL(pnorm_kernel<0>, dim3(g), dim3(256), 0, st, stats_T, ld,
                       x0, fw, B, S, p, eps, d_out, accept, guard);
  ABC_LAUNCH_CHECK("pnorm_kernel");
  return kOk;
}

int abc_sim_linear_gaussian_f64(const double* theta, int64_t B, int d,
                                const double* A, const double* c, int S,
                                double sigma, uint64_t seed, uint64_t sid,
                                uint64_t offset, double* out_T, int64_t ld,
                                hipStream_t st) {
  ABC_REQUIRE(d >= 1 && d <= 32 && S >= 1 && B >= 0 && ld >= B,
              "sim_linear_gaussian: bad sizes (d <= 32)");
  if (B == 0) return kOk;
  ABC_REQUIRE(theta && A && out_T, "sim_linear_gaussian: null pointer");
  hipLaunchKernelGGL(sim_linear_gaussian_kernel, dim3(ceil_div(B, 256)),
                     dim3(256), 0, st, theta, B, d, A, c, S, sigma, seed, sid,
                     offset, out_T, ld);
  ABC_LAUNCH_CHECK("sim_linear_gaussian_kernel");
  return kOk;
}

int abc_sim_linear_gaussian_pnorm_stats_f64(
    const double* theta, int64_t B, int d, const double* A, const double* c, int S,
    double sigma, uint64_t seed, uint64_t sid, uint64_t offset, const double* x0,
    const double* fw, double p, double eps, double* d_out, uint8_t* accept,
    uint8_t* guard, double* out_T, int64_t ld, hipStream_t st);

int abc_sim_linear_gaussian_pnorm_f64(const double* theta, int64_t B, int d,
                                      const double* A, const double* c, int S,
                                      double sigma, uint64_t seed, uint64_t sid,
                                      uint64_t offset, const double* x0,
                                      const double* fw, double p, double eps,
                                      double* d_out, uint8_t* accept,
                                      uint8_t* guard, hipStream_t st) {
  return abc_sim_linear_gaussian_pnorm_stats_f64(theta, B, d, A, c, S, sigma, seed,
                                                 sid, offset, x0, fw, p, eps, d_out,
                                                 accept, guard, nullptr, 0, st);
}

// The same pass writing the statistics too (stat-major [S][ld], the columns
// sim_linear_gaussian_kernel writes): the kept-statistics rounds of the
// sampler (History, adaptive distances) no longer read them back for the
// distance (round 6)
int abc_sim_linear_gaussian_pnorm_stats_f64(
    const double* theta, int64_t B, int d, const double* A, const double* c, int S,
    double sigma, uint64_t seed, uint64_t sid, uint64_t offset, const double* x0,
    const double* fw, double p, double eps, double* d_out, uint8_t* accept,
    uint8_t* guard, double* out_T, int64_t ld, hipStream_t st) {
  ABC_REQUIRE(d >= 1 && d <= 32 && S >= 1 && B >= 0,
              "sim_linear_gaussian_pnorm: bad sizes (d <= 32)");
  ABC_REQUIRE(!out_T || ld >= B, "sim_linear_gaussian_pnorm: ld < B");
  ABC_REQUIRE(p >= 1.0, "sim_linear_gaussian_pnorm: It must be p >= 1");
  if (B == 0) return kOk;
  ABC_REQUIRE(theta && A && x0 && fw && d_out,
              "sim_linear_gaussian_pnorm: null pointer");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
  const size_t lds = static_cast<size_t>(S) * (d + 1) * sizeof(double);
  const bool in_lds = lds <= 48 * 1024;
#define LK(PM, DM, LA)                                                             \
  hipLaunchKernelGGL((sim_lg_pnorm_kernel<PM, DM, LA>), dim3(g), dim3(256),         \
                     LA ? lds : 0, st, theta, B, d, A, c, S, sigma, seed, sid,      \
                     offset, x0, fw, p, eps, d_out, accept, guard, out_T, ld)
#define LD(PM, DM) \
  if (in_lds) {    \
    LK(PM, DM, true);  \
  } else {         \
    LK(PM, DM, false); \
  }
#define L(PM)                  \
  if (d <= 8) {                \
    LD(PM, 8)                  \
  } else if (d <= 16) {        \
    LD(PM, 16)                 \
  } else if (d <= 24) {        \
    LD(PM, 24)                 \
  } else {                     \
    LD(PM, 32)                 \
  }
  if (std::isinf(p)) {
    L(3)
  } else if (p == 1.0) {
    L(1)
  } else if (p == 2.0) {
    L(2)
  } else {
    L(0)
  }
#undef L
#undef LD
#undef LK
  ABC_LAUNCH_CHECK("sim_lg_pnorm_kernel");
  return kOk;
}

int abc_sim_gaussian_mean_f64(const double* theta, int64_t B, double sigma,
                              uint64_t seed, uint64_t sid, uint64_t offset,
                              double* out, hipStream_t st) {
  ABC_REQUIRE(B >= 0, "sim_gaussian_mean: bad sizes");
  if (B == 0) return kOk;
  hipLaunchKernelGGL(sim_gaussian_mean_kernel, dim3(ceil_div(B, 256)),
                     dim3(256), 0, st, theta, B, sigma, seed, sid, offset, out);
  ABC_LAUNCH_CHECK("sim_gaussian_mean_kernel");
  return kOk;
}

}  // extern "C"

namespace abc {
// Loads this translation unit's code object (HIP loads each one lazily, at
// the first launch of one of its kernels: ~4 ms for local_mfma's inside
// C4's first weighted generation); abc_preload calls every unit's hook.
int preload_distance() { return preload_kernel(pnorm_kernel<2>); }
}  // namespace abc
