// Exact-inference ABC: stochastic kernels, stochastic
// acceptance and the tempered sums behind the temperature schemes.
//
// IndependentNormalKernel.__call__  (pyabc/distance/kernel.py:256-282):
//   log pd = -0.5 * (c + np.sum(diff**2 / var)),  c = np.sum(log 2 + log pi + log var)
// IndependentLaplaceKernel.__call__ (pyabc/distance/kernel.py:332-357):
//   log pd = -(c + np.sum(|diff| / b)),           c = np.sum(log 2 + log b)
// diff = x - x_0 over the kernel's (sorted) keys.  The constant c is a
// per-kernel scalar computed once on the host with numpy; the per-particle
// sum is numpy's float64 pairwise summation (0 + pairwise: eight strided
// accumulators per <=128 block, halves split at a multiple of 8), restated
// here term for term, so the log-density is bit-identical to the reference.
//
// StochasticAcceptor.__call__ (pyabc/acceptor/acceptor.py:440-473):
//   acc = exp((pd - c) * (1/T))  [SCALE_LOG]   or  (pd / c) ** (1/T)  [SCALE_LIN]
//   accept iff acc >= u,  u ~ U[0,1)
//   weight = 0 if acc == 0, acc / min(1, acc) with importance weighting, else 1
// exp / pow are the device libm; the reference's numpy exp / libm pow can
// differ by an ulp, so every particle whose acc lies within 4 ulp of u is
// flagged (guard band) and the parity tests assert the band is empty.
//
// Layout: statistics stat-major stats_T[S][ld] (one column per evaluation),
// lane b walks s = 0..S-1 with coalesced rows, as the p-norm kernel does.
// HBM-bound: 8 S + 8 (u, when injected) + 8 + 8 + 1 + 1 bytes per evaluation.
#include "common.hpp"
#include "philox.hpp"

namespace abc {

namespace {

// numpy pairwise_sum of n <= 128 terms starting at lo
template <class F>
__device__ inline double np_pw_block(const F& term, int lo, int n) {
#pragma clang fp contract(off)
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += term(lo + i);
    return r;
  }
  double r0 = term(lo + 0), r1 = term(lo + 1), r2 = term(lo + 2),
         r3 = term(lo + 3), r4 = term(lo + 4), r5 = term(lo + 5),
         r6 = term(lo + 6), r7 = term(lo + 7);
  const int lim = n - (n % 8);
  int i = 8;
  for (; i < lim; i += 8) {
    r0 += term(lo + i + 0);
    r1 += term(lo + i + 1);
    r2 += term(lo + i + 2);
    r3 += term(lo + i + 3);
    r4 += term(lo + i + 4);
    r5 += term(lo + i + 5);
    r6 += term(lo + i + 6);
    r7 += term(lo + i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += term(lo + i);
  return res;
}

// recursive halves (numpy: n2 = n / 2; n2 -= n2 % 8), DEPTH levels deep
template <int DEPTH, class F>
__device__ inline double np_pw(const F& term, int lo, int n) {
#pragma clang fp contract(off)
  if constexpr (DEPTH == 0) {
    return np_pw_block(term, lo, n);
  } else {
    if (n <= 128) return np_pw_block(term, lo, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_pw<DEPTH - 1>(term, lo, n2) + np_pw<DEPTH - 1>(term, lo + n2, n - n2);
  }
}

constexpr int kPwDepth = 5;          // S <= 128 * 2^5 = 4096
constexpr int kMaxStats = 128 << kPwDepth;

__device__ inline double ulp_of(double x) {
  const double a = fabs(x);
  return nextafter(a, INFINITY) - a;
}

// acceptance of one evaluation: probability, decision, weight, guard flag
__device__ inline void stochastic_decide(double pd, double pdf_norm,
                                         double inv_temp, int log_scale,
                                         int apply_iw, double u,
                                         uint8_t& accept, double& weight,
                                         uint8_t& guard) {
#pragma clang fp contract(off)
  const double acc = log_scale ? exp((pd - pdf_norm) * inv_temp)
                               : pow(pd / pdf_norm, inv_temp);
  accept = acc >= u ? 1 : 0;
  weight = acc == 0.0 ? 0.0 : (apply_iw ? acc / fmin(1.0, acc) : 1.0);
  guard = (acc < 1.0 && fabs(acc - u) <= 4.0 * ulp_of(fmax(acc, u))) ? 1 : 0;
}

__device__ inline double philox_u01(uint64_t seed, uint64_t stream, uint64_t i) {
  const u32x4 b = philox_block(seed, stream, i >> 1);
  return (i & 1) ? u53(b.z, b.w) : u53(b.x, b.y);
}

}  // namespace

// KIND 0: independent normal (prm = var), 1: independent Laplace (prm = b)
template <int KIND>
__global__ __launch_bounds__(256) void stochastic_kernel_kernel(
    const double* __restrict__ stats_T, int64_t ld,
    const double* __restrict__ x0, const double* __restrict__ prm, int S,
    double c, int64_t B, double* __restrict__ pd_out,
    // fused acceptance (accept == nullptr: density only)
    double pdf_norm, double inv_temp, int apply_iw,
    const double* __restrict__ u_in, uint64_t seed, uint64_t stream,
    uint64_t offset, uint8_t* __restrict__ accept, double* __restrict__ accw,
    uint8_t* __restrict__ guard) {
#pragma clang fp contract(off)  // diff*diff, /var, + separately rounded
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* col = stats_T + b;
  auto term = [&](int s) -> double {
    const double diff = col[static_cast<int64_t>(s) * ld] - x0[s];
    if (KIND == 0) return (diff * diff) / prm[s];
    return fabs(diff) / prm[s];
  };
  const double sum = 0.0 + np_pw<kPwDepth>(term, 0, S);
  const double pd = KIND == 0 ? -0.5 * (c + sum) : -(c + sum);
  pd_out[b] = pd;
  if (accept) {
    const double u = u_in ? u_in[b] : philox_u01(seed, stream, offset + b);
    uint8_t a, g;
    double w;
    stochastic_decide(pd, pdf_norm, inv_temp, 1, apply_iw, u, a, w, g);
    accept[b] = a;
    if (accw) accw[b] = w;
    if (guard) guard[b] = g;
  }
}

__global__ __launch_bounds__(256) void stochastic_accept_kernel(
    const double* __restrict__ pd, int64_t B, double pdf_norm, double inv_temp,
    int log_scale, int apply_iw, const double* __restrict__ u_in, uint64_t seed,
    uint64_t stream, uint64_t offset, uint8_t* __restrict__ accept,
    double* __restrict__ accw, uint8_t* __restrict__ guard) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double u = u_in ? u_in[b] : philox_u01(seed, stream, offset + b);
  uint8_t a, g;
  double w;
  stochastic_decide(pd[b], pdf_norm, inv_temp, log_scale, apply_iw, u, a, w, g);
  accept[b] = a;
  if (accw) accw[b] = w;
  if (guard) guard[b] = g;
}

// w = (prior_const * s_i) / exp(logpd_i)   (smc.py:776-792 with the
// acceptance weight: prior_pd * acceptance_weight * 1 / transition_pd);
// logpd == nullptr (t = 0): w = prior_const * s_i   (smc.py:762-770)
__global__ __launch_bounds__(256) void importance_scaled_kernel(
    const double* __restrict__ logpd, const double* __restrict__ s,
    double prior_const, int64_t M, double* __restrict__ w) {
#pragma clang fp contract(off)
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= M) return;
  const double pr = s ? prior_const * s[i] : prior_const;
  w[i] = logpd ? pr / exp(logpd[i]) : pr;
}

// Tempered sums for the temperature schemes (epsilon/temperature.py:306-345
// AcceptanceRateScheme objective, :695-742 EssScheme).  Particle weight
//   w_i = (w ? w[i] : 1) * (lnum ? exp(lnum[i] - (lden ? lden[i] : 0)) : 1)
// (the AcceptanceRateScheme's importance weight t_pd / t_pd_prev from the two
// transition log-densities), and for every beta_k
//   v_i = exp((pd_i - c) beta_k)  [log]  or  (pd_i / c)^beta_k  [lin],
//   v_i = min(v_i, 1) when clamp,
//   out[0] = sum w_i, out[1] = sum w_i^2,
//   out[2 + 2k] = sum w_i v_i,  out[3 + 2k] = sum (w_i v_i)^2.
// Deterministic: the grid is a function of n, fixed per-block tree,
// fixed-order final sum over the block partials.
constexpr int kTsBlock = 256;
constexpr int kTsMaxK = 16;
constexpr int kTsGrid = 512;

__global__ __launch_bounds__(kTsBlock) void tempered_sums_kernel(
    const double* __restrict__ pd, const double* __restrict__ wl,
    const double* __restrict__ lnum, const double* __restrict__ lden,
    int64_t n, double c, int log_scale, const double* __restrict__ betas,
    int K, int clamp, double* __restrict__ partial /* [grid][2K+2] */) {
#pragma clang fp contract(off)
  __shared__ double lds[kTsBlock / 64];
  double a[kTsMaxK], q[kTsMaxK], bk[kTsMaxK];
  double sw = 0.0, sw2 = 0.0;
#pragma unroll
  for (int k = 0; k < kTsMaxK; ++k) {
    a[k] = 0.0;
    q[k] = 0.0;
    bk[k] = k < K ? betas[k] : 0.0;
  }
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kTsBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kTsBlock + threadIdx.x;
       i < n; i += stride) {
    const double p = pd[i];
    double w = wl ? wl[i] : 1.0;
    if (lnum) w *= exp(lnum[i] - (lden ? lden[i] : 0.0));
    sw += w;
    sw2 += w * w;
    const double x = log_scale ? (p - c) : (p / c);
#pragma unroll
    for (int k = 0; k < kTsMaxK; ++k) {
      if (k < K) {
        double v = log_scale ? exp(x * bk[k]) : pow(x, bk[k]);
        if (clamp) v = fmin(v, 1.0);
        const double wv = w * v;
        a[k] += wv;
        q[k] += wv * wv;
      }
    }
  }
  const int64_t base = static_cast<int64_t>(blockIdx.x) * (2 * K + 2);
  const double s0 = block_sum<double, kTsBlock>(sw, lds);
  const double s1 = block_sum<double, kTsBlock>(sw2, lds);
  if (threadIdx.x == 0) {
    partial[base] = s0;
    partial[base + 1] = s1;
  }
  for (int k = 0; k < K; ++k) {
    const double sa = block_sum<double, kTsBlock>(a[k], lds);
    const double sq = block_sum<double, kTsBlock>(q[k], lds);
    if (threadIdx.x == 0) {
      partial[base + 2 + 2 * k] = sa;
      partial[base + 3 + 2 * k] = sq;
    }
  }
}

// One wave per output: lane l adds the block partials l, l + 64, ... in
// order, then a fixed xor tree (one thread per output walked the <= 512
// partials as a dependent chain: ~54 us per call, 42 calls per generation in
// the exact-inference run's temperature bisection).
__global__ __launch_bounds__(64) void tempered_sums_finish(
    const double* __restrict__ partial, int grid, int width,
    double* __restrict__ out) {
  const int j = blockIdx.x;
  const int lane = threadIdx.x;
  double s = 0.0;
  for (int g = lane; g < grid; g += 64) s += partial[static_cast<int64_t>(g) * width + j];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[j] = s;
}

}  // namespace abc

using namespace abc;

extern "C" {

int abc_stochastic_kernel_f64(const double* stats_T, int64_t ld,
                              const double* x0, const double* prm, int S,
                              int kind, double c, int64_t B, double* pd_out,
                              double pdf_norm, double inv_temp, int apply_iw,
                              const double* u, uint64_t seed, uint64_t stream,
                              uint64_t offset, uint8_t* accept, double* accw,
                              uint8_t* guard, hipStream_t st) {
  ABC_REQUIRE(B >= 0 && S >= 1 && ld >= B, "stochastic_kernel: bad sizes");
  ABC_REQUIRE(S <= kMaxStats, "stochastic_kernel: S > %d unsupported",
              kMaxStats);
  ABC_REQUIRE(kind == 0 || kind == 1,
              "stochastic_kernel: kind must be 0 (normal) or 1 (laplace)");
  if (B == 0) return kOk;
  ABC_REQUIRE(stats_T && x0 && prm && pd_out, "stochastic_kernel: null pointer");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
  if (kind == 0)
    hipLaunchKernelGGL(stochastic_kernel_kernel<0>, dim3(g), dim3(256), 0, st,
                       stats_T, ld, x0, prm, S, c, B, pd_out, pdf_norm,
                       inv_temp, apply_iw, u, seed, stream, offset, accept,
                       accw, guard);
  else
    hipLaunchKernelGGL(stochastic_kernel_kernel<1>, dim3(g), dim3(256), 0, st,
                       stats_T, ld, x0, prm, S, c, B, pd_out, pdf_norm,
                       inv_temp, apply_iw, u, seed, stream, offset, accept,
                       accw, guard);
  ABC_LAUNCH_CHECK("stochastic_kernel_kernel");
  return kOk;
}

int abc_stochastic_accept_f64(const double* pd, int64_t B, double pdf_norm,
                              double inv_temp, int log_scale, int apply_iw,
                              const double* u, uint64_t seed, uint64_t stream,
                              uint64_t offset, uint8_t* accept, double* accw,
                              uint8_t* guard, hipStream_t st) {
  ABC_REQUIRE(B >= 0, "stochastic_accept: bad sizes");
  if (B == 0) return kOk;
  ABC_REQUIRE(pd && accept, "stochastic_accept: null pointer");
  hipLaunchKernelGGL(stochastic_accept_kernel, dim3(ceil_div(B, 256)),
                     dim3(256), 0, st, pd, B, pdf_norm, inv_temp, log_scale,
                     apply_iw, u, seed, stream, offset, accept, accw, guard);
  ABC_LAUNCH_CHECK("stochastic_accept_kernel");
  return kOk;
}

int abc_importance_weights_scaled_f64(const double* logpd, const double* s,
                                      double prior_const, int64_t M, double* w,
                                      hipStream_t st) {
  ABC_REQUIRE(M >= 0, "importance_weights_scaled: bad sizes");
  if (M == 0) return kOk;
  ABC_REQUIRE(w, "importance_weights_scaled: null pointer");
  hipLaunchKernelGGL(importance_scaled_kernel, dim3(ceil_div(M, 256)),
                     dim3(256), 0, st, logpd, s, prior_const, M, w);
  ABC_LAUNCH_CHECK("importance_scaled_kernel");
  return kOk;
}

size_t abc_tempered_sums_workspace_bytes(int K) {
  return static_cast<size_t>(kTsGrid) * (2 * (K > 0 ? K : 1) + 2) *
         sizeof(double);
}

int abc_tempered_sums_f64(const double* pd, const double* w,
                          const double* logw_num, const double* logw_den,
                          int64_t n, double c, int log_scale,
                          const double* betas, int K, int clamp, double* out,
                          void* ws, size_t ws_bytes, hipStream_t st) {
  ABC_REQUIRE(n >= 0 && K >= 0 && K <= kTsMaxK,
              "tempered_sums: bad sizes (0 <= K <= %d)", kTsMaxK);
  ABC_REQUIRE(pd && (betas || K == 0) && out && ws,
              "tempered_sums: null pointer");
  ABC_REQUIRE(ws_bytes >= abc_tempered_sums_workspace_bytes(K),
              "tempered_sums: workspace too small");
  const int grid = static_cast<int>(stream_grid(n, kTsBlock, kTsGrid));
  double* partial = static_cast<double*>(ws);
  hipLaunchKernelGGL(tempered_sums_kernel, dim3(grid), dim3(kTsBlock), 0, st,
                     pd, w, logw_num, logw_den, n, c, log_scale, betas, K,
                     clamp, partial);
  ABC_LAUNCH_CHECK("tempered_sums_kernel");
  hipLaunchKernelGGL(tempered_sums_finish, dim3(2 * K + 2), dim3(64), 0, st,
                     partial, grid, 2 * K + 2, out);
  ABC_LAUNCH_CHECK("tempered_sums_finish");
  return kOk;
}

}  // extern "C"

namespace abc {
// Loads this translation unit's code object (HIP loads each one lazily, at
// the first launch of one of its kernels: ~4 ms for local_mfma's inside
// C4's first weighted generation); abc_preload calls every unit's hook.
int preload_stochastic() { return preload_kernel(stochastic_kernel_kernel<0>); }
}  // namespace abc
