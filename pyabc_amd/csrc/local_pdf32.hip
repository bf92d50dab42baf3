// LocalTransition density, fp32 pair loop (reference:
// pyabc/transition/local_transition.py:103-110):
//   pdf(theta) = sum_n w_n N(theta; X_n, C_n) / sum w
// One thread per evaluation point, the previous population's particles in
// pairs streaming through the scalar path (packed fp32), exact (hi, lo)
// centred differences and the symmetric quadratic form; see DESIGN.md
// section 4 "LocalTransition density pass" for what bounds it and the two
// alternatives measured against it (tile pruning, the feature-form GEMM on
// the f32 matrix cores).
#include "common.hpp"
#include "local_common.hpp"

namespace abc {
namespace {

// fp32 pass (precision="f32", 1e-5 relative): the same sum with the
// population centred on X[0] in fp64, the packed coefficients pre-scaled by
// log2(e)/2 and lc by log2(e), so a term is one v_exp_f32 of (lc2_n - q'_n);
// 16 terms are added in fp32, then into fp64.  Centred coordinates are kept
// as an fp32 (hi, lo) pair, x - X[0] = hi + lo, and the pair difference is
// (th_hi - X_hi) + (th_lo - X_lo): its error is ~2^-24 of the difference
// itself, not of the distance R to X[0], so the density's accuracy does not
// degrade with the population's extent over the local bandwidth (a single
// fp32 rounding of x - X[0] costs ~ sqrt(q) (R / sigma) 2^-23 relative).
// Layout: particles in PAIRS (n, n + 1) interleaved per coordinate, so one
// 64-bit scalar load feeds a packed-fp32 operand (v_pk_*_f32) that serves
// two particles at once: X2[(n / 2) * D + q] = (x_n, x_{n+1}), the same for
// the lo parts, coef2[(n / 2) * NC + t] and lc2[n / 2].  The count is padded
// to even with a particle of lc = -inf (exp2 -> 0).
template <int D>
__global__ __launch_bounds__(256) void local_pack32_kernel(
    const double* __restrict__ X, const double* __restrict__ coef,
    const double* __restrict__ lc, const unsigned long long* __restrict__ lc_max_key,
    int64_t N, float* __restrict__ X32, float* __restrict__ X32lo,
    float* __restrict__ coef32, float* __restrict__ lc32) {
  constexpr int NC = D * (D + 1) / 2;
  const int64_t n = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (n >= ((N + 1) & ~int64_t{1})) return;
  const int64_t pr = n >> 1;
  const int h = static_cast<int>(n & 1);
  if (n >= N) {  // padding particle of an odd count
#pragma unroll
    for (int q = 0; q < D; ++q) {
      X32[(pr * D + q) * 2 + h] = 0.0f;
      X32lo[(pr * D + q) * 2 + h] = 0.0f;
    }
#pragma unroll
    for (int t = 0; t < NC; ++t) coef32[(pr * NC + t) * 2 + h] = 0.0f;
    lc32[n] = -INFINITY;
    return;
  }
  const double L = key_f64(*lc_max_key);
  constexpr double kLog2e = 1.4426950408889634;
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const double c = X[n * D + q] - X[q];
    const float hi = static_cast<float>(c);
    X32[(pr * D + q) * 2 + h] = hi;
    X32lo[(pr * D + q) * 2 + h] = static_cast<float>(c - static_cast<double>(hi));
  }
#pragma unroll
  for (int t = 0; t < NC; ++t)
    coef32[(pr * NC + t) * 2 + h] = static_cast<float>(coef[n * NC + t] * (0.5 * kLog2e));
  lc32[n] = static_cast<float>((lc[n] - L) * kLog2e);
}

// Two particles per packed-fp32 lane pair: the (hi, lo) differences, the
// quadratic form's FMAs and the exponent arguments of particles n and n + 1
// run as v_pk_add / v_pk_fma / v_pk_mul on SGPR-pair operands, about half
// the VALU instructions of the one-particle loop; two v_exp_f32 per pair.
// Terms of 8 pairs are added in fp32 (even and odd particles apart), then
// into fp64.  nchunk is even, so no pair straddles two chunks.
template <int D>
__global__ __launch_bounds__(256) void local_pdf32_kernel(
    const float* __restrict__ pts, const float* __restrict__ ptslo, int64_t M,
    const f32x2* __restrict__ X2, const f32x2* __restrict__ X2lo,
    const f32x2* __restrict__ coef2, const f32x2* __restrict__ lc2, int64_t N,
    int split, int64_t nchunk, double* __restrict__ part) {
  constexpr int NC = D * (D + 1) / 2;
  const int s = blockIdx.x % split;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x / split) * 256 + threadIdx.x;
  const int64_t i = i0 < M ? i0 : M - 1;
  f32x2 th[D], tl[D];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const float a = pts[i * D + q], b = ptslo[i * D + q];
    th[q] = f32x2{a, a};
    tl[q] = f32x2{b, b};
  }
  double acc = 0.0;
  const int64_t n0 = static_cast<int64_t>(s) * nchunk;  // even
  int64_t n1 = n0 + nchunk;
  const int64_t npair = (N + 1) & ~int64_t{1};
  if (n1 > npair) n1 = npair;
  for (int64_t b = n0; b < n1; b += 16) {
    const int64_t be = b + 16 < n1 ? b + 16 : n1;
    f32x2 a2 = f32x2{0.0f, 0.0f};
    for (int64_t n = b; n < be; n += 2) {
      const int64_t pr = n >> 1;
      f32x2 dl[D];
#pragma unroll
      for (int q = 0; q < D; ++q)
        dl[q] = (th[q] - X2[pr * D + q]) + (tl[q] - X2lo[pr * D + q]);
      const f32x2* c = coef2 + pr * NC;
      f32x2 qf = f32x2{0.0f, 0.0f};
      int t = 0;
#pragma unroll
      for (int a = 0; a < D; ++a) {
        f32x2 r = c[t++] * dl[a];
#pragma unroll
        for (int bb = a + 1; bb < D; ++bb)
          r = __builtin_elementwise_fma(c[t++], dl[bb], r);
        qf = __builtin_elementwise_fma(dl[a], r, qf);
      }
      const f32x2 e = lc2[pr] - qf;
      a2 += f32x2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
    }
    acc += static_cast<double>(a2.x + a2.y);
  }
  if (i0 < M) part[static_cast<int64_t>(s) * M + i0] = acc;
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" {

size_t abc_local_logpdf_workspace_bytes(int64_t M, int64_t N);

size_t abc_local_logpdf_f32_workspace_bytes(int64_t M, int64_t N) {
  // the fp64 layout, then X32[N][8] | X32lo[N][8] | coef32[N][36] | lc32[N]
  // | pts32[M][8] | pts32lo[M][8]
  // (N padded to even: particle pairs)
  return abc_local_logpdf_workspace_bytes(M, N) +
         static_cast<size_t>(N + 1) * 4 * 53 + static_cast<size_t>(M) * 4 * 16 + 512;
}

int abc_local_logpdf_f32(const double* pts, int64_t M, const double* X,
                         const double* w, const double* inv_covs,
                         const double* dets, int64_t N, int d,
                         double* out_logpdf, void* ws, size_t ws_bytes,
                         hipStream_t st) {
  ABC_REQUIRE(M >= 0 && N >= 1, "local_logpdf_f32: bad sizes");
  if (M == 0) return kOk;
  ABC_REQUIRE(d >= 1 && d <= 8, "local_logpdf_f32: unsupported d=%d (d <= 8)", d);
  ABC_REQUIRE(pts && X && w && inv_covs && dets && out_logpdf && ws,
              "local_logpdf_f32: null pointer");
  ABC_REQUIRE(ws_bytes >= abc_local_logpdf_f32_workspace_bytes(M, N),
              "local_logpdf_f32: workspace too small");
  int split;
  int64_t nchunk;
  local_plan(M, N, split, nchunk);
  nchunk += nchunk & 1;  // even: particle pairs never straddle two chunks
  const int64_t Np = N + (N & 1);
  char* base = static_cast<char*>(ws);
  double* logsumw = reinterpret_cast<double*>(base);
  unsigned long long* lc_max_key = reinterpret_cast<unsigned long long*>(base + 8);
  int* n_fix = reinterpret_cast<int*>(base + 16);
  double* lc = reinterpret_cast<double*>(base + 64);
  double* coef = lc + N;
  double* part = coef + N * 36;
  int* fix_rows = reinterpret_cast<int*>(part + static_cast<int64_t>(split) * M);
  float* X32 = reinterpret_cast<float*>(
      base + ((abc_local_logpdf_workspace_bytes(M, N) + 255) / 256) * 256);
  float* X32lo = X32 + Np * 8;
  float* coef32 = X32lo + Np * 8;
  float* lc32 = coef32 + Np * 36;
  float* pts32 = lc32 + Np;
  float* pts32lo = pts32 + M * 8;
  ABC_HIP(hipMemsetAsync(base + 8, 0, 16, st));
  local_sumw(w, N, split, part, logsumw, st);
  hipLaunchKernelGGL(local_const_kernel, dim3(ceil_div(N, 256)), dim3(256), 0,
                     st, w, dets, inv_covs, N, d, lc, coef, lc_max_key);
  const unsigned grid = static_cast<unsigned>(ceil_div(M, 256) * split);
  // rows whose fp32 sum is below 2^-60 take the exact fp64 fixup: the terms
  // lost to fp32 underflow (< 2^-126 each) are then < 2^-40 of the sum
  const double thresh = 8.673617379884035e-19;
#define L(DD)                                                                    \
  hipLaunchKernelGGL((local_pack32_kernel<DD>), dim3(ceil_div(Np, 256)), dim3(256), \
                     0, st, X, coef, lc, lc_max_key, N, X32, X32lo, coef32,    \
                     lc32);                                                      \
  hipLaunchKernelGGL((local_pts32_kernel<DD>), dim3(ceil_div(M, 256)), dim3(256),  \
                     0, st, pts, M, X, pts32, pts32lo);                          \
  hipLaunchKernelGGL((local_pdf32_kernel<DD>), dim3(grid), dim3(256), 0, st,       \
                     pts32, pts32lo, M, reinterpret_cast<const f32x2*>(X32),     \
                     reinterpret_cast<const f32x2*>(X32lo),                      \
                     reinterpret_cast<const f32x2*>(coef32),                     \
                     reinterpret_cast<const f32x2*>(lc32), N, split, nchunk,     \
                     part);                                                      \
  hipLaunchKernelGGL(local_pdf_final_kernel, dim3(ceil_div(M, 256)), dim3(256),  \
                     0, st, part, M, split, lc_max_key, logsumw, out_logpdf,     \
                     n_fix, fix_rows, thresh);                                   \
  hipLaunchKernelGGL((local_pdf_fixup_kernel<DD>), dim3(1024), dim3(256), 0, st, \
                     pts, X, coef, lc, N, logsumw, n_fix, fix_rows, out_logpdf);
  switch (d) {
    case 1: L(1) break;
    case 2: L(2) break;
    case 3: L(3) break;
    case 4: L(4) break;
    case 5: L(5) break;
    case 6: L(6) break;
    case 7: L(7) break;
    case 8: L(8) break;
  }
#undef L
  ABC_LAUNCH_CHECK("local_logpdf_f32 kernels");
  return kOk;
}

}  // extern "C"

namespace abc {
// Loads this translation unit's code object (HIP loads each one lazily, at
// the first launch of one of its kernels: ~4 ms for local_mfma's inside
// C4's first weighted generation); abc_preload calls every unit's hook.
int preload_local_pdf32() { return preload_kernel(local_sumw_part_kernel); }
}  // namespace abc
