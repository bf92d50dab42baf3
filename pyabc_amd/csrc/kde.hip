// KDE importance-weight pass: the O(M*N*d) transition density of
// MultivariateNormalTransition.pdf (reference: pyabc/transition/
// multivariatenormal.py:102-125, called per accepted particle from
// pyabc/smc.py:722-733 and 776-792).
//
//   pd(theta_i) = sum_j w_j N(theta_i; X_j, cov)
//               = exp(c) * sum_j 2^(lw2_j - |y_i - y_j|^2)      (*)
//
// with y = (x - mu) U sqrt(log2(e)/2) (U = scipy _PSD pseudo-inverse root of
// cov, built on the host), lw2_j = log2 w_j - L, L = max_j log2 w_j and
// c = ln2 L - (rank ln 2pi + log_pdet)/2.  The previous population is packed
// once per generation as P[Npad][D+1] = (y_j, lw2_j) rows; padding rows have
// lw2 = -1e30 so they contribute exactly 0.
//
// Main kernel (VALU-bound, no MFMA: D <= 32 is too thin): each thread keeps R
// new rows y_i in VGPRs; the block's j-range streams through the SCALAR path
// (wave-uniform s_load of P rows, SGPR operands of v_sub/v_fma), so there is
// no LDS traffic and no barrier in the inner loop.  Per pair: D subs, D FMAs
// (the first seeded with lw2_j), one v_exp_f32, one add.  The fp32 kernel
// holds its rows in PAIRS (float2) so the subs and FMAs issue as
// v_pk_add_f32 / v_pk_fma_f32 with the SGPR operand broadcast to both halves:
// one wave-instruction does two pairs' work, which keeps a single wave at the
// SIMD's issue rate (measured +25 % over scalar v_sub/v_fma at d = 8, same
// bits: each lane still evaluates the identical fp32 expression).  fp32 sums are
// flushed into fp64 every CH pairs.  The j-range is cut into nseg fixed
// segments (a function of npad only); SPLIT blocks per row block each take
// nseg/SPLIT consecutive segments (split index = block % SPLIT, so with
// SPLIT % 8 == 0 every XCD streams its own j-ranges through its own L2) and
// write one fp64 partial per segment; the finalize kernel sums the nseg
// partials in fixed order.  A row's result is therefore independent of M
// and of the launch shape (deterministic, and identical across GPU counts).
// Rows whose sum falls below 2^-60 (f32) are re-evaluated by a two-pass
// (fp64 max, then fp64 sum) fixup kernel, so underflow of the fixed global
// offset never loses a row; in the fp32 and MFMA passes each term
// 2^(acc - max) is ldexp of v_exp_f32 on the fraction (~1.2e-7 relative per
// term), in the fp64 pass fp64 exp2 (1e-12).
#include <cstdlib>

#include "common.hpp"
#include "kde_internal.hpp"

namespace abc {

constexpr double kLn2 = 0.6931471805599453;
constexpr float kPadLw = -1.0e30f;

template <typename T>
struct KdeCfg;
template <>
struct KdeCfg<float> {
  static constexpr double underflow = 8.673617379884035e-19;  // 2^-60
};
template <>
struct KdeCfg<double> {
  static constexpr double underflow = 1.0e-280;
};

__device__ __forceinline__ float fast_exp2(float x) {
  return __builtin_amdgcn_exp2f(x);
}
__device__ __forceinline__ double fast_exp2(double x) { return exp2(x); }

// ---------------------------------------------------------------------------
// packing: whitening of new rows and of the previous population
// ---------------------------------------------------------------------------
template <typename T, int D>
__global__ __launch_bounds__(256) void whiten_kernel(
    const double* __restrict__ X, int64_t n, int d,
    const double* __restrict__ mu, const double* __restrict__ Us,
    T* __restrict__ Y, int ldy) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double xc[D];
#pragma unroll
  for (int l = 0; l < D; ++l) xc[l] = l < d ? X[i * d + l] - mu[l] : 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    double acc = 0.0;
#pragma unroll
    for (int l = 0; l < D; ++l)
      if (l < d && k < d) acc = fma(xc[l], Us[l * d + k], acc);
    Y[i * ldy + k] = static_cast<T>(acc);
  }
}

__global__ __launch_bounds__(256) void max_key_kernel(
    const double* __restrict__ w, int64_t n,
    unsigned long long* __restrict__ out_key) {
  uint64_t m = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    m = max(m, f64_key(w[i]));
  block_atomic_max_u64<256>(out_key, static_cast<unsigned long long>(m));
}

template <typename T, int D>
__global__ __launch_bounds__(256) void pack_prev_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t n,
    int d, const double* __restrict__ mu, const double* __restrict__ Us,
    T* __restrict__ P, int64_t npad,
    const unsigned long long* __restrict__ max_key,
    double* __restrict__ lw2max_out) {
  // The block's 256 rows of X and the whitening matrix are staged in LDS
  // (coalesced row loads instead of one 8 d-byte row per lane; the matrix
  // read from LDS instead of uniform loads), and the
  // packed rows leave through LDS as whole contiguous lines.  Each row's
  // arithmetic is unchanged (same products, same fma order).
  constexpr int kRowsB = 256;
  constexpr size_t kBuf = sizeof(double) * kRowsB * D > sizeof(T) * kRowsB * (D + 1)
                              ? sizeof(double) * kRowsB * D
                              : sizeof(T) * kRowsB * (D + 1);
  __shared__ double Ush[D * D];
  __shared__ double mus[D];
  __shared__ __attribute__((aligned(16))) unsigned char buf[kBuf];
  double* Xs = reinterpret_cast<double*>(buf);
  T* Ps = reinterpret_cast<T*>(buf);
  const int tid = threadIdx.x;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kRowsB;
  const int64_t i = r0 + tid;
  const double L = log2(key_f64(*max_key));
  if (i == 0 && lw2max_out) *lw2max_out = L;
  for (int q = tid; q < d * d; q += kRowsB) Ush[(q / d) * D + q % d] = Us[q];
  for (int q = tid; q < d; q += kRowsB) mus[q] = mu[q];
  const int nr = r0 < n ? static_cast<int>(min<int64_t>(kRowsB, n - r0)) : 0;
  for (int q = tid; q < nr * d; q += kRowsB) Xs[q] = X[r0 * d + q];
  __syncthreads();
  T row[D + 1];
  if (i < n) {
    // row of the matrix by row: each output's fma chain still runs over l
    // in ascending order (the same bits as the column-wise form)
    double acc[D];
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = 0.0;
#pragma unroll
    for (int l = 0; l < D; ++l) {
      if (l < d) {
        const double xl = Xs[tid * d + l] - mus[l];
#pragma unroll
        for (int k = 0; k < D; ++k)
          if (k < d) acc[k] = fma(xl, Ush[l * D + k], acc[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < D; ++k) row[k] = static_cast<T>(acc[k]);
    const double wi = w[i];
    double lw = wi > 0.0 ? log2(wi) - L : -1.0e300;
    if (lw < static_cast<double>(kPadLw)) lw = kPadLw;
    row[D] = static_cast<T>(lw);
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) row[k] = T(0);
    row[D] = static_cast<T>(kPadLw);
  }
  __syncthreads();  // every lane is done reading Xs
#pragma unroll
  for (int k = 0; k <= D; ++k) Ps[tid * (D + 1) + k] = row[k];
  __syncthreads();
  const int64_t nb = r0 < npad ? min<int64_t>(kRowsB, npad - r0) : 0;
  T* dst = P + r0 * (D + 1);
  for (int64_t q = tid; q < nb * (D + 1); q += kRowsB) dst[q] = Ps[q];
}

// ---------------------------------------------------------------------------
// main pass
// ---------------------------------------------------------------------------
template <typename T, int D, int R, int U, int CH>
__global__ __launch_bounds__(256) void kde_main_kernel(
    const T* __restrict__ Ynew, int64_t M, const T* __restrict__ P,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t rows_per_block = 256 * R;

  T yi[R][D];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int64_t row = rb * rows_per_block + r * 256 + threadIdx.x;
    if (row >= M) row = M - 1;
#pragma unroll
    for (int k = 0; k < D; ++k) yi[r][k] = Ynew[row * D + k];
  }
  for (int g = 0; g < spb; ++g) {
    const int seg = s * spb + g;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    int64_t j1 = j0 + jseg;
    if (j1 > npad) j1 = npad;
    double S[R];
#pragma unroll
    for (int r = 0; r < R; ++r) S[r] = 0.0;
    for (int64_t jc = j0; jc < j1; jc += CH) {
      int64_t je = jc + CH;
      if (je > j1) je = j1;
      T sacc[R];
#pragma unroll
      for (int r = 0; r < R; ++r) sacc[r] = T(0);
      for (int64_t j = jc; j < je; j += U) {
        const T* __restrict__ pj = P + j * (D + 1);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const T lw = pj[u * (D + 1) + D];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            T acc = lw;
#pragma unroll
            for (int k = 0; k < D; ++k) {
              const T df = yi[r][k] - pj[u * (D + 1) + k];
              acc = fma(-df, df, acc);
            }
            sacc[r] += fast_exp2(acc);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) S[r] += static_cast<double>(sacc[r]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t row = rb * rows_per_block + r * 256 + threadIdx.x;
      if (row < M) partial[static_cast<int64_t>(seg) * M + row] = S[r];
    }
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// fp32 main pass, rows held in pairs: lane t of block rb owns rows
// rb*256*2*R2 + (2r+h)*256 + t (h = half of the float2), the same row map as
// kde_main_kernel with R = 2*R2.  Block (rb, s) covers the spb consecutive
// j-segments s*spb .. s*spb+spb-1 and writes one fp64 partial per segment.
template <int D, int R2, int U, int CH>
__global__ __launch_bounds__(256) void kde_main_pk_kernel(
    const float* __restrict__ Ynew, int64_t M, const float* __restrict__ P,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int R = 2 * R2;
  constexpr int W = U * (D + 1);
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t rows_per_block = 256 * R;

  f32x2 yi[R2][D];
#pragma unroll
  for (int r = 0; r < R2; ++r) {
    int64_t ra = rb * rows_per_block + (2 * r) * 256 + threadIdx.x;
    int64_t rc = ra + 256;
    if (ra >= M) ra = M - 1;
    if (rc >= M) rc = M - 1;
#pragma unroll
    for (int k = 0; k < D; ++k) yi[r][k] = f32x2{Ynew[ra * D + k], Ynew[rc * D + k]};
  }
  for (int g = 0; g < spb; ++g) {
    const int seg = s * spb + g;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    // int32 trip counts keep the loop control on the scalar unit
    const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
    const float* __restrict__ base = P + j0 * (D + 1);
    double S[R];
#pragma unroll
    for (int r = 0; r < R; ++r) S[r] = 0.0;
    for (int jc = 0; jc < nj; jc += CH) {
      const int je = min(jc + CH, nj);
      f32x2 sacc[R2];
#pragma unroll
      for (int r = 0; r < R2; ++r) sacc[r] = f32x2{0.f, 0.f};
      for (int j = jc; j < je; j += U) {
        const float* __restrict__ pj = base + static_cast<int64_t>(j) * (D + 1);
        float cu[W];
#pragma unroll
        for (int q = 0; q < W; ++q) cu[q] = pj[q];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float lw = cu[u * (D + 1) + D];
#pragma unroll
          for (int r = 0; r < R2; ++r) {
            f32x2 acc = f32x2{lw, lw};
#pragma unroll
            for (int k = 0; k < D; ++k) {
              const float pk = cu[u * (D + 1) + k];
              const f32x2 df = yi[r][k] - f32x2{pk, pk};
              acc = __builtin_elementwise_fma(-df, df, acc);
            }
            sacc[r] += f32x2{fast_exp2(acc.x), fast_exp2(acc.y)};
          }
        }
      }
#pragma unroll
      for (int r = 0; r < R2; ++r) {
        S[2 * r] += static_cast<double>(sacc[r].x);
        S[2 * r + 1] += static_cast<double>(sacc[r].y);
      }
    }
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      const int64_t ra = rb * rows_per_block + (2 * r) * 256 + threadIdx.x;
      const int64_t rc = ra + 256;
      double* out = partial + static_cast<int64_t>(seg) * M;
      if (ra < M) out[ra] = S[2 * r];
      if (rc < M) out[rc] = S[2 * r + 1];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void kde_finalize_kernel(
    const double* __restrict__ partial, int64_t M, int nseg,
    const double* __restrict__ lw2max, double log_const,
    double* __restrict__ out_logpd, int* __restrict__ n_fix,
    int* __restrict__ fix_rows, double thr) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= M) return;
  double S = 0.0;
  for (int s = 0; s < nseg; ++s) S += partial[static_cast<int64_t>(s) * M + i];
  const double off = kLn2 * (*lw2max) + log_const;
  if (!(S >= thr)) {
    const int slot = atomicAdd(n_fix, 1);
    fix_rows[slot] = static_cast<int>(i);
    out_logpd[i] = -INFINITY;
  } else {
    out_logpd[i] = log(S) + off;
  }
}

// two-pass evaluation (fp64 max, then fp64 sum) for rows whose fixed-offset
// sum underflowed.  A block takes RB fixup rows at once, so each pass over
// the population serves RB rows (one row per block re-read P from L2 per
// row: 37.6 ms per launch on the exact-inference records, 3.2x the MFMA
// pass).  Grid-stride over the device-side count: 1024 blocks, so a launch
// with few or no fixup rows costs only the empty blocks' exit.  A row's
// arithmetic (thread j-stride, fixed reduction order) does not depend on RB
// or on which rows share its block.
// F32EXP: each term 2^(acc - max) as ldexp of v_exp_f32 on the fraction
// (~1.2e-7 relative per term) -- the fp32 pass and the MFMA pass, whose
// contract is 1e-5; otherwise fp64 exp2 (the fp64 pass's 1e-12 contract).
constexpr int kFixupBlocks = 1024;
template <int D>
constexpr int kFixupRows = D <= 4 ? 8 : (D <= 8 ? 4 : (D <= 16 ? 2 : 1));
template <typename T, int D, bool F32EXP>
__global__ __launch_bounds__(256) void kde_fixup_kernel(
    const T* __restrict__ Ynew, const T* __restrict__ P, int64_t npad,
    const double* __restrict__ lw2max, double log_const,
    const int* __restrict__ n_fix, const int* __restrict__ fix_rows,
    double* __restrict__ out_logpd) {
  constexpr int RB = kFixupRows<D>;
  __shared__ double red[RB][4];
  const int count = *n_fix;
  const int ngroups = (count + RB - 1) / RB;
  const double off = kLn2 * (*lw2max) + log_const;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    T yi[RB][D];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int f = g * RB + r;
      const int64_t src = fix_rows[f < count ? f : g * RB];
#pragma unroll
      for (int k = 0; k < D; ++k) yi[r][k] = Ynew[src * D + k];
    }
    double m[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) m[r] = -INFINITY;
    for (int64_t j = threadIdx.x; j < npad; j += 256) {
      const T* pj = P + j * (D + 1);
      T pv[D + 1];
#pragma unroll
      for (int k = 0; k <= D; ++k) pv[k] = pj[k];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        T acc = pv[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const T df = yi[r][k] - pv[k];
          acc = fma(-df, df, acc);
        }
        m[r] = fmax(m[r], static_cast<double>(acc));
      }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const double v = wave_max(m[r]);
      if (lane == 0) red[r][wid] = v;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RB; ++r)
      m[r] = fmax(fmax(red[r][0], red[r][1]), fmax(red[r][2], red[r][3]));
    __syncthreads();
    double sum[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) sum[r] = 0.0;
    for (int64_t j = threadIdx.x; j < npad; j += 256) {
      const T* pj = P + j * (D + 1);
      T pv[D + 1];
#pragma unroll
      for (int k = 0; k <= D; ++k) pv[k] = pj[k];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        T acc = pv[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const T df = yi[r][k] - pv[k];
          acc = fma(-df, df, acc);
        }
        const double x = static_cast<double>(acc) - m[r];
        if constexpr (F32EXP) {
          // 2^x for x = acc - m <= 0 (exact in fp64): the integer part by
          // ldexp, the fraction in [0, 1) on v_exp_f32 (~1.2e-7 relative
          // per term; fp64 exp2 issued 3x the instructions)
          const double fl = floor(fmax(x, -2000.0));
          const float fr = static_cast<float>(x - fl);
          sum[r] += ldexp(static_cast<double>(__builtin_amdgcn_exp2f(fr)),
                          static_cast<int>(fl));
        } else {
          sum[r] += exp2(x);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const double v = wave_sum(sum[r]);
      if (lane == 0) red[r][wid] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int f = g * RB + r;
        if (f < count) {
          const double S = ((red[r][0] + red[r][1]) + red[r][2]) + red[r][3];
          out_logpd[fix_rows[f]] =
              (m[r] > -1.0e29) ? kLn2 * (m[r] + log2(S)) + off : -INFINITY;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int padded_dim(int d) {
  static const int dims[] = {1, 2, 3, 4, 6, 8, 12, 16, 20, 24, 32};
  for (int v : dims)
    if (d <= v) return v;
  return -1;
}

constexpr int kRowPad = 64;  // Npad multiple (>= U, == CH)
constexpr int kCH = 64;

// rows per thread; fp32: R = 2*R2 rows in float2 pairs, R2 and the j-unroll
// U picked per D from the tools/probes/kde_variants.hip sweep on MI355X.
// Small launches drop to fewer rows per thread (tier 1, 2) to fill the chip;
// the tier only changes how rows map to lanes, never a row's arithmetic.
template <typename T, int D>
struct RowsPerThread;
template <int D>
struct RowsPerThread<double, D> {
  static constexpr int value = D <= 8 ? 4 : 2;
};
template <int D>
struct RowsPerThread<float, D> {
  static constexpr int pairs = D <= 8 ? 4 : 2;
  static constexpr int unroll = D <= 8 ? 1 : 2;
  static constexpr int value = 2 * pairs;
};

// The j-range [0, npad) is cut into nseg fixed segments that depend on npad
// ONLY (a power of two, <= 64, segments of >= ~1024 rows, multiples of CH).
// Every row's density is the fixed-order fp64 sum of its nseg segment sums,
// each a sequential fp64 sum of 64-pair fp32 chunk sums -- so a row's bits
// do not depend on M, on the launch shape, or on how many ranks share the
// rows (multi-GPU results equal single-GPU results bit for bit).
static int kde_segments(int64_t npad) {
  const int64_t q = npad / 1024;
  int n = 1;
  while (n < 64 && 2 * n <= q) n *= 2;
  return n;
}

struct Plan {
  int split;    // blocks per row block (power of two, divides nseg)
  int nseg;     // j-segments (power of two)
  int spb;      // segments per block = nseg / split
  int jseg;     // rows per segment (multiple of kCH)
  int tier;     // 0: full rows per thread, 1: half, 2: quarter
  int rows_per_thread;
  int64_t row_blocks;
};

template <typename T, int D>
static Plan make_plan(int64_t M, int64_t npad) {
  constexpr int R = RowsPerThread<T, D>::value;
  constexpr int64_t target_blocks = 8192;  // ~4 waves of 2048 resident blocks
  Plan p;
  p.nseg = kde_segments(npad);
  p.jseg = static_cast<int>(ceil_div(ceil_div(npad, p.nseg), kCH) * kCH);
  constexpr int min_rows = sizeof(T) == 4 ? 2 : 1;  // fp32: one float2 pair
  p.tier = 0;
  while (p.tier < 2 && (R >> (p.tier + 1)) >= min_rows &&
         ceil_div(M, 256 * (R >> p.tier)) * p.nseg < target_blocks)
    ++p.tier;
  // tuning override (tools/bench_kde.py sweeps): ABC_KDE_TIER=0|1|2
  {
    const int t = tuning_knob(kKnobKdeTier, -1);
    if (t >= 0 && t <= 2 && (R >> t) >= min_rows) p.tier = t;
  }
  p.rows_per_thread = R >> p.tier;
  p.row_blocks = ceil_div(M, 256 * p.rows_per_thread);
  int split = 1;
  while (split < p.nseg && p.row_blocks * split < target_blocks) split *= 2;
  p.split = split;
  p.spb = p.nseg / split;
  return p;
}

template <typename T>
static size_t ws_bytes_impl(int64_t M, int64_t npad, int d) {
  // partial[nseg*M] doubles + n_fix (16 B) + fix_rows[M] ints
  if (padded_dim(d) < 0) return 0;
  const int64_t nseg = kde_segments(npad);
  return static_cast<size_t>(nseg * M) * 8 + 16 + static_cast<size_t>(M) * 4 + 256;
}

template <int D, int R2>
static void launch_pk(const Plan& p, unsigned grid, const float* Ynew,
                      int64_t M, const float* P, int64_t npad, double* partial,
                      hipStream_t stream) {
  constexpr int U = RowsPerThread<float, D>::unroll;
  hipLaunchKernelGGL((kde_main_pk_kernel<D, R2, U, kCH>), dim3(grid), dim3(256),
                     0, stream, Ynew, M, P, npad, p.split, p.spb, p.jseg,
                     partial);
}

template <typename T, int D, int R>
static void launch_generic(const Plan& p, unsigned grid, const T* Ynew,
                           int64_t M, const T* P, int64_t npad,
                           double* partial, hipStream_t stream) {
  hipLaunchKernelGGL((kde_main_kernel<T, D, R, 2, kCH>), dim3(grid), dim3(256),
                     0, stream, Ynew, M, P, npad, p.split, p.spb, p.jseg,
                     partial);
}

template <typename T, int D>
static int logpdf_impl(const T* Ynew, int64_t M, const T* P, int64_t npad,
                       const double* lw2max, double log_const,
                       double* out_logpd, void* ws, size_t ws_bytes,
                       hipStream_t stream) {
  const Plan p = make_plan<T, D>(M, npad);
  const size_t need = static_cast<size_t>(p.nseg * M) * 8 + 16 +
                      static_cast<size_t>(M) * 4;
  ABC_REQUIRE(ws_bytes >= need, "kde: workspace too small (%zu < %zu)",
              ws_bytes, need);
  char* base = static_cast<char*>(ws);
  double* partial = reinterpret_cast<double*>(base);
  int* n_fix = reinterpret_cast<int*>(base + static_cast<size_t>(p.nseg * M) * 8);
  int* fix_rows = n_fix + 4;
  ABC_HIP(hipMemsetAsync(n_fix, 0, 16, stream));
  const unsigned grid = static_cast<unsigned>(p.row_blocks * p.split);
  if constexpr (sizeof(T) == 4) {
    constexpr int R2 = RowsPerThread<float, D>::pairs;
    if (p.tier == 0)
      launch_pk<D, R2>(p, grid, Ynew, M, P, npad, partial, stream);
    else if (p.tier == 1 || R2 < 4)
      launch_pk<D, (R2 > 1 ? R2 / 2 : 1)>(p, grid, Ynew, M, P, npad, partial,
                                          stream);
    else
      launch_pk<D, 1>(p, grid, Ynew, M, P, npad, partial, stream);
    ABC_LAUNCH_CHECK("kde_main_pk_kernel");
  } else {
    constexpr int R = RowsPerThread<T, D>::value;
    if (p.tier == 0)
      launch_generic<T, D, R>(p, grid, Ynew, M, P, npad, partial, stream);
    else if (p.tier == 1 || R < 4)
      launch_generic<T, D, (R > 1 ? R / 2 : 1)>(p, grid, Ynew, M, P, npad,
                                                partial, stream);
    else
      launch_generic<T, D, 1>(p, grid, Ynew, M, P, npad, partial, stream);
    ABC_LAUNCH_CHECK("kde_main_kernel");
  }
  hipLaunchKernelGGL((kde_finalize_kernel<T>), dim3(ceil_div(M, 256)),
                     dim3(256), 0, stream, partial, M, p.nseg, lw2max,
                     log_const, out_logpd, n_fix, fix_rows,
                     KdeCfg<T>::underflow);
  ABC_LAUNCH_CHECK("kde_finalize_kernel");
  hipLaunchKernelGGL((kde_fixup_kernel<T, D, sizeof(T) == 4>), dim3(kFixupBlocks),
                     dim3(256), 0, stream,
                     Ynew, P, npad, lw2max, log_const, n_fix, fix_rows,
                     out_logpd);
  ABC_LAUNCH_CHECK("kde_fixup_kernel");
  return kOk;
}

template <typename T>
static int logpdf_dispatch(const T* Ynew, int64_t M, const T* P, int64_t npad,
                           int d, const double* lw2max, double log_const,
                           double* out, void* ws, size_t wsb,
                           hipStream_t st) {
  ABC_REQUIRE(M >= 0 && npad >= 0, "kde: negative size");
  ABC_REQUIRE(npad % kRowPad == 0, "kde: npad must be a multiple of %d", kRowPad);
  if (M == 0) return kOk;
  ABC_REQUIRE(npad > 0, "kde: empty previous population");
  ABC_REQUIRE(Ynew && P && lw2max && out && ws, "kde: null pointer");
  switch (padded_dim(d)) {
#define CASE(DD) \
  case DD:       \
    return logpdf_impl<T, DD>(Ynew, M, P, npad, lw2max, log_const, out, ws, wsb, st);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default:
      set_error("kde: unsupported dimension d=%d (max 32)", d);
      return kUnsupported;
  }
}

template <typename T>
static int whiten_dispatch(const double* X, int64_t n, int d, const double* mu,
                           const double* Us, T* Y, hipStream_t st) {
  ABC_REQUIRE(n >= 0, "whiten: negative n");
  if (n == 0) return kOk;
  const int D = padded_dim(d);
  const unsigned g = static_cast<unsigned>(ceil_div(n, 256));
  switch (D) {
#define CASE(DD)                                                             \
  case DD:                                                                   \
    hipLaunchKernelGGL((whiten_kernel<T, DD>), dim3(g), dim3(256), 0, st, X, \
                       n, d, mu, Us, Y, DD);                                 \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default:
      set_error("whiten: unsupported dimension d=%d", d);
      return kUnsupported;
  }
  ABC_LAUNCH_CHECK("whiten_kernel");
  return kOk;
}

template <typename T>
static int pack_dispatch(const double* X, const double* w, int64_t n, int d,
                         const double* mu, const double* Us, T* P,
                         int64_t npad, double* lw2max, void* ws,
                         hipStream_t st) {
  ABC_REQUIRE(n > 0 && npad >= n && npad % kRowPad == 0,
              "pack_prev: need 0 < n <= npad, npad %% %d == 0", kRowPad);
  ABC_REQUIRE(ws != nullptr, "pack_prev: null workspace");
  unsigned long long* key = static_cast<unsigned long long*>(ws);
  ABC_HIP(hipMemsetAsync(key, 0, 8, st));
  hipLaunchKernelGGL(max_key_kernel, dim3(stream_grid(n, 256, 1024)),
                     dim3(256), 0, st, w, n, key);
  ABC_LAUNCH_CHECK("max_key_kernel");
  const unsigned g = static_cast<unsigned>(ceil_div(npad, 256));
  switch (padded_dim(d)) {
#define CASE(DD)                                                            \
  case DD:                                                                  \
    hipLaunchKernelGGL((pack_prev_kernel<T, DD>), dim3(g), dim3(256), 0, st, \
                       X, w, n, d, mu, Us, P, npad, key, lw2max);           \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default:
      set_error("pack_prev: unsupported dimension d=%d", d);
      return kUnsupported;
  }
  ABC_LAUNCH_CHECK("pack_prev_kernel");
  return kOk;
}

// ---------------------------------------------------------------------------
// abc_kde_logsum (SURVEY 8(b) minimum set): the same pass on rows the caller
// has already whitened with scipy's U, and log-weights:
//   out_i = log_offset + log sum_j exp(logw_j - |y_i - y_j|^2 / 2)
// The rows are rescaled by sqrt(log2(e)/2) and the log-weights moved to
// log2 units relative to their maximum, then the packed-population pass of
// logpdf_impl runs unchanged (finalize adds ln2 * max + log_offset).
// ---------------------------------------------------------------------------
constexpr double kSqrtHalfLog2e = 0.84932180028801907;  // sqrt(log2(e) / 2)
constexpr double kLog2e = 1.4426950408889634;

template <typename T>
__global__ __launch_bounds__(256) void logw_max_kernel(
    const T* __restrict__ logw, int64_t n, unsigned long long* __restrict__ key) {
  uint64_t m = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const double v = static_cast<double>(logw[i]);
    if (v == v) m = max(m, f64_key(v));  // NaN ignored
  }
  block_atomic_max_u64<256>(key, static_cast<unsigned long long>(m));
}

template <typename T, int D>
__global__ __launch_bounds__(256) void logsum_pack_kernel(
    const T* __restrict__ Yp, const T* __restrict__ logw, int64_t n, int d,
    T* __restrict__ P, int64_t npad, const unsigned long long* __restrict__ key,
    double* __restrict__ lw2max_out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const double L = key_f64(*key) * kLog2e;
  if (i == 0) *lw2max_out = L;
  if (i >= npad) return;
  T* row = P + i * (D + 1);
  if (i >= n) {
#pragma unroll
    for (int k = 0; k < D; ++k) row[k] = T(0);
    row[D] = static_cast<T>(kPadLw);
    return;
  }
#pragma unroll
  for (int k = 0; k < D; ++k)
    row[k] = k < d ? static_cast<T>(static_cast<double>(Yp[i * d + k]) *
                                    kSqrtHalfLog2e)
                   : T(0);
  double lw = static_cast<double>(logw[i]) * kLog2e - L;
  if (!(lw >= static_cast<double>(kPadLw))) lw = kPadLw;  // -inf / NaN
  row[D] = static_cast<T>(lw);
}

template <typename T, int D>
__global__ __launch_bounds__(256) void logsum_rows_kernel(
    const T* __restrict__ Yn, int64_t M, int d, T* __restrict__ Y) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= M) return;
#pragma unroll
  for (int k = 0; k < D; ++k)
    Y[i * D + k] = k < d ? static_cast<T>(static_cast<double>(Yn[i * d + k]) *
                                          kSqrtHalfLog2e)
                         : T(0);
}

template <typename T>
__global__ __launch_bounds__(256) void store_out_kernel(const double* __restrict__ src,
                                                        int64_t M,
                                                        T* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < M) out[i] = static_cast<T>(src[i]);
}

template <typename T>
size_t logsum_ws_bytes(int64_t M, int64_t N, int d) {
  const int D = padded_dim(d);
  if (D < 0 || M < 0 || N < 0) return 0;
  const int64_t npad = ceil_div(N > 0 ? N : 1, kRowPad) * kRowPad;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  return 256 + al(static_cast<size_t>(npad) * (D + 1) * sizeof(T)) +
         al(static_cast<size_t>(M) * D * sizeof(T)) +
         al(static_cast<size_t>(M) * 8) + ws_bytes_impl<T>(M, npad, d);
}

template <typename T>
int logsum_impl(const T* Ynew, const T* Yprev, const T* logw, int64_t M,
                int64_t N, int d, T log_offset, T* out, void* ws,
                size_t ws_bytes, hipStream_t st) {
  ABC_REQUIRE(M >= 0 && N > 0, "kde_logsum: need M >= 0, N > 0");
  const int D = padded_dim(d);
  if (D < 0) {
    set_error("kde_logsum: unsupported dimension d=%d (max 32)", d);
    return kUnsupported;
  }
  if (M == 0) return kOk;
  ABC_REQUIRE(Ynew && Yprev && logw && out && ws, "kde_logsum: null pointer");
  ABC_REQUIRE(ws_bytes >= logsum_ws_bytes<T>(M, N, d),
              "kde_logsum: workspace too small");
  const int64_t npad = ceil_div(N, kRowPad) * kRowPad;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  char* base = static_cast<char*>(ws);
  unsigned long long* key = reinterpret_cast<unsigned long long*>(base);
  double* lw2max = reinterpret_cast<double*>(base + 64);
  char* q = base + 256;
  T* P = reinterpret_cast<T*>(q);
  q += al(static_cast<size_t>(npad) * (D + 1) * sizeof(T));
  T* Y = reinterpret_cast<T*>(q);
  q += al(static_cast<size_t>(M) * D * sizeof(T));
  double* tmp = reinterpret_cast<double*>(q);
  q += al(static_cast<size_t>(M) * 8);
  const size_t rest = ws_bytes - static_cast<size_t>(q - base);
  ABC_HIP(hipMemsetAsync(key, 0, 8, st));
  hipLaunchKernelGGL((logw_max_kernel<T>), dim3(stream_grid(N, 256, 1024)),
                     dim3(256), 0, st, logw, N, key);
  switch (D) {
#define CASE(DD)                                                               \
  case DD:                                                                     \
    hipLaunchKernelGGL((logsum_pack_kernel<T, DD>), dim3(ceil_div(npad, 256)), \
                       dim3(256), 0, st, Yprev, logw, N, d, P, npad, key,      \
                       lw2max);                                                \
    hipLaunchKernelGGL((logsum_rows_kernel<T, DD>), dim3(ceil_div(M, 256)),    \
                       dim3(256), 0, st, Ynew, M, d, Y);                       \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
  }
  ABC_LAUNCH_CHECK("kde_logsum pack kernels");
  const int rc = logpdf_dispatch<T>(Y, M, P, npad, d, lw2max,
                                    static_cast<double>(log_offset), tmp, q,
                                    rest, st);
  if (rc != kOk) return rc;
  hipLaunchKernelGGL((store_out_kernel<T>), dim3(ceil_div(M, 256)), dim3(256),
                     0, st, tmp, M, out);
  ABC_LAUNCH_CHECK("kde_logsum store");
  return kOk;
}

// shared with kde_mfma.hip (kde_internal.hpp): the two-pass fixup of the
// rows the MFMA pass could not resolve on the matrix cores (outside the grid
// range, offsets beyond the piece range), in fp64 on the fp64 whitened rows.
// An fp32 copy of a far row (|y| ~ 30 in log2 units) carries ~2e-6 absolute
// error per coordinate, i.e. up to 5e-5 relative on the density through
// |y_i - y_j|^2, so these rows are evaluated from the fp64 rows
// (tests/test_gpu_fullsize.py, constructed rows beyond the population); each
// term's 2^x is v_exp_f32 on the fraction (~1.2e-7 relative, inside the
// pass's 1e-5 contract; the fp64 pass keeps fp64 exp2).
int kde_fixup_rows_mfma(const double* Ynew, const double* P, int64_t npad,
                        int d, const double* lw2max, double log_const,
                        const int* n_fix, const int* fix_rows,
                        double* out_logpd, hipStream_t stream) {
  switch (padded_dim(d)) {
#define CASE(DD)                                                              \
  case DD:                                                                    \
    hipLaunchKernelGGL((kde_fixup_kernel<double, DD, true>), dim3(kFixupBlocks), \
                       dim3(256), 0, stream, Ynew, P, npad, lw2max, log_const, \
                       n_fix, fix_rows, out_logpd);                           \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default:
      set_error("kde: unsupported dimension d=%d (max 32)", d);
      return kUnsupported;
  }
  ABC_LAUNCH_CHECK("kde_fixup_kernel");
  return kOk;
}

int kde_padded_dim(int d) { return padded_dim(d); }
int kde_num_segments(int64_t npad) { return kde_segments(npad); }
int kde_pack_direct_f64(const double* X, const double* w, int64_t n, int d,
                        const double* mu, const double* Us, double* P,
                        int64_t npad, double* lw2max, void* ws,
                        hipStream_t st) {
  return pack_dispatch<double>(X, w, n, d, mu, Us, P, npad, lw2max, ws, st);
}

}  // namespace abc

using namespace abc;

extern "C" {

int abc_kde_padded_dim(int d) { return padded_dim(d); }
int abc_kde_row_pad(void) { return kRowPad; }

size_t abc_kde_workspace_bytes(int64_t M, int64_t npad, int d) {
  // one size for every pass (their plans may split differently; the MFMA
  // pass adds its refine lists and fragments)
  const size_t a = ws_bytes_impl<float>(M, npad, d);
  const size_t b = ws_bytes_impl<double>(M, npad, d);
  const size_t c = kde_mfma_ws_bytes(M, npad, d);
  return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

int abc_kde_segments(int64_t npad) { return kde_segments(npad); }

int abc_kde_split(int64_t M, int64_t npad, int d) {
  switch (padded_dim(d)) {
#define CASE(DD) \
  case DD: return make_plan<float, DD>(M, npad).split;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default: return -1;
  }
}

size_t abc_kde_logsum_workspace_bytes_f32(int64_t M, int64_t N, int d) {
  return logsum_ws_bytes<float>(M, N, d);
}
size_t abc_kde_logsum_workspace_bytes_f64(int64_t M, int64_t N, int d) {
  return logsum_ws_bytes<double>(M, N, d);
}
int abc_kde_logsum_f32(const float* Ynew, const float* Yprev, const float* logw,
                       int64_t M, int64_t N, int d, float log_offset,
                       float* out_log_sum, void* ws, size_t ws_bytes,
                       hipStream_t st) {
  return logsum_impl<float>(Ynew, Yprev, logw, M, N, d, log_offset,
                            out_log_sum, ws, ws_bytes, st);
}
int abc_kde_logsum_f64(const double* Ynew, const double* Yprev,
                       const double* logw, int64_t M, int64_t N, int d,
                       double log_offset, double* out_log_sum, void* ws,
                       size_t ws_bytes, hipStream_t st) {
  return logsum_impl<double>(Ynew, Yprev, logw, M, N, d, log_offset,
                             out_log_sum, ws, ws_bytes, st);
}

int abc_whiten_f32(const double* X, int64_t n, int d, const double* mu,
                   const double* Us, float* Y, hipStream_t st) {
  return whiten_dispatch<float>(X, n, d, mu, Us, Y, st);
}
int abc_whiten_f64(const double* X, int64_t n, int d, const double* mu,
                   const double* Us, double* Y, hipStream_t st) {
  return whiten_dispatch<double>(X, n, d, mu, Us, Y, st);
}

int abc_kde_pack_prev_f32(const double* X, const double* w, int64_t n, int d,
                          const double* mu, const double* Us, float* P,
                          int64_t npad, double* lw2max, void* ws,
                          hipStream_t st) {
  return pack_dispatch<float>(X, w, n, d, mu, Us, P, npad, lw2max, ws, st);
}
int abc_kde_pack_prev_f64(const double* X, const double* w, int64_t n, int d,
                          const double* mu, const double* Us, double* P,
                          int64_t npad, double* lw2max, void* ws,
                          hipStream_t st) {
  return pack_dispatch<double>(X, w, n, d, mu, Us, P, npad, lw2max, ws, st);
}

int abc_kde_logpdf_f32(const float* Ynew, int64_t M, const float* P,
                       int64_t npad, int d, const double* lw2max,
                       double log_const, double* out_logpd, void* ws,
                       size_t ws_bytes, hipStream_t st) {
  return logpdf_dispatch<float>(Ynew, M, P, npad, d, lw2max, log_const,
                                out_logpd, ws, ws_bytes, st);
}
int abc_kde_logpdf_f64(const double* Ynew, int64_t M, const double* P,
                       int64_t npad, int d, const double* lw2max,
                       double log_const, double* out_logpd, void* ws,
                       size_t ws_bytes, hipStream_t st) {
  return logpdf_dispatch<double>(Ynew, M, P, npad, d, lw2max, log_const,
                                 out_logpd, ws, ws_bytes, st);
}

}  // extern "C"

namespace abc {
// Loads this translation unit's code object (HIP loads each one lazily, at
// the first launch of one of its kernels: ~4 ms for local_mfma's inside
// C4's first weighted generation); abc_preload calls every unit's hook.
int preload_kde() { return preload_kernel(whiten_kernel<double, 8>); }
}  // namespace abc
