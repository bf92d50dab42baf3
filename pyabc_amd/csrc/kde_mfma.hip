// KDE importance-weight pass on the matrix cores: exact-grid bf16 MFMA.
// Same quantity as kde.hip (MultivariateNormalTransition.pdf, reference
// pyabc/transition/multivariatenormal.py:102-125 via smc.py:722-733):
//
//   pd(theta_i) = exp(c) * sum_j 2^(e_ij),  e_ij = lw2_j - |y_i - y_j|^2
//
// expanded as e_ij = a_j + b_i + 2 y_i.y_j with a_j = lw2_j - |y_j|^2 and
// b_i = -|y_i|^2.  The expansion cancels catastrophically in fp32 (a plain
// fp32 GEMM form loses 4e-5 relative at N = 1e6, d = 8), so every operand is
// split into bf16 pieces that make the large part of the sum EXACT:
//
//   y = y1 + y2 + y3   y1 = g*rint(y/g) on a fixed power-of-two grid g with
//                      |y1/g| <= 256 (8 significant bits: exact in bf16),
//                      y2 = bf16(y - y1), y3 = bf16(y - y1 - y2)
//   a = aH0 + aH1 + aH2 + aL0 + aL1   (aH* bf16 multiples of G = g^2 holding
//                      rint(a/G)*G exactly, aL* = bf16 pieces of the rest)
//
// hi = sum_k 2 y1_ik y1_jk + aH + bH is a sum of multiples of G below
// 2^24 G, so the fp32 MFMA accumulation is exact in ANY order; lo (the
// seven y1/y2/y3 cross products per dimension + aL + bL) is small (|lo| <~
// 4) and accumulates with ~1e-7 absolute error.  e = hi + lo is rounded
// once, so the exponent carries one fp32 rounding at |e| -- tighter than
// the direct fp32 difference form of kde.hip (max 9e-6 vs 3e-5 relative on
// rows far outside the population, SURVEY 8(a3) tolerance 1e-5).
//
// MFMA mapping (v_mfma_f32_32x32x16_bf16): A = previous population (rows =
// j), B = new rows (columns = i), K = the piece slots.  KH chunks of 16
// slots feed the hi accumulator, KL chunks the lo accumulator; each lane
// owns one new row (column lane&31) and 16 j's of the 32-row tile, so per
// pair the VALU does only  v_add (hi+lo), v_exp_f32, v_add (row sum).
// The j-range uses kde.hip's fixed segments, each lane's values are summed in
// register order and the two lane halves combined in a fixed order, so a
// row's bits are independent of M, of the launch shape and of the number of
// ranks.  Rows whose sum underflows -- and new rows outside the grid range
// (|y| > 256 g, flagged by b = -inf) -- go through kde.hip's exact fixup,
// in fp64 on the fp64 whitened rows (Ynew [M][D], P [npad][D+1]).
#include <cmath>

#include "common.hpp"
#include "kde_internal.hpp"

namespace abc {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr double kLwFloor = -160.0;  // 2^-160 is 0 in fp32: no term changes
constexpr int kWaves = 4;            // waves per block

template <int D>
struct Mk {
  static constexpr int KH = (D + 6 + 15) / 16;      // y1.y1, aH x3, bH x3
  static constexpr int KL = (7 * D + 4 + 15) / 16;  // 7 cross terms, aL, bL
  static constexpr int KT = KH + KL;
  static constexpr int IB = D <= 8 ? 3 : (D <= 24 ? 2 : 1);  // i-tiles/wave
  // row padding unit in i-tiles per wave: every IB the launch may pick
  // (1, 2, 3 at D <= 8) divides it
  static constexpr int PADIB = D <= 8 ? 6 : IB;
};

__device__ inline unsigned short bf16_rne(float x) {
  unsigned u = __float_as_uint(x);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return static_cast<unsigned short>(u >> 16);
}
__device__ inline unsigned short bf16_trunc(float x) {
  return static_cast<unsigned short>(__float_as_uint(x) >> 16);
}
__device__ inline float bf16_f(unsigned short b) {
  return __uint_as_float(static_cast<unsigned>(b) << 16);
}
constexpr unsigned short kBf16One = 0x3F80;
constexpr unsigned short kBf16NegInf = 0xFF80;

// y -> (y1, y2, y3) bf16 bits, scaled by `side` (1 for the population, 2 for
// new rows: exact); returns |y1 + y2 + y3|^2 (the represented point)
template <int D>
__device__ inline double split_row(const double* y, double g, float side,
                                   unsigned short* y1, unsigned short* y2,
                                   unsigned short* y3) {
  double n2 = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const double v1 = rint(y[k] / g) * g;
    const double r = y[k] - v1;
    const unsigned short b2 = bf16_rne(static_cast<float>(r));
    const double v2 = bf16_f(b2);
    const unsigned short b3 = bf16_rne(static_cast<float>(r - v2));
    const double v3 = bf16_f(b3);
    y1[k] = bf16_rne(side * static_cast<float>(v1));
    y2[k] = bf16_rne(side * static_cast<float>(v2));
    y3[k] = bf16_rne(side * static_cast<float>(v3));
    const double yt = v1 + v2 + v3;
    n2 = fma(yt, yt, n2);
  }
  return n2;
}

// v -> three bf16 multiples of G summing to rint(v/G)*G exactly, plus two
// bf16 pieces of the remainder (|rem| <= G/2)
__device__ inline void split_value(double v, double G, unsigned short* h,
                                   unsigned short* l) {
  double q = rint(v / G);
  q = fmin(fmax(q, -8388607.0), 8388607.0);  // |q| < 2^23 (bounds in DESIGN)
  const float qf = static_cast<float>(q);     // exact integer
  const unsigned short h0 = bf16_trunc(qf);
  const float r1 = qf - bf16_f(h0);
  const unsigned short h1 = bf16_trunc(r1);
  const float r2 = r1 - bf16_f(h1);
  const unsigned short h2 = bf16_trunc(r2);  // r2 - h2 == 0
  const float Gf = static_cast<float>(G);
  h[0] = bf16_rne(bf16_f(h0) * Gf);
  h[1] = bf16_rne(bf16_f(h1) * Gf);
  h[2] = bf16_rne(bf16_f(h2) * Gf);
  const double lo = v - q * G;  // exact (Sterbenz / q == 0)
  const unsigned short l0 = bf16_rne(static_cast<float>(lo));
  l[0] = l0;
  l[1] = bf16_rne(static_cast<float>(lo - static_cast<double>(bf16_f(l0))));
}

// Slot k of the population (A) and new-row (B) operands.
//  hi  k < D: y1 | 2y1        k = D..D+2: aH | 1     k = D+3..D+5: 1 | bH
//  lo  k' = 7m + q (m < D):   q: 0 y2|2y1  1 y3|2y1  2 y1|2y2  3 y1|2y3
//                                4 y2|2y2  5 y3|2y2  6 y2|2y3
//      k' = 7D, 7D+1: aL | 1  k' = 7D+2, 7D+3: 1 | bL
template <int D, bool kA>
__device__ inline unsigned short slot(int k, const unsigned short* y1,
                                      const unsigned short* y2,
                                      const unsigned short* y3,
                                      const unsigned short* h,
                                      const unsigned short* l) {
  constexpr int KH = Mk<D>::KH;
  if (k < 16 * KH) {
    if (k < D) return y1[k];
    if (k < D + 3) return kA ? h[k - D] : kBf16One;
    if (k < D + 6) return kA ? kBf16One : h[k - D - 3];
    return 0;
  }
  const int kk = k - 16 * KH;
  if (kk < 7 * D) {
    const int m = kk / 7, q = kk % 7;
    if (kA) {
      switch (q) {
        case 0: case 4: case 6: return y2[m];
        case 1: case 5: return y3[m];
        default: return y1[m];
      }
    } else {
      switch (q) {
        case 0: case 1: return y1[m];
        case 2: case 4: case 5: return y2[m];
        default: return y3[m];
      }
    }
  }
  if (kk < 7 * D + 2) return kA ? l[kk - 7 * D] : kBf16One;
  if (kk < 7 * D + 4) return kA ? kBf16One : l[kk - 7 * D - 2];
  return 0;
}

// fragment layout [tile][chunk c][lane][8]: lane = 32h + (particle % 32),
// element e = slot 16c + 8h + e
template <int D, bool kA>
__device__ inline void store_frags(bf16x8* __restrict__ F, int64_t p,
                                   const unsigned short* y1,
                                   const unsigned short* y2,
                                   const unsigned short* y3,
                                   const unsigned short* h,
                                   const unsigned short* l) {
  constexpr int KT = Mk<D>::KT;
  const int64_t tile = p >> 5;
  const int r = static_cast<int>(p & 31);
#pragma unroll
  for (int c = 0; c < KT; ++c) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[e] = static_cast<short>(slot<D, kA>(16 * c + 8 * hh + e, y1, y2, y3, h, l));
      F[(tile * KT + c) * 64 + 32 * hh + r] = v;
    }
  }
}

template <int D>
__device__ inline void whiten_row(const double* __restrict__ X, int64_t i,
                                  int d, const double* __restrict__ mu,
                                  const double* __restrict__ Us, double* y) {
  double xc[D];
#pragma unroll
  for (int l = 0; l < D; ++l) xc[l] = l < d ? X[i * d + l] - mu[l] : 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    double acc = 0.0;
#pragma unroll
    for (int l = 0; l < D; ++l)
      if (l < d && k < d) acc = fma(xc[l], Us[l * d + k], acc);
    y[k] = acc;
  }
}

template <int D>
__global__ __launch_bounds__(256) void ymax_kernel(
    const double* __restrict__ X, int64_t n, int d,
    const double* __restrict__ mu, const double* __restrict__ Us,
    unsigned long long* __restrict__ key) {
  double m = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    double y[D];
    whiten_row<D>(X, i, d, mu, Us, y);
#pragma unroll
    for (int k = 0; k < D; ++k) m = fmax(m, fabs(y[k]));
  }
  block_atomic_max_u64<256>(key, static_cast<unsigned long long>(f64_key(m)));
}

__device__ inline double grid_from_key(const unsigned long long* key) {
  const double m = key_f64(*key);
  int E = 0;
  if (m > 0.0) frexp(m, &E);  // m < 2^E
  return fmax(ldexp(1.0, E - 7), 0.015625);  // 256 g = 2^(E+1) >= 2 max|y|
}

template <int D>
__global__ __launch_bounds__(256) void pack_prev_frag_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t n,
    int d, const double* __restrict__ mu, const double* __restrict__ Us,
    int64_t npad, const double* __restrict__ lw2max,
    const unsigned long long* __restrict__ ykey, double* __restrict__ gscale,
    bf16x8* __restrict__ A) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const double g = grid_from_key(ykey);
  if (j == 0) *gscale = g;
  if (j >= npad) return;
  double y[D];
  double lw = kLwFloor;
  if (j < n) {
    whiten_row<D>(X, j, d, mu, Us, y);
    const double wj = w[j];
    if (wj > 0.0) lw = fmax(log2(wj) - *lw2max, kLwFloor);
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) y[k] = 0.0;
  }
  unsigned short y1[D], y2[D], y3[D], h[3], l[2];
  const double n2 = split_row<D>(y, g, 1.0f, y1, y2, y3);
  split_value(lw - n2, g * g, h, l);
  store_frags<D, true>(A, j, y1, y2, y3, h, l);
}

template <int D>
__global__ __launch_bounds__(256) void pack_new_frag_kernel(
    const double* __restrict__ theta, int64_t M, int64_t mpad, int d,
    const double* __restrict__ mu, const double* __restrict__ Us,
    const double* __restrict__ gscale, double* __restrict__ Ydir,
    bf16x8* __restrict__ B) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= mpad) return;
  const double g = *gscale;
  double y[D];
  bool ok = i < M;
  if (ok) {
    whiten_row<D>(theta, i, d, mu, Us, y);
#pragma unroll
    for (int k = 0; k < D; ++k) {
      Ydir[i * D + k] = y[k];
      ok = ok && fabs(y[k]) <= 256.0 * g;  // NaN -> not ok
    }
  }
  unsigned short y1[D], y2[D], y3[D], h[3], l[2];
  if (ok) {
    const double n2 = split_row<D>(y, g, 2.0f, y1, y2, y3);
    split_value(-n2, g * g, h, l);
  } else {  // padding / out-of-grid row: e = -inf, exact fixup if i < M
#pragma unroll
    for (int k = 0; k < D; ++k) y1[k] = y2[k] = y3[k] = 0;
    h[0] = kBf16NegInf;
    h[1] = h[2] = l[0] = l[1] = 0;
  }
  store_frags<D, false>(B, i, y1, y2, y3, h, l);
}

// Folded accumulation (KL <= kFoldKL, i.e. D <= 8, the VALU-bound shapes):
// the exact hi products first, then the lo chain accumulated ON TOP of them
// in the same accumulator, so the MFMA delivers e = hi + lo itself and the
// VALU add per pair disappears (143.6 vs 156.6 ms at N = M = 1e6, d = 8).
// hi is exact in any order (multiples of G below 2^24 G); each of the KL lo
// MFMAs then rounds at |e| instead of once, so a term's exponent carries
// about (KL + 1) / 2 ulps of |e| instead of 1/2: relative error ~8e-8 |e|
// at KL = 4.  A row's error is the t-weighted mean of its terms' errors,
// bounded by ~8e-8 log2(N / S) for a row sum S; rows with S < 2^-32 (dominant
// exponents beyond ~32) take the exact fp64 fixup (kMfmaFixupSum), so the
// bound is ~4e-6 at N = 1e6 (measured: tests/test_gpu_fullsize.py, DESIGN
// section 4).  The opt-in LDS / DMA variants keep the split order.
constexpr int kFoldKL = 4;

// one (32-row tile, i-tile) product: hi (exact) and lo accumulators, or the
// folded e in hi
template <int KH, int KL>
__device__ __forceinline__ void mfma_step(const bf16x8* a, const bf16x8* b,
                                          f32x16& hi, f32x16& lo) {
  hi = f32x16{};
#pragma unroll
  for (int c = 0; c < KH; ++c)
    hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[c], b[c], hi, 0, 0, 0);
  if constexpr (KL <= kFoldKL) {
#pragma unroll
    for (int c = 0; c < KL; ++c)
      hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[KH + c], b[KH + c], hi, 0,
                                                   0, 0);
  } else {
    lo = f32x16{};
#pragma unroll
    for (int c = 0; c < KL; ++c)
      lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[KH + c], b[KH + c], lo, 0,
                                                   0, 0);
  }
}

// sum of 2^(hi+lo) over the lane's 16 values: 16 independent exps, then a
// fixed pairwise tree (v, v+8), (v, v+4), (v, v+2), (v, v+1)
__device__ __forceinline__ float tile_sum_split(const f32x16& hi,
                                                const f32x16& lo) {
  float e[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) e[v] = __builtin_amdgcn_exp2f(hi[v] + lo[v]);
#pragma unroll
  for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
    for (int v = 0; v < w; ++v) e[v] += e[v + w];
  return e[0];
}

// the same after mfma_step (folded: e is in hi)
template <int KL>
__device__ __forceinline__ float tile_sum(const f32x16& hi, const f32x16& lo) {
  if constexpr (KL > kFoldKL) {
    return tile_sum_split(hi, lo);
  } else {
    float e[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) e[v] = __builtin_amdgcn_exp2f(hi[v]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int v = 0; v < w; ++v) e[v] += e[v + w];
    return e[0];
  }
}

// VALU instructions of one step's sum (16 exps + the tree + the row add,
// plus the 16 hi + lo adds when not folded): the sched_group_barrier share
template <int KL>
constexpr int step_valu() { return KL <= kFoldKL ? 32 : 48; }

// Ablation forms of one step (tuning diagnostics only, ABC_KDE_MFMA_ABL):
// 1 no exp, 2 no MFMA, 3 neither (adds only), 4 MFMA only.  The results are
// meaningless; they time the pipes separately.
template <int ABL, int KH, int KL>
__device__ __forceinline__ void abl_step(const bf16x8* a, const bf16x8* b,
                                         f32x16& hi, f32x16& lo) {
  if constexpr (ABL == 5) {
    // fold: the lo chain first, then the exact hi products on top of it as
    // the MFMA's C operand (accuracy probe; saves the VALU hi + lo add)
    lo = f32x16{};
#pragma unroll
    for (int c = 0; c < KL; ++c)
      lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[KH + c], b[KH + c], lo, 0, 0, 0);
    hi = lo;
#pragma unroll
    for (int c = 0; c < KH; ++c)
      hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[c], b[c], hi, 0, 0, 0);
  } else if constexpr (ABL == 6) {
    // fold the other way: the exact hi products first, then the lo chain
    // accumulated on top of them (rounding at |e|, not at the hi partials)
    hi = f32x16{};
#pragma unroll
    for (int c = 0; c < KH; ++c)
      hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[c], b[c], hi, 0, 0, 0);
#pragma unroll
    for (int c = 0; c < KL; ++c)
      hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[KH + c], b[KH + c], hi, 0, 0, 0);
  } else if constexpr (ABL == 2 || ABL == 3) {
    asm volatile("" : "+v"(hi), "+v"(lo));
  } else {
    mfma_step<KH, KL>(a, b, hi, lo);
  }
}
// (the ablated sum is consumed by an empty asm and replaced by 1, so no row
// reaches the exact fixup)
template <int ABL, int KL>
__device__ __forceinline__ float abl_sum(const f32x16& hi, const f32x16& lo) {
  if constexpr (ABL == 0) return tile_sum<KL>(hi, lo);
  if constexpr (ABL == 5 || ABL == 6) {
    float e[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) e[v] = __builtin_amdgcn_exp2f(hi[v]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int v = 0; v < w; ++v) e[v] += e[v + w];
    return e[0];
  }
  float r;
  if constexpr (ABL == 2) {
    r = tile_sum_split(hi, lo);
  } else if constexpr (ABL == 4) {
    r = hi[0] + lo[0];
  } else {
    float e[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) e[v] = hi[v] + lo[v];
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int v = 0; v < w; ++v) e[v] += e[v + w];
    r = e[0];
  }
  asm volatile("" ::"v"(r));
  return 1.0f;
}

// main pass.  Block (rb, s): wave w owns i-tiles (rb*kWaves + w)*IB + t and
// walks the spb consecutive j-segments s*spb ..; per segment one fp64 partial
// per row.  64-row chunks (two 32-row tiles) are summed in fp32, then added
// into fp64.
template <int KH, int KL, int IB, bool PIPE, bool SCHED, int ABL = 0>
__device__ __forceinline__ void kde_mfma_body(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t t0 = (rb * kWaves + wave) * IB;

  bf16x8 bq[IB][KT];
#pragma unroll
  for (int t = 0; t < IB; ++t)
#pragma unroll
    for (int c = 0; c < KT; ++c) bq[t][c] = Bfr[((t0 + t) * KT + c) * 64 + lane];

  for (int gi = 0; gi < spb; ++gi) {
    const int seg = s * spb + gi;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
    const bf16x8* __restrict__ Aseg = Afr + (j0 >> 5) * KT * 64 + lane;
    double S[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) S[t] = 0.0;
    // a[0] / a[1]: the two 32-row tiles of the current 64-row chunk.  Each
    // tile's fragments are requested one half-chunk before their first MFMA
    // (tile 1 while tile 0 computes, the next chunk's tile 0 while tile 1
    // computes), so the L2 latency runs under the VALU work.
    bf16x8 a[2][KT];
    if (nj > 0) {
#pragma unroll
      for (int c = 0; c < KT; ++c) a[0][c] = Aseg[c * 64];
    }
    for (int jc = 0; jc < nj; jc += 64) {
      const bf16x8* __restrict__ ap = Aseg + (jc >> 5) * KT * 64;
      // next chunk's first tile (re-read of this one on the last chunk)
      const bf16x8* __restrict__ an =
          Aseg + (((jc + 64 < nj) ? jc + 64 : jc) >> 5) * KT * 64;
      float sacc[IB];
#pragma unroll
      for (int t = 0; t < IB; ++t) sacc[t] = 0.0f;
      if constexpr (PIPE) {
        // 2*IB (tile, i-tile) steps; the MFMAs of step q+1 issue before the
        // VALU of step q, on a second accumulator pair
#pragma unroll
        for (int c = 0; c < KT; ++c) a[1][c] = ap[(KT + c) * 64];
        f32x16 hi[2], lo[2];
        abl_step<ABL, KH, KL>(a[0], bq[0], hi[0], lo[0]);
#pragma unroll
        for (int q = 0; q < 2 * IB; ++q) {
          if (q + 1 < 2 * IB)
            abl_step<ABL, KH, KL>(a[(q + 1) / IB], bq[(q + 1) % IB],
                              hi[(q + 1) & 1], lo[(q + 1) & 1]);
          if (q + 1 == IB) {  // last MFMA reading tile 0 is issued
#pragma unroll
            for (int c = 0; c < KT; ++c) a[0][c] = an[c * 64];
          }
          sacc[q % IB] += abl_sum<ABL, KL>(hi[q & 1], lo[q & 1]);
          if constexpr (SCHED) {
            // interleave: each MFMA of step q+1 followed by a share of step
            // q's VALU (16 exp, 16 tree/row adds, 16 hi + lo adds unless folded)
            constexpr int VPG = (step_valu<KL>() + KT - 1) / KT;
            if (q + 1 < 2 * IB) {
#pragma unroll
              for (int m = 0; m < KT; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, VPG, 0);
              }
            } else {
              __builtin_amdgcn_sched_group_barrier(0x002, step_valu<KL>(), 0);
            }
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < KT; ++c) a[1][c] = ap[(KT + c) * 64];
#pragma unroll
        for (int q = 0; q < 2 * IB; ++q) {
          f32x16 hi, lo;
          abl_step<ABL, KH, KL>(a[q / IB], bq[q % IB], hi, lo);
          sacc[q % IB] += abl_sum<ABL, KL>(hi, lo);
          if (q + 1 == IB) {
#pragma unroll
            for (int c = 0; c < KT; ++c) a[0][c] = an[c * 64];
          }
        }
      }
#pragma unroll
      for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sacc[t]);
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double tot = S[t] + __shfl_xor(S[t], 32, 64);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * M + i] = tot;
    }
  }
}

template <int KH, int KL, int IB, bool PIPE, bool SCHED = false>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  kde_mfma_body<KH, KL, IB, PIPE, SCHED>(Bfr, M, Afr, npad, split, spb, jseg,
                                         partial);
}

template <int KH, int KL, int ABL>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_abl_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  kde_mfma_body<KH, KL, 3, true, true, ABL>(Bfr, M, Afr, npad, split, spb,
                                            jseg, partial);
}

// The same pass software-pipelined ACROSS 64-row chunks: the MFMAs of step
// q+1 -- for the last step of a chunk, step 0 of the next chunk -- are
// issued interleaved with the VALU of step q (sched_group_barrier: one MFMA,
// then a share of the 48 VALU instructions), so no step's exp/add block
// runs without matrix work beside it.  A row's arithmetic and summation
// order are those of kde_mfma_kernel: the rows are bit-identical.
template <int KH, int KL, int IB>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_sw_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int NS = 2 * IB;                  // steps per 64-row chunk
  constexpr int VPG = (step_valu<KL>() + KT - 1) / KT;  // VALU per gap
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t t0 = (rb * kWaves + wave) * IB;

  bf16x8 bq[IB][KT];
#pragma unroll
  for (int t = 0; t < IB; ++t)
#pragma unroll
    for (int c = 0; c < KT; ++c) bq[t][c] = Bfr[((t0 + t) * KT + c) * 64 + lane];

  for (int gi = 0; gi < spb; ++gi) {
    const int seg = s * spb + gi;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
    const bf16x8* __restrict__ Aseg = Afr + (j0 >> 5) * KT * 64 + lane;
    double S[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) S[t] = 0.0;
    if (nj > 0) {
      bf16x8 a[2][KT];
      f32x16 hi[2], lo[2];
#pragma unroll
      for (int c = 0; c < KT; ++c) a[0][c] = Aseg[c * 64];
#pragma unroll
      for (int c = 0; c < KT; ++c) a[1][c] = Aseg[(KT + c) * 64];
      mfma_step<KH, KL>(a[0], bq[0], hi[0], lo[0]);
      for (int jc = 0; jc < nj; jc += 64) {
        const bool more = jc + 64 < nj;
        // next chunk's tiles (a re-read of this chunk's on the last one)
        const bf16x8* __restrict__ an =
            Aseg + ((more ? jc + 64 : jc) >> 5) * KT * 64;
        float sacc[IB];
#pragma unroll
        for (int t = 0; t < IB; ++t) sacc[t] = 0.0f;
#pragma unroll
        for (int q = 0; q < NS; ++q) {
          if (q + 1 < NS)
            mfma_step<KH, KL>(a[(q + 1) / IB], bq[(q + 1) % IB],
                              hi[(q + 1) & 1], lo[(q + 1) & 1]);
          else if (more)  // step 0 of the next chunk (tile 0 loaded below)
            mfma_step<KH, KL>(a[0], bq[0], hi[0], lo[0]);
          if (q + 1 == IB) {  // last MFMA reading tile 0 issued
#pragma unroll
            for (int c = 0; c < KT; ++c) a[0][c] = an[c * 64];
          }
          if (q + 2 == NS) {  // last MFMA reading tile 1 issued
#pragma unroll
            for (int c = 0; c < KT; ++c) a[1][c] = an[(KT + c) * 64];
          }
          sacc[q % IB] += tile_sum<KL>(hi[q & 1], lo[q & 1]);
          if (q + 1 < NS || more) {
#pragma unroll
            for (int m = 0; m < KT; ++m) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, VPG, 0);
            }
          }
        }
#pragma unroll
        for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sacc[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double tot = S[t] + __shfl_xor(S[t], 32, 64);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * M + i] = tot;
    }
  }
}

// L1-relief form: the A fragments of each 64-row chunk are copied ONCE per
// block into LDS by LDS-DMA (global_load_lds_dwordx4: no staging registers,
// double-buffered, one barrier per chunk) and every wave of the block reads
// them from LDS (128 B/clk/CU) instead of each wave pulling its own 10 KiB
// per chunk through the vector L1 (64 B/clk/CU: the MFMA path alone ran
// 114 ms at N = M = 1e6, d = 8, L1-bound, tools/kde_variants.py ablations).
// NW waves per block share one copy; each keeps IB i-tiles of B in
// registers.  Per-lane arithmetic and summation order are those of
// kde_mfma_body: rows are bit-identical.
template <int KH, int KL, int IB, int NW, bool SCHED, int ABL = 0>
__global__ __launch_bounds__(64 * NW) void kde_mfma_dmab_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int CH = 2 * KT;  // 1-KiB fragments per 64-row chunk
  __shared__ bf16x8 As[2][CH][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t t0 = (rb * NW + wave) * IB;

  bf16x8 bq[IB][KT];
#pragma unroll
  for (int t = 0; t < IB; ++t)
#pragma unroll
    for (int c = 0; c < KT; ++c) bq[t][c] = Bfr[((t0 + t) * KT + c) * 64 + lane];

  for (int gi = 0; gi < spb; ++gi) {
    const int seg = s * spb + gi;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
    const bf16x8* __restrict__ Aseg = Afr + (j0 >> 5) * KT * 64;
    double S[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) S[t] = 0.0;
    // fragment f of a chunk = contiguous 1 KiB at Aseg + (chunk*2*KT + f)*64
    auto fill = [&](int buf, int jc) {
      const bf16x8* __restrict__ src = Aseg + (jc >> 5) * KT * 64;
      for (int f = wave; f < CH; f += NW)
        __builtin_amdgcn_global_load_lds(
            src + f * 64 + lane,
            (__attribute__((address_space(3))) void*)&As[buf][f][0], 16, 0, 0);
    };
    __syncthreads();  // the previous segment's readers are done with As
    if (nj > 0) fill(0, 0);
    int buf = 0;
    for (int jc = 0; jc < nj; jc += 64) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // chunk jc landed (each wave waited for its own pieces) and every wave
      // is done with chunk jc - 64, whose buffer is refilled now
      __syncthreads();
      if (jc + 64 < nj) fill(buf ^ 1, jc + 64);
      const bf16x8(*Ab)[64] = As[buf];
      float sacc[IB];
#pragma unroll
      for (int t = 0; t < IB; ++t) sacc[t] = 0.0f;
      bf16x8 a[2][KT];
#pragma unroll
      for (int c = 0; c < KT; ++c) a[0][c] = Ab[c][lane];
#pragma unroll
      for (int c = 0; c < KT; ++c) a[1][c] = Ab[KT + c][lane];
      f32x16 hi[2], lo[2];
      abl_step<ABL, KH, KL>(a[0], bq[0], hi[0], lo[0]);
#pragma unroll
      for (int q = 0; q < 2 * IB; ++q) {
        if (q + 1 < 2 * IB)
          abl_step<ABL, KH, KL>(a[(q + 1) / IB], bq[(q + 1) % IB],
                            hi[(q + 1) & 1], lo[(q + 1) & 1]);
        sacc[q % IB] += abl_sum<ABL, KL>(hi[q & 1], lo[q & 1]);
        if constexpr (SCHED) {
          constexpr int VPG = (step_valu<KL>() + KT - 1) / KT;
          if (q + 1 < 2 * IB) {
#pragma unroll
            for (int m = 0; m < KT; ++m) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, VPG, 0);
            }
          } else {
            __builtin_amdgcn_sched_group_barrier(0x002, step_valu<KL>(), 0);
          }
        }
      }
#pragma unroll
      for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sacc[t]);
      buf ^= 1;
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double tot = S[t] + __shfl_xor(S[t], 32, 64);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * M + i] = tot;
    }
  }
}

// Occupancy form for large d (MFMA-bound): one i-tile per wave, the A
// fragments of each 64-row chunk copied once per block into LDS by LDS-DMA
// (global_load_lds_dwordx4, no staging registers; double-buffered, one
// barrier per chunk) and read back one fragment ahead of its MFMA (sched
// groups DS_READ 1 / MFMA 1), so a wave holds only its B fragments, one
// accumulator pair and the exp block: three waves per SIMD at d = 20
// instead of one, and the MFMA chain of one wave runs beside the VALU of
// another.  Per-lane arithmetic and order are those of kde_mfma_kernel at
// IB = 1: rows are bit-identical.
template <int KH, int KL>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_dma_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int CH = 2 * KT;  // 1-KiB fragments per 64-row chunk
  __shared__ bf16x8 As[2][CH][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t t0 = rb * kWaves + wave;

  bf16x8 bq[KT];
#pragma unroll
  for (int c = 0; c < KT; ++c) bq[c] = Bfr[(t0 * KT + c) * 64 + lane];

  for (int gi = 0; gi < spb; ++gi) {
    const int seg = s * spb + gi;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
    const bf16x8* __restrict__ Aseg = Afr + (j0 >> 5) * KT * 64;
    double S = 0.0;
    // fragment f of a chunk = (tile f / KT, slot chunk f % KT): contiguous
    // 1 KiB at Aseg + (chunk * 2 * KT + f) * 64; wave w copies f = w, w+4..
    auto fill = [&](int buf, int jc) {
      const bf16x8* __restrict__ src = Aseg + (jc >> 5) * KT * 64;
      for (int f = wave; f < CH; f += kWaves)
        __builtin_amdgcn_global_load_lds(
            src + f * 64 + lane,
            (__attribute__((address_space(3))) void*)&As[buf][f][0], 16, 0, 0);
    };
    __syncthreads();  // the previous segment's readers are done with As
    if (nj > 0) fill(0, 0);
    int buf = 0;
    for (int jc = 0; jc < nj; jc += 64) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // chunk jc landed (every wave waited for its own pieces) and every
      // wave finished chunk jc - 64, whose buffer is refilled next
      __syncthreads();
      if (jc + 64 < nj) fill(buf ^ 1, jc + 64);
      float sacc = 0.0f;
#pragma unroll
      for (int tile = 0; tile < 2; ++tile) {
        f32x16 hi = f32x16{}, lo = f32x16{};
#pragma unroll
        for (int c = 0; c < KH; ++c) {
          hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(As[buf][tile * KT + c][lane],
                                                       bq[c], hi, 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
#pragma unroll
        for (int c = 0; c < KL; ++c) {
          lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              As[buf][tile * KT + KH + c][lane], bq[KH + c], lo, 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        sacc += tile_sum_split(hi, lo);
      }
      S += static_cast<double>(sacc);
      buf ^= 1;  // the next top barrier also ends every read of this buffer
    }
    const double tot = S + __shfl_xor(S, 32, 64);
    const int64_t i = t0 * 32 + lane;
    if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * M + i] = tot;
  }
}

// MFMA-bound form for d > 8.  Per 32x32 tile a wave runs KT = KH + KL
// MFMAs; with A streamed per wave from L2 (kde_mfma_kernel) every MFMA needs
// 1 KiB of A per 32 cycles, i.e. 128 B/clk/CU at IB = 1 and 64 at IB = 2 --
// the vector L1's whole bandwidth, so the matrix pipe ran at ~50 % (21 ms at
// N = M = 262144, d = 20).  Here the A fragments of each 64-row chunk are
// copied ONCE per block into LDS by LDS-DMA (double-buffered, one barrier
// per chunk), and each fragment read back from LDS (ds_read_b128) feeds IB
// MFMAs, one per i-tile held in registers: LDS serves 128/IB B/clk/CU, L2
// only 1/(kWaves*IB) of the A bytes.  A wave holds B (IB*KT fragments), the
// 2*IB accumulators and one A fragment in flight, so two waves share a SIMD
// and one wave's exp block runs beside another's MFMA chain.  Per-lane
// arithmetic and summation order are those of kde_mfma_body (split hi / lo
// accumulators, tile 0 then tile 1 of each chunk): the rows are
// bit-identical to kde_mfma_kernel's.
template <int KH, int KL, int IB, bool FOLD>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_lds2_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int CH = 2 * KT;  // 1-KiB fragments per 64-row chunk
  __shared__ bf16x8 As[2][CH][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t t0 = (rb * kWaves + wave) * IB;

  bf16x8 bq[IB][KT];
#pragma unroll
  for (int t = 0; t < IB; ++t)
#pragma unroll
    for (int c = 0; c < KT; ++c) bq[t][c] = Bfr[((t0 + t) * KT + c) * 64 + lane];

  for (int gi = 0; gi < spb; ++gi) {
    const int seg = s * spb + gi;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
    const bf16x8* __restrict__ Aseg = Afr + (j0 >> 5) * KT * 64;
    double S[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) S[t] = 0.0;
    // fragment f of a chunk = contiguous 1 KiB at Aseg + (chunk*2*KT + f)*64
    auto fill = [&](int buf, int jc) {
      const bf16x8* __restrict__ src = Aseg + (jc >> 5) * KT * 64;
      for (int f = wave; f < CH; f += kWaves)
        __builtin_amdgcn_global_load_lds(
            src + f * 64 + lane,
            (__attribute__((address_space(3))) void*)&As[buf][f][0], 16, 0, 0);
    };
    __syncthreads();  // the previous segment's readers are done with As
    if (nj > 0) fill(0, 0);
    int buf = 0;
    for (int jc = 0; jc < nj; jc += 64) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // chunk jc landed (each wave waited for its own pieces) and every wave
      // is done with chunk jc - 64, whose buffer is refilled now
      __syncthreads();
      if (jc + 64 < nj) fill(buf ^ 1, jc + 64);
      const bf16x8(*Ab)[64] = As[buf];
      float sacc[IB];
#pragma unroll
      for (int t = 0; t < IB; ++t) sacc[t] = 0.0f;
#pragma unroll
      for (int tile = 0; tile < 2; ++tile) {
        f32x16 hi[IB], lo[IB];
#pragma unroll
        for (int t = 0; t < IB; ++t) hi[t] = lo[t] = f32x16{};
#pragma unroll
        for (int c = 0; c < KT; ++c) {
          const bf16x8 a = Ab[tile * KT + c][lane];
#pragma unroll
          for (int t = 0; t < IB; ++t) {
            if (c < KH || FOLD)
              hi[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bq[t][c], hi[t],
                                                              0, 0, 0);
            else
              lo[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bq[t][c], lo[t],
                                                              0, 0, 0);
          }
          // one fragment read ahead of its IB MFMAs, no early hoisting
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, IB, 0);
        }
#pragma unroll
        for (int t = 0; t < IB; ++t)
          sacc[t] += FOLD ? tile_sum<0>(hi[t], lo[t]) : tile_sum_split(hi[t], lo[t]);
      }
#pragma unroll
      for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sacc[t]);
      buf ^= 1;  // the next top barrier also ends every read of this buffer
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double tot = S[t] + __shfl_xor(S[t], 32, 64);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * M + i] = tot;
    }
  }
}

// ---- hand-interleaved folded LDS-DMA pass (d > 8, opt-in ABC_KDE_MFMA_LDS2=2)
// The VALU of one 32-row tile (per i-tile: 16 v_exp_f32, the 15-add tree and
// the row add) is cut into slices placed in the gaps of the NEXT tile's MFMA
// chain, one slice after each MFMA, with sched_barrier fences so the compiler
// keeps exactly that order: an MFMA holds vector issue for 8 of its 32
// cycles, and a slice of two exps and one add (20 issue cycles) runs in the
// other 24 (MI355X_MICROARCH.md, MFMA gap fillers).  Per i-tile the 32 ops
// are  e0 e8  e1 e9 a0  e2 e10 a1 ... e7 e15 a6  a7  b0..b3  c0 c1  d0  s
// (a: v + 8, b: v + 4, c: v + 2, d: v + 1, s: the row add) -- the tree of
// tile_sum, so the rows are bit-identical to the FOLD lds2 kernel's.
struct TileSumState {
  float e[16];
};
template <int O>
__device__ __forceinline__ void tile_sum_op(const f32x16& acc, TileSumState& st,
                                            float& sacc) {
  if constexpr (O < 2) {
    st.e[8 * O] = __builtin_amdgcn_exp2f(acc[8 * O]);
  } else if constexpr (O < 23) {
    // the exps of pair v one slice ahead of the add of pair v - 1, so no
    // add waits on the transcendental it follows
    constexpr int v = 1 + (O - 2) / 3, k = (O - 2) % 3;
    if constexpr (k == 0) st.e[v] = __builtin_amdgcn_exp2f(acc[v]);
    else if constexpr (k == 1) st.e[v + 8] = __builtin_amdgcn_exp2f(acc[v + 8]);
    else st.e[v - 1] += st.e[v - 1 + 8];
  } else if constexpr (O == 23) {
    st.e[7] += st.e[15];
  } else if constexpr (O < 28) {
    st.e[O - 24] += st.e[O - 24 + 4];
  } else if constexpr (O < 30) {
    st.e[O - 28] += st.e[O - 28 + 2];
  } else if constexpr (O == 30) {
    st.e[0] += st.e[1];
  } else {
    sacc += st.e[0];
  }
}
template <int G, int PER, int O = G * PER>
__device__ __forceinline__ void tile_sum_slice(const f32x16& acc, TileSumState& st,
                                               float& sacc) {
  if constexpr (O < 32 && O < (G + 1) * PER) {
    tile_sum_op<O>(acc, st, sacc);
    tile_sum_slice<G, PER, O + 1>(acc, st, sacc);
  }
}
// one gap's slice: gap g of the KT * IB gaps serves i-tile g / KT
template <int KT, int IB, int G>
__device__ __forceinline__ void gap_slice(const f32x16 (&acc)[IB],
                                          TileSumState (&st)[IB],
                                          float (&sacc)[IB]) {
  constexpr int t = G / KT, gi = G % KT;
  constexpr int PER = (32 + KT - 1) / KT;
  if constexpr (t < IB) tile_sum_slice<gi, PER>(acc[t], st[t], sacc[t]);
}

// MFMA chain of one tile (folded) with the previous tile's VALU in its gaps
template <int KT, int IB, bool VALU, int C = 0>
__device__ __forceinline__ void lds_chain(const bf16x8 (*Ab)[64], int tile, int lane,
                                          const bf16x8 (&bq)[IB][KT],
                                          f32x16 (&acc)[IB],
                                          const f32x16 (&prev)[IB],
                                          TileSumState (&st)[IB],
                                          float (&sacc)[IB], bf16x8 (&a)[2]) {
  if constexpr (C < KT) {
    // fragment C + 2 is read while C's MFMAs run (a[C & 1] holds C)
    bf16x8 nxt = a[(C + 1) & 1];
    if constexpr (C + 2 < KT) nxt = Ab[tile * KT + C + 2][lane];
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[C & 1], bq[t][C], acc[t],
                                                       0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (VALU) {
        if (t == 0) gap_slice<KT, IB, C * IB + 0>(prev, st, sacc);
        if (t == 1) gap_slice<KT, IB, C * IB + 1>(prev, st, sacc);
        if (t == 2) gap_slice<KT, IB, C * IB + 2>(prev, st, sacc);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    a[C & 1] = nxt;
    lds_chain<KT, IB, VALU, C + 1>(Ab, tile, lane, bq, acc, prev, st, sacc, a);
  }
}

template <int KH, int KL, int IB>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_lds2f_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int CH = 2 * KT;
  static_assert(IB <= 3, "gap_slice serves at most 3 i-tiles");
  __shared__ bf16x8 As[2][CH][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t t0 = (rb * kWaves + wave) * IB;

  bf16x8 bq[IB][KT];
#pragma unroll
  for (int t = 0; t < IB; ++t)
#pragma unroll
    for (int c = 0; c < KT; ++c) bq[t][c] = Bfr[((t0 + t) * KT + c) * 64 + lane];

  for (int gi = 0; gi < spb; ++gi) {
    const int seg = s * spb + gi;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
    const bf16x8* __restrict__ Aseg = Afr + (j0 >> 5) * KT * 64;
    double S[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) S[t] = 0.0;
    auto fill = [&](int buf, int jc) {
      const bf16x8* __restrict__ src = Aseg + (jc >> 5) * KT * 64;
      for (int f = wave; f < CH; f += kWaves)
        __builtin_amdgcn_global_load_lds(
            src + f * 64 + lane,
            (__attribute__((address_space(3))) void*)&As[buf][f][0], 16, 0, 0);
    };
    __syncthreads();
    if (nj > 0) fill(0, 0);
    int buf = 0;
    f32x16 accA[IB], accB[IB];
    TileSumState st[IB];
    float sprev[IB], scur[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) sprev[t] = scur[t] = 0.0f;
    for (int jc = 0; jc < nj; jc += 64) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (jc + 64 < nj) fill(buf ^ 1, jc + 64);
      const bf16x8(*Ab)[64] = As[buf];
      bf16x8 a[2];
#pragma unroll
      for (int t = 0; t < IB; ++t) accA[t] = f32x16{};
      a[0] = Ab[0][lane];
      a[1] = Ab[1][lane];
      if (jc == 0) {  // tile 0, nothing to retire yet
        lds_chain<KT, IB, false>(Ab, 0, lane, bq, accA, accB, st, sprev, a);
      } else {        // tile 0 || tile 1 of the previous chunk
        lds_chain<KT, IB, true>(Ab, 0, lane, bq, accA, accB, st, sprev, a);
#pragma unroll
        for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sprev[t]);
      }
#pragma unroll
      for (int t = 0; t < IB; ++t) {
        accB[t] = f32x16{};
        scur[t] = 0.0f;
      }
      a[0] = Ab[KT][lane];
      a[1] = Ab[KT + 1][lane];
      // tile 1 || tile 0 of this chunk
      lds_chain<KT, IB, true>(Ab, 1, lane, bq, accB, accA, st, scur, a);
#pragma unroll
      for (int t = 0; t < IB; ++t) sprev[t] = scur[t];
      buf ^= 1;
    }
    if (nj > 0) {  // retire the last tile
#pragma unroll
      for (int t = 0; t < IB; ++t) sprev[t] += tile_sum<0>(accB[t], accB[t]);
#pragma unroll
      for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sprev[t]);
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double tot = S[t] + __shfl_xor(S[t], 32, 64);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * M + i] = tot;
    }
  }
}

// The same pass with the A fragments of each 64-row chunk staged once per
// block in LDS (double-buffered) and shared by the kWaves waves, which walk
// the same j-segments.  Where the register version needs more than 256
// VGPRs (d > 8: one wave per SIMD, MFMA chain and VALU back to back) this
// frees the a[2][KT] registers, and L2 serves each fragment once per block
// instead of once per wave.  Per-lane arithmetic and order are those of
// kde_mfma_kernel<.., PIPE = false>: the two give bit-identical rows.
template <int KH, int KL, int IB>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_lds_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int CH = 2 * KT * 64;  // fragments of one 64-row chunk
  constexpr int PER = (CH + 64 * kWaves - 1) / (64 * kWaves);
  __shared__ bf16x8 As[2][CH];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t t0 = (rb * kWaves + wave) * IB;

  bf16x8 bq[IB][KT];
#pragma unroll
  for (int t = 0; t < IB; ++t)
#pragma unroll
    for (int c = 0; c < KT; ++c) bq[t][c] = Bfr[((t0 + t) * KT + c) * 64 + lane];

  for (int gi = 0; gi < spb; ++gi) {
    const int seg = s * spb + gi;
    const int64_t j0 = static_cast<int64_t>(seg) * jseg;
    const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
    const bf16x8* __restrict__ Aseg = Afr + (j0 >> 5) * KT * 64;
    double S[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) S[t] = 0.0;
    bf16x8 stage[PER];
    if (nj > 0) {
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int idx = threadIdx.x + q * 64 * kWaves;
        if (idx < CH) As[0][idx] = Aseg[idx];
      }
    }
    __syncthreads();
    int buf = 0;
    for (int jc = 0; jc < nj; jc += 64) {
      const bool more = jc + 64 < nj;
      if (more) {  // next chunk into registers; written after this compute
        const bf16x8* __restrict__ an = Aseg + ((jc + 64) >> 5) * KT * 64;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
          const int idx = threadIdx.x + q * 64 * kWaves;
          if (idx < CH) stage[q] = an[idx];
        }
      }
      const bf16x8* __restrict__ Ab = As[buf];
      float sacc[IB];
#pragma unroll
      for (int t = 0; t < IB; ++t) sacc[t] = 0.0f;
#pragma unroll
      for (int q = 0; q < 2 * IB; ++q) {
        const int tile = q / IB, it = q % IB;
        f32x16 hi = f32x16{}, lo = f32x16{};
#pragma unroll
        for (int c = 0; c < KH; ++c)
          hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              Ab[(tile * KT + c) * 64 + lane], bq[it][c], hi, 0, 0, 0);
#pragma unroll
        for (int c = 0; c < KL; ++c)
          lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              Ab[(tile * KT + KH + c) * 64 + lane], bq[it][KH + c], lo, 0, 0, 0);
        sacc[it] += tile_sum_split(hi, lo);
      }
#pragma unroll
      for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sacc[t]);
      if (more) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
          const int idx = threadIdx.x + q * 64 * kWaves;
          if (idx < CH) As[buf ^ 1][idx] = stage[q];
        }
      }
      __syncthreads();
      buf ^= 1;
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double tot = S[t] + __shfl_xor(S[t], 32, 64);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * M + i] = tot;
    }
  }
}

template <int D>
int64_t mpad_rows(int64_t M) {
  constexpr int rows = 32 * kWaves * Mk<D>::PADIB;
  return ceil_div(M, rows) * rows;
}

int64_t mpad_for(int d, int64_t M) {
  switch (kde_padded_dim(d)) {
#define CASE(DD) \
  case DD: return mpad_rows<DD>(M);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default: return -1;
  }
}

int kt_for(int d) {
  switch (kde_padded_dim(d)) {
#define CASE(DD) \
  case DD: return Mk<DD>::KT;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default: return -1;
  }
}

struct MPlan {
  int split, nseg, spb, jseg;
  int64_t row_blocks;
};

template <int D>
MPlan make_mplan(int64_t M, int64_t npad, int ib) {
  // many short blocks: at N = M = 1e6 split 1 -> 32 is 181 -> 163 ms
  // (tools/bench_kde.py msplit); split % 8 == 0 pins each j-segment set to
  // one XCD's L2 (blocks go round-robin over the 8 XCDs)
  constexpr int64_t target_blocks = 65536;
  MPlan p;
  p.nseg = kde_num_segments(npad);
  p.jseg = static_cast<int>(ceil_div(ceil_div(npad, p.nseg), 64) * 64);
  p.row_blocks = mpad_rows<D>(M) / (32 * kWaves * ib);
  int split = 1;
  while (split < p.nseg && p.row_blocks * split < target_blocks) split *= 2;
  if (const char* env = getenv("ABC_KDE_MFMA_SPLIT")) {  // tuning override
    const int v = atoi(env);
    if (v >= 1 && v <= p.nseg && (p.nseg % v) == 0) split = v;
  }
  p.split = split;
  p.spb = p.nseg / split;
  return p;
}

template <int D, int IB>
void launch_mfma(const MPlan& p, const bf16x8* Bfr, int64_t M,
                 const bf16x8* Afr, int64_t npad, double* partial,
                 hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(p.row_blocks * p.split);
  // software pipelining pays at D <= 8 (VALU-bound); at larger D the
  // MFMA chain dominates and the lower register count wins (bench_kde sweep)
  bool pipe = D <= 8;
  if (const char* env = getenv("ABC_KDE_MFMA_PIPE")) pipe = atoi(env) != 0;
  bool lds = false;
  if (const char* env = getenv("ABC_KDE_MFMA_LDS")) lds = atoi(env) != 0;
  // sched_group_barrier interleave of step q+1's MFMAs with step q's VALU:
  // 156.4 -> 151.2 ms at N = M = 1e6, d = 8 with SLP-packed adds, but with
  // plain adds (no SLP, Makefile) the hardware's own interleave is faster:
  // 143.4 (sched) vs 139.2 ms (tools/kde_ab.py); slower at d = 4 and 20
  bool sched = false;
  if (const char* env = getenv("ABC_KDE_MFMA_SCHED")) sched = atoi(env) != 0;
  bool sw = false;
  if (const char* env = getenv("ABC_KDE_MFMA_SW")) sw = atoi(env) != 0;
  int dmab = 0;  // LDS-DMA shared A: 1 = 4 waves per block, 2 = 8 waves
  if (const char* env = getenv("ABC_KDE_MFMA_DMAB")) dmab = atoi(env);
  // LDS-DMA A with IB MFMAs per LDS fragment: the MFMA-bound shapes (d > 8)
  // (default at d > 8: d = 20 21.5 -> 20.4 ms, d = 12 18.6 -> 15.1, d = 24
  // 27.0 -> 23.8 at N = M = 262144, rows bit-identical; tools/kde_variants.py)
  // 2 (default at d > 8): the hand-interleaved folded form, d = 20 19.5 ->
  // 17.3 ms at N = M = 262144, full-size error 6.3e-6 (split form: 1.5e-6);
  // 1: the split form (kde_mfma_lds2_kernel); 0: the register kernel
  int lds2 = D > 8 ? 2 : 0;
  if (const char* env = getenv("ABC_KDE_MFMA_LDS2")) lds2 = atoi(env);
  if constexpr (D > 8) {
    if (lds2 == 2) {
      hipLaunchKernelGGL((kde_mfma_lds2f_kernel<Mk<D>::KH, Mk<D>::KL, IB>),
                         dim3(grid), dim3(64 * kWaves), 0, st, Bfr, M, Afr, npad,
                         p.split, p.spb, p.jseg, partial);
      return;
    }
    if (lds2) {
      bool fold = false;
      if (const char* env = getenv("ABC_KDE_MFMA_FOLD")) fold = atoi(env) != 0;
      if (fold)
        hipLaunchKernelGGL((kde_mfma_lds2_kernel<Mk<D>::KH, Mk<D>::KL, IB, true>),
                           dim3(grid), dim3(64 * kWaves), 0, st, Bfr, M, Afr,
                           npad, p.split, p.spb, p.jseg, partial);
      else
        hipLaunchKernelGGL((kde_mfma_lds2_kernel<Mk<D>::KH, Mk<D>::KL, IB, false>),
                           dim3(grid), dim3(64 * kWaves), 0, st, Bfr, M, Afr,
                           npad, p.split, p.spb, p.jseg, partial);
      return;
    }
  }
  if constexpr (D <= 8) {
    if (dmab == 1 || dmab == 2) {
#define DMAB(NW, SC)                                                           \
  hipLaunchKernelGGL((kde_mfma_dmab_kernel<Mk<D>::KH, Mk<D>::KL, IB, NW, SC>),  \
                     dim3(grid / (NW / kWaves)), dim3(64 * NW), 0, st, Bfr, M, \
                     Afr, npad, p.split, p.spb, p.jseg, partial)
      int abl = 0;
      if (const char* env = getenv("ABC_KDE_MFMA_ABL")) abl = atoi(env);
      if (abl == 4) {  // MFMA + LDS-DMA only (diagnostic)
        hipLaunchKernelGGL((kde_mfma_dmab_kernel<Mk<D>::KH, Mk<D>::KL, IB, 4,
                                                 false, 4>),
                           dim3(grid), dim3(256), 0, st, Bfr, M, Afr, npad,
                           p.split, p.spb, p.jseg, partial);
        return;
      }
      if (abl == 2) {  // exp + adds only (diagnostic)
        hipLaunchKernelGGL((kde_mfma_dmab_kernel<Mk<D>::KH, Mk<D>::KL, IB, 4,
                                                 false, 2>),
                           dim3(grid), dim3(256), 0, st, Bfr, M, Afr, npad,
                           p.split, p.spb, p.jseg, partial);
        return;
      }
      if (dmab == 2 && (p.row_blocks & 1) == 0) {
        if (sched) DMAB(8, true);
        else DMAB(8, false);
      } else {  // 8-wave blocks need an even row-block count
        if (sched) DMAB(4, true);
        else DMAB(4, false);
      }
#undef DMAB
      return;
    }
  }
  if constexpr (D == 8 && IB == 3) {
    int abl = 0;
    if (const char* env = getenv("ABC_KDE_MFMA_ABL")) abl = atoi(env);
    if (abl >= 1 && abl <= 6) {
#define ABLK(A)                                                                \
  hipLaunchKernelGGL((kde_mfma_abl_kernel<Mk<D>::KH, Mk<D>::KL, A>), dim3(grid), \
                     dim3(64 * kWaves), 0, st, Bfr, M, Afr, npad, p.split,     \
                     p.spb, p.jseg, partial)
      if (abl == 1) ABLK(1);
      else if (abl == 5) ABLK(5);
      else if (abl == 6) ABLK(6);
      else if (abl == 2) ABLK(2);
      else if (abl == 3) ABLK(3);
      else ABLK(4);
#undef ABLK
      return;
    }
  }
  if (sw)
    hipLaunchKernelGGL((kde_mfma_sw_kernel<Mk<D>::KH, Mk<D>::KL, IB>),
                       dim3(grid), dim3(64 * kWaves), 0, st, Bfr, M, Afr, npad,
                       p.split, p.spb, p.jseg, partial);
  else if (sched)
    hipLaunchKernelGGL((kde_mfma_kernel<Mk<D>::KH, Mk<D>::KL, IB, true, true>),
                       dim3(grid), dim3(64 * kWaves), 0, st, Bfr, M, Afr, npad,
                       p.split, p.spb, p.jseg, partial);
  else if (lds)
    hipLaunchKernelGGL((kde_mfma_lds_kernel<Mk<D>::KH, Mk<D>::KL, IB>),
                       dim3(grid), dim3(64 * kWaves), 0, st, Bfr, M, Afr, npad,
                       p.split, p.spb, p.jseg, partial);
  else if (pipe)
    hipLaunchKernelGGL((kde_mfma_kernel<Mk<D>::KH, Mk<D>::KL, IB, true>),
                       dim3(grid), dim3(64 * kWaves), 0, st, Bfr, M, Afr, npad,
                       p.split, p.spb, p.jseg, partial);
  else
    hipLaunchKernelGGL((kde_mfma_kernel<Mk<D>::KH, Mk<D>::KL, IB, false>),
                       dim3(grid), dim3(64 * kWaves), 0, st, Bfr, M, Afr, npad,
                       p.split, p.spb, p.jseg, partial);
}

template <int D>
int logpdf_mfma_impl(const bf16x8* Bfr, const double* Ynew, int64_t M,
                     const bf16x8* Afr, const double* P, int64_t npad, int d,
                     const double* lw2max, double log_const, double* out,
                     void* ws, size_t ws_bytes, hipStream_t st) {
  // i-tiles per wave: Mk<D>::IB (the row padding unit) or half of it
  // (tuning override ABC_KDE_MFMA_IB); a row's arithmetic is the same
  constexpr int IBF = Mk<D>::IB;
  constexpr int IBH = IBF > 1 ? IBF / 2 : 1;
  constexpr int IB2 = IBF == 3 ? 2 : IBF;  // the third choice at D <= 8
  int ib = IBF;
  if (const char* env = getenv("ABC_KDE_MFMA_IB")) {
    const int v = atoi(env);
    if (v == IBH || v == IB2) ib = v;
  }
  bool dma = false;
  if (const char* env = getenv("ABC_KDE_MFMA_DMA")) dma = atoi(env) != 0;
  if (dma) ib = 1;
  const MPlan p = make_mplan<D>(M, npad, ib);
  const size_t need = static_cast<size_t>(p.nseg * M) * 8 + 16 +
                      static_cast<size_t>(M) * 4;
  ABC_REQUIRE(ws_bytes >= need, "kde_mfma: workspace too small (%zu < %zu)",
              ws_bytes, need);
  char* base = static_cast<char*>(ws);
  double* partial = reinterpret_cast<double*>(base);
  int* n_fix = reinterpret_cast<int*>(base + static_cast<size_t>(p.nseg * M) * 8);
  int* fix_rows = n_fix + 4;
  ABC_HIP(hipMemsetAsync(n_fix, 0, 16, st));
  if (dma)
    hipLaunchKernelGGL((kde_mfma_dma_kernel<Mk<D>::KH, Mk<D>::KL>),
                       dim3(static_cast<unsigned>(p.row_blocks * p.split)),
                       dim3(64 * kWaves), 0, st, Bfr, M, Afr, npad, p.split,
                       p.spb, p.jseg, partial);
  else if (ib == IBF)
    launch_mfma<D, IBF>(p, Bfr, M, Afr, npad, partial, st);
  else if (ib == IB2)
    launch_mfma<D, IB2>(p, Bfr, M, Afr, npad, partial, st);
  else
    launch_mfma<D, IBH>(p, Bfr, M, Afr, npad, partial, st);
  ABC_LAUNCH_CHECK("kde_mfma_kernel");
  return kde_finish_mfma(partial, M, p.nseg, Ynew, P, npad, d, lw2max,
                         log_const, out, n_fix, fix_rows, st);
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" {

size_t abc_kde_mfma_prev_bytes(int64_t npad, int d) {
  const int kt = kt_for(d);
  if (kt < 0 || npad < 0) return 0;
  return static_cast<size_t>(ceil_div(npad, 32)) * kt * 64 * 16;
}

int64_t abc_kde_mfma_new_rows(int64_t M, int d) { return mpad_for(d, M); }

size_t abc_kde_mfma_new_bytes(int64_t M, int d) {
  const int kt = kt_for(d);
  const int64_t mp = mpad_for(d, M);
  if (kt < 0 || mp < 0) return 0;
  return static_cast<size_t>(mp / 32) * kt * 64 * 16;
}

int abc_kde_pack_prev_mfma(const double* X, const double* w, int64_t n, int d,
                           const double* mu, const double* Us, double* P,
                           void* Afr, int64_t npad, double* lw2max,
                           double* gscale, void* ws, hipStream_t st) {
  ABC_REQUIRE(Afr && gscale && ws, "pack_prev_mfma: null pointer");
  const int D = kde_padded_dim(d);
  if (D < 0) {
    set_error("pack_prev_mfma: unsupported dimension d=%d (max 32)", d);
    return kUnsupported;
  }
  const int rc = kde_pack_direct_f64(X, w, n, d, mu, Us, P, npad, lw2max, ws, st);
  if (rc != kOk) return rc;
  unsigned long long* ykey =
      reinterpret_cast<unsigned long long*>(static_cast<char*>(ws) + 64);
  ABC_HIP(hipMemsetAsync(ykey, 0, 8, st));
  const unsigned gr = static_cast<unsigned>(ceil_div(npad, 256));
  switch (D) {
#define CASE(DD)                                                               \
  case DD:                                                                     \
    hipLaunchKernelGGL((ymax_kernel<DD>), dim3(stream_grid(n, 256, 1024)),     \
                       dim3(256), 0, st, X, n, d, mu, Us, ykey);               \
    hipLaunchKernelGGL((pack_prev_frag_kernel<DD>), dim3(gr), dim3(256), 0, st, \
                       X, w, n, d, mu, Us, npad, lw2max, ykey, gscale,         \
                       static_cast<bf16x8*>(Afr));                             \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
  }
  ABC_LAUNCH_CHECK("pack_prev_frag_kernel");
  return kOk;
}

int abc_kde_pack_new_mfma(const double* theta, int64_t M, int d,
                          const double* mu, const double* Us,
                          const double* gscale, double* Ynew, void* Bfr,
                          hipStream_t st) {
  ABC_REQUIRE(M >= 0, "pack_new_mfma: negative M");
  const int D = kde_padded_dim(d);
  if (D < 0) {
    set_error("pack_new_mfma: unsupported dimension d=%d (max 32)", d);
    return kUnsupported;
  }
  if (M == 0) return kOk;
  ABC_REQUIRE(theta && mu && Us && gscale && Ynew && Bfr,
              "pack_new_mfma: null pointer");
  const int64_t mp = mpad_for(d, M);
  const unsigned gr = static_cast<unsigned>(ceil_div(mp, 256));
  switch (D) {
#define CASE(DD)                                                              \
  case DD:                                                                    \
    hipLaunchKernelGGL((pack_new_frag_kernel<DD>), dim3(gr), dim3(256), 0, st, \
                       theta, M, mp, d, mu, Us, gscale, Ynew,                 \
                       static_cast<bf16x8*>(Bfr));                            \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
  }
  ABC_LAUNCH_CHECK("pack_new_frag_kernel");
  return kOk;
}

int abc_kde_logpdf_mfma(const void* Bfr, const double* Ynew, int64_t M,
                        const void* Afr, const double* P, int64_t npad, int d,
                        const double* lw2max, double log_const,
                        double* out_logpd, void* ws, size_t ws_bytes,
                        hipStream_t st) {
  ABC_REQUIRE(M >= 0 && npad >= 0, "kde_mfma: negative size");
  ABC_REQUIRE(npad % kKdeRowPad == 0, "kde_mfma: npad must be a multiple of %d",
              kKdeRowPad);
  if (M == 0) return kOk;
  ABC_REQUIRE(npad > 0, "kde_mfma: empty previous population");
  ABC_REQUIRE(Bfr && Ynew && Afr && P && lw2max && out_logpd && ws,
              "kde_mfma: null pointer");
  const bf16x8* B = static_cast<const bf16x8*>(Bfr);
  const bf16x8* A = static_cast<const bf16x8*>(Afr);
  switch (kde_padded_dim(d)) {
#define CASE(DD)                                                          \
  case DD:                                                                \
    return logpdf_mfma_impl<DD>(B, Ynew, M, A, P, npad, d, lw2max,        \
                                log_const, out_logpd, ws, ws_bytes, st);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default:
      set_error("kde_mfma: unsupported dimension d=%d (max 32)", d);
      return kUnsupported;
  }
}

}  // extern "C"
