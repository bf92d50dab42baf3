// KDE importance-weight pass on the matrix cores: exact-grid MFMA.
// Same quantity as kde.hip (MultivariateNormalTransition.pdf, reference
// pyabc/transition/multivariatenormal.py:102-125 via smc.py:722-733):
//
//   pd(theta_i) = exp(c) * sum_j 2^(e_ij),  e_ij = lw2_j - |y_i - y_j|^2
//
// expanded as e_ij = a_j + b_i + 2 y_i.y_j with a_j = lw2_j - |y_j|^2 and
// b_i = -|y_i|^2.  The expansion cancels catastrophically in fp32 (a plain
// fp32 GEMM form loses 4e-5 relative at N = 1e6, d = 8), so every operand is
// split into 16-bit pieces that make the large part of the sum EXACT.  The
// default (round 4, every d up to 24) is f16 (Mk<D>::SCH, below):
//
//   y = y1 + r2 + r3   y1 = g*rint(y/g) on a power-of-two grid g from the
//                      population's largest norm (|y1/g| <= 2043: f16
//                      integers), r2 = f16(y - y1), r3 = f16(rest)
//   a = aH0 + aH1 + aL0 + aL1   (aH* f16 multiples of G = g^2 holding
//                      rint(a/G)*G exactly, aL* = f16 pieces of the rest)
//
// hi = sum_k 2 y1_ik y1_jk + aH + bH is a sum of multiples of G below
// 2^24 G, so the fp32 MFMA accumulation is exact in ANY order; lo (five
// cross products per dimension + aL + bL) is small and accumulates on top
// of hi in the same accumulator (folded: the MFMA delivers e itself; a hi
// chunk never carries lo products -- an MFMA's internal sum is not exact,
// tools/probes/mfma_acc_round.hip).  The bf16 scheme of rounds 1-3 (seven
// cross terms, 8-bit y1) and the split f16 form (lo x 2^10 in its own
// accumulator, one rounding at |e|) are kept for d > 24 and as build options.
//
// MFMA mapping (v_mfma_f32_32x32x16_f16): A = previous population (rows =
// j), B = new rows (columns = i), K = the piece slots.  KH chunks of 16
// slots carry the hi products, KL chunks the lo products; each lane owns one
// new row (column lane&31) and 16 j's of the 32-row tile, so per pair the
// VALU does only v_exp_f32 and the row-sum add (plus the hi + lo add where
// the accumulation is split).  The j-range uses kde.hip's fixed segments,
// each lane's values are summed in register order and the two lane halves
// combined in a fixed order, so a row's bits are independent of M, of the
// launch shape and of the number of ranks.  Rows whose sum underflows -- and
// new rows outside the grid range (flagged by b = -inf) -- go through
// kde.hip's exact fixup, in fp64 on the fp64 whitened rows (Ynew [M][D],
// P [npad][D+1]).
#include <cmath>

#include "common.hpp"
#include "kde_internal.hpp"

namespace abc {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr double kLwFloor = -160.0;  // 2^-160 is 0 in fp32: no term changes
constexpr int kWaves = 4;            // waves per block

// Block -> (j-segment set s, row block rb).  split > 0: row-block major
// (the split blocks of one row block adjacent); split < 0: segment major
// (|split| sets, the row blocks of one set adjacent) -- the blocks resident
// together on an XCD then stream the same A segments, so its L2 serves
// them.  A row's arithmetic is the same either way.
__device__ inline void block_coords(int split, int& s, int64_t& rb) {
  if (split > 0) {
    s = static_cast<int>(blockIdx.x % split);
    rb = blockIdx.x / split;
  } else {
    const int64_t nrb = gridDim.x / (-split);
    s = static_cast<int>(blockIdx.x / nrb);
    rb = blockIdx.x % nrb;
  }
}

// Piece scheme per dimension class (compile-time; tools/kde_ab.py prices two
// builds on one box):
//   0 bf16 y1.y1, aH x3, bH x3 | seven cross terms per dimension, aL, bL
//     (folded when KL <= kFoldKL) -- d <= 8 up to round 3
//     (-DABC_KDE_SCHEME_SMALL=0);
//   1 f16 y1.y1, aH x2, bH x2 | five cross terms, aL, bL, the lo pieces
//     x 2^10, split accumulation (hi exact, lo apart, e = fma(lo, 2^-10, hi))
//     -- d > 24 (and 8 < d <= 24 with -DABC_KDE_SCHEME_LARGE=1);
//   2 the same f16 pieces unscaled, every chunk accumulated onto one fp32
//     value (folded: no hi + lo add per pair; the KL lo chunks each round at
//     |e|) -- d <= 24.  At d <= 8 it replaces scheme 0 (round 4, same box,
//     N = M = 1e6: d = 8 128.3 -> 115.3 ms, 4 MFMAs per tile instead of 5,
//     max row error on the kde_variants rows 4.3e-6 -> 3.0e-6; d = 2 91.7 ->
//     83.9 ms, 3.2e-6 -> 9.8e-7; d = 4 96.4 -> 95.1 ms).  Needs the MFMA to keep f16 denormal inputs
//     (tools/probes/mfma_f16_denorm.hip: outputs down to 2^-24).  Same box,
//     N = M = 1e6, d = 20: 209.7 ms against 232.2 ms split; max row error
//     on the kde_variants rows 4.5e-6 against 7.5e-7 (d = 12 / 16 / 24:
//     3.8 / 4.2 / 5.4e-6; d = 32 would be 6.2e-6, so it stays split).
// Rejected (measured): the lo slots packed into the hi chunks' spare slots
// (8 MFMAs at d = 20 instead of 9) -- a chunk mixing the large, cancelling hi
// products with lo products loses the lo bits inside the MFMA (row errors
// 1.4e-5 -- 1.6e-5 at d = 16, 24; tools/probes/mfma_acc_round.hip: the
// 32x32x16 MFMA is not one exact sum + one rounding).
#ifndef ABC_KDE_SCHEME_SMALL
#define ABC_KDE_SCHEME_SMALL 2
#endif
#ifndef ABC_KDE_SCHEME_LARGE
#define ABC_KDE_SCHEME_LARGE 2
#endif

#ifndef ABC_KDE_IB_LARGE
#define ABC_KDE_IB_LARGE 3
#endif
// i-tiles per wave at d = 8 (the headline): 4 since round 6 -- each LDS
// fragment read feeds four MFMAs; 167 VGPRs, three waves per SIMD instead
// of four.  Same box, interleaved, rows bit-identical (tools/ab_ib.sh,
// calls r06ab / r06ac): N = M = 1e6 111.9 -> 110.6 and 113.1 -> 112.2 ms;
// IB = 5 / 6 (two waves per SIMD) 113.5 / 112.2.  At d = 2 and 4 the same
// change measured slower (80.8 -> 82.7, 94.1 -> 158.8 ms), so the other
// d <= 8 keep IB = 3 (build option ABC_KDE_IB_D8 for A/B)
#ifndef ABC_KDE_IB_D8
#define ABC_KDE_IB_D8 4
#endif

template <int D>
struct Mk {
  static constexpr int SCH =
      D <= 8 ? ABC_KDE_SCHEME_SMALL : (D <= 24 ? ABC_KDE_SCHEME_LARGE : 1);
  static_assert(SCH >= 0 && SCH <= 2 && (SCH != 1 || D > 8),
                "piece scheme 0..2 (1 only for d > 8)");
  static constexpr bool F16 = SCH != 0;
  static constexpr int KH = F16 ? (D + 4 + 15) / 16 : (D + 6 + 15) / 16;
  static constexpr int KL = F16 ? (5 * D + 4 + 15) / 16 : (7 * D + 4 + 15) / 16;
  static constexpr int KT = KH + KL;
  static constexpr int LO0 = 16 * KH;  // first lo slot
  // i-tiles per wave: 3 up to d = 24 (round 5 at d > 8: each LDS fragment
  // read feeds three MFMAs instead of two -- the d = 20 probe ladder,
  // profiles/r05_issue_probe.json, prices a ds_read_b128 at ~9 ns per tile
  // step); 1 for the split scheme above d = 24
  static constexpr int IB =
      D == 8 ? ABC_KDE_IB_D8 : D <= 8 ? 3 : D <= 24 ? ABC_KDE_IB_LARGE : 1;
  // row padding unit in i-tiles per wave: every IB the launch may pick
  // (IB, IB / 2, and 2 when IB = 3) divides it
  static constexpr int PADIB =
      D <= 8 ? (IB == 4 ? 4 : IB == 5 ? 10 : 6)
             : D <= 24 ? (IB == 4 ? 12 : 6) : IB;
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

// ---- f16 pieces (d > 8) -------------------------------------------------------
// The bf16 scheme spends 7 cross products per dimension because bf16 keeps 8
// bits; with f16's 11 bits the same exactness takes five, on a grid eight
// times finer:
//   y1 = g rint(y/g) with the grid from the population's largest NORM,
//        |y_j| < 2^E -> g = 2^(E-10): |y1/g| <= 1027 (population), <= 2043
//        (new rows, |y_i| <= 2040 g; others take the exact fixup) -- f16
//        integers;
//   r = y - y1 (|r| <= g/2) -> r2 = f16(r 2^10), r3 = f16((r - r2) 2^10):
//        22 bits below g/2; lo = y1.r2, y1.r3, r2.y1, r3.y1, r2.r2 per
//        dimension + aL + bL (r2.r3, r3.r2 <= D g^2 2^-12 are dropped:
//        numpy emulation tools/probes/kde_f16lo_emul.py, max row error 6.6e-7
//        -- 8.2e-7 at d = 12, 20, 24 against 1.2e-6 -- 1.7e-6 for the bf16
//        scheme);
//   hi = sum 2 y1_i y1_j + aH + bH: multiples of G = g^2, |sum|/G <= 2^23.4
//        (Cauchy-Schwarz: 2 * 2043 * 1027, |a|/G <= 160/G + 1027^2 with
//        g >= 2^-7, |b|/G <= 2043^2), so exact in any order;
//   every lo piece carries 2^10 (r2.r2 2^5 per side) so the pieces that
//   matter are NORMAL f16 numbers whatever the MFMA does with f16
//   denormals; e = fma(lo_acc, 2^-10, hi), one rounding as before.  aH, bH
//   pieces (up to ~2^(2E+2)) are scaled by 2^-K against a partner 2^K,
//   K = max(0, 2E - 13), to stay below the f16 maximum.  A population whose
//   largest norm reaches 2^14 (E > 13) is packed with e = -inf everywhere:
//   every row then takes the exact fixup.
constexpr int kF16GridBits = 10;   // g = 2^(E - 10)
constexpr double kF16MinGrid = 0.0078125;  // 2^-7: 160 / G <= 2^21.3
constexpr int kF16MaxE = 13;
constexpr float kF16LoScale = 1024.0f;     // lo pieces x 2^10
constexpr float kF16LoUnscale = 0.0009765625f;
constexpr unsigned short kF16One = 0x3C00;
constexpr unsigned short kF16NegInf = 0xFC00;

__device__ inline unsigned short f16_bits(float x) {  // RNE
  return __builtin_bit_cast(unsigned short, static_cast<_Float16>(x));
}
__device__ inline float f16_f(unsigned short b) {
  return static_cast<float>(__builtin_bit_cast(_Float16, b));
}
// grid exponent E (|y| < 2^E) -> the aH / bH scale K
__device__ inline int f16_shift(double g) {
  int E = 0;
  frexp(g, &E);                        // g = 2^(E - 1 - 10) * 2^1 ...
  E = E - 1 + kF16GridBits;            // g = 2^(E - 10)
  const int K = 2 * E - 13;
  return K > 0 ? K : 0;
}

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

// f16 pieces of one row (scaled as above), `side` 1 (population) or 2
// (new rows, exact); returns |y1 + r2 + r3|^2 (the represented point)
template <int D, bool SCALED>
__device__ inline double split_row_f16(const double* y, double g, float side,
                                       unsigned short* y1, unsigned short* r2,
                                       unsigned short* r3, unsigned short* r2h) {
  constexpr float LS = SCALED ? kF16LoScale : 1.0f;
  constexpr float LU = SCALED ? kF16LoUnscale : 1.0f;
  double n2 = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const double v1 = rint(y[k] / g) * g;
    const double r = y[k] - v1;                       // exact
    const unsigned short b2 = f16_bits(static_cast<float>(r * LS));
    const double v2 = static_cast<double>(f16_f(b2)) * LU;
    const unsigned short b3 = f16_bits(static_cast<float>((r - v2) * LS));
    const double v3 = static_cast<double>(f16_f(b3)) * LU;
    y1[k] = f16_bits(side * static_cast<float>(v1));
    r2[k] = f16_bits(side * f16_f(b2));
    r3[k] = f16_bits(side * f16_f(b3));
    // r2.r2: 2^5 per side when scaled, the plain pieces when not
    r2h[k] = SCALED ? f16_bits(side * static_cast<float>(v2 * 32.0)) : r2[k];
    const double yt = v1 + v2 + v3;
    n2 = fma(yt, yt, n2);
  }
  return n2;
}

// v -> two f16 pieces holding rint(v/G) G exactly (|rint(v/G)| < 2^22:
// 11 + 11 bits), each x 2^-K, plus two f16 pieces of the remainder x 2^10
template <bool SCALED>
__device__ inline void split_value_f16(double v, double G, int K,
                                       unsigned short* h, unsigned short* l) {
  double q = rint(v / G);
  q = fmin(fmax(q, -4194303.0), 4194303.0);
  const double q0 = trunc(q / 2048.0) * 2048.0;     // top 11 bits
  const double q1 = q - q0;                         // |q1| < 2^11
  const double sc = ldexp(G, -K);
  h[0] = f16_bits(static_cast<float>(q0 * sc));     // exact (11 bits)
  h[1] = f16_bits(static_cast<float>(q1 * sc));
  const double lo = (v - q * G) * (SCALED ? kF16LoScale : 1.0f);  // exact
  const unsigned short l0 = f16_bits(static_cast<float>(lo));
  l[0] = l0;
  l[1] = f16_bits(static_cast<float>(lo - static_cast<double>(f16_f(l0))));
}

// Slot k of the f16 operands (d > 8):
//  hi  k < D: y1 | 2y1     k = D, D+1: aH 2^-K | 2^K   k = D+2, D+3: 2^K | bH 2^-K
//  lo  from slot LO0 = 16 KH, k' = 5m + q (m < D): q: 0 r2|2y1  1 r3|2y1  2 y1|2r2  3 y1|2r3
//                                4 r2 2^-5|2r2 2^-5 (x 2^10 included above)
//      k' = 5D, 5D+1: aL | 1   k' = 5D+2, 5D+3: 1 | bL
template <int D, bool kA>
__device__ inline unsigned short slot_f16(int k, const unsigned short* y1,
                                          const unsigned short* r2,
                                          const unsigned short* r3,
                                          const unsigned short* r2h,
                                          const unsigned short* h,
                                          const unsigned short* l,
                                          unsigned short kpow) {
  constexpr int LO0 = Mk<D>::LO0;
  if (k < LO0) {
    if (k < D) return y1[k];
    if (k < D + 2) return kA ? h[k - D] : kpow;
    if (k < D + 4) return kA ? kpow : h[k - D - 2];
    return 0;
  }
  const int kk = k - LO0;
  if (kk < 5 * D) {
    const int m = kk / 5, q = kk % 5;
    switch (q) {
      case 0: return kA ? r2[m] : y1[m];
      case 1: return kA ? r3[m] : y1[m];
      case 2: return kA ? y1[m] : r2[m];
      case 3: return kA ? y1[m] : r3[m];
      default: return r2h[m];
    }
  }
  if (kk < 5 * D + 2) return kA ? l[kk - 5 * D] : kF16One;
  if (kk < 5 * D + 4) return kA ? kF16One : l[kk - 5 * D - 2];
  return 0;
}

template <int D, bool kA>
__device__ inline void store_frags_f16(bf16x8* __restrict__ F, int64_t p,
                                       const unsigned short* y1,
                                       const unsigned short* r2,
                                       const unsigned short* r3,
                                       const unsigned short* r2h,
                                       const unsigned short* h,
                                       const unsigned short* l,
                                       unsigned short kpow) {
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
        v[e] = static_cast<short>(
            slot_f16<D, kA>(16 * c + 8 * hh + e, y1, r2, r3, r2h, h, l, kpow));
      F[(tile * KT + c) * 64 + 32 * hh + r] = v;
    }
  }
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

// Block-staged whitening (round 6; the pattern of
// kde.hip's pack_prev_kernel): the block's 256 rows of X arrive in LDS by
// coalesced loads (one 8d-byte row per lane otherwise), and the whitening
// matrix is read from LDS instead of being hoisted into SGPRs (114 SGPR
// spills in pack_prev_frag_kernel at d = 20).  Row r0 + threadIdx.x gets
// whiten_row's y: the same products, each output's fma chain over l in
// ascending order -- the same bits.  Every thread of the block calls it.
template <int D>
struct WhitenLds {
  static constexpr int LD = D | 1;  // odd row stride: fewer bank conflicts
  double Ush[D * D];
  double mus[D];
  double Xs[256 * LD];
};

template <int D>
__device__ inline void whiten_block(const double* __restrict__ X, int64_t r0,
                                    int64_t n, int d, const double* __restrict__ mu,
                                    const double* __restrict__ Us, WhitenLds<D>& s,
                                    double (&y)[D]) {
  constexpr int LD = WhitenLds<D>::LD;
  const int tid = threadIdx.x;
  for (int q = tid; q < d * d; q += 256) s.Ush[(q / d) * D + q % d] = Us[q];
  for (int q = tid; q < d; q += 256) s.mus[q] = mu[q];
  const int nr = r0 < n ? static_cast<int>(n - r0 < 256 ? n - r0 : 256) : 0;
  for (int q = tid; q < nr * d; q += 256) s.Xs[(q / d) * LD + q % d] = X[r0 * d + q];
  __syncthreads();
  double acc[D];
#pragma unroll
  for (int k = 0; k < D; ++k) acc[k] = 0.0;
  if (tid < nr) {
#pragma unroll
    for (int l = 0; l < D; ++l) {
      if (l < d) {
        const double xl = s.Xs[tid * LD + l] - s.mus[l];
#pragma unroll
        for (int k = 0; k < D; ++k)
          if (k < d) acc[k] = fma(xl, s.Ush[l * D + k], acc[k]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < D; ++k) y[k] = acc[k];
}

template <int D>
__global__ __launch_bounds__(256) void ymax_kernel(
    const double* __restrict__ X, int64_t n, int d,
    const double* __restrict__ mu, const double* __restrict__ Us,
    unsigned long long* __restrict__ key) {
  __shared__ WhitenLds<D> s;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * 256;
  double y[D];
  whiten_block<D>(X, r0, n, d, mu, Us, s, y);
  double m = 0.0;
  if (r0 + threadIdx.x < n) {
    if constexpr (Mk<D>::F16) {  // largest norm
      double n2 = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) n2 = fma(y[k], y[k], n2);
      m = sqrt(n2);
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) m = fmax(m, fabs(y[k]));
    }
  }
  block_atomic_max_u64<256>(key, static_cast<unsigned long long>(f64_key(m)));
}

__device__ inline double grid_from_key(const unsigned long long* key) {
  const double m = key_f64(*key);
  int E = 0;
  if (m > 0.0) frexp(m, &E);  // m < 2^E
  return fmax(ldexp(1.0, E - 7), 0.015625);  // 256 g = 2^(E+1) >= 2 max|y|
}
// f16 scheme: from the largest norm, |y| < 2^E -> g = 2^(E - 10) (floor
// 2^-7); a negative value flags E > kF16MaxE (the all-fixup packing)
__device__ inline double grid_from_key_f16(const unsigned long long* key) {
  const double m = key_f64(*key);
  int E = 0;
  if (m > 0.0) frexp(m, &E);
  if (E > kF16MaxE) return -1.0;
  return fmax(ldexp(1.0, E - kF16GridBits), kF16MinGrid);
}

template <int D>
__global__ __launch_bounds__(256) void pack_prev_frag_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t n,
    int d, const double* __restrict__ mu, const double* __restrict__ Us,
    int64_t npad, const double* __restrict__ lw2max,
    const unsigned long long* __restrict__ ykey, double* __restrict__ gscale,
    bf16x8* __restrict__ A) {
  __shared__ WhitenLds<D> s;
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const double g = Mk<D>::F16 ? grid_from_key_f16(ykey) : grid_from_key(ykey);
  if (j == 0) *gscale = g;
  double y[D];
  whiten_block<D>(X, static_cast<int64_t>(blockIdx.x) * blockDim.x, n, d, mu, Us,
                  s, y);  // zeros beyond n
  if (j >= npad) return;
  double lw = kLwFloor;
  if (j < n) {
    const double wj = w[j];
    if (wj > 0.0) lw = fmax(log2(wj) - *lw2max, kLwFloor);
  }
  if constexpr (Mk<D>::F16) {
    unsigned short y1[D], r2[D], r3[D], r2h[D], h[2], l[2];
    if (g > 0.0) {
      const int K = f16_shift(g);
      constexpr bool SC = Mk<D>::SCH == 1;
      const double n2 = split_row_f16<D, SC>(y, g, 1.0f, y1, r2, r3, r2h);
      split_value_f16<SC>(lw - n2, g * g, K, h, l);
      store_frags_f16<D, true>(A, j, y1, r2, r3, r2h, h, l,
                               f16_bits(ldexpf(1.0f, K)));
    } else {  // E > kF16MaxE: e = -inf for every pair (all rows to the fixup)
#pragma unroll
      for (int k = 0; k < D; ++k) y1[k] = r2[k] = r3[k] = r2h[k] = 0;
      h[0] = kF16NegInf;
      h[1] = l[0] = l[1] = 0;
      store_frags_f16<D, true>(A, j, y1, r2, r3, r2h, h, l, kF16One);
    }
  } else {
    unsigned short y1[D], y2[D], y3[D], h[3], l[2];
    const double n2 = split_row<D>(y, g, 1.0f, y1, y2, y3);
    split_value(lw - n2, g * g, h, l);
    store_frags<D, true>(A, j, y1, y2, y3, h, l);
  }
}

// Per-row offsets (round 5).  Row i's exponents are taken relative to
// m_i (log2 units, <= 0): e'_ij = e_ij - m_i, packed as b'_i = -|y_i|^2 - m_i
// (still split into exact multiples of G plus a remainder, so hi stays exact;
// |b'| <= 2^22 G is checked), and the finalize adds ln2 m_i back.  The
// folded chain rounds each lo MFMA at |e'| instead of |e|, so a row whose
// dominant terms sit near its own offset is as accurate as a row near the
// largest weight ("Accuracy of the folded
// accumulation").  m_i comes from the row's parent (the particle its
// proposal was resampled from: e_self = lw2_p - |y_i - y_p|^2, floored, at
// most 64 below the global offset, plus kParentShift = 3, the typical log2
// of the other terms' mass relative to it) or from the refine below.
constexpr double kRowOffMin = -64.0;
constexpr double kF16MaxQ = 4.19e6;  // |b'| / G bound (two 11-bit pieces: 4194303)

// f16 B fragments of one whitened row with offset m (false: not packable --
// outside the grid range or b' beyond the two-piece range; the fragments
// then carry e = -inf)
template <int D>
__device__ inline bool pack_row_new(const double* y, double g, double m,
                                    bf16x8* __restrict__ B, int64_t slot) {
  double n2 = 0.0;
  bool ok = g > 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    ok = ok && fabs(y[k]) <= 256.0 * g;  // NaN -> not ok
    n2 = fma(y[k], y[k], n2);
  }
  if constexpr (Mk<D>::F16) {
    ok = g > 0.0 && sqrt(n2) <= 2040.0 * g;  // the norm bound of the f16 scheme
    ok = ok && fabs(-n2 - m) <= kF16MaxQ * g * g;
    unsigned short y1[D], r2[D], r3[D], r2h[D], h[2], l[2];
    unsigned short kpow = kF16One;
    if (ok) {
      const int K = f16_shift(g);
      kpow = f16_bits(ldexpf(1.0f, K));
      constexpr bool SC = Mk<D>::SCH == 1;
      const double n2r = split_row_f16<D, SC>(y, g, 2.0f, y1, r2, r3, r2h);
      split_value_f16<SC>(-n2r - m, g * g, K, h, l);
    } else {  // padding / out-of-grid row: e = -inf
#pragma unroll
      for (int k = 0; k < D; ++k) y1[k] = r2[k] = r3[k] = r2h[k] = 0;
      h[0] = kF16NegInf;
      h[1] = l[0] = l[1] = 0;
    }
    store_frags_f16<D, false>(B, slot, y1, r2, r3, r2h, h, l, kpow);
  } else {
    unsigned short y1[D], y2[D], y3[D], h[3], l[2];
    ok = ok && fabs(-n2 - m) <= 8.0e6 * g * g;  // three bf16 pieces: 2^23
    if (ok) {
      const double n2r = split_row<D>(y, g, 2.0f, y1, y2, y3);
      split_value(-n2r - m, g * g, h, l);
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) y1[k] = y2[k] = y3[k] = 0;
      h[0] = kBf16NegInf;
      h[1] = h[2] = l[0] = l[1] = 0;
    }
    store_frags<D, false>(B, slot, y1, y2, y3, h, l);
  }
  return ok;
}

// parent offset of row i (see above): P is the fp64 direct population
// [npad][D + 1] (y_j, lw2_j)
template <int D>
__device__ inline double parent_offset(const double* y, const double* __restrict__ P,
                                       int64_t p, double shift) {
  const double* pp = P + p * (D + 1);
  double e = pp[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const double df = y[k] - pp[k];
    e = fma(-df, df, e);
  }
  return e == e ? fmin(fmax(floor(e), kRowOffMin), 0.0) + shift : 0.0;
}

template <int D>
__global__ __launch_bounds__(256) void pack_new_frag_kernel(
    const double* __restrict__ theta, int64_t M, int64_t mpad, int d,
    const double* __restrict__ mu, const double* __restrict__ Us,
    const double* __restrict__ gscale, const double* __restrict__ P,
    int64_t npad, const int64_t* __restrict__ parent, double pshift,
    double* __restrict__ Ydir, double* __restrict__ row_off,
    bf16x8* __restrict__ B) {
  __shared__ WhitenLds<D> s;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  double y[D];
  whiten_block<D>(theta, static_cast<int64_t>(blockIdx.x) * blockDim.x, M, d, mu,
                  Us, s, y);
  if (i >= mpad) return;
  const double g = *gscale;
  double m = 0.0;
  if (i < M) {
#pragma unroll
    for (int k = 0; k < D; ++k) Ydir[i * D + k] = y[k];
    // parents only where KL >= 4 lo MFMAs fold (d > 8): at d <= 8 the
    // global offset already keeps every bench row within the routing range
    // (log2 S in [-5.1, -0.9] at N = 1e6) while the parent's term is not
    // the dominant one (the sum is 2^6.8 times it at the median), so the
    // offset would only push rows out of range (tools/kde_offsets.py,
    // gpurun_out/r05d)
    if (parent && Mk<D>::SCH == 2 && Mk<D>::KL >= 4) {
      const int64_t p = parent[i];
      if (p >= 0 && p < npad) m = parent_offset<D>(y, P, p, pshift);
    }
    if (row_off) row_off[i] = m;
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) y[k] = NAN;  // padding: e = -inf
  }
  pack_row_new<D>(y, g, m, B, i);
}

// the 32x32x16 MFMA of the piece scheme: f16 (d > 8) or bf16 (d <= 8); the
// fragments are 16-bit patterns either way
template <bool F16>
__device__ __forceinline__ f32x16 mfma_op(const bf16x8& a, const bf16x8& b,
                                          const f32x16& c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// e = hi + lo, rounded once (the f16 lo accumulator carries 2^10)
template <bool F16>
__device__ __forceinline__ float combine(float hi, float lo) {
  if constexpr (F16)
    return __builtin_fmaf(lo, kF16LoUnscale, hi);
  else
    return hi + lo;
}

// Folded accumulation (KL <= kFoldKL, i.e. D <= 8, the VALU-bound shapes):
// the exact hi products first, then the lo chain accumulated ON TOP of them
// in the same accumulator, so the MFMA delivers e = hi + lo itself and the
// VALU add per pair disappears (143.6 vs 156.6 ms at N = M = 1e6, d = 8).
// hi is exact in any order (multiples of G below 2^24 G); each of the KL lo
// MFMAs then rounds at |e| instead of once, so a term's exponent carries
// about (KL + 1) / 2 ulps of |e| instead of 1/2: relative error ~8e-8 |e|
// at KL = 4.  A row's error is the t-weighted mean of its terms' errors,
// bounded by ~8e-8 log2(N / S) for a row sum S.  Since round 5 rows are
// evaluated relative to their own offset and re-evaluated with a new one
// when the sum leaves the routing range (Route, the refine below), which
// keeps the rounding at |e'| small; DESIGN.md section 4 derives the per-row
// bound (tests/test_gpu_kde_band.py evaluates it row by row).  The f16
// scheme 2 (8 < d <= 24) folds the same way.
constexpr int kFoldKL = 4;

// one (32-row tile, i-tile) product: hi (exact) and lo accumulators, or the
// folded e in hi
// folded: the bf16 scheme with few lo chunks (d <= 8)
template <int KL, int SCH>
constexpr bool kFolded = SCH == 2 || (SCH == 0 && KL <= kFoldKL);

template <int KH, int KL, int SCH>
__device__ __forceinline__ void mfma_step(const bf16x8* a, const bf16x8* b,
                                          f32x16& hi, f32x16& lo) {
  hi = f32x16{};
#pragma unroll
  for (int c = 0; c < KH; ++c) hi = mfma_op<(SCH != 0)>(a[c], b[c], hi);
  if constexpr (kFolded<KL, SCH>) {
#pragma unroll
    for (int c = 0; c < KL; ++c) hi = mfma_op<(SCH != 0)>(a[KH + c], b[KH + c], hi);
  } else {
    lo = f32x16{};
#pragma unroll
    for (int c = 0; c < KL; ++c) lo = mfma_op<(SCH != 0)>(a[KH + c], b[KH + c], lo);
  }
}

// sum of 2^(hi+lo) over the lane's 16 values: 16 independent exps, then a
// fixed pairwise tree (v, v+8), (v, v+4), (v, v+2), (v, v+1)
template <int SCH>
__device__ __forceinline__ float tile_sum_split(const f32x16& hi,
                                                const f32x16& lo) {
  float e[16];
#pragma unroll
  for (int v = 0; v < 16; ++v)
    e[v] = __builtin_amdgcn_exp2f(combine<(SCH == 1)>(hi[v], lo[v]));
#pragma unroll
  for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
    for (int v = 0; v < w; ++v) e[v] += e[v + w];
  return e[0];
}

// the same after mfma_step (folded: e is in hi)
template <int KL, int SCH>
__device__ __forceinline__ float tile_sum(const f32x16& hi, const f32x16& lo) {
  if constexpr (!kFolded<KL, SCH>) {
    return tile_sum_split<SCH>(hi, lo);
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

// largest e over the lane's 16 values (the refine's max pass, MODE 1):
// the same folded / split e as tile_sum exponentiates
template <int KL, int SCH>
__device__ __forceinline__ float tile_max(const f32x16& hi, const f32x16& lo) {
  float e[16];
#pragma unroll
  for (int v = 0; v < 16; ++v)
    e[v] = kFolded<KL, SCH> ? hi[v] : combine<(SCH == 1)>(hi[v], lo[v]);
#pragma unroll
  for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
    for (int v = 0; v < w; ++v) e[v] = fmaxf(e[v], e[v + w]);
  return e[0];
}

// MODE 0: sum of 2^e (the density pass); MODE 1: max of e (the refine's
// offset pass).  Same MFMA chain either way.
template <int MODE, int KL, int SCH>
__device__ __forceinline__ void tile_acc(float& sacc, const f32x16& hi,
                                         const f32x16& lo) {
  if constexpr (MODE == 0)
    sacc += tile_sum<KL, SCH>(hi, lo);
  else
    sacc = fmaxf(sacc, tile_max<KL, SCH>(hi, lo));
}

// main pass.  Block (rb, s): wave w owns i-tiles (rb*kWaves + w)*IB + t and
// walks the spb consecutive j-segments s*spb ..; per segment one fp64 partial
// per row (partial[seg * ld + i], ld >= M).  64-row chunks (two 32-row tiles)
// are summed in fp32, then added into fp64 (MODE 1: maxima instead).
template <int KH, int KL, int IB, bool PIPE, int SCH, int MODE = 0>
__device__ __forceinline__ void kde_mfma_rows(
    const bf16x8* __restrict__ Bfr, int64_t M, int64_t ld,
    const bf16x8* __restrict__ Afr, int64_t npad, int s, int64_t rb, int spb,
    int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr float kInit = MODE == 0 ? 0.0f : -INFINITY;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
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
    for (int t = 0; t < IB; ++t) S[t] = kInit;
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
      for (int t = 0; t < IB; ++t) sacc[t] = kInit;
      if constexpr (PIPE) {
        // 2*IB (tile, i-tile) steps; the MFMAs of step q+1 issue before the
        // VALU of step q, on a second accumulator pair
#pragma unroll
        for (int c = 0; c < KT; ++c) a[1][c] = ap[(KT + c) * 64];
        f32x16 hi[2], lo[2];
        mfma_step<KH, KL, SCH>(a[0], bq[0], hi[0], lo[0]);
#pragma unroll
        for (int q = 0; q < 2 * IB; ++q) {
          if (q + 1 < 2 * IB)
            mfma_step<KH, KL, SCH>(a[(q + 1) / IB], bq[(q + 1) % IB],
                                   hi[(q + 1) & 1], lo[(q + 1) & 1]);
          if (q + 1 == IB) {  // last MFMA reading tile 0 is issued
#pragma unroll
            for (int c = 0; c < KT; ++c) a[0][c] = an[c * 64];
          }
          tile_acc<MODE, KL, SCH>(sacc[q % IB], hi[q & 1], lo[q & 1]);
        }
      } else {
#pragma unroll
        for (int c = 0; c < KT; ++c) a[1][c] = ap[(KT + c) * 64];
#pragma unroll
        for (int q = 0; q < 2 * IB; ++q) {
          f32x16 hi, lo;
          mfma_step<KH, KL, SCH>(a[q / IB], bq[q % IB], hi, lo);
          tile_acc<MODE, KL, SCH>(sacc[q % IB], hi, lo);
          if (q + 1 == IB) {
#pragma unroll
            for (int c = 0; c < KT; ++c) a[0][c] = an[c * 64];
          }
        }
      }
#pragma unroll
      for (int t = 0; t < IB; ++t) {
        if constexpr (MODE == 0)
          S[t] += static_cast<double>(sacc[t]);
        else
          S[t] = fmax(S[t], static_cast<double>(sacc[t]));
      }
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double o = __shfl_xor(S[t], 32, 64);
      const double tot = MODE == 0 ? S[t] + o : fmax(S[t], o);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * ld + i] = tot;
    }
  }
}

template <int KH, int KL, int IB, bool PIPE, int SCH>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  int s;
  int64_t rb;
  block_coords(split, s, rb);
  kde_mfma_rows<KH, KL, IB, PIPE, SCH>(Bfr, M, M, Afr, npad, s, rb, spb, jseg,
                                       partial);
}

// The same pass over a device-counted row list (the refine of flagged rows,
// below): rows [0, *count) of Bfr, partial[seg * ld + row]; blocks take
// (segment, row block) pairs grid-stride, so an empty list costs only the
// blocks' exit.  A row's arithmetic is that of kde_mfma_kernel.
template <int KH, int KL, int IB, bool PIPE, int SCH, int MODE>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_list_kernel(
    const bf16x8* __restrict__ Bfr, const int* __restrict__ count, int64_t ld,
    const bf16x8* __restrict__ Afr, int64_t npad, int nseg, int jseg,
    double* __restrict__ partial) {
  const int64_t M = *count;
  const int64_t nrb = ceil_div(M, 32 * kWaves * IB);
  const int s = static_cast<int>(blockIdx.x % nseg);
  const int64_t stride = gridDim.x / nseg;
  for (int64_t rb = blockIdx.x / nseg; rb < nrb; rb += stride)
    kde_mfma_rows<KH, KL, IB, PIPE, SCH, MODE>(Bfr, M, ld, Afr, npad, s, rb, 1,
                                               jseg, partial);
}

// ---- hand-interleaved LDS-DMA passes (d > 8) --------------------------------
// The VALU of one 32-row tile is cut into slices placed in the gaps of the
// NEXT tile's MFMA chain, one slice after each MFMA, with sched_barrier
// fences so the compiler keeps exactly that order: an MFMA holds vector
// issue for 8 of its 32 cycles, and the slice runs in the other 24
// (MI355X_MICROARCH.md, MFMA gap fillers).  Every op works in place on the
// retiring tile's accumulators (no separate exp registers).
//
// Sum ops of one i-tile (32): the exps of pair v are issued one slice ahead
// of the add of pair v - 1, so no add waits on the transcendental it follows:
//   e0 e8  e1 e9 a0  e2 e10 a1 ... e7 e15 a6  a7  b0..b3  c0 c1  d0  s
// (a: v += v + 8, b: v + 4, c: v + 2, d: v + 1, s: the row add) -- the tree
// of tile_sum, so the rows are bit-identical to the plain passes'.
template <int O>
__device__ __forceinline__ void sum_op(f32x16& x, float& sacc) {
  if constexpr (O < 2) {
    x[8 * O] = __builtin_amdgcn_exp2f(x[8 * O]);
  } else if constexpr (O < 23) {
    constexpr int v = 1 + (O - 2) / 3, k = (O - 2) % 3;
    if constexpr (k == 0) x[v] = __builtin_amdgcn_exp2f(x[v]);
    else if constexpr (k == 1) x[v + 8] = __builtin_amdgcn_exp2f(x[v + 8]);
    else x[v - 1] += x[v - 1 + 8];
  } else if constexpr (O == 23) {
    x[7] += x[15];
  } else if constexpr (O < 28) {
    x[O - 24] += x[O - 24 + 4];
  } else if constexpr (O < 30) {
    x[O - 28] += x[O - 28 + 2];
  } else if constexpr (O == 30) {
    x[0] += x[1];
  } else {
    sacc += x[0];
  }
}

// Split accumulation (hi and lo accumulators, e = hi + lo rounded once).
// The lo accumulators are single-buffered: the next chain's first lo MFMA of
// i-tile t comes after its KH * IB + t hi MFMAs, so the retiring tile's
// 16 IB  hi += lo  adds (i-tile by i-tile) go in the first GA = KH*IB+IB-1
// gaps, and the 32 IB sum ops (i-tiles interleaved op by op) in the rest.
template <int KT, int KH, int IB>
struct SplitPlan {
  static constexpr int NG = KT * IB;
  static constexpr int GA = KH * IB + IB - 1;
  static constexpr int NA = 16 * IB;
  static constexpr int NS = 32 * IB;
  static constexpr int a0(int g) { return g * NA / GA; }
  static constexpr int s0(int g) { return (g - GA) * NS / (NG - GA); }
};
template <int KT, int KH, int IB, int SCH, int Q, int QE>
__device__ __forceinline__ void split_add_ops(f32x16 (&h)[IB],
                                              const f32x16 (&l)[IB]) {
  if constexpr (Q < QE) {
    h[Q / 16][Q % 16] = combine<(SCH == 1)>(h[Q / 16][Q % 16], l[Q / 16][Q % 16]);
    split_add_ops<KT, KH, IB, SCH, Q + 1, QE>(h, l);
  }
}
template <int IB, int Q, int QE>
__device__ __forceinline__ void split_sum_ops(f32x16 (&h)[IB], float (&sacc)[IB]) {
  if constexpr (Q < QE) {
    sum_op<Q / IB>(h[Q % IB], sacc[Q % IB]);
    split_sum_ops<IB, Q + 1, QE>(h, sacc);
  }
}
template <int KT, int KH, int IB, int SCH, int G>
__device__ __forceinline__ void split_gap_ops(f32x16 (&h)[IB], const f32x16 (&l)[IB],
                                              float (&sacc)[IB]) {
  using P = SplitPlan<KT, KH, IB>;
  if constexpr (G < P::GA) {
    split_add_ops<KT, KH, IB, SCH, P::a0(G), P::a0(G + 1)>(h, l);
  } else {
    split_sum_ops<IB, P::s0(G), P::s0(G + 1)>(h, sacc);
  }
}

// MFMA chain of one tile with the previous tile's VALU in its gaps.  acc:
// this tile's hi accumulators; prev: the retiring tile's; lo: the lo
// accumulators (read as the retiring tile's lo by the first gaps, then
// overwritten by this chain).
template <int KT, int KH, int IB, int SCH, bool VALU, int C = 0>
__device__ __forceinline__ void lds_chain(const bf16x8 (*Ab)[64], int tile, int lane,
                                          const bf16x8 (&bq)[IB][KT],
                                          f32x16 (&acc)[IB], f32x16 (&prev)[IB],
                                          f32x16 (&lo)[IB], float (&sacc)[IB],
                                          bf16x8 (&a)[2]) {
  if constexpr (C < KT) {
    // fragment C + 2 is read while C's MFMAs run (a[C & 1] holds C)
    bf16x8 nxt = a[(C + 1) & 1];
    if constexpr (C + 2 < KT) nxt = Ab[tile * KT + C + 2][lane];
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      if (C >= KH)
        lo[t] = mfma_op<(SCH != 0)>(a[C & 1], bq[t][C], C == KH ? f32x16{} : lo[t]);
      else
        acc[t] = mfma_op<(SCH != 0)>(a[C & 1], bq[t][C], C == 0 ? f32x16{} : acc[t]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (VALU) {
        // t is a compile-time constant after unrolling; each branch names
        // its gap index
#define ABC_GAP(TT) \
  if (t == TT) split_gap_ops<KT, KH, IB, SCH, C * IB + TT>(prev, lo, sacc);
        ABC_GAP(0)
        ABC_GAP(1)
        ABC_GAP(2)
#undef ABC_GAP
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    a[C & 1] = nxt;
    lds_chain<KT, KH, IB, SCH, VALU, C + 1>(Ab, tile, lane, bq, acc, prev, lo,
                                             sacc, a);
  }
}

// The split accumulation (d > 24) with A fragments shared through LDS by
// LDS-DMA (double-buffered, one barrier per 64-row chunk; each fragment
// read feeds IB MFMAs) and the VALU hand-placed in the MFMA gaps; rows
// bit-identical to the register kernel's.  d = 20, N = M = 262144: 19.3 (lds2) -> 18.0 ms.
// (The folded accumulation in the same schedule ran 16.8 ms but its error
// reached 6.3e-6 at N = M = 1e6 against 1.5e-6 -- DESIGN.md section 4 --
// and was dropped.)
template <int KH, int KL, int IB, int SCH>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_lds2i_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int CH = 2 * KT;
  static_assert(IB <= 3, "the gap ops serve at most 3 i-tiles");
  __shared__ bf16x8 As[2][CH][64];
  const int lane = threadIdx.x & 63;
  // wave-uniform: the LDS-DMA fill loop and its M0 address stay scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int s;
  int64_t rb;
  block_coords(split, s, rb);
  split = split < 0 ? -split : split;
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
    f32x16 accA[IB], accB[IB], lo[IB];
    float sprev[IB], scur[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) sprev[t] = scur[t] = 0.0f;
    for (int jc = 0; jc < nj; jc += 64) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (jc + 64 < nj) fill(buf ^ 1, jc + 64);
      const bf16x8(*Ab)[64] = As[buf];
      bf16x8 a[2];
      a[0] = Ab[0][lane];
      a[1] = Ab[1][lane];
      if (jc == 0) {  // tile 0, nothing to retire yet
        lds_chain<KT, KH, IB, SCH, false>(Ab, 0, lane, bq, accA, accB, lo, sprev,
                                          a);
      } else {        // tile 0 || tile 1 of the previous chunk
        lds_chain<KT, KH, IB, SCH, true>(Ab, 0, lane, bq, accA, accB, lo, sprev,
                                         a);
#pragma unroll
        for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sprev[t]);
      }
#pragma unroll
      for (int t = 0; t < IB; ++t) scur[t] = 0.0f;
      a[0] = Ab[KT][lane];
      a[1] = Ab[KT + 1][lane];
      // tile 1 || tile 0 of this chunk
      lds_chain<KT, KH, IB, SCH, true>(Ab, 1, lane, bq, accB, accA, lo, scur, a);
#pragma unroll
      for (int t = 0; t < IB; ++t) sprev[t] = scur[t];
      buf ^= 1;
    }
    if (nj > 0) {  // retire the last tile
#pragma unroll
      for (int t = 0; t < IB; ++t)
        sprev[t] += tile_sum_split<SCH>(accB[t], lo[t]);
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

// ---- folded, hand-interleaved LDS-DMA pass (d <= 8) -------------------------
// The register kernel's arithmetic (hi products first, the lo chain on top
// in the same accumulator, then tile_sum's exps and tree) with the A
// fragments shared by the block through LDS (as kde_mfma_lds2i_kernel) and
// the retiring tile's 32 IB sum ops spread evenly over the next chain's
// KT IB MFMA gaps.  Rows bit-identical to kde_mfma_kernel's.
template <int KT, int IB>
struct FoldPlan {
  static constexpr int NG = KT * IB;
  static constexpr int NS = 32 * IB;
  static constexpr int s0(int g) { return g * NS / NG; }
};
template <int KT, int IB, int G>
__device__ __forceinline__ void fold_gap_ops(f32x16 (&h)[IB], float (&sacc)[IB]) {
  using P = FoldPlan<KT, IB>;
  split_sum_ops<IB, P::s0(G), P::s0(G + 1)>(h, sacc);
}
template <int KT, int IB, int SCH, bool VALU, int C = 0>
__device__ __forceinline__ void lds_chain_f(const bf16x8 (*Ab)[64], int tile, int lane,
                                            const bf16x8 (&bq)[IB][KT],
                                            f32x16 (&acc)[IB], f32x16 (&prev)[IB],
                                            float (&sacc)[IB], bf16x8 (&a)[2]) {
  if constexpr (C < KT) {
    bf16x8 nxt = a[(C + 1) & 1];
    if constexpr (C + 2 < KT) nxt = Ab[tile * KT + C + 2][lane];
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      acc[t] = mfma_op<(SCH != 0)>(a[C & 1], bq[t][C], C == 0 ? f32x16{} : acc[t]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (VALU) {
#define ABC_GAP(TT) \
  if constexpr (TT < IB) if (t == TT) fold_gap_ops<KT, IB, C * IB + TT>(prev, sacc);
        ABC_GAP(0)
        ABC_GAP(1)
        ABC_GAP(2)
        ABC_GAP(3)
        ABC_GAP(4)
        ABC_GAP(5)
#undef ABC_GAP
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    a[C & 1] = nxt;
    lds_chain_f<KT, IB, SCH, VALU, C + 1>(Ab, tile, lane, bq, acc, prev, sacc, a);
  }
}

// waves per SIMD the folded LDS pass is compiled for (register budget
// 512 / waves).  The headline d = 8 form needs 129 VGPRs unconstrained, one
// over the 4-wave budget: held to 128 (2 spilled outside the loop) it runs
// 114.5 vs 115.5 ms at N = M = 1e6, interleaved (gpurun_out/r04x).  d = 20
// held to 3 waves (168 VGPRs, 6 spilled): 206.8 vs 206.0 ms -- no hint.
#ifndef ABC_KDE_LDS2G_WAVES
#define ABC_KDE_LDS2G_WAVES 1
#endif
constexpr int lds2g_waves(int KT, int IB, bool PIPE) {
  return ABC_KDE_LDS2G_WAVES == 0 ? 1
         : ABC_KDE_LDS2G_WAVES >= 2 && KT > 4 ? ABC_KDE_LDS2G_WAVES
         : (PIPE ? KT * IB <= 8 : KT * IB <= 12) ? 4
         : (!PIPE && KT * IB <= 18) ? 3 : 1;
}

// 32-row tiles of A per LDS stage of the folded pass (one barrier per
// stage): 4 since round 4 (2 before); the issue probe with the kernel's
// memory path (tools/probes/issue_probe.hip variants 9 / 11) measures 124.3
// vs 119.0 ns per tile step at 4 waves per SIMD for 2 vs 4; the kernel,
// interleaved on one box (gpurun_out/r04aj): 122.9 / 122.8 -> 121.1 /
// 121.1 ms at N = M = 1e6, d = 8; 222.0 -> 221.0 ms at d = 20
#ifndef ABC_KDE_STAGE_TILES
#define ABC_KDE_STAGE_TILES 4
#endif
// d > 8 (KT = 9 / 10 fragments per tile): 4 tiles per stage too since
// round 5 (72 / 80 KB of LDS per block, still two blocks per CU): at IB = 3,
// N = M = 1e6, d = 20 the launch ran 199.4 / 201.5-201.9 ms (min / median)
// against 200.8-200.9 / 203.6 ms with 2-tile stages, rows bit-identical
// (tools/build_variant.sh + tools/lib_ab.py tools/kde_time.py, gpurun_out/
// r05y).  Issuing the next stage's LDS-DMA pieces a share before each tile's
// chain instead of all at the stage start measured slower at both d = 8
// (116.1 vs 111.5 ms) and d = 20 (206.4 vs 200.9 ms) and was not kept.
#ifndef ABC_KDE_STAGE_TILES_LARGE
#define ABC_KDE_STAGE_TILES_LARGE 4
#endif
constexpr int lds2g_stage_tiles(int KT) {
  return KT <= 4 ? ABC_KDE_STAGE_TILES : ABC_KDE_STAGE_TILES_LARGE;
}

// W: waves per block (4).  Measured and not kept (round 5): 8 waves per
// block at d = 20, IB = 3 -- every wave's share of the LDS-DMA refill
// halves -- ran 199.2 / 199.5 ms against 196.9 / 198.7 ms, interleaved
// (gpurun_out/r05h)
template <int KH, int KL, int IB, int SCH, bool PIPE = true, int W = kWaves>
__global__ __launch_bounds__(64 * W)
__attribute__((amdgpu_waves_per_eu(lds2g_waves(KH + KL, IB, PIPE))))
void kde_mfma_lds2g_kernel(
    const bf16x8* __restrict__ Bfr, int64_t M, const bf16x8* __restrict__ Afr,
    int64_t npad, int split, int spb, int jseg, double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int TPS = lds2g_stage_tiles(KT);  // 32-row tiles per LDS stage
  constexpr int CH = TPS * KT;
  static_assert(kFolded<KL, SCH>, "folded accumulation only");
  static_assert(IB <= 6, "the gap ops serve at most 6 i-tiles");
  static_assert(TPS % 2 == 0, "stages hold whole 64-row chunks");
  __shared__ bf16x8 As[2][CH][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int s;
  int64_t rb;
  block_coords(split, s, rb);
  split = split < 0 ? -split : split;
  const int64_t t0 = (rb * W + wave) * IB;

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
    // tiles [jc/32, jc/32 + nt) into buffer buf (nt: TPS, or 2 for the
    // segment's last 64 rows)
    auto fill = [&](int buf, int jc, int nt) {
      const bf16x8* __restrict__ src = Aseg + (jc >> 5) * KT * 64;
      for (int f = wave; f < nt * KT; f += W)
        __builtin_amdgcn_global_load_lds(
            src + f * 64 + lane,
            (__attribute__((address_space(3))) void*)&As[buf][f][0], 16, 0, 0);
    };
    auto stage_tiles = [&](int jc) { return min(TPS, (nj - jc) >> 5); };
    __syncthreads();
    if (nj > 0) fill(0, 0, stage_tiles(0));
    int buf = 0;
    f32x16 accA[IB], accB[IB];
    // fp32 sum of the current 64-row chunk (two tiles) per i-tile: the
    // retiring tile's terms are added during the next tile's chain; a chunk
    // goes into fp64 once both of its tiles are in (the plain passes'
    // grouping, so the rows are bit-identical to theirs)
    float sc[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) sc[t] = 0.0f;
    for (int jc = 0; jc < nj;) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int nt = stage_tiles(jc);
      const int jn = jc + 32 * nt;
      if (jn < nj) fill(buf ^ 1, jn, stage_tiles(jn));
      const bf16x8(*Ab)[64] = As[buf];
      // tiles u0 (even: accA) and u0 + 1 (odd: accB) of the stage; each
      // chain carries the VALU of the tile before it (the other set)
      auto pair = [&](int u0, bool first) {
        if constexpr (!PIPE) {
          // no overlap inside the wave: each tile's chain, then its sum
          // (the same per-lane arithmetic and grouping)
#pragma unroll
          for (int t = 0; t < IB; ++t) sc[t] = 0.0f;
#pragma unroll
          for (int u = u0; u < u0 + 2; ++u) {
            bf16x8 a[2];
            a[0] = Ab[u * KT][lane];
            a[1] = Ab[u * KT + 1][lane];
            lds_chain_f<KT, IB, SCH, false>(Ab, u, lane, bq, accA, accA, sc, a);
#pragma unroll
            for (int t = 0; t < IB; ++t) sc[t] += tile_sum<KL, SCH>(accA[t], accA[t]);
          }
#pragma unroll
          for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sc[t]);
          return;
        }
        bf16x8 a[2];
        a[0] = Ab[u0 * KT][lane];
        a[1] = Ab[u0 * KT + 1][lane];
        if (first) {
          lds_chain_f<KT, IB, SCH, false>(Ab, u0, lane, bq, accA, accB, sc, a);
        } else {
          lds_chain_f<KT, IB, SCH, true>(Ab, u0, lane, bq, accA, accB, sc, a);
#pragma unroll
          for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sc[t]);
        }
#pragma unroll
        for (int t = 0; t < IB; ++t) sc[t] = 0.0f;
        a[0] = Ab[(u0 + 1) * KT][lane];
        a[1] = Ab[(u0 + 1) * KT + 1][lane];
        lds_chain_f<KT, IB, SCH, true>(Ab, u0 + 1, lane, bq, accB, accA, sc, a);
      };
      pair(0, jc == 0);
#pragma unroll
      for (int u0 = 2; u0 < TPS; u0 += 2)
        if (u0 < nt) pair(u0, false);
      buf ^= 1;
      jc = jn;
    }
    if (PIPE && nj > 0) {
#pragma unroll
      for (int t = 0; t < IB; ++t) sc[t] += tile_sum<KL, SCH>(accB[t], accB[t]);
#pragma unroll
      for (int t = 0; t < IB; ++t) S[t] += static_cast<double>(sc[t]);
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double tot = S[t] + __shfl_xor(S[t], 32, 64);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(seg) * M + i] = tot;
    }
  }
}

// The refine's passes over a device-counted row list (MODE 0 density, 1
// max), folded schemes: the unpipelined LDS-DMA form of
// kde_mfma_lds2g_kernel (A fragments shared by the block's four waves
// through LDS) with blocks taking (segment, row block) pairs grid-stride.
// A row's arithmetic is the main pass's (the register list kernel, which
// streams A per wave from L2, served the round's first measurements: 1.6 ms
// per launch for ~4000 rows at d = 20, N = 1e6).
template <int KH, int KL, int IB, int SCH, int MODE>
__global__ __launch_bounds__(64 * kWaves) void kde_mfma_lds_list_kernel(
    const bf16x8* __restrict__ Bfr, const int* __restrict__ count, int64_t ld,
    const bf16x8* __restrict__ Afr, int64_t npad, int nseg, int jseg,
    double* __restrict__ partial) {
  constexpr int KT = KH + KL;
  constexpr int TPS = lds2g_stage_tiles(KT);
  constexpr int CH = TPS * KT;
  constexpr float kInit = MODE == 0 ? 0.0f : -INFINITY;
  static_assert(kFolded<KL, SCH>, "folded accumulation only");
  __shared__ bf16x8 As[2][CH][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t M = *count;
  const int64_t nrb = ceil_div(M, 32 * kWaves * IB);
  const int s = static_cast<int>(blockIdx.x % nseg);
  const int64_t stride = gridDim.x / nseg;
  const int64_t j0 = static_cast<int64_t>(s) * jseg;
  const int nj = static_cast<int>(j0 < npad ? min<int64_t>(jseg, npad - j0) : 0);
  const bf16x8* __restrict__ Aseg = Afr + (j0 >> 5) * KT * 64;
  auto fill = [&](int buf, int jc, int nt) {
    const bf16x8* __restrict__ src = Aseg + (jc >> 5) * KT * 64;
    for (int f = wave; f < nt * KT; f += kWaves)
      __builtin_amdgcn_global_load_lds(
          src + f * 64 + lane,
          (__attribute__((address_space(3))) void*)&As[buf][f][0], 16, 0, 0);
  };
  auto stage_tiles = [&](int jc) { return min(TPS, (nj - jc) >> 5); };
  for (int64_t rb = blockIdx.x / nseg; rb < nrb; rb += stride) {
    const int64_t t0 = (rb * kWaves + wave) * IB;
    bf16x8 bq[IB][KT];
#pragma unroll
    for (int t = 0; t < IB; ++t)
#pragma unroll
      for (int c = 0; c < KT; ++c) bq[t][c] = Bfr[((t0 + t) * KT + c) * 64 + lane];
    double S[IB];
#pragma unroll
    for (int t = 0; t < IB; ++t) S[t] = kInit;
    __syncthreads();  // the previous row block's readers are done with As
    if (nj > 0) fill(0, 0, stage_tiles(0));
    int buf = 0;
    f32x16 acc[IB];
    for (int jc = 0; jc < nj;) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int nt = stage_tiles(jc);
      const int jn = jc + 32 * nt;
      if (jn < nj) fill(buf ^ 1, jn, stage_tiles(jn));
      const bf16x8(*Ab)[64] = As[buf];
#pragma unroll
      for (int u0 = 0; u0 < TPS; u0 += 2) {
        if (u0 < nt) {
          float sc[IB];
#pragma unroll
          for (int t = 0; t < IB; ++t) sc[t] = kInit;
#pragma unroll
          for (int u = u0; u < u0 + 2; ++u) {
            bf16x8 a[2];
            a[0] = Ab[u * KT][lane];
            a[1] = Ab[u * KT + 1][lane];
            lds_chain_f<KT, IB, SCH, false>(Ab, u, lane, bq, acc, acc, sc, a);
#pragma unroll
            for (int t = 0; t < IB; ++t) tile_acc<MODE, KL, SCH>(sc[t], acc[t], acc[t]);
          }
#pragma unroll
          for (int t = 0; t < IB; ++t) {
            if constexpr (MODE == 0)
              S[t] += static_cast<double>(sc[t]);
            else
              S[t] = fmax(S[t], static_cast<double>(sc[t]));
          }
        }
      }
      buf ^= 1;
      jc = jn;
    }
#pragma unroll
    for (int t = 0; t < IB; ++t) {
      const double o = __shfl_xor(S[t], 32, 64);
      const double tot = MODE == 0 ? S[t] + o : fmax(S[t], o);
      const int64_t i = (t0 + t) * 32 + lane;
      if (lane < 32 && i < M) partial[static_cast<int64_t>(s) * ld + i] = tot;
    }
  }
}

// d = 8 takes IB = 4 from kIb4MinRows rows and IB = 3 below: the larger
// blocks cost more at a rank's share of the rows (same box, interleaved,
// rows bit-identical, tools/ab_lib.sh, call r06ai: N = 1e6, M = 1e6 108.0
// against 108.7 ms, M = 5e5 54.1 / 54.3, M = 125 000 14.0-14.4 / 13.8 --
// 326 row blocks of 384 against 245 of 512 for 768 resident blocks)
constexpr int64_t kIb4MinRows = 375000;
template <int D>
constexpr bool kIbBySize = D == 8 && Mk<D>::IB == 4;
template <int D>
int ib_full(int64_t M) {
  return kIbBySize<D> && M < kIb4MinRows ? 3 : Mk<D>::IB;
}
// row padding unit in i-tiles per wave (every IB the launch may pick at
// this M divides it)
template <int D>
int padib(int64_t M) {
  if constexpr (kIbBySize<D>) return M < kIb4MinRows ? 6 : 4;
  return Mk<D>::PADIB;
}

template <int D>
int64_t mpad_rows(int64_t M) {
  const int64_t rows = int64_t{32} * kWaves * padib<D>(M);
  return ceil_div(M, rows) * rows;
}
// the refine's row list: any IB of the list kernel divides 12
template <int D>
int64_t list_pad_rows(int64_t M) {
  constexpr int64_t rows = int64_t{32} * kWaves * 12;
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
  bool smajor;  // segment-major block order (block_coords)
};

template <int D>
MPlan make_mplan(int64_t M, int64_t npad, int ib, bool smajor) {
  // many short blocks: at N = M = 1e6 split 1 -> 32 is 181 -> 163 ms
  // (tools/bench_kde.py msplit); split % 8 == 0 pins each j-segment set to
  // one XCD's L2 (blocks go round-robin over the 8 XCDs)
  constexpr int64_t target_blocks = 65536;
  MPlan p;
  p.nseg = kde_num_segments(npad);
  p.jseg = static_cast<int>(ceil_div(ceil_div(npad, p.nseg), 64) * 64);
  p.row_blocks = mpad_rows<D>(M) / (32 * kWaves * ib);
  // segment major: one segment per block, so the blocks an XCD runs
  // together share one segment of A in its L2 (fetch per launch at N = M =
  // 1e6, d = 8: 80 GB row-block major, 25.8 GB segment major with 4
  // segments per block, 14.5 GB with 1; time 131.1 -> 130.3 ms)
  p.smajor = smajor;
  int split = 1;
  if (smajor)
    split = p.nseg;
  else
    while (split < p.nseg && p.row_blocks * split < target_blocks) split *= 2;
  {  // tuning override
    const int v = tuning_knob(kKnobKdeMfmaSplit, 0);
    if (v >= 1 && v <= p.nseg && (p.nseg % v) == 0) split = v;
  }
  p.split = split;
  p.spb = p.nseg / split;
  return p;
}

// Runtime knobs (tuning only; tests/test_gpu_kernels.py
// test_kde_mfma_launch_knobs_bit_identical checks that each leaves every row
// unchanged): ABC_KDE_MFMA_SPLIT (j-segment blocks per row block),
// ABC_KDE_MFMA_IB (i-tiles per wave), ABC_KDE_MFMA_PIPE (software
// pipelining of the register kernel), ABC_KDE_MFMA_LDS2 (0: the register
// kernel; folded schemes: 1 or 2 the folded LDS-DMA pass, hand-interleaved,
// 3 the same without in-wave pipelining (d <= 8 default on large
// populations); split schemes: 1 LDS-DMA A fragments, 2 the same
// hand-interleaved),
// ABC_KDE_MFMA_SMAJOR (1: segment-major block order, one segment per block).
// Read once per process (common.hpp tuning_knob; abc_tuning_reload).

template <int D, int IB>
void launch_mfma(const MPlan& p, const bf16x8* Bfr, int64_t M,
                 const bf16x8* Afr, int64_t npad, double* partial, int lds2g,
                 hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(p.row_blocks * p.split);
  const dim3 block(64 * kWaves);
  const int split = p.smajor ? -p.split : p.split;
  if constexpr (D > 8 && Mk<D>::SCH == 2) {
    // the folded f16 scheme: the LDS-DMA folded pass, pipelined
    // (ABC_KDE_MFMA_LDS2 1 or 2, the default) or not (3: one accumulator
    // set), or the register kernel (0); rows bit-identical.  d = 20,
    // N = M = 1e6, one process (gpurun_out/r05d): IB = 2 pipelined (round
    // 4) 210.3 / 210.4 ms, IB = 3 unpipelined 215.9 ms, IB = 3 pipelined
    // 198.9 ms
    const int lds2 = tuning_knob(kKnobKdeMfmaLds2, 2);
    if (lds2 == 3) {  // no in-wave pipelining
      hipLaunchKernelGGL((kde_mfma_lds2g_kernel<Mk<D>::KH, Mk<D>::KL, IB, Mk<D>::SCH, false>),
                         dim3(grid), block, 0, st, Bfr, M, Afr, npad, split,
                         p.spb, p.jseg, partial);
      return;
    }
    if (lds2 != 0) {
      hipLaunchKernelGGL((kde_mfma_lds2g_kernel<Mk<D>::KH, Mk<D>::KL, IB, Mk<D>::SCH>),
                         dim3(grid), block, 0, st, Bfr, M, Afr, npad, split,
                         p.spb, p.jseg, partial);
      return;
    }
  } else if constexpr (D > 8) {
    // the split schemes (d > 24): the hand-interleaved LDS-DMA pass, or the
    // register kernel (0); rows bit-identical.  (The LDS-DMA pass with the
    // compiler's schedule, rounds 2-4, is gone: 19.3 vs 17.9 ms at d = 20,
    // N = M = 262144.)
    const int lds2 = tuning_knob(kKnobKdeMfmaLds2, 2);
    if (lds2 != 0) {
      hipLaunchKernelGGL((kde_mfma_lds2i_kernel<Mk<D>::KH, Mk<D>::KL, IB, Mk<D>::SCH>),
                         dim3(grid), block, 0, st, Bfr, M, Afr, npad, split,
                         p.spb, p.jseg, partial);
      return;
    }
  }
  if constexpr (D <= 8) {
    // the folded pass with LDS-DMA A fragments and hand-placed VALU
    // (kde_mfma_lds2g_kernel); rows bit-identical
    if (lds2g == 3) {  // no in-wave pipelining (tuning; rows bit-identical)
      hipLaunchKernelGGL((kde_mfma_lds2g_kernel<Mk<D>::KH, Mk<D>::KL, IB, Mk<D>::SCH, false>),
                         dim3(grid), block, 0, st, Bfr, M, Afr, npad, split,
                         p.spb, p.jseg, partial);
      return;
    }
    if (lds2g) {
      hipLaunchKernelGGL((kde_mfma_lds2g_kernel<Mk<D>::KH, Mk<D>::KL, IB, Mk<D>::SCH>),
                         dim3(grid), block, 0, st, Bfr, M, Afr, npad, split,
                         p.spb, p.jseg, partial);
      return;
    }
  }
  // software pipelining pays at D <= 8 (VALU-bound); at larger D the MFMA
  // chain dominates and the lower register count wins (bench_kde sweep)
  if (tuning_knob(kKnobKdeMfmaPipe, D <= 8) != 0)
    hipLaunchKernelGGL((kde_mfma_kernel<Mk<D>::KH, Mk<D>::KL, IB, true, Mk<D>::SCH>),
                       dim3(grid), block, 0, st, Bfr, M, Afr, npad, split,
                       p.spb, p.jseg, partial);
  else
    hipLaunchKernelGGL((kde_mfma_kernel<Mk<D>::KH, Mk<D>::KL, IB, false, Mk<D>::SCH>),
                       dim3(grid), block, 0, st, Bfr, M, Afr, npad, split,
                       p.spb, p.jseg, partial);
}

// ---- refine: flagged rows re-evaluated with their own offset (round 5) -----
// Pass 1 evaluates every row relative to its offset m_i (0, or its parent's
// term shifted up by kParentShift).  Rows whose sum S_i falls below lo
// (offset 0; the sum is then <= N) or leaves [2^-kParentWin, 2^kParentWin]
// (a parent offset) are refined on the matrix cores instead of going to the
// fp64 fixup:
//   * S_i in the normal range: m_i += floor(log2 S_i) (the dominant terms
//     then sit in [-log2 n_eff - 1, 0]);
//   * S_i underflowed: one max pass of the same folded e over the row list
//     (MODE 1), m_i += floor(max_j e'_ij);
//   then the density pass again over the list with the new offsets.  Rows
// outside the grid range, or whose offset leaves the two-piece range of b',
// and any row the second pass still cannot resolve, take the exact fp64
// fixup.  lo: the folded scheme's routing bound: a row
// without an offset whose sum stays at or above lo keeps the derived bound
// under 1e-5 / 1.5 -- 2^-26 where KL <= 2 lo MFMAs fold (d <= 4: band rows
// e_max in [-40, -16] bound at 5.2e-6 / 5.4e-6 / 6.2e-6 / 9.1e-6 for 2^-24 /
// -26 / -28 / -30, tools/route_bound.py; 2^-24 until round 5), 2^-12
// where KL = 3 (d = 6, 8; 2^-16 measured a 6.76e-6 bound on rows at
// e = -16, tests/test_gpu_kde_band.py), 2^-4 where KL = 4 ... 8
// (8 < d <= 24).  The split and bf16 schemes keep the 2^-32 of rounds 1-4.
// Rows with a parent offset (d > 8; round 6): the sum
// relative to the parent's own term is >= 1 by construction (the parent's
// term floored into [1, 2)); its spread comes from the other terms --
// quantiles 0.1 / 50 / 90 / 99 / 99.9 % of log2 S' = 0.03 / 1.97 / 7.7 /
// 13.9 / 19.1 on C5's rows (N = 1e6, d = 20; tools/kde_route.py, call
// r06a).  The offset is the parent's floored term + kParentShift = 3 and
// the row stays on the folded pass while S'' = S' 2^-3 lies in [2^-7, 2^7]:
// a one-term-dominated row then has its dominant exponent within |e''| < 8
// (derived bound <= 4.8e-6), and the refine takes the 4.6 % of C5's rows
// with S' > 2^10 (211.1 ms against ~201 ms unrouted).  Measured with the
// derived bound evaluated on EVERY row (tools/probes/kde_bound.hip, call
// r06e): max 6.29e-6 <= 1e-5 / 1.5 on C5's 1e6 rows; window 2^8 left 18
// rows above the bar, shift 2 refined 6.5 % of the rows.  A wrong parent
// (S'' far outside the window) is refined like any other flagged row.  The
// round-5 window [2^-16, 2^16] with no shift left rows at a 1.5e-5 bound.
constexpr int kParentShift = 3;
constexpr int kParentWin = 7;
// routing experiments (tools/kde_route.py; ABC_KDE_PARENT_SHIFT / _WIN
// override the two above): the parent offset's shift and the parent rows'
// window [1 / phi, phi]
inline double parent_shift() { return tuning_knob(kKnobKdeParentShift, kParentShift); }
inline double parent_window() {
  const int u = tuning_knob(kKnobKdeParentWin, kParentWin);
  return ldexp(1.0, u < 1 ? 1 : (u > 60 ? 60 : u));
}

template <int D>
struct Route {
  static constexpr bool kFold = Mk<D>::SCH == 2;
  static constexpr double lo =
      !kFold ? 0x1p-32
             : (Mk<D>::KL <= 2 ? 0x1p-26 : (Mk<D>::KL <= 3 ? 0x1p-12 : 0x1p-4));
};
constexpr double kLn2d = 0.6931471805599453;
constexpr int kListBlocks = 8192;  // (segment, row block) blocks of a list pass

// workspace of the MFMA pass: [nseg][M] fp64 partials, the 16 counters
// (cnt[0] fp64-fixup rows, [1] flagged, [2] refine list, [3] max list), then
// the lists and the refine's B fragments
struct MfmaWs {
  double* partial;
  int* cnt;
  int *rows1, *rows2, *rowsx, *rows3;
  double *s1, *m2, *mxo;
  bf16x8* Bbuf;
};
inline size_t al256(size_t b) { return (b + 255) / 256 * 256; }

template <int D>
size_t mfma_ws_layout(int64_t M, int nseg, char* base, MfmaWs* w) {
  const size_t m = static_cast<size_t>(M);
  size_t off = static_cast<size_t>(nseg) * m * 8;  // counters right after
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off = al256(off + bytes);
    return p;
  };
  char* part = base;
  char* cnt = take(64);
  char* r1 = take(4 * m);
  char* s1 = take(8 * m);
  char* r2 = take(4 * m);
  char* m2 = take(8 * m);
  char* rx = take(4 * m);
  char* mx = take(8 * m);
  char* r3 = take(4 * m);
  char* bb = take(static_cast<size_t>(list_pad_rows<D>(M) / 32) * Mk<D>::KT * 64 * 16);
  if (w) {
    w->partial = reinterpret_cast<double*>(part);
    w->cnt = reinterpret_cast<int*>(cnt);
    w->rows1 = reinterpret_cast<int*>(r1);
    w->s1 = reinterpret_cast<double*>(s1);
    w->rows2 = reinterpret_cast<int*>(r2);
    w->m2 = reinterpret_cast<double*>(m2);
    w->rowsx = reinterpret_cast<int*>(rx);
    w->mxo = reinterpret_cast<double*>(mx);
    w->rows3 = reinterpret_cast<int*>(r3);
    w->Bbuf = reinterpret_cast<bf16x8*>(bb);
  }
  return off;
}

// pass-1 finalize: the fixed-order segment sum; rows at or above lo (rows
// without an offset) or inside [plo, phi] (rows with a parent offset) are
// final, the rest join the refine list
__global__ __launch_bounds__(256) void mfma_finalize_kernel(
    const double* __restrict__ partial, int64_t M, int nseg,
    const double* __restrict__ row_off, const double* __restrict__ lw2max,
    double log_const, double lo, double plo, double phi, double* __restrict__ out,
    int* __restrict__ cnt, int* __restrict__ rows1, double* __restrict__ s1) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= M) return;
  double S = 0.0;
  for (int s = 0; s < nseg; ++s) S += partial[static_cast<int64_t>(s) * M + i];
  const double m = row_off ? row_off[i] : 0.0;
  const double off = kLn2d * (*lw2max) + log_const;
  // m == 0: the global offset (every e <= 0), whatever the row's origin
  const bool keep = m == 0.0 ? S >= lo : (S >= plo && S <= phi);
  if (keep) {
    out[i] = log(S) + off + kLn2d * m;
  } else {
    const int f = atomicAdd(cnt + 1, 1);
    rows1[f] = static_cast<int>(i);
    s1[f] = S;
    out[i] = -INFINITY;
  }
}

template <int D>
__device__ inline bool on_grid(const double* y, double g) {
  double n2 = 0.0;
  bool ok = g > 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    ok = ok && fabs(y[k]) <= 256.0 * g;
    n2 = fma(y[k], y[k], n2);
  }
  if constexpr (Mk<D>::F16) ok = g > 0.0 && sqrt(n2) <= 2040.0 * g;
  return ok;
}

// flagged rows -> refine list (offset from the sum), max list (sum
// underflowed; packed with the pass-1 offset for the max pass) or fixup
template <int D>
__global__ __launch_bounds__(256) void refine_classify_kernel(
    int* __restrict__ cnt, const int* __restrict__ rows1,
    const double* __restrict__ s1, const double* __restrict__ row_off,
    const double* __restrict__ Ynew, const double* __restrict__ gscale,
    int* __restrict__ rows2, double* __restrict__ m2, int* __restrict__ rowsx,
    double* __restrict__ mxo, int* __restrict__ rows3, bf16x8* __restrict__ Bbuf) {
  const int n1 = cnt[1];
  const double g = gscale ? *gscale : -1.0;  // no grid: every row to the fixup
  for (int f = blockIdx.x * blockDim.x + threadIdx.x; f < n1;
       f += gridDim.x * blockDim.x) {
    const int row = rows1[f];
    const double m = row_off ? row_off[row] : 0.0;
    const double S = s1[f];
    double y[D];
#pragma unroll
    for (int k = 0; k < D; ++k) y[k] = Ynew[static_cast<int64_t>(row) * D + k];
    if (!on_grid<D>(y, g)) {
      rows3[atomicAdd(cnt, 1)] = row;
    } else if (S > 0x1p-100 && S < 0x1p+100) {
      const int q = atomicAdd(cnt + 2, 1);
      rows2[q] = row;
      m2[q] = m + floor(log2(S));
    } else {
      const int q = atomicAdd(cnt + 3, 1);
      rowsx[q] = row;
      mxo[q] = m;
      pack_row_new<D>(y, g, m, Bbuf, q);
    }
  }
}

// max list -> refine list with m += floor(max e'), or fixup
__global__ __launch_bounds__(256) void refine_after_max_kernel(
    int* __restrict__ cnt, const int* __restrict__ rowsx,
    const double* __restrict__ mxo, const double* __restrict__ partial,
    int64_t ld, int nseg, int* __restrict__ rows2, double* __restrict__ m2,
    int* __restrict__ rows3) {
  const int nx = cnt[3];
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nx;
       q += gridDim.x * blockDim.x) {
    double mx = -INFINITY;
    for (int s = 0; s < nseg; ++s)
      mx = fmax(mx, partial[static_cast<int64_t>(s) * ld + q]);
    if (mx > -1.0e30 && mx < 1.0e30) {
      const int r = atomicAdd(cnt + 2, 1);
      rows2[r] = rowsx[q];
      m2[r] = mxo[q] + floor(mx);
    } else {
      rows3[atomicAdd(cnt, 1)] = rowsx[q];
    }
  }
}

// B fragments of the refine list with the new offsets (an unpackable offset
// marks the row for the fixup: m2 = NaN)
template <int D>
__global__ __launch_bounds__(256) void refine_pack_kernel(
    const int* __restrict__ cnt, const int* __restrict__ rows2,
    double* __restrict__ m2, const double* __restrict__ Ynew,
    const double* __restrict__ gscale, bf16x8* __restrict__ Bbuf) {
  const int n2 = cnt[2];
  const double g = gscale ? *gscale : -1.0;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n2;
       q += gridDim.x * blockDim.x) {
    double y[D];
    const int64_t row = rows2[q];
#pragma unroll
    for (int k = 0; k < D; ++k) y[k] = Ynew[row * D + k];
    if (!pack_row_new<D>(y, g, m2[q], Bbuf, q)) m2[q] = NAN;
  }
}

__global__ __launch_bounds__(256) void refine_finalize_kernel(
    int* __restrict__ cnt, const int* __restrict__ rows2,
    const double* __restrict__ m2, const double* __restrict__ partial,
    int64_t ld, int nseg, const double* __restrict__ lw2max, double log_const,
    double* __restrict__ out, int* __restrict__ rows3) {
  const int n2 = cnt[2];
  const double off = kLn2d * (*lw2max) + log_const;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n2;
       q += gridDim.x * blockDim.x) {
    double S = 0.0;
    for (int s = 0; s < nseg; ++s) S += partial[static_cast<int64_t>(s) * ld + q];
    const double mm = m2[q];
    if (mm == mm && S >= 0x1p-32 && S < 0x1p+100)
      out[rows2[q]] = log(S) + off + kLn2d * mm;
    else
      rows3[atomicAdd(cnt, 1)] = rows2[q];
  }
}

template <int D, int MODE>
void launch_list(const bf16x8* Bbuf, const int* count, int64_t ld,
                 const bf16x8* Afr, int64_t npad, int nseg, int jseg,
                 double* partial, hipStream_t st) {
  const int rbs = kListBlocks / nseg > 0 ? kListBlocks / nseg : 1;
  if constexpr (kFolded<Mk<D>::KL, Mk<D>::SCH>) {
    hipLaunchKernelGGL((kde_mfma_lds_list_kernel<Mk<D>::KH, Mk<D>::KL, Mk<D>::IB,
                                               Mk<D>::SCH, MODE>),
                       dim3(rbs * nseg), dim3(64 * kWaves), 0, st, Bbuf, count, ld,
                       Afr, npad, nseg, jseg, partial);
    return;
  }
  // the split schemes: the register kernel (it holds IB x KT B fragments
  // and two A tiles: IB = 2 above d = 8 keeps it in registers)
  constexpr int IB = D <= 8 ? Mk<D>::IB : (Mk<D>::IB > 2 ? 2 : Mk<D>::IB);
  hipLaunchKernelGGL((kde_mfma_list_kernel<Mk<D>::KH, Mk<D>::KL, IB, (D <= 8),
                                           Mk<D>::SCH, MODE>),
                     dim3(rbs * nseg), dim3(64 * kWaves), 0, st, Bbuf, count, ld,
                     Afr, npad, nseg, jseg, partial);
}

template <int D>
int logpdf_mfma_impl(const bf16x8* Bfr, const double* Ynew,
                     const double* row_off, int64_t M, const bf16x8* Afr,
                     const double* P, int64_t npad, int d,
                     const double* lw2max, const double* gscale,
                     double log_const, double* out, void* ws, size_t ws_bytes,
                     hipStream_t st) {
  // i-tiles per wave: Mk<D>::IB (the row padding unit) or a divisor of it
  // (tuning override ABC_KDE_MFMA_IB); a row's arithmetic is the same
  constexpr int IBF = Mk<D>::IB;
  constexpr int IBH = IBF > 1 ? IBF / 2 : 1;
  constexpr int IB2 = IBF == 3 ? 2 : IBF;  // the third choice at D <= 8
  // this M's i-tiles per wave and its alternatives (d = 8: IB by size)
  const int ibf = ib_full<D>(M);
  const int ibh = ibf > 1 ? ibf / 2 : 1;
  const int ib2 = ibf == 3 ? 2 : ibf;
  // D <= 8 on a large population: the LDS-DMA folded pass at IB = 2 (three
  // waves per SIMD) is the default -- 133.4-133.7 -> 131.1-131.3 ms at
  // N = M = 1e6, d = 8, interleaved A/B in one process (gpurun_out/lds2g2);
  // IB = 3 there ran 136.5 ms, IB = 1 149 ms.  Small populations keep the
  // register kernel (equal at N = 1e5, d = 4).
  // Round 4: the same pass WITHOUT in-wave pipelining (mode 3: each tile's
  // chain, then its sums; one accumulator set) at IB = 3 holds four waves
  // per SIMD in 128 VGPRs and reads each A fragment for three i-tiles:
  // 115.9-116.1 -> 112.7-112.9 ms at N = M = 1e6, d = 8, and 93.2 -> 91.1 ms
  // at d = 4, interleaved (gpurun_out/r04ao, r04ap); rows bit-identical.
  // (At d > 8 the pipelined form stays: 204.8 vs 208.4 ms at d = 20.)  From
  // 2^16 rows on (config 2, N = 1e5, d = 4: 1.07-1.14 -> 1.04-1.11 ms
  // against the register kernel, interleaved, gpurun_out/r04aq).
  const int lds2g =
      D <= 8 ? tuning_knob(kKnobKdeMfmaLds2, npad >= (int64_t{1} << 16) ? 3 : 0) : 0;
  int ib = lds2g == 1 ? ib2 : ibf;
  const int v = tuning_knob(kKnobKdeMfmaIb, ib);
  if (v == ibf || v == ibh || v == ib2) ib = v;
  // segment-major block order on large populations (the A fragments no
  // longer fit the L2s; ABC_KDE_MFMA_SMAJOR overrides, rows bit-identical)
  const bool smajor =
      tuning_knob(kKnobKdeMfmaSmajor, npad >= (int64_t{1} << 18) ? 1 : 0) != 0;
  const MPlan p = make_mplan<D>(M, npad, ib, smajor);
  const size_t need = mfma_ws_layout<D>(M, p.nseg, nullptr, nullptr);
  ABC_REQUIRE(ws_bytes >= need, "kde_mfma: workspace too small (%zu < %zu)",
              ws_bytes, need);
  MfmaWs w;
  mfma_ws_layout<D>(M, p.nseg, static_cast<char*>(ws), &w);
  ABC_HIP(hipMemsetAsync(w.cnt, 0, 64, st));
  if (ib == IBF)
    launch_mfma<D, IBF>(p, Bfr, M, Afr, npad, w.partial, lds2g, st);
  else if (ib == IB2)
    launch_mfma<D, IB2>(p, Bfr, M, Afr, npad, w.partial, lds2g, st);
  else if (ib == IBH)
    launch_mfma<D, IBH>(p, Bfr, M, Afr, npad, w.partial, lds2g, st);
  else if constexpr (kIbBySize<D>) {
    if (ib == 3)
      launch_mfma<D, 3>(p, Bfr, M, Afr, npad, w.partial, lds2g, st);
    else
      launch_mfma<D, 1>(p, Bfr, M, Afr, npad, w.partial, lds2g, st);
  }
  ABC_LAUNCH_CHECK("kde_mfma_kernel");
  const unsigned gm = static_cast<unsigned>(ceil_div(M, 256));
  const unsigned gl = stream_grid(M, 256, 1024);
  // the folded scheme's routing bound with or without the grid: without it
  // (the legacy abc_kde_logpdf_mfma) the flagged rows go straight to the
  // fp64 fixup -- the same 1e-5 contract, only the cost differs (round 6,
  // the 2^-32 of rounds 1-4 left derived bounds of 1.27e-5 at
  // d = 8 and 2.9e-5 at d = 20 on this entry)
  const double lo = Route<D>::lo;
  const double phi = parent_window();
  hipLaunchKernelGGL(mfma_finalize_kernel, dim3(gm), dim3(256), 0, st, w.partial,
                     M, p.nseg, row_off, lw2max, log_const, lo, 1.0 / phi, phi,
                     out, w.cnt, w.rows1, w.s1);
  hipLaunchKernelGGL(refine_classify_kernel<D>, dim3(gl), dim3(256), 0, st, w.cnt,
                     w.rows1, w.s1, row_off, Ynew, gscale, w.rows2, w.m2, w.rowsx,
                     w.mxo, w.rows3, w.Bbuf);
  ABC_LAUNCH_CHECK("kde_mfma refine classify");
  launch_list<D, 1>(w.Bbuf, w.cnt + 3, M, Afr, npad, p.nseg, p.jseg, w.partial, st);
  ABC_LAUNCH_CHECK("kde_mfma_list_kernel (max)");
  hipLaunchKernelGGL(refine_after_max_kernel, dim3(gl), dim3(256), 0, st, w.cnt,
                     w.rowsx, w.mxo, w.partial, M, p.nseg, w.rows2, w.m2, w.rows3);
  hipLaunchKernelGGL(refine_pack_kernel<D>, dim3(gl), dim3(256), 0, st, w.cnt,
                     w.rows2, w.m2, Ynew, gscale, w.Bbuf);
  ABC_LAUNCH_CHECK("kde_mfma refine pack");
  launch_list<D, 0>(w.Bbuf, w.cnt + 2, M, Afr, npad, p.nseg, p.jseg, w.partial, st);
  ABC_LAUNCH_CHECK("kde_mfma_list_kernel (sum)");
  hipLaunchKernelGGL(refine_finalize_kernel, dim3(gl), dim3(256), 0, st, w.cnt,
                     w.rows2, w.m2, w.partial, M, p.nseg, lw2max, log_const, out,
                     w.rows3);
  ABC_LAUNCH_CHECK("kde_mfma refine finalize");
  return kde_fixup_rows_mfma(Ynew, P, npad, d, lw2max, log_const, w.cnt, w.rows3,
                             out, st);
}

}  // namespace

size_t kde_mfma_ws_bytes(int64_t M, int64_t npad, int d) {
  const int nseg = kde_num_segments(npad);
  switch (kde_padded_dim(d)) {
#define CASE(DD) \
  case DD: return mfma_ws_layout<DD>(M, nseg, nullptr, nullptr);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default: return 0;
  }
}
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
    hipLaunchKernelGGL((ymax_kernel<DD>), dim3(ceil_div(n > 0 ? n : 1, 256)),  \
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

int abc_kde_pack_new_mfma_rows(const double* theta, int64_t M, int d,
                               const double* mu, const double* Us,
                               const double* gscale, const double* P,
                               int64_t npad, const int64_t* parent,
                               double* Ynew, void* Bfr, double* row_off,
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
  ABC_REQUIRE(!parent || (P && npad > 0),
              "pack_new_mfma: parents need the packed population P");
  const int64_t mp = mpad_for(d, M);
  const unsigned gr = static_cast<unsigned>(ceil_div(mp, 256));
  const double pshift = parent_shift();
  switch (D) {
#define CASE(DD)                                                              \
  case DD:                                                                    \
    hipLaunchKernelGGL((pack_new_frag_kernel<DD>), dim3(gr), dim3(256), 0, st, \
                       theta, M, mp, d, mu, Us, gscale, P, npad, parent,     \
                       pshift, Ynew, row_off, static_cast<bf16x8*>(Bfr));    \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
  }
  ABC_LAUNCH_CHECK("pack_new_frag_kernel");
  return kOk;
}

int abc_kde_pack_new_mfma(const double* theta, int64_t M, int d,
                          const double* mu, const double* Us,
                          const double* gscale, double* Ynew, void* Bfr,
                          hipStream_t st) {
  return abc_kde_pack_new_mfma_rows(theta, M, d, mu, Us, gscale, nullptr, 0,
                                    nullptr, Ynew, Bfr, nullptr, st);
}

static int logpdf_mfma_entry(const void* Bfr, const double* Ynew,
                             const double* row_off, int64_t M, const void* Afr,
                             const double* P, int64_t npad, int d,
                             const double* lw2max, const double* gscale,
                             double log_const, double* out_logpd, void* ws,
                             size_t ws_bytes, hipStream_t st) {
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
#define CASE(DD)                                                               \
  case DD:                                                                     \
    return logpdf_mfma_impl<DD>(B, Ynew, row_off, M, A, P, npad, d, lw2max,    \
                                gscale, log_const, out_logpd, ws, ws_bytes, st);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(6) CASE(8) CASE(12) CASE(16)
    CASE(20) CASE(24) CASE(32)
#undef CASE
    default:
      set_error("kde_mfma: unsupported dimension d=%d (max 32)", d);
      return kUnsupported;
  }
}

int abc_kde_logpdf_mfma(const void* Bfr, const double* Ynew, int64_t M,
                        const void* Afr, const double* P, int64_t npad, int d,
                        const double* lw2max, double log_const,
                        double* out_logpd, void* ws, size_t ws_bytes,
                        hipStream_t st) {
  return logpdf_mfma_entry(Bfr, Ynew, nullptr, M, Afr, P, npad, d, lw2max,
                           nullptr, log_const, out_logpd, ws, ws_bytes, st);
}

int abc_kde_logpdf_mfma_rows(const void* Bfr, const double* Ynew,
                             const double* row_off, int64_t M, const void* Afr,
                             const double* P, int64_t npad, int d,
                             const double* lw2max, const double* gscale,
                             double log_const, double* out_logpd, void* ws,
                             size_t ws_bytes, hipStream_t st) {
  ABC_REQUIRE(gscale, "kde_mfma: null grid");
  return logpdf_mfma_entry(Bfr, Ynew, row_off, M, Afr, P, npad, d, lw2max,
                           gscale, log_const, out_logpd, ws, ws_bytes, st);
}

}  // extern "C"

namespace abc {
// Loads this translation unit's code object (HIP loads each one lazily, at
// the first launch of one of its kernels: ~4 ms for local_mfma's inside
// C4's first weighted generation); abc_preload calls every unit's hook.
int preload_kde_mfma() { return preload_kernel(ymax_kernel<8>); }
}  // namespace abc
