// LocalTransition density on the matrix cores (reference:
// pyabc/transition/local_transition.py:103-110):
//   pdf(theta) = sum_n w_n N(theta; X_n, C_n) / sum w
//
// "z form": with P_n = C_n^-1 = L_n L_n^T (Cholesky, L lower),
//   q_n(theta) = |z_n|^2,  z_na = sum_b L_ba (theta_b - X_nb)
// is a GEMM of the [N * d, d] matrix of the L_n columns with the [d, M]
// matrix of evaluation points -- on the f16 matrix cores -- followed per pair
// by d squares, one exp and one add on the VALU (the pair loop of
// local_pdf32.hip spends 47 packed instructions per two pairs on the
// symmetric form instead).
//
// Exactness (as the MVN pass, kde_mfma.hip): every operand is split into
// f16 pieces so that the large part of z is exact in the fp32 accumulator.
//  * coordinates: u' = (x - X_0) 2^s_b per dimension (powers of two putting
//    the population's |x'_b| below 1), then u' = t1 + r on the grid
//    g = 2^-8 (|t1 / g| <= 2048 for |u'| <= 7.9; rows beyond take the exact
//    fixup), r -> r2 = f16(r 2^12), r3 = f16((r - r2) 2^12);
//  * columns: l = L_{.a} 2^-s_b sqrt(log2(e)/2) 2^F_n (q in log2 units; F_n
//    a per-particle power of two putting the largest column norm at 2^11),
//    l = l1 + l2 + l3 with l1 on the grid G_a = 2^(e_a - 11) of its norm
//    (|l1 / G_a| <= 2048), l2, l3 = f16 pieces of the rest x 2^12;
//  * hi = sum_b l1_b (t1_b 2^12) - kappa1 2^12, kappa1 = l1 . x1 (x1 the
//    particle on the grid g): multiples of G_a g 2^12 whose absolute sum
//    is below 2^23 of them (Cauchy-Schwarz: 2048 * 2048 + 2^20.5), so the
//    fp32 accumulation is exact in any order;
//  * lo (x 2^12): l1.r2, l1.r3, l2.t1, l3.t1, l2.r2 (2^6 per side) per
//    dimension, minus kappa_lo = l1.(x' - x1) + (l2 + l3).x' -- on top of
//    hi in the same accumulator (the MVN pass's folded form), so the MFMA
//    delivers acc = 2^(12 + F_n) z;
//  * q = 2^(-24 - 2 F_n) sum acc^2: e = fma(sum acc^2, cf_n, lc2_n) with the
//    per-particle cf_n = -2^(-24 - 2 F_n), lc2_n = (lc_n - max lc) log2(e).
// numpy emulation of this arithmetic (tools/probes/local_zform_emul.py):
// 4.6e-7 on rows drawn from the transition, 3.1e-6 on rows 3 local sigma
// out (log density -31); rows whose sum falls below 2^-32 take the exact
// fp64 fixup, as in the MVN pass.  A particle whose Cholesky fails, whose
// column norms span more than 2^16, or whose local bandwidth is below ~1/400
// of the population's extent (the pieces' precision floor) sets a flag that
// sends every row to the exact fp64 pass (correct, slower; C4's populations
// sit at ~1/16).
//
// Layout: 32-row MFMA tiles of (particle, component) rows, DP = 8 rows per
// particle for d = 5..8 (4 particles per tile, the rows placed so that each
// lane holds two particles whole: lz_row) and DP = 4
// for d <= 4 (8 particles per tile, a particle whole in one lane).  The
// particles stream through LDS (LDS-DMA, TPB = 4 particle tiles per buffer
// with their (lc2, cf) pairs, double buffered); each wave holds IB = 4
// 32-point tiles of the evaluation points in registers (128 VGPRs: four
// waves per SIMD).  The VALU stages of one (particle tile, point tile)
// product run in the MFMA gaps of the next ones (lz_kernel).  The particle
// range is cut into segments that depend on N only and each row's terms are
// summed in a fixed order (fp32 over 4 particle tiles, then fp64), so a
// row's bits do not depend on M, the launch shape or the number of ranks.
// N = M = 2e5, d = 6: 21 ms for the whole pass (35.7 ms fp32 pair loop),
// at the SIMD's issue bound.
#include <cmath>

#include "common.hpp"
#include "local_common.hpp"

// the fp64 pass's workspace (local.hip): logsumw, lc_max_key, n_fix | lc |
// coef | part[split][M] | fix_rows[M] -- shared by this pass
extern "C" size_t abc_local_logpdf_workspace_bytes(int64_t M, int64_t N);

namespace abc {
namespace {

typedef short h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#ifndef ABC_LZ_WAVES
#define ABC_LZ_WAVES 4
#endif
constexpr int kLzWaves = ABC_LZ_WAVES;  // waves per block sharing the LDS stream
constexpr double kLzGrid = 0.00390625;       // g = 2^-8
constexpr double kLzRowNorm = 7.9;           // |u'| bound of the grid
constexpr float kLzLo = 4096.0f;             // lo pieces x 2^12
constexpr float kLzHalf = 64.0f;             // l2.r2: 2^6 per side
constexpr int kLzTopE = 11;                  // largest column norm -> 2^11
constexpr int kLzMinE = -5;                  // smallest kept: 2^-5 (denormal floor)
constexpr int kLzMaxE = 9;                   // largest unscaled column norm 2^9
constexpr unsigned short kLzOne = 0x3C00;    // f16 1.0
constexpr unsigned short kLzHiPartner = 0x6C00;  // f16 4096.0
// rows whose term sum falls below this take the exact fp64 fixup
constexpr double kLzFixupSum = 2.3283064365386963e-10;  // 2^-32

constexpr int kLzUnitTiles = 8;  // particle tiles per segment unit
constexpr int kLzFlush = 4;      // particle tiles summed in fp32 per fp64 add
constexpr int kLzMaxIB = 4;      // point tiles per wave, largest

template <int D>
struct Lz {
  static constexpr int DP = D <= 4 ? 4 : 8;  // rows per particle
  static constexpr int PT = 32 / DP;         // particles per 32-row tile
  static constexpr int KL = (5 * D + 2 + 15) / 16;
  static constexpr int KT = 1 + KL;          // hi: D + 2 <= 10 slots
  static constexpr int IB = 4;               // point tiles per wave
  static constexpr int TPB = 4;              // particle tiles per LDS buffer
};

__device__ inline unsigned short h16(float x) {  // RNE
  return __builtin_bit_cast(unsigned short, static_cast<_Float16>(x));
}
__device__ inline float h16f(unsigned short b) {
  return static_cast<float>(__builtin_bit_cast(_Float16, b));
}

// largest |X_nb - X_0b| per dimension (ordered keys)
template <int D>
__global__ __launch_bounds__(256) void lz_dims_kernel(const double* __restrict__ X,
                                                      int64_t N,
                                                      unsigned long long* __restrict__ keys) {
  double m[D];
#pragma unroll
  for (int b = 0; b < D; ++b) m[b] = 0.0;
  for (int64_t n = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; n < N;
       n += static_cast<int64_t>(gridDim.x) * 256) {
#pragma unroll
    for (int b = 0; b < D; ++b) m[b] = fmax(m[b], fabs(X[n * D + b] - X[b]));
  }
#pragma unroll
  for (int b = 0; b < D; ++b) {
    block_atomic_max_u64<256>(&keys[b], static_cast<unsigned long long>(f64_key(m[b])));
    __syncthreads();
  }
}

// 2^s_b: the scale putting the population's |x'_b| below 1
__device__ inline double lz_dim_scale(const unsigned long long* keys, int b) {
  const double m = key_f64(keys[b]);
  int E = 0;
  if (m > 0.0) frexp(m, &E);  // m < 2^E
  return ldexp(1.0, -E);
}

// A-operand fragment of row r (of its 32-row tile) for chunk c: slot
// 16 c + 8 hh + e -> F[(tile * KT + c) * 64 + 32 hh + r]
template <int KT>
__device__ inline void lz_store_row(h16x8* __restrict__ F, int64_t tile, int r,
                                    const unsigned short (&v)[16 * KT]) {
#pragma unroll
  for (int c = 0; c < KT; ++c)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      h16x8 x;
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = static_cast<short>(v[16 * c + 8 * hh + e]);
      F[(tile * KT + c) * 64 + 32 * hh + r] = x;
    }
}

// Row of component a of tile particle p.  The accumulator holds row
// 8 (v >> 2) + 4 h + (v & 3) in lane half h, value v.  DP = 8: particle p
// takes groups 2 (p & 1), 2 (p & 1) + 1 of half p >> 1, so a lane holds
// particles 2h (values 0-7) and 2h + 1 (values 8-15) whole -- no exchange
// between the halves; DP = 4: rows 4 p .. 4 p + 3 (group p >> 1, half p & 1).
template <int DP>
__device__ __forceinline__ int lz_row(int p, int a) {
  if constexpr (DP == 8)
    return 8 * (2 * (p & 1) + (a >> 2)) + 4 * (p >> 1) + (a & 3);
  else
    return DP * p + a;
}

// One thread per particle: Cholesky of inv_n, the scaled columns, their
// pieces and the kappa constants -> DP rows of A fragments; (lc2, cf) in
// the lane order of the main kernel
template <int D>
__global__ __launch_bounds__(128) void lz_pack_prev_kernel(
    const double* __restrict__ X, const double* __restrict__ invs,
    const double* __restrict__ lc, const unsigned long long* __restrict__ lc_max_key,
    int64_t N, int64_t npad, const unsigned long long* __restrict__ dkeys,
    h16x8* __restrict__ A, float2* __restrict__ lcT, int* __restrict__ gflag) {
  using P = Lz<D>;
  constexpr int KT = P::KT, DP = P::DP, PT = P::PT;
  const int64_t n = static_cast<int64_t>(blockIdx.x) * 128 + threadIdx.x;
  if (n >= npad) return;
  const int64_t tile = n / PT;
  const int pin = static_cast<int>(n % PT);
  // lane order of (lc2, cf): DP = 8 natural; DP = 4 -> [4 h + k] = 2 k + h
  const int64_t lslot = tile * PT + (DP == 8 ? pin : (pin & 1) * 4 + (pin >> 1));
  unsigned short v[DP][16 * KT];
#pragma unroll
  for (int a = 0; a < DP; ++a)
#pragma unroll
    for (int k = 0; k < 16 * KT; ++k) v[a][k] = 0;
  bool ok = n < N;
  float2 lcv = make_float2(-INFINITY, 0.0f);
  if (ok) {
    double sc[D], xs[D], x1[D];
#pragma unroll
    for (int b = 0; b < D; ++b) {
      sc[b] = lz_dim_scale(dkeys, b);
      xs[b] = (X[n * D + b] - X[b]) * sc[b];
      x1[b] = rint(xs[b] / kLzGrid) * kLzGrid;
    }
    // Cholesky P = L L^T (row-major symmetric inv_n)
    double L[D][D];
    const double* Pn = invs + n * D * D;
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int j = 0; j < D; ++j) L[i][j] = 0.0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double s = Pn[j * D + j];
#pragma unroll
      for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
      ok = ok && s > 0.0;
      const double djj = s > 0.0 ? sqrt(s) : 1.0;
      L[j][j] = djj;
#pragma unroll
      for (int i = j + 1; i < D; ++i) {
        double t = 0.5 * (Pn[i * D + j] + Pn[j * D + i]);
#pragma unroll
        for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
        L[i][j] = t / djj;
      }
    }
    // scaled columns lhat_ba = L_ba 2^-s_b sqrt(log2 e / 2); their norms
    const double c = 0.84932180028801907;  // sqrt(log2(e) / 2)
    double lh[D][D];  // [a][b]
    int ea[D];
    int emax = -1000, emin = 1000;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      double nn = 0.0;
#pragma unroll
      for (int b = 0; b < D; ++b) {
        lh[a][b] = b >= a ? L[b][a] / sc[b] * c : 0.0;
        nn = fma(lh[a][b], lh[a][b], nn);
      }
      int E = 0;
      frexp(sqrt(nn), &E);  // |l| < 2^E
      ea[a] = nn > 0.0 ? E : -1000;
      if (nn > 0.0) {
        emax = ea[a] > emax ? ea[a] : emax;
        emin = ea[a] < emin ? ea[a] : emin;
      }
      ok = ok && nn > 0.0 && nn == nn;
    }
    // precision: the pieces hold u' to 2^-31 (22 bits below g / 2), so
    // |l| must stay below 2^9 (z to ~2e-7; in the scaled coordinates the
    // column norm is ~ 1 / (local sigma / population extent)): a population
    // wider than ~400 local bandwidths takes the exact path
    ok = ok && emax <= kLzMaxE;
    const int F = kLzTopE - emax;
    ok = ok && emin + F >= kLzMinE;
    if (ok) {
#pragma unroll
      for (int a = 0; a < D; ++a) {
        const double G = ldexp(1.0, ea[a] + F - kLzTopE);
        double l1[D], l2v[D], l3v[D];
        double k1 = 0.0, klo = 0.0;
#pragma unroll
        for (int b = 0; b < D; ++b) {
          const double l = ldexp(lh[a][b], F);
          l1[b] = rint(l / G) * G;
          const unsigned short p2 = h16(static_cast<float>((l - l1[b]) * kLzLo));
          l2v[b] = static_cast<double>(h16f(p2)) / kLzLo;
          const unsigned short p3 =
              h16(static_cast<float>((l - l1[b] - l2v[b]) * kLzLo));
          l3v[b] = static_cast<double>(h16f(p3)) / kLzLo;
          const unsigned short ph = h16(static_cast<float>(l2v[b] * kLzHalf));
          // hi slot b: l1 | t1 2^12
          v[a][b] = h16(static_cast<float>(l1[b]));
          // lo slots 5 b + q
          v[a][16 + 5 * b + 0] = v[a][b];  // l1 | r2
          v[a][16 + 5 * b + 1] = v[a][b];  // l1 | r3
          v[a][16 + 5 * b + 2] = p2;       // l2 2^12 | t1
          v[a][16 + 5 * b + 3] = p3;       // l3 2^12 | t1
          v[a][16 + 5 * b + 4] = ph;       // l2 2^6 | r2 2^6
          k1 = fma(l1[b], x1[b], k1);      // exact (multiples of G g)
          klo += l1[b] * (xs[b] - x1[b]) + (l2v[b] + l3v[b]) * xs[b];
        }
        // -kappa1 in two f16 pieces (K = kappa1 / (G g) < 2^21: 11 + 11 bits)
        const double Gg = G * kLzGrid;
        const double K = rint(k1 / Gg);
        const double K0 = trunc(K / 2048.0) * 2048.0;
        v[a][D] = h16(static_cast<float>(-K0 * Gg));
        v[a][D + 1] = h16(static_cast<float>(-(K - K0) * Gg));
        // -kappa_lo x 2^12 in two pieces
        const double kl = -klo * kLzLo;
        const unsigned short q0 = h16(static_cast<float>(kl));
        v[a][16 + 5 * D] = q0;
        v[a][16 + 5 * D + 1] = h16(static_cast<float>(kl - static_cast<double>(h16f(q0))));
      }
      const double L0 = key_f64(*lc_max_key);
      lcv = make_float2(static_cast<float>((lc[n] - L0) * 1.4426950408889634),
                        -ldexpf(1.0f, -24 - 2 * F));
    } else {
      atomicOr(gflag, 1);
    }
  }
#pragma unroll
  for (int a = 0; a < DP; ++a) lz_store_row<KT>(A, tile, lz_row<DP>(pin, a), v[a]);
  lcT[lslot] = lcv;
}

// One thread per evaluation point: its pieces in B-operand order
template <int D>
__global__ __launch_bounds__(256) void lz_pack_new_kernel(
    const double* __restrict__ pts, int64_t M, int64_t mpad,
    const double* __restrict__ X, const unsigned long long* __restrict__ dkeys,
    h16x8* __restrict__ B, int* __restrict__ rflag) {
  constexpr int KT = Lz<D>::KT;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= mpad) return;
  unsigned short v[16 * KT];
#pragma unroll
  for (int k = 0; k < 16 * KT; ++k) v[k] = 0;
  bool ok = i < M;
  double us[D];
  if (ok) {
    double nn = 0.0;
#pragma unroll
    for (int b = 0; b < D; ++b) {
      us[b] = (pts[i * D + b] - X[b]) * lz_dim_scale(dkeys, b);
      nn = fma(us[b], us[b], nn);
    }
    ok = sqrt(nn) <= kLzRowNorm;  // NaN -> false
  }
  if (ok) {
#pragma unroll
    for (int b = 0; b < D; ++b) {
      const double t1 = rint(us[b] / kLzGrid) * kLzGrid;
      const double r = us[b] - t1;
      const unsigned short r2 = h16(static_cast<float>(r * kLzLo));
      const double r2v = static_cast<double>(h16f(r2)) / kLzLo;
      const unsigned short r3 = h16(static_cast<float>((r - r2v) * kLzLo));
      const unsigned short t1b = h16(static_cast<float>(t1));
      v[b] = h16(static_cast<float>(t1 * kLzLo));  // exact: |t1| < 8
      v[16 + 5 * b + 0] = r2;
      v[16 + 5 * b + 1] = r3;
      v[16 + 5 * b + 2] = t1b;
      v[16 + 5 * b + 3] = t1b;
      v[16 + 5 * b + 4] = h16(static_cast<float>(r2v * kLzHalf));
    }
    v[D] = v[D + 1] = kLzHiPartner;
    v[16 + 5 * D] = v[16 + 5 * D + 1] = kLzOne;
  }
  if (i < M) rflag[i] = ok ? 0 : 1;
  const int64_t tile = i >> 5;
  const int r = static_cast<int>(i & 31);
#pragma unroll
  for (int c = 0; c < KT; ++c)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      h16x8 x;
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = static_cast<short>(v[16 * c + 8 * hh + e]);
      B[(tile * KT + c) * 64 + 32 * hh + r] = x;
    }
}

__device__ __forceinline__ f32x16 lz_mfma(const h16x8& a, const h16x8& b,
                                          const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                __builtin_bit_cast(f16x8, b), c, 0,
                                                0, 0);
}

// The terms of one (particle tile, point tile) for this lane's point, in
// three stages so the kernel can place them between the MFMAs of the next
// product: stages 0, 1 the squares of particle group G (DP = 8: particle
// 2h + G, values 8G .. 8G + 7, whole by lz_row; DP = 4: particles 2 (2G) + h
// and 2 (2G + 1) + h, values 4k .. 4k + 3), only the D real components;
// stage 2 the 2 (DP = 8) or 4 (DP = 4) exps and their sum in a fixed order.
template <int D, int DP, int G>
__device__ __forceinline__ void lz_squares(const f32x16& acc, float (&q)[4]) {
  if constexpr (DP == 8) {
    float x = acc[8 * G] * acc[8 * G];
#pragma unroll
    for (int j = 1; j < D; ++j) x = __builtin_fmaf(acc[8 * G + j], acc[8 * G + j], x);
    q[G] = x;
  } else {
    float x = acc[8 * G] * acc[8 * G], y = acc[8 * G + 4] * acc[8 * G + 4];
#pragma unroll
    for (int j = 1; j < D; ++j) {
      x = __builtin_fmaf(acc[8 * G + j], acc[8 * G + j], x);
      y = __builtin_fmaf(acc[8 * G + 4 + j], acc[8 * G + 4 + j], y);
    }
    q[2 * G] = x;
    q[2 * G + 1] = y;
  }
}
template <int DP>
__device__ __forceinline__ float lz_exps(const float (&q)[4], const float2* lcp) {
  if constexpr (DP == 8) {
    const float t0 = __builtin_amdgcn_exp2f(__builtin_fmaf(q[0], lcp[0].y, lcp[0].x));
    const float t1 = __builtin_amdgcn_exp2f(__builtin_fmaf(q[1], lcp[1].y, lcp[1].x));
    return t0 + t1;
  } else {
    float t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      t[k] = __builtin_amdgcn_exp2f(__builtin_fmaf(q[k], lcp[k].y, lcp[k].x));
    return (t[0] + t[1]) + (t[2] + t[3]);
  }
}
// Block (segment s, row block rb), segment major; wave w owns point tiles
// (rb * kLzWaves + w) * IB ...  Per segment one fp64 partial per point; the
// fp32 terms are flushed into it every kLzFlush particle tiles whatever TPB (the
// particle tiles per LDS buffer) and IB, so a row's bits do not depend on
// either (tuning knobs ABC_LZ_IB, ABC_LZ_TPB).
template <int D, int IB, int TPB>
__global__ __launch_bounds__(64 * kLzWaves) void lz_kernel(
    const h16x8* __restrict__ Bfr, int64_t M, const h16x8* __restrict__ Afr,
    const float2* __restrict__ lcT, int64_t npad, int nseg, int64_t seg_len,
    const int* __restrict__ gflag, double* __restrict__ part) {
  using P = Lz<D>;
  constexpr int KT = P::KT, PT = P::PT, DP = P::DP;
  constexpr int CH = TPB * KT;  // fragments per LDS buffer
  constexpr int NL = DP == 8 ? 2 : 4;
  static_assert(TPB % 2 == 0 && kLzUnitTiles % TPB == 0, "TPB: 2, 4 or 8");
  constexpr int LCF = TPB * PT * 2;  // lc floats per buffer (64 or more)
  __shared__ h16x8 As[2][CH][64];
  // (lc2, cf) of the buffer's TPB PT particles, DMA'd with it
  __shared__ float Lc[2][LCF < 64 ? 64 : LCF];
  if (*gflag) return;  // every row takes the exact fixup
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nrb = gridDim.x / nseg;
  const int s = static_cast<int>(blockIdx.x / nrb);
  const int64_t rb = blockIdx.x % nrb;
  const int64_t t0 = (rb * kLzWaves + wave) * IB;
  const int h = lane >> 5;
  h16x8 bq[IB][KT];
#pragma unroll
  for (int t = 0; t < IB; ++t)
#pragma unroll
    for (int c = 0; c < KT; ++c) bq[t][c] = Bfr[((t0 + t) * KT + c) * 64 + lane];
  const int64_t p0 = static_cast<int64_t>(s) * seg_len;
  int64_t p1 = p0 + seg_len;
  if (p1 > npad) p1 = npad;
  const int64_t tile0 = p0 / PT, ntile = (p1 - p0) / PT;  // a multiple of TPB
  const h16x8* __restrict__ Aseg = Afr + tile0 * KT * 64;
  const float* __restrict__ Lseg = reinterpret_cast<const float*>(lcT + tile0 * PT);
  auto fill = [&](int buf, int64_t tl) {
    const h16x8* __restrict__ src = Aseg + tl * KT * 64;
    for (int f = wave; f < CH; f += kLzWaves)
      __builtin_amdgcn_global_load_lds(
          src + f * 64 + lane, (__attribute__((address_space(3))) void*)&As[buf][f][0],
          16, 0, 0);
    // one dword per lane and piece of 64; lcT carries 512 bytes of slack
    if (wave == kLzWaves - 1)
#pragma unroll
      for (int pc = 0; pc < (LCF + 63) / 64; ++pc)
        __builtin_amdgcn_global_load_lds(
            Lseg + tl * PT * 2 + 64 * pc + lane,
            (__attribute__((address_space(3))) void*)&Lc[buf][64 * pc], 4, 0, 0);
  };
  double S[IB];
  float sacc[IB];
#pragma unroll
  for (int t = 0; t < IB; ++t) S[t] = 0.0;
  if (ntile > 0) fill(0, 0);
  int buf = 0;
  for (int64_t tl = 0; tl < ntile; tl += TPB) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tl + TPB < ntile) fill(buf ^ 1, tl + TPB);
    const float2* __restrict__ Lb = reinterpret_cast<const float2*>(&Lc[buf][0]);
    // A fragments of particle tile u, read one product before their first
    // MFMA (a ring of two)
    h16x8 a[2][KT];
#pragma unroll
    for (int c = 0; c < KT; ++c) a[0][c] = As[buf][c][lane];
    // the TPB IB (particle tile, point tile) products of this buffer,
    // software pipelined: stage s of product p runs in MFMA gap
    // KT (p + 1) + 1 + s (counting gaps over the products), i.e. from the
    // second MFMA of product p + 1 on -- its accumulator has landed by then
    // (hand-placed; an MFMA holds the vector issue for 8 of its 32 cycles,
    // MI355X_MICROARCH.md)
    constexpr int NQ = TPB * IB;
    f32x16 acc[3];
    float qv[2][4];
#pragma unroll
    for (int q = 0; q < NQ + 3; ++q) {
      if (q < NQ) acc[q % 3] = f32x16{};
#pragma unroll
      for (int c = 0; c < KT; ++c) {
        if (q < NQ) acc[q % 3] = lz_mfma(a[(q / IB) & 1][c], bq[q % IB][c], acc[q % 3]);
        __builtin_amdgcn_sched_barrier(0);
        // the next particle tile's fragments, one product ahead
        if (c == 0 && q % IB == IB - 1 && q / IB + 1 < TPB) {
          const int un = q / IB + 1;
#pragma unroll
          for (int cc = 0; cc < KT; ++cc) a[un & 1][cc] = As[buf][un * KT + cc][lane];
        }
        // the stages due in this gap, older products first
#pragma unroll
        for (int st = 2; st >= 0; --st) {
          const int pos = KT * q + c - 1 - st;  // = KT (p + 1) for stage st of p
          if (pos < 0 || pos % KT != 0) continue;
          const int p = pos / KT - 1;
          if (p < 0 || p >= NQ) continue;
          const int u = p / IB, t = p % IB;
          if (st == 0) {
            // the accumulator stays allocated whole until here: its unread
            // padding values must not be reused as temporaries while the
            // MFMA that writes them is in flight (a write-after-write
            // hazard the compiler pads with s_nop)
            asm volatile("" ::"v"(acc[p % 3]));
            lz_squares<D, DP, 0>(acc[p % 3], qv[p & 1]);
          }
          if (st == 1) lz_squares<D, DP, 1>(acc[p % 3], qv[p & 1]);
          if (st == 2) {
            float2 lcv[NL];
#pragma unroll
            for (int k = 0; k < NL; ++k) lcv[k] = Lb[u * PT + (DP == 8 ? 2 * h : 4 * h) + k];
            const float v = lz_exps<DP>(qv[p & 1], lcv);
            // fp32 over kLzFlush consecutive particle tiles, then into fp64
            const int tg = TPB % kLzFlush == 0 ? u % kLzFlush
                                               : static_cast<int>((tl + u) % kLzFlush);
            sacc[t] = tg == 0 ? v : sacc[t] + v;
            if (tg == kLzFlush - 1) S[t] += static_cast<double>(sacc[t]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    buf ^= 1;
  }
#pragma unroll
  for (int t = 0; t < IB; ++t) {
    const double tot = S[t] + __shfl_xor(S[t], 32, 64);
    const int64_t i = (t0 + t) * 32 + lane;
    if (lane < 32 && i < M) part[static_cast<int64_t>(s) * M + i] = tot;
  }
}

__global__ __launch_bounds__(256) void lz_final_kernel(
    const double* __restrict__ part, int64_t M, int nseg,
    const unsigned long long* __restrict__ lc_max_key,
    const double* __restrict__ logsumw, const int* __restrict__ gflag,
    const int* __restrict__ rflag, double* __restrict__ out,
    int* __restrict__ n_fix, int* __restrict__ fix_rows) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= M) return;
  double S = 0.0;
  for (int s = 0; s < nseg; ++s) S += part[s * M + i];
  if (!*gflag && !rflag[i] && S >= kLzFixupSum) {
    out[i] = key_f64(*lc_max_key) + log(S) - *logsumw;
  } else {
    fix_rows[atomicAdd(n_fix, 1)] = static_cast<int>(i);
    out[i] = -INFINITY;
  }
}

struct LzPlan {
  int64_t npad, mpad, seg_len;
  int nseg;
  size_t a_bytes, b_bytes, lc_bytes;
};

template <int D>
LzPlan lz_plan(int64_t M, int64_t N) {
  using P = Lz<D>;
  LzPlan p;
  int split;
  int64_t nchunk;
  local_plan(M, N, split, nchunk);
  const int64_t unit = kLzUnitTiles * P::PT;  // any LDS buffer size divides it
  p.seg_len = ceil_div(nchunk, unit) * unit;
  p.npad = ceil_div(N, unit) * unit;
  p.nseg = static_cast<int>(ceil_div(p.npad, p.seg_len));
  const int64_t rows = 32 * kLzWaves * kLzMaxIB;  // every IB divides it
  p.mpad = ceil_div(M, rows) * rows;
  p.a_bytes = static_cast<size_t>(p.npad / P::PT) * P::KT * 64 * 16;
  p.b_bytes = static_cast<size_t>(p.mpad / 32) * P::KT * 64 * 16;
  p.lc_bytes = static_cast<size_t>(p.npad) * 8 + 512;  // + the DMA's slack
  return p;
}

size_t lz_extra_bytes(int64_t M, int64_t N, int d) {
  LzPlan p{};
  switch (d) {
#define C(DD) \
  case DD: p = lz_plan<DD>(M, N); break;
    C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8)
#undef C
    default: return 0;
  }
  // dims keys (64) + flag (64) + rflag[M] + lcT + A + B, 256-aligned pieces
  return 128 + static_cast<size_t>(M) * 4 + 256 + p.lc_bytes + 256 + p.a_bytes +
         256 + p.b_bytes + 256;
}

template <int D>
int lz_run(const double* pts, int64_t M, const double* X, const double* w,
           const double* invs, const double* dets, int64_t N, double* out,
           void* ws, hipStream_t st) {
  const LzPlan p = lz_plan<D>(M, N);
  char* base = static_cast<char*>(ws);
  double* logsumw = reinterpret_cast<double*>(base);
  unsigned long long* lc_max_key = reinterpret_cast<unsigned long long*>(base + 8);
  int* n_fix = reinterpret_cast<int*>(base + 16);
  double* lc = reinterpret_cast<double*>(base + 64);
  double* coef = lc + N;
  double* part = coef + N * 36;
  int split;
  int64_t nchunk;
  local_plan(M, N, split, nchunk);
  int* fix_rows = reinterpret_cast<int*>(part + static_cast<int64_t>(split) * M);
  char* ex = base + ((abc_local_logpdf_workspace_bytes(M, N) + 255) / 256) * 256;
  unsigned long long* dkeys = reinterpret_cast<unsigned long long*>(ex);
  int* gflag = reinterpret_cast<int*>(ex + 64);
  int* rflag = reinterpret_cast<int*>(ex + 128);
  char* q = ex + 128 + ((static_cast<size_t>(M) * 4 + 255) / 256) * 256;
  float2* lcT = reinterpret_cast<float2*>(q);
  q += ((p.lc_bytes + 255) / 256) * 256;
  h16x8* A = reinterpret_cast<h16x8*>(q);
  q += ((p.a_bytes + 255) / 256) * 256;
  h16x8* B = reinterpret_cast<h16x8*>(q);
  ABC_HIP(hipMemsetAsync(base + 8, 0, 16, st));
  ABC_HIP(hipMemsetAsync(ex, 0, 128, st));
  local_sumw(w, N, split, part, logsumw, st);
  // the packed coefficients only for fixup rows (local_coef_kernel below)
  hipLaunchKernelGGL(local_const_kernel, dim3(ceil_div(N, 256)), dim3(256), 0, st,
                     w, dets, invs, N, D, lc, static_cast<double*>(nullptr), lc_max_key);
  hipLaunchKernelGGL(lz_dims_kernel<D>, dim3(stream_grid(N, 256, 512)), dim3(256),
                     0, st, X, N, dkeys);
  hipLaunchKernelGGL(lz_pack_prev_kernel<D>, dim3(ceil_div(p.npad, 128)), dim3(128),
                     0, st, X, invs, lc, lc_max_key, N, p.npad, dkeys, A, lcT, gflag);
  hipLaunchKernelGGL(lz_pack_new_kernel<D>, dim3(ceil_div(p.mpad, 256)), dim3(256),
                     0, st, pts, M, p.mpad, X, dkeys, B, rflag);
  // point tiles per wave and particle tiles per LDS buffer: defaults, or
  // the tuning knobs (rows bit-identical)
  int ib = Lz<D>::IB, tpb = Lz<D>::TPB;
  {
    const int v = tuning_knob(kKnobLzIb, ib);
    if (v == 1 || v == 2 || v == 4) ib = v;
  }
  {
    const int v = tuning_knob(kKnobLzTpb, tpb);
    if (v == 2 || v == 4 || v == 8) tpb = v;
  }
  const unsigned grid =
      static_cast<unsigned>(p.mpad / (32 * kLzWaves * ib) * p.nseg);
#define LZ_LAUNCH(IBV, TPBV)                                                          \
  hipLaunchKernelGGL((lz_kernel<D, IBV, TPBV>), dim3(grid), dim3(64 * kLzWaves), 0, st, \
                     B, M, A, lcT, p.npad, p.nseg, p.seg_len, gflag, part)
  if (tpb == 2) {
    if (ib == 4) LZ_LAUNCH(4, 2); else if (ib == 2) LZ_LAUNCH(2, 2); else LZ_LAUNCH(1, 2);
  } else if (tpb == 4) {
    if (ib == 4) LZ_LAUNCH(4, 4); else if (ib == 2) LZ_LAUNCH(2, 4); else LZ_LAUNCH(1, 4);
  } else {
    if (ib == 4) LZ_LAUNCH(4, 8); else if (ib == 2) LZ_LAUNCH(2, 8); else LZ_LAUNCH(1, 8);
  }
#undef LZ_LAUNCH
  hipLaunchKernelGGL(lz_final_kernel, dim3(ceil_div(M, 256)), dim3(256), 0, st, part,
                     M, p.nseg, lc_max_key, logsumw, gflag, rflag, out, n_fix,
                     fix_rows);
  hipLaunchKernelGGL(local_coef_kernel, dim3(ceil_div(N, 256)), dim3(256), 0, st, invs,
                     N, D, coef, n_fix);
  hipLaunchKernelGGL(local_pdf_fixup_kernel<D>, dim3(1024), dim3(256), 0, st, pts, X,
                     coef, lc, N, logsumw, n_fix, fix_rows, out);
  return kOk;
}

}  // namespace
}  // namespace abc

using namespace abc;

extern "C" {

size_t abc_local_logpdf_mfma_workspace_bytes(int64_t M, int64_t N, int d) {
  if (M < 1) M = 1;
  if (N < 1) N = 1;
  return ((abc_local_logpdf_workspace_bytes(M, N) + 255) / 256) * 256 +
         lz_extra_bytes(M, N, d);
}

int abc_local_logpdf_mfma(const double* pts, int64_t M, const double* X,
                          const double* w, const double* inv_covs,
                          const double* dets, int64_t N, int d,
                          double* out_logpdf, void* ws, size_t ws_bytes,
                          hipStream_t st) {
  ABC_REQUIRE(M >= 0 && N >= 1, "local_logpdf_mfma: bad sizes");
  if (M == 0) return kOk;
  ABC_REQUIRE(d >= 1 && d <= 8, "local_logpdf_mfma: unsupported d=%d (d <= 8)", d);
  ABC_REQUIRE(pts && X && w && inv_covs && dets && out_logpdf && ws,
              "local_logpdf_mfma: null pointer");
  ABC_REQUIRE(ws_bytes >= abc_local_logpdf_mfma_workspace_bytes(M, N, d),
              "local_logpdf_mfma: workspace too small");
  int rc = kOk;
  switch (d) {
#define C(DD)                                                                  \
  case DD:                                                                     \
    rc = lz_run<DD>(pts, M, X, w, inv_covs, dets, N, out_logpdf, ws, st);      \
    break;
    C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8)
#undef C
  }
  if (rc != kOk) return rc;
  ABC_LAUNCH_CHECK("local_logpdf_mfma kernels");
  return kOk;
}

}  // extern "C"

namespace abc {
// Loads this translation unit's code object (HIP loads each one lazily, at
// the first launch of one of its kernels: ~4 ms for local_mfma's inside
// C4's first weighted generation); abc_preload calls every unit's hook.
int preload_local_mfma() { return preload_kernel(local_sumw_part_kernel); }
}  // namespace abc
