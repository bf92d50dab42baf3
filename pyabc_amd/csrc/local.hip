// LocalTransition (reference: pyabc/transition/local_transition.py:13-145):
//   fit:  nbr = cKDTree(X).query(X, k+1)[:, 1:]                       (:82-83)
//         C_n = np.cov(X[nbr_n] - X_n, aweights = w[nbr_n]/sum) * scaling
//         (|sum C| == 0 -> C_kk = |X_0k|); while det(C) <= 0: C += 1e-3 I
//         inv_n = inv(C_n), det_n                                     (:112-139)
//   pdf:  sum_n w_n exp(-q_n/2) / sqrt((2 pi)^d det_n) / sum w,
//         q_n = (theta - X_n)^T inv_n (theta - X_n)                   (:103-110)
//
// kNN: one wave per 8 rows streams every candidate through a provably safe
// packed-fp32 filter; passing candidates' indices go to a per-row LDS
// buffer that is re-ranked by EXACT fp64 squared distance (sequential over
// dimensions, no FMA contraction, as the reference tree computes them) in
// registers and cut back to k, setting the pruning threshold tau.
// cov/det/inv: 8 lanes per particle for the weighted moments of the k
// neighbour deltas, then LU with partial pivoting for det and inverse (fp64).
// pdf: one thread per evaluation point; the previous population's
// (X_n, packed symmetric inv_n, log(w_n / norm_n)) stream through the scalar
// path (wave-uniform), d(d+1)/2 + d FMAs per pair for the quadratic form,
// fp64 terms under one global offset, exact fixup for underflowing rows.
#include "common.hpp"
#include "philox.hpp"
#include "spatial.hpp"
#include "local_common.hpp"

namespace abc {


// 1: the wave's query rows are held in VGPRs (uniform, the compiler put
// them in SGPRs and the kernel sat at 100 SGPRs, spilling to VGPR lanes):
// knn 4.10 -> 3.93 ms at C4's shape, interleaved (gpurun_out/r05ax)
#ifndef ABC_KNN_XR_VGPR
#define ABC_KNN_XR_VGPR 1
#endif
constexpr int kKnnRows = 4;     // rows per wave (one wave per block; 8 before
                                // round 5: 7.6 -> 6.1 ms, tools/knn_ab.py)
constexpr int kMaxK = 192;      // k > 64: buffer of 256 = k kept + 64 appended

// Separately rounded fp64 ops: hipcc contracts a*b+c into an FMA by default
// (-ffp-contract=fast, and __dmul_rn/__dadd_rn are plain operators), so the
// pragma keeps the reference's sub / mul / add sequence.
__device__ inline double dsub(double a, double b) {
#pragma clang fp contract(off)
  return a - b;
}
__device__ inline double dadd(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ inline double dmul(double a, double b) {
#pragma clang fp contract(off)
  return a * b;
}

// fp32 filter of the kNN candidate test.  Coordinates are centred on X[0]
// and rounded to fp32 once (knn_prep_kernel, A = max |x - x0| in fp64); the
// filter distance d2f = sum fl32(xf_j - xf_i)^2 then satisfies
//   |d2f - d2| <= (d+2) 2^-24 d2 + 2^-22 A sqrt(d d2)
// so  d2 < tau  =>  d2f < T(tau) = tau (1 + (d+4) 2^-22) + 2^-20 A sqrt(d tau)
// (both terms 4x the bound), rounded up to fp32.  Only lanes passing the
// filter compute the exact fp64 distance (the reference's sub/mul/add
// sequence) and take the exact test d2 < tau, so the neighbour sets, their
// order and their distances are exactly those of the all-fp64 scan.
__device__ inline float knn_filter_bound(double tau, int d, double A) {
  if (!(tau < INFINITY)) return INFINITY;
  const double T = tau * (1.0 + (d + 4) * 0x1p-22) +
                   0x1p-20 * A * sqrt(static_cast<double>(d) * tau) + 1e-300;
  return __double2float_ru(T);
}

// Tiled prep (spatial.hpp): fp32 centred coordinates in Hilbert order (one
// wave per tile of 64 sorted positions, padding positions at kFar), the
// tile's bounding box of those fp32 values, and the coordinate bound A.
constexpr float kFar = 1e30f;  // (kFar - x)^2 overflows to +inf

template <int D>
__global__ __launch_bounds__(256) void knn_prep_kernel(
    const double* __restrict__ X, int64_t N, const int32_t* __restrict__ perm,
    int T, float* __restrict__ Xs, double* __restrict__ Xd,
    float* __restrict__ tbox, unsigned long long* __restrict__ amax) {
  const int lane = threadIdx.x & 63;
  const int t = static_cast<int>((static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) >> 6);
  const int64_t s = static_cast<int64_t>(t) * kTile + lane;
  const bool valid = t < T && s < N;
  double m = 0.0;
  float xf[D];
#pragma unroll
  for (int q = 0; q < D; ++q) xf[q] = kFar;
  if (valid) {
    const int64_t n = perm[s];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const double x = X[n * D + q];
      Xd[s * D + q] = x;
      const double v = x - X[q];
      xf[q] = static_cast<float>(v);
      m = fmax(m, fabs(v));
    }
  }
  if (t < T) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      Xs[s * D + q] = xf[q];
      float lo = valid ? xf[q] : INFINITY, hi = valid ? xf[q] : -INFINITY;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, o, 64));
        hi = fmaxf(hi, __shfl_xor(hi, o, 64));
      }
      if (lane == 0) {
        tbox[(static_cast<int64_t>(t) * 2) * D + q] = lo;
        tbox[(static_cast<int64_t>(t) * 2 + 1) * D + q] = hi;
      }
    }
  }
  block_atomic_max_u64<256>(
      amax, static_cast<unsigned long long>(__double_as_longlong(m)));
}

// (d2, idx) lexicographic order, ascending; the reference breaks no ties
// (tie-free inputs), the index order makes the result deterministic
__device__ inline bool knn_less(double a, int ia, double b, int ib) {
  return a < b || (a == b && ia < ib);
}

// Bitonic sort of H*64 (d2, idx) pairs held in registers (with the
// candidates' sorted positions as payload), element i = h*64 + lane: strides
// < 64 exchange across lanes (shuffles), stride >= 64 within a lane.
template <int H>
__device__ inline void reg_bitonic(double (&v)[H], int (&ix)[H], int (&ps)[H],
                                   int lane) {
#pragma unroll
  for (int size = 2; size <= H * 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 64) {
        const int hs = stride / 64;
#pragma unroll
        for (int h = 0; h < H; ++h) {
          if (h & hs) continue;
          const int i = h * 64 + lane;
          const bool up = (i & size) == 0;
          const int g = h | hs;
          const bool gt = knn_less(v[g], ix[g], v[h], ix[h]);
          if (gt == up) {
            const double tv = v[h];
            v[h] = v[g];
            v[g] = tv;
            const int ti = ix[h];
            ix[h] = ix[g];
            ix[g] = ti;
            const int tp = ps[h];
            ps[h] = ps[g];
            ps[g] = tp;
          }
        }
      } else {
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const int i = h * 64 + lane;
          const bool up = (i & size) == 0;
          const bool lower = (lane & stride) == 0;
          const double pv = __shfl_xor(v[h], stride, 64);
          const int pi = __shfl_xor(ix[h], stride, 64);
          const int pp = __shfl_xor(ps[h], stride, 64);
          // the lower element keeps the min when ascending
          const bool p_less = knn_less(pv, pi, v[h], ix[h]);
          const bool take = (lower == up) ? p_less : !p_less;
          if (take) {
            v[h] = pv;
            ix[h] = pi;
            ps[h] = pp;
          }
        }
      }
    }
  }
}

// Exact fp64 squared distance (the reference's sequential sub/mul/add).
template <int D>
__device__ inline double knn_exact_d2(const double* __restrict__ X, int64_t i,
                                      int64_t j) {
  double d2 = 0.0;
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const double df = dsub(X[j * D + q], X[i * D + q]);
    d2 = dadd(d2, dmul(df, df));
  }
  return d2;
}

// Sort one row's candidate buffer (cnt sorted positions) by exact distance
// and original index; keep the first k (written back), return tau = the k-th
// exact distance; with out pointers, write the final neighbours (original
// indices) instead.  The exact distances read the fp64 coordinates in the
// spatial order (Xd: the same values as X, so the same d2), where a tile's
// candidates are contiguous.
template <int D, int H>
__device__ inline double knn_sort_cut(const double* __restrict__ Xd,
                                      const int32_t* __restrict__ perm,
                                      int64_t rs, int* __restrict__ buf,
                                      int cnt, int k, int lane,
                                      int32_t* __restrict__ out_idx,
                                      double* __restrict__ out_d2) {
  double v[H];
  int ix[H], ps[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const int i = h * 64 + lane;
    if (i < cnt) {
      ps[h] = buf[i];
      ix[h] = perm[ps[h]];
      // the row itself passes the filter (d2f = 0); it ranks last
      v[h] = ps[h] == rs ? INFINITY : knn_exact_d2<D>(Xd, rs, ps[h]);
    } else {
      ix[h] = 0x7fffffff;
      ps[h] = 0;
      v[h] = INFINITY;
    }
  }
  reg_bitonic<H>(v, ix, ps, lane);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const int i = h * 64 + lane;
    if (i < k) {
      if (out_idx) {
        out_idx[i] = ix[h];
        if (out_d2) out_d2[i] = v[h];
      } else {
        buf[i] = ps[h];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const int hk = (k - 1) / 64, lk = (k - 1) % 64;
  double tk = 0.0;
#pragma unroll
  for (int h = 0; h < H; ++h)
    if (h == hk) tk = v[h];
  return __shfl(tk, lk, 64);
}

// k <= 64 (H = 1): the row's best 64 (exact d2, index) pairs stay sorted in
// registers (element i in lane i) and the passing candidates' sorted
// positions collect in a 64-slot LDS buffer.  A full buffer is ranked by
// exact distance (bitonic sort, descending) and merged into the kept set
// (elementwise min of an ascending and a descending run is bitonic and holds
// the 64 smallest of both; six merge stages sort it), which sets tau = the
// k-th kept distance: 27 compare-exchange stages over one register per lane
// instead of the 28 over two of a full 128-element re-rank, and the kept
// pairs are never re-read or recomputed.
__device__ inline void knn_cmpx(double& v, int& ix, int stride, bool up, int lane) {
  const double pv = __shfl_xor(v, stride, 64);
  const int pi = __shfl_xor(ix, stride, 64);
  const bool lower = (lane & stride) == 0;
  const bool p_less = knn_less(pv, pi, v, ix);
  if ((lower == up) ? p_less : !p_less) {
    v = pv;
    ix = pi;
  }
}

template <int D>
__device__ inline double knn_merge(const double* __restrict__ Xd,
                                   const int32_t* __restrict__ perm, int64_t rs,
                                   const int* __restrict__ buf, int cnt, int k,
                                   int lane, double& kv, int& ki) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  double v = INFINITY;
  int ix = 0x7fffffff;
  if (lane < cnt) {
    const int ps = buf[lane];
    ix = perm[ps];
    // the row itself passes the filter (d2f = 0); it ranks last
    v = ps == rs ? INFINITY : knn_exact_d2<D>(Xd, rs, ps);
  }
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1)
      knn_cmpx(v, ix, stride, (lane & size) != 0, lane);  // descending
  if (knn_less(v, ix, kv, ki)) {
    kv = v;
    ki = ix;
  }
#pragma unroll
  for (int stride = 32; stride > 0; stride >>= 1) knn_cmpx(kv, ki, stride, true, lane);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return __shfl(kv, k - 1, 64);
}

// One wave per R rows (R consecutive rows of the Hilbert order), no block
// barriers.  Candidates stream tile by tile (64 sorted positions, one per
// lane; fp32 centred coordinates) against the wave's rows (packed-fp32
// pairs in VGPRs); lanes passing the fp32 filter append the candidate's
// ORIGINAL index to the row's LDS buffer; a full buffer is re-ranked by exact
// fp64 distance in registers (reg_bitonic) and cut back to k, which sets tau.
// Tiles: first the wave's home tile and its two neighbours (they fill the
// buffers and set tau), then all others in order, 64 at a time: lane l
// tests tile tb + l against every row (box distance with the filter's own
// rounded operations, spatial.hpp) and only tiles some row could take a
// candidate from are streamed.  The skipped tiles hold no candidate the
// filter would pass, so sets, order and distances are those of the full
// scan.  The per-step test is ONE compare per row: padding positions carry
// coordinates whose d2f is +inf, rows past the list a threshold of -inf, and
// the row itself (d2f = 0) is dropped by the exact ranking (knn_sort_cut).
// The kernel is VALU-bound (PMC at C4's shape: VALU busy ~90 % of the
// cycles, ~4.5e4 VALU per wave, a third of them in the ~5 re-rankings per
// row); keeping the next tile's coordinates in flight measured no faster.
template <int D>
__device__ inline void knn_load(const float* __restrict__ Xs, int t, int lane,
                                float (&x)[D]) {
  const int64_t j = static_cast<int64_t>(t) * kTile + lane;
#pragma unroll
  for (int q = 0; q < D; ++q) x[q] = Xs[j * D + q];
}

template <int D, int H, int R>
__device__ inline void knn_step(const float (&xj)[D],
                                const int32_t* __restrict__ perm,
                                const double* __restrict__ Xd, int t,
                                const f32x2 (&xrf)[R / 2][D], float (&Tf)[R],
                                int (&cnt)[R], const int64_t (&rs)[R],
                                int (&buf)[R][H * 64], double (&kv)[R],
                                int (&ki)[R], int k, double A, int lane) {
  constexpr int CAP = H * 64;
  const int64_t j = static_cast<int64_t>(t) * kTile + lane;
  float d2f[R];
#pragma unroll
  for (int p = 0; p < R / 2; ++p) {
    f32x2 acc = f32x2{0.f, 0.f};
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const f32x2 df = xrf[p][q] - f32x2{xj[q], xj[q]};
      acc = __builtin_elementwise_fma(df, df, acc);
    }
    d2f[2 * p] = acc.x;
    d2f[2 * p + 1] = acc.y;
  }
  uint64_t m[R];
  uint64_t any = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    m[r] = __ballot(d2f[r] < Tf[r]);
    any |= m[r];
  }
  if (!any) return;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (!m[r]) continue;
    bool cand = d2f[r] < Tf[r];
    if (cnt[r] + __popcll(m[r]) > CAP) {
      double tau;
      if constexpr (H == 1) {
        tau = knn_merge<D>(Xd, perm, rs[r], buf[r], cnt[r], k, lane, kv[r], ki[r]);
        cnt[r] = 0;
      } else {
        tau = knn_sort_cut<D, H>(Xd, perm, rs[r], buf[r], cnt[r], k, lane, nullptr,
                                 nullptr);
        cnt[r] = k;
      }
      Tf[r] = knn_filter_bound(tau, D, A);
      cand = cand && d2f[r] < Tf[r];
      m[r] = __ballot(cand);
    }
    if (cand) buf[r][cnt[r] + __popcll(m[r] & ((1ull << lane) - 1ull))] = static_cast<int>(j);
    cnt[r] += __popcll(m[r]);
  }
}

template <int D, int H, int R>
__global__ __launch_bounds__(64) void knn_kernel(
    const double* __restrict__ Xd, const float* __restrict__ Xs,
    const int32_t* __restrict__ perm, const float* __restrict__ tbox, int T,
    const unsigned long long* __restrict__ amax, int k,
    const int32_t* __restrict__ rows, const int* __restrict__ nrows_p,
    int64_t rlo, int32_t* __restrict__ nbr, double* __restrict__ nbr_d2) {
  // rows[] = sorted positions of the query rows; row r's output is row r - rlo
  constexpr int CAP = H * 64;
  __shared__ int buf[R][CAP];
  const int lane = threadIdx.x;
  const int64_t nrows = *nrows_p;
  const int64_t w0 = static_cast<int64_t>(blockIdx.x) * R;
  if (w0 >= nrows) return;
  const double A = __longlong_as_double(static_cast<long long>(*amax));

  f32x2 xrf[R / 2][D];   // rows in pairs for packed fp32 math
  float xr[R][D];
  int64_t row[R], rs[R];
  double kv[R];  // H = 1: the kept set, sorted across lanes
  int ki[R];
  float Tf[R];
  int cnt[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t li = w0 + r < nrows ? w0 + r : nrows - 1;
    const int64_t sp = rows[li];
    rs[r] = sp;
    row[r] = perm[sp];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      xr[r][q] = Xs[sp * D + q];
#if ABC_KNN_XR_VGPR
      asm volatile("" : "+v"(xr[r][q]));  // keep the rows out of the SGPRs
#endif
    }
    Tf[r] = w0 + r < nrows ? INFINITY : -INFINITY;
    cnt[r] = 0;
    kv[r] = INFINITY;
    ki[r] = 0x7fffffff;
  }
#pragma unroll
  for (int p = 0; p < R / 2; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) xrf[p][q] = f32x2{xr[2 * p][q], xr[2 * p + 1][q]};

  const int home = static_cast<int>(rows[w0] / kTile);
  const int wlo = home > 0 ? home - 1 : 0;
  const int whi = home + 1 < T ? home + 1 : T - 1;
  float xj[D];
  for (int t = wlo; t <= whi; ++t) {
    knn_load<D>(Xs, t, lane, xj);
    knn_step<D, H, R>(xj, perm, Xd, t, xrf, Tf, cnt, rs, buf, kv, ki, k, A, lane);
  }
  for (int tb = 0; tb < T; tb += 64) {
    const int t = tb + lane;
    bool need = false;
    if (t < T && (t < wlo || t > whi)) {
      const float* lo = tbox + static_cast<int64_t>(t) * 2 * D;
#pragma unroll
      for (int r = 0; r < R; ++r) need = need || box_dist2<D>(xr[r], lo, lo + D) < Tf[r];
    }
    uint64_t mask = __ballot(need);
    while (mask) {
      const int tt = tb + __builtin_ctzll(mask);
      mask &= mask - 1;
      knn_load<D>(Xs, tt, lane, xj);
      knn_step<D, H, R>(xj, perm, Xd, tt, xrf, Tf, cnt, rs, buf, kv, ki, k, A, lane);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if constexpr (H == 1) {
      if (w0 + r < nrows) {
        if (cnt[r] > 0) knn_merge<D>(Xd, perm, rs[r], buf[r], cnt[r], k, lane, kv[r], ki[r]);
        if (lane < k) {
          nbr[(row[r] - rlo) * k + lane] = ki[r];
          if (nbr_d2) nbr_d2[(row[r] - rlo) * k + lane] = kv[r];
        }
      }
    } else {
      if (w0 + r < nrows)
        knn_sort_cut<D, H>(Xd, perm, rs[r], buf[r], cnt[r], k, lane,
                           nbr + (row[r] - rlo) * k,
                           nbr_d2 ? nbr_d2 + (row[r] - rlo) * k : nullptr);
    }
  }
}

// ---------------------------------------------------------------------------
// LU with partial pivoting (the reference's np.linalg.det / inv on the
// host is LAPACK's getrf order); EXACT = (d == D): every loop bound is a
// compile-time constant, so the d x d arrays stay in registers (the
// runtime-d form keeps them in scratch).
template <int D, bool EXACT>
__device__ inline double lu_det_inv(double (&a)[D][D], double (&inv)[D][D],
                                    int d_arg, bool want_inv) {
  const int d = EXACT ? D : d_arg;
  int piv[D];
  double det = 1.0;
#pragma unroll
  for (int i = 0; i < d; ++i) piv[i] = i;
#pragma unroll
  for (int c = 0; c < d; ++c) {
    int p = c;
    double best = fabs(a[c][c]);
#pragma unroll
    for (int r = c + 1; r < d; ++r)
      if (fabs(a[r][c]) > best) {
        best = fabs(a[r][c]);
        p = r;
      }
    if (p != c) {
      if constexpr (EXACT) {  // the same swap with static indices
#pragma unroll
        for (int r = c + 1; r < D; ++r)
          if (r == p) {
#pragma unroll
            for (int q = 0; q < D; ++q) {
              const double t = a[c][q];
              a[c][q] = a[r][q];
              a[r][q] = t;
            }
            const int t = piv[c];
            piv[c] = piv[r];
            piv[r] = t;
          }
      } else {
        for (int q = 0; q < d; ++q) {
          const double t = a[c][q];
          a[c][q] = a[p][q];
          a[p][q] = t;
        }
        const int t = piv[c];
        piv[c] = piv[p];
        piv[p] = t;
      }
      det = -det;
    }
    const double diag = a[c][c];
    det *= diag;
    if (diag == 0.0) continue;
#pragma unroll
    for (int r = c + 1; r < d; ++r) {
      const double f = a[r][c] / diag;
      a[r][c] = f;
#pragma unroll
      for (int q = c + 1; q < d; ++q) a[r][q] = fma(-f, a[c][q], a[r][q]);
    }
  }
  if (want_inv) {
#pragma unroll
    for (int col = 0; col < d; ++col) {
      double y[D];
#pragma unroll
      for (int i = 0; i < d; ++i) {
        double s = piv[i] == col ? 1.0 : 0.0;
#pragma unroll
        for (int q = 0; q < i; ++q) s = fma(-a[i][q], y[q], s);
        y[i] = s;
      }
#pragma unroll
      for (int i = d - 1; i >= 0; --i) {
        double s = y[i];
#pragma unroll
        for (int q = i + 1; q < d; ++q) s = fma(-a[i][q], inv[q][col], s);
        inv[i][col] = s / a[i][i];
      }
    }
  }
  return det;
}

// cov/det/inv: kCovLanes lanes per particle share its k neighbour gathers
// (one thread per particle ran 0.9 ms at C4's N = 2e5, d = 6, k = 50: three
// dependent gather chains of k steps each at ~3 waves per SIMD).
constexpr int kCovLanes = 8;

__device__ inline double cov_group_sum(double v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

template <int D, bool EXACT>
__global__ __launch_bounds__(128) void local_cov_kernel(
    const double* __restrict__ X, const double* __restrict__ w, int64_t N,
    int d_arg, const int32_t* __restrict__ nbr, int k, double scaling,
    int64_t rlo, int64_t rhi, double* __restrict__ covs,
    double* __restrict__ invs, double* __restrict__ dets) {
  const int d = EXACT ? D : d_arg;
  // particles [rlo, rhi), kCovLanes lanes per particle (lane s takes the
  // neighbours t = s, s + 8, ...; the partial sums meet in a fixed xor
  // tree, identical on every lane of the group); nbr and the outputs are
  // indexed from rlo
  const int sub = threadIdx.x & (kCovLanes - 1);
  const int64_t n = rlo + (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) /
                              kCovLanes;
  if (rlo + (static_cast<int64_t>(blockIdx.x) * blockDim.x) / kCovLanes >= rhi) return;
  const bool live = n < rhi;
  const int64_t nn = live ? n : rhi - 1;  // idle groups still join the shuffles
  nbr -= rlo * k;
  covs -= rlo * d * d;
  invs -= rlo * d * d;
  dets -= rlo;
  double xn[D];
#pragma unroll
  for (int q = 0; q < d; ++q) xn[q] = X[nn * d + q];
  // local weights lw = w[nbr] / sum
  double sw = 0.0;
  for (int t = sub; t < k; t += kCovLanes) sw += w[nbr[nn * k + t]];
  sw = cov_group_sum(sw);
  double v1 = 0.0, v2 = 0.0, mu[D];
#pragma unroll
  for (int q = 0; q < d; ++q) mu[q] = 0.0;
  for (int t = sub; t < k; t += kCovLanes) {
    const int64_t j = nbr[nn * k + t];
    const double lw = w[j] / sw;
    v1 += lw;
    v2 += lw * lw;
#pragma unroll
    for (int q = 0; q < d; ++q) mu[q] = fma(lw, X[j * d + q] - xn[q], mu[q]);
  }
  v1 = cov_group_sum(v1);
  v2 = cov_group_sum(v2);
#pragma unroll
  for (int q = 0; q < d; ++q) mu[q] = cov_group_sum(mu[q]) / v1;
  double C[D][D];
#pragma unroll
  for (int a = 0; a < d; ++a)
#pragma unroll
    for (int b = 0; b < d; ++b) C[a][b] = 0.0;
  for (int t = sub; t < k; t += kCovLanes) {
    const int64_t j = nbr[nn * k + t];
    const double lw = w[j] / sw;
    double dl[D];
#pragma unroll
    for (int q = 0; q < d; ++q) dl[q] = (X[j * d + q] - xn[q]) - mu[q];
#pragma unroll
    for (int a = 0; a < d; ++a)
#pragma unroll
      for (int b = a; b < d; ++b) C[a][b] = fma(lw * dl[a], dl[b], C[a][b]);
  }
#pragma unroll
  for (int a = 0; a < d; ++a)
#pragma unroll
    for (int b = a; b < d; ++b) C[a][b] = cov_group_sum(C[a][b]);
  if (!live || sub != 0) return;
  double fact = v1 - v2 / v1;
  if (fact <= 0.0) fact = 0.0;
  double csum = 0.0;
#pragma unroll
  for (int a = 0; a < d; ++a)
#pragma unroll
    for (int b = a; b < d; ++b) {
      C[a][b] = C[a][b] * (1.0 / fact);
      C[b][a] = C[a][b];
    }
  if (k == 1) {  // smart_cov of ONE delta row: diag(|delta_0|) (util.py:8-11)
    const int64_t j = nbr[n * k];
#pragma unroll
    for (int a = 0; a < d; ++a)
#pragma unroll
      for (int b = 0; b < d; ++b)
        C[a][b] = a == b ? fabs(X[j * d + a] - xn[a]) : 0.0;
  }
#pragma unroll
  for (int a = 0; a < d; ++a)
#pragma unroll
    for (int b = 0; b < d; ++b) csum += C[a][b];
  if (fabs(csum) == 0.0) {
#pragma unroll
    for (int q = 0; q < d; ++q) C[q][q] = fabs(X[q]);
  }
#pragma unroll
  for (int a = 0; a < d; ++a)
#pragma unroll
    for (int b = 0; b < d; ++b) C[a][b] *= scaling;
  double work[D][D], inv[D][D];
  double det;
  for (int it = 0; it < 100000; ++it) {
#pragma unroll
    for (int a = 0; a < d; ++a)
#pragma unroll
      for (int b = 0; b < d; ++b) work[a][b] = C[a][b];
    det = lu_det_inv<D, EXACT>(work, inv, d, false);
    if (!(det <= 0.0)) break;  // reference: while det <= 0 (NaN exits)
#pragma unroll
    for (int q = 0; q < d; ++q) C[q][q] += 1e-3;
  }
#pragma unroll
  for (int a = 0; a < d; ++a)
#pragma unroll
    for (int b = 0; b < d; ++b) work[a][b] = C[a][b];
  lu_det_inv<D, EXACT>(work, inv, d, true);
#pragma unroll
  for (int a = 0; a < d; ++a)
#pragma unroll
    for (int b = 0; b < d; ++b) {
      covs[n * d * d + a * d + b] = C[a][b];
      invs[n * d * d + a * d + b] = inv[a][b];
    }
  dets[n] = det;
}

// Main pass: one thread per evaluation point, the previous population's
// (X_n, coef_n, lc_n) streaming through the scalar path (wave-uniform n).
// Terms are exp(lc_n - q_n/2 - L) <= 1 (q >= 0), summed in fp64 without a
// running max; the n-range is cut into a fixed number of chunks (a function
// of N only) whose partial sums are added in fixed order.
template <int D>
__global__ __launch_bounds__(256) void local_pdf_kernel(
    const double* __restrict__ pts, int64_t M, const double* __restrict__ X,
    const double* __restrict__ coef, const double* __restrict__ lc,
    const unsigned long long* __restrict__ lc_max_key, int64_t N, int split,
    int64_t nchunk, double* __restrict__ part) {
  constexpr int NC = D * (D + 1) / 2;
  const int s = blockIdx.x % split;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x / split) * 256 + threadIdx.x;
  const int64_t i = i0 < M ? i0 : M - 1;
  const double L = key_f64(*lc_max_key);
  double th[D];
#pragma unroll
  for (int q = 0; q < D; ++q) th[q] = pts[i * D + q];
  double acc = 0.0;
  const int64_t n0 = static_cast<int64_t>(s) * nchunk;
  int64_t n1 = n0 + nchunk;
  if (n1 > N) n1 = N;
  for (int64_t n = n0; n < n1; ++n) {
    double dl[D];
#pragma unroll
    for (int q = 0; q < D; ++q) dl[q] = th[q] - X[n * D + q];
    const double qf = local_qform<D>(dl, coef + n * NC);
    acc += exp(fma(-0.5, qf, lc[n] - L));
  }
  if (i0 < M) part[static_cast<int64_t>(s) * M + i0] = acc;
}


// LocalTransition.rvs_single (local_transition.py:141-145):
//   idx ~ choice(N, p=w); theta ~ N(X[idx], C[idx]).
// The index is the same CDF search as the global kernel (bit-exact for the
// same u); the Gaussian draw uses the Cholesky factor of C[idx] (numpy uses
// an SVD factor: same distribution, different map from z to theta).
// EXACT (d == D, d <= 8): compile-time loops keep the factor in registers;
// with the runtime bound the d x d factor lived in scratch (528 B per lane
// at D = 8, tools/spill_report.py).  Same operations in the same order.
template <int D, bool EXACT>
__global__ __launch_bounds__(256) void propose_local_kernel(
    const double* __restrict__ X, int64_t N, int d,
    const double* __restrict__ cdf, const double* __restrict__ covs,
    const double* __restrict__ lo, const double* __restrict__ scale,
    uint64_t seed, uint64_t sid, uint64_t offset, int64_t B,
    double* __restrict__ theta, int64_t* __restrict__ idx_out,
    uint8_t* __restrict__ sup) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t ui = offset + static_cast<uint64_t>(b);
  const u32x4 ub = philox_block(seed, 2 * sid, ui >> 1);
  const double u = (ui & 1) ? u53(ub.z, ub.w) : u53(ub.x, ub.y);
  int64_t lo_i = 0, hi_i = N;
  while (lo_i < hi_i) {
    const int64_t mid = (lo_i + hi_i) >> 1;
    if (cdf[mid] <= u) lo_i = mid + 1; else hi_i = mid;
  }
  const int64_t idx = lo_i < N ? lo_i : N - 1;
  const int dd = EXACT ? D : d;
  constexpr int kUnroll = EXACT ? D : 1;
  double L[D][D];
  const double* C = covs + idx * dd * dd;
#pragma unroll kUnroll
  for (int i = 0; i < dd; ++i)
#pragma unroll kUnroll
    for (int j = 0; j <= i; ++j) {
      double s = C[i * dd + j];
#pragma unroll kUnroll
      for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
      if (i == j)
        L[i][i] = sqrt(s > 0.0 ? s : 0.0);
      else
        L[i][j] = L[j][j] > 0.0 ? s / L[j][j] : 0.0;
    }
  double z[D];
  const uint64_t zi0 = ui * static_cast<uint64_t>(dd);
#pragma unroll kUnroll
  for (int k = 0; k < dd; ++k) {
    const uint64_t zi = zi0 + k;
    double c0, c1;
    box_muller(philox_block(seed, 2 * sid + 1, zi >> 1), c0, c1);
    z[k] = (zi & 1) ? c1 : c0;
  }
  bool ok = true;
#pragma unroll kUnroll
  for (int i = 0; i < dd; ++i) {
    double s = 0.0;
#pragma unroll kUnroll
    for (int k = 0; k <= i; ++k) s = fma(L[i][k], z[k], s);
    const double th = X[idx * dd + i] + s;
    theta[b * dd + i] = th;
    if (lo) {
      const double x = (th - lo[i]) / scale[i];
      ok = ok && x >= 0.0 && x <= 1.0;
    }
  }
  idx_out[b] = lo_i;
  sup[b] = ok ? 1 : 0;
}

// fp32-storage entry points (SURVEY 8(b) abc_knn_topk_f32 /
// abc_local_cov_f32): the fp32 inputs are widened into the workspace and the
// fp64 kernels run on them (every fp32 value is exact in fp64, so the kNN
// sets are those of the fp32 points), results rounded to fp32 on the way out.
template <typename S, typename D>
__global__ __launch_bounds__(256) void convert_kernel(const S* __restrict__ src,
                                                      int64_t n,
                                                      D* __restrict__ dst) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256)
    dst[i] = static_cast<D>(src[i]);
}
template <typename S, typename D>
void convert(const S* src, int64_t n, D* dst, hipStream_t st) {
  if (n > 0)
    hipLaunchKernelGGL((convert_kernel<S, D>), dim3(stream_grid(n, 256, 2048)),
                       dim3(256), 0, st, src, n, dst);
}

}  // namespace abc

using namespace abc;

extern "C" {

int abc_propose_local_philox_f64(const double* X, int64_t N, int d,
                                 const double* cdf, const double* covs,
                                 const double* lo, const double* scale,
                                 uint64_t seed, uint64_t sid, uint64_t offset,
                                 int64_t B, double* theta, int64_t* idx,
                                 uint8_t* in_support, hipStream_t st) {
  ABC_REQUIRE(N > 0 && B >= 0 && d >= 1 && d <= 16, "propose_local: bad sizes");
  if (B == 0) return kOk;
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
  switch (d) {
#define PL(DD, EX)                                                              \
  hipLaunchKernelGGL((propose_local_kernel<DD, EX>), dim3(g), dim3(256), 0, st, \
                     X, N, d, cdf, covs, lo, scale, seed, sid, offset, B, theta, \
                     idx, in_support)
    case 1: PL(1, true); break;
    case 2: PL(2, true); break;
    case 3: PL(3, true); break;
    case 4: PL(4, true); break;
    case 5: PL(5, true); break;
    case 6: PL(6, true); break;
    case 7: PL(7, true); break;
    case 8: PL(8, true); break;
    default: PL(16, false); break;
#undef PL
  }
  ABC_LAUNCH_CHECK("propose_local_kernel");
  return kOk;
}

size_t abc_knn_workspace_bytes(int64_t N, int k) {
  (void)k;
  // amax | rows[N] | fp32 sorted centred coordinates [T*64][8] | fp64
  // sorted coordinates [T*64][8] | spatial index
  const int64_t T = ceil_div(N > 0 ? N : 1, kTile);
  return 256 + al256(static_cast<size_t>(N > 0 ? N : 1) * 4) +
         al256(static_cast<size_t>(T) * kTile * 8 * 4) +
         al256(static_cast<size_t>(T) * kTile * 8 * 8) + spatial_ws_bytes(N > 0 ? N : 1);
}

int abc_knn_rows_f64(const double* X, int64_t N, int d, int k, int64_t row0,
                     int64_t nrows, int32_t* nbr, double* nbr_d2, void* ws,
                     size_t ws_bytes, hipStream_t st) {
  ABC_REQUIRE(N > 1 && k >= 1 && k <= N - 1, "knn: need 1 <= k <= N-1");
  ABC_REQUIRE(k <= kMaxK, "knn: k=%d exceeds the one-pass limit %d", k, kMaxK);
  ABC_REQUIRE(N < (1ll << 31), "knn: N must fit int32 indices");
  ABC_REQUIRE(row0 >= 0 && nrows >= 0 && row0 + nrows <= N,
              "knn: rows [%lld, %lld) outside [0, %lld)", (long long)row0,
              (long long)(row0 + nrows), (long long)N);
  if (nrows == 0) return kOk;
  ABC_REQUIRE(X && nbr && ws, "knn: null pointer");
  ABC_REQUIRE(ws_bytes >= abc_knn_workspace_bytes(N, k), "knn: workspace too small");
  ABC_REQUIRE(d >= 1 && d <= 8, "knn: unsupported d=%d (d <= 8)", d);
  char* q = static_cast<char*>(ws);
  unsigned long long* amax = reinterpret_cast<unsigned long long*>(q);
  q += 256;
  int32_t* rows = reinterpret_cast<int32_t*>(q);
  q += al256(static_cast<size_t>(N) * 4);
  const int64_t T = ceil_div(N, kTile);
  float* Xs = reinterpret_cast<float*>(q);
  q += al256(static_cast<size_t>(T) * kTile * 8 * 4);
  double* Xd = reinterpret_cast<double*>(q);
  q += al256(static_cast<size_t>(T) * kTile * 8 * 8);
  SpatialWs v = spatial_ws(q, N);
  ABC_HIP(hipMemsetAsync(amax, 0, 8, st));
  // rows per wave: kKnnRows, or 8 (tuning knob ABC_KNN_ROWS; the neighbour
  // sets, order and distances are the same; 2 and 16 measured slower)
  const int rpw = tuning_knob(kKnobKnnRows, kKnnRows);
  const int64_t rlo = row0, rhi = row0 + nrows;
#define KNN_R(DD, H, RR)                                                          \
  hipLaunchKernelGGL((knn_kernel<DD, H, RR>), dim3(ceil_div(nrows, RR)), dim3(64), \
                     0, st, Xd, Xs, v.perm, v.tbox, v.T, amax, k, rows, v.count,  \
                     rlo, nbr, nbr_d2)
#define KNN(DD, H)                                                               \
  do {                                                                           \
    if (rpw == 8) KNN_R(DD, H, 8);                                               \
    else KNN_R(DD, H, kKnnRows);                                                 \
  } while (0)
#define L(DD)                                                                    \
  {                                                                              \
    const int rc = spatial_sort_population<DD>(X, N, v, st);                     \
    if (rc != kOk) return rc;                                                    \
    hipLaunchKernelGGL((knn_prep_kernel<DD>), dim3(ceil_div(T, 4)), dim3(256), 0, \
                       st, X, N, v.perm, v.T, Xs, Xd, v.tbox, amax);             \
    hipLaunchKernelGGL(sp_rows_in_range_kernel, dim3(ceil_div(N, 256)), dim3(256), \
                       0, st, v.perm, N, rlo, rhi, rows, v.count);               \
    if (k <= 64) KNN(DD, 1); else KNN(DD, 4);                                    \
  }
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
#undef KNN
  ABC_LAUNCH_CHECK("knn_kernel");
  return kOk;
}

int abc_knn_f64(const double* X, int64_t N, int d, int k, int32_t* nbr,
                double* nbr_d2, void* ws, size_t ws_bytes, hipStream_t st) {
  return abc_knn_rows_f64(X, N, d, k, 0, N, nbr, nbr_d2, ws, ws_bytes, st);
}

int abc_local_cov_rows_f64(const double* X, const double* w, int64_t N, int d,
                           const int32_t* nbr, int k, int64_t row0,
                           int64_t nrows, double scaling, double* covs,
                           double* inv_covs, double* dets, hipStream_t st) {
  ABC_REQUIRE(N >= 1 && k >= 1, "local_cov: bad sizes");
  ABC_REQUIRE(row0 >= 0 && nrows >= 0 && row0 + nrows <= N,
              "local_cov: rows outside [0, N)");
  if (nrows == 0) return kOk;
  const unsigned g = static_cast<unsigned>(ceil_div(nrows * kCovLanes, 128));
  const int64_t rlo = row0, rhi = row0 + nrows;
#define L(DD, EX)                                                                \
  hipLaunchKernelGGL((local_cov_kernel<DD, EX>), dim3(g), dim3(128), 0, st, X, w, \
                     N, d, nbr, k, scaling, rlo, rhi, covs, inv_covs, dets);
  // d <= 6: one instantiation per d (register-resident d x d arrays; at
  // d = 7, 8 those need 262 / 360 VGPRs and the compile time explodes)
  switch (d) {
    case 1: L(1, true) break;
    case 2: L(2, true) break;
    case 3: L(3, true) break;
    case 4: L(4, true) break;
    case 5: L(5, true) break;
    case 6: L(6, true) break;
    default:
      if (d <= 8) {
        L(8, false)
      } else if (d <= 16) {
        L(16, false)
      } else {
        set_error("local_cov: unsupported d=%d (d <= 16)", d);
        return kUnsupported;
      }
  }
#undef L
  ABC_LAUNCH_CHECK("local_cov_kernel");
  return kOk;
}

int abc_local_cov_f64(const double* X, const double* w, int64_t N, int d,
                      const int32_t* nbr, int k, double scaling, double* covs,
                      double* inv_covs, double* dets, hipStream_t st) {
  return abc_local_cov_rows_f64(X, w, N, d, nbr, k, 0, N, scaling, covs,
                                inv_covs, dets, st);
}

// The n-range is cut into a fixed number of chunks that depends on N only,
// so a row's log-sum-exp does not depend on M or on how rows are shared
// between ranks (multi-GPU results equal single-GPU results bit for bit).
size_t abc_local_logpdf_workspace_bytes(int64_t M, int64_t N) {
  int split;
  int64_t nchunk;
  local_plan(M > 0 ? M : 1, N > 0 ? N : 1, split, nchunk);
  // logsumw, lc_max_key, n_fix (64 B) | lc[N] | coef[N][36] (d <= 8)
  // | part[split][M] | fix_rows[M]
  return 64 + static_cast<size_t>(N) * 8 * 37 +
         static_cast<size_t>(split) * M * 8 + static_cast<size_t>(M) * 4 + 512;
}

int abc_local_logpdf_f64(const double* pts, int64_t M, const double* X,
                         const double* w, const double* inv_covs,
                         const double* dets, int64_t N, int d,
                         double* out_logpdf, void* ws, size_t ws_bytes,
                         hipStream_t st) {
  ABC_REQUIRE(M >= 0 && N >= 1, "local_logpdf: bad sizes");
  if (M == 0) return kOk;
  ABC_REQUIRE(d >= 1 && d <= 8, "local_logpdf: unsupported d=%d (d <= 8)", d);
  ABC_REQUIRE(pts && X && w && inv_covs && dets && out_logpdf && ws,
              "local_logpdf: null pointer");
  ABC_REQUIRE(ws_bytes >= abc_local_logpdf_workspace_bytes(M, N),
              "local_logpdf: workspace too small");
  int split;
  int64_t nchunk;
  local_plan(M, N, split, nchunk);
  char* base = static_cast<char*>(ws);
  double* logsumw = reinterpret_cast<double*>(base);
  unsigned long long* lc_max_key = reinterpret_cast<unsigned long long*>(base + 8);
  int* n_fix = reinterpret_cast<int*>(base + 16);
  double* lc = reinterpret_cast<double*>(base + 64);
  double* coef = lc + N;
  double* part = coef + N * 36;
  int* fix_rows = reinterpret_cast<int*>(part + static_cast<int64_t>(split) * M);
  ABC_HIP(hipMemsetAsync(base + 8, 0, 16, st));
  local_sumw(w, N, split, part, logsumw, st);
  hipLaunchKernelGGL(local_const_kernel, dim3(ceil_div(N, 256)), dim3(256), 0,
                     st, w, dets, inv_covs, N, d, lc, coef, lc_max_key);
  const unsigned grid = static_cast<unsigned>(ceil_div(M, 256) * split);
#define L(DD)                                                                   \
  hipLaunchKernelGGL((local_pdf_kernel<DD>), dim3(grid), dim3(256), 0, st, pts,  \
                     M, X, coef, lc, lc_max_key, N, split, nchunk, part);       \
  hipLaunchKernelGGL(local_pdf_final_kernel, dim3(ceil_div(M, 256)), dim3(256), \
                     0, st, part, M, split, lc_max_key, logsumw, out_logpdf,    \
                     n_fix, fix_rows, 1e-280);                                  \
  hipLaunchKernelGGL((local_pdf_fixup_kernel<DD>), dim3(64), dim3(256), 0, st,  \
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
  ABC_LAUNCH_CHECK("local_logpdf kernels");
  return kOk;
}

size_t abc_knn_topk_f32_workspace_bytes(int64_t N, int d, int k) {
  return al256(static_cast<size_t>(N) * d * 8) +
         al256(static_cast<size_t>(N) * k * 8) + abc_knn_workspace_bytes(N, k);
}

int abc_knn_topk_f32(const float* X, int64_t N, int d, int k, int32_t* nbr,
                     float* nbr_d2, void* ws, size_t ws_bytes, hipStream_t st) {
  ABC_REQUIRE(N >= 1 && d >= 1 && k >= 1, "knn_topk_f32: bad sizes");
  ABC_REQUIRE(X && nbr && nbr_d2 && ws, "knn_topk_f32: null pointer");
  ABC_REQUIRE(ws_bytes >= abc_knn_topk_f32_workspace_bytes(N, d, k),
              "knn_topk_f32: workspace too small");
  char* q = static_cast<char*>(ws);
  double* Xd = reinterpret_cast<double*>(q);
  q += al256(static_cast<size_t>(N) * d * 8);
  double* d2 = reinterpret_cast<double*>(q);
  q += al256(static_cast<size_t>(N) * k * 8);
  convert(X, N * d, Xd, st);
  const int rc = abc_knn_rows_f64(Xd, N, d, k, 0, N, nbr, d2, q,
                                  ws_bytes - static_cast<size_t>(
                                                 q - static_cast<char*>(ws)),
                                  st);
  if (rc != kOk) return rc;
  convert(d2, N * k, nbr_d2, st);
  ABC_LAUNCH_CHECK("knn_topk_f32");
  return kOk;
}

size_t abc_local_cov_f32_workspace_bytes(int64_t N, int d) {
  return al256(static_cast<size_t>(N) * d * 8) + al256(static_cast<size_t>(N) * 8) +
         2 * al256(static_cast<size_t>(N) * d * d * 8) +
         al256(static_cast<size_t>(N) * 8);
}

int abc_local_cov_f32(const float* X, const float* w, int64_t N, int d,
                      const int32_t* nbr, int k, double scaling, float* covs,
                      float* inv_covs, float* dets, void* ws, size_t ws_bytes,
                      hipStream_t st) {
  ABC_REQUIRE(N >= 1 && d >= 1 && k >= 1, "local_cov_f32: bad sizes");
  ABC_REQUIRE(X && w && nbr && covs && inv_covs && dets && ws,
              "local_cov_f32: null pointer");
  ABC_REQUIRE(ws_bytes >= abc_local_cov_f32_workspace_bytes(N, d),
              "local_cov_f32: workspace too small");
  char* q = static_cast<char*>(ws);
  double* Xd = reinterpret_cast<double*>(q);
  q += al256(static_cast<size_t>(N) * d * 8);
  double* wd = reinterpret_cast<double*>(q);
  q += al256(static_cast<size_t>(N) * 8);
  double* C = reinterpret_cast<double*>(q);
  q += al256(static_cast<size_t>(N) * d * d * 8);
  double* Ci = reinterpret_cast<double*>(q);
  q += al256(static_cast<size_t>(N) * d * d * 8);
  double* dt = reinterpret_cast<double*>(q);
  convert(X, N * d, Xd, st);
  convert(w, N, wd, st);
  const int rc = abc_local_cov_rows_f64(Xd, wd, N, d, nbr, k, 0, N, scaling, C,
                                        Ci, dt, st);
  if (rc != kOk) return rc;
  convert(C, N * d * d, covs, st);
  convert(Ci, N * d * d, inv_covs, st);
  convert(dt, N, dets, st);
  ABC_LAUNCH_CHECK("local_cov_f32");
  return kOk;
}

}  // extern "C"

namespace abc {
// Loads this translation unit's code object (HIP loads each one lazily, at
// the first launch of one of its kernels: ~4 ms for local_mfma's inside
// C4's first weighted generation); abc_preload calls every unit's hook.
int preload_local() { return preload_kernel(local_sumw_part_kernel); }
}  // namespace abc
