// Proposal generation: MultivariateNormalTransition.rvs + prior support.
//
// Reference semantics (pyabc/transition/multivariatenormal.py:87-95 and
// pyabc/smc.py:602-645, numpy legacy RandomState):
//   cdf = cumsum(w); cdf /= cdf[-1]            (sequential fp64)
//   idx = cdf.searchsorted(u, side='right')    (u = random_sample())
//   theta = X[idx] + z @ A,  A = sqrt(s)[:,None] * V  from svd(cov)
//   valid iff prior.pdf(theta) > 0; for RV('uniform', lo, scale) scipy tests
//   0 <= (theta - lo) / scale <= 1 in fp64 (random_variables.py:425-452).
// The CDF is built by ONE lane in sequential order so that it is bit-identical
// to numpy's; the resampled indices are then bit-exact for injected u.
// Production proposals draw u and z from Philox4x32-10 inside the kernel
// (no u/z round trip through HBM); the parity entry point takes them as
// inputs.  Out-of-support draws are not evaluations: an order-preserving
// compaction assigns proposal ids to in-support draws only.
#include "common.hpp"
#include "philox.hpp"

namespace abc {

// ---------------------------------------------------------------------------
// Exact sequential fp64 cumsum, evaluated in parallel.
//
// numpy's cumsum is the chain c_k = fl(c_{k-1} + w_k).  While c stays in one
// binade [2^e, 2^(e+1)) every double there is an integer multiple of
// u = 2^(e-52), so with C = c/u (an integer < 2^53) and v = w * 2^(52-e)
// (exact scaling) the rounded sum is fl(c + w) = u * (C + floor(v) +
// [frac(v) > 1/2]) -- except when frac(v) == 1/2 (a tie, resolved by the
// parity of the result) or when the sum leaves the binade.  Inside a binade
// the chain is therefore an INTEGER prefix sum of increments that do not
// depend on the chain itself, and a whole 1024-element tile advances it by
// one precomputed integer T_t.
//
//   1. cdf_tile_sum    (tiles in parallel)  approximate fp64 tile sums
//   2. cdf_prefix      (one block)          approximate tile-start prefixes
//   3. cdf_tile_plan   (tiles in parallel)  the tile's binade e_t from its
//      approximate prefix range (with a relative margin far above the
//      chain's accumulated rounding), its integer increment total T_t under
//      grid e_t; ties / negative / non-finite / binade-straddling tiles are
//      marked slow
//   4. cdf_chain       (one wave)           walks the tiles: a run of fast
//      tiles of one binade is advanced in parallel (C_in = run start + prefix
//      of T_t), each step VERIFIED against the exact chain value (c in
//      binade e_t and C + T_t <= 2^53 - 2, i.e. no element leaves the
//      binade); any other tile runs the exact walk (exact_tile_wave: integer
//      increments, wave scan, real fp64 add at the first tie / binade exit,
//      re-grid, continue) -- ~1 slow tile per binade crossing; the first
//      kHeadSeq elements (binade exits at ~1, 2, 4, ... elements) by one
//      lane in numpy's own order (head_seq_wave)
//   5. cdf_write       (tiles in parallel)  rebuilds every fast tile's
//      elements from its exact start value C_t and the in-tile integer
//      prefix, and divides by the last value (numpy's cdf /= cdf[-1])
//
// The plan only decides which tiles take which path; the chain kernel checks
// every fast step exactly, so the result is bit-identical to the sequential
// chain for any input.
constexpr int kCdfThreads = 256;
constexpr int kCdfItems = 4;
constexpr int kCdfTile = kCdfThreads * kCdfItems;
constexpr int kCdfSlow = -100000;
constexpr int kChainChunk = 2048;       // tile records per LDS batch
constexpr long long kBinadeTop = (1ll << 53) - 2;

constexpr int kWaveItems = kCdfTile / 64;  // one wave walks a whole tile

__device__ inline long long wave_incl_scan(long long v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Cross-lane steps of the single-wave walks on DPP (row shifts within the
// 16-lane rows, then the row-15 / lane-31 broadcasts): a VALU operand
// modifier per step instead of a ds_bpermute round trip through LDS -- the
// walks are latency-bound, one wave on the chip.
template <int CTRL, int ROWS = 0xf>
__device__ inline double dpp_f64_zero(double v) {  // out-of-row lanes read 0
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS,
                                             0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS,
                                             0xf, true);
  return __hiloint2double(hi, lo);
}

// inclusive prefix sum over the 64 lanes (adds of +0.0 elsewhere: the
// values summed here are non-negative integers held in fp64)
__device__ inline double wave_incl_scan_f64(double v) {
  v += dpp_f64_zero<0x111>(v);       // row_shr:1
  v += dpp_f64_zero<0x112>(v);       // row_shr:2
  v += dpp_f64_zero<0x114>(v);       // row_shr:4
  v += dpp_f64_zero<0x118>(v);       // row_shr:8
  v += dpp_f64_zero<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f64_zero<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}

__device__ inline double wave_shr1_f64(double v) {  // lane l gets l - 1; 0 at 0
  return dpp_f64_zero<0x138>(v);                    // wave_shr:1
}

__device__ inline long long readlane_i64(long long v, int l) {
  const unsigned lo = __builtin_amdgcn_readlane(static_cast<int>(v), l);
  const unsigned hi = __builtin_amdgcn_readlane(static_cast<int>(v >> 32), l);
  return static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo);
}

__device__ inline double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

template <int CTRL, int ROWS = 0xf>
__device__ inline int dpp_min_step(int v) {  // disabled lanes keep INT_MAX
  return min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, CTRL, ROWS, 0xf,
                                            false));
}

// minimum over the 64 lanes, wave-uniform (an SGPR)
__device__ inline int wave_min_int(int v) {
  v = dpp_min_step<0x111>(v);
  v = dpp_min_step<0x112>(v);
  v = dpp_min_step<0x114>(v);
  v = dpp_min_step<0x118>(v);
  v = dpp_min_step<0x142, 0xa>(v);
  v = dpp_min_step<0x143, 0xc>(v);
  return __builtin_amdgcn_readlane(v, 63);
}

// The exact chain over w[base, base + tile_n) by ONE wave (no barriers):
// integer increments on the current binade grid, a wave scan, the real fp64
// add at the first tie / binade exit, re-grid, continue.  The integers are
// held in fp64: every partial sum up to the first break is an integer below
// 2^53 and therefore exact (and a sum at or past 2^53 still compares >= the
// representable bound after rounding), which avoids int64<->fp64
// conversions on this latency-bound single-wave path.  c (wave-uniform) in
// and out; raw (un-normalised) values written to cdf.
__device__ void exact_tile_wave(const double* __restrict__ w, int64_t base,
                                int tile_n, double& c,
                                double* __restrict__ cdf) {
  const int lane = threadIdx.x & 63;
  double wv[kWaveItems];
#pragma unroll
  for (int q = 0; q < kWaveItems; ++q) {
    const int k = lane * kWaveItems + q;
    wv[q] = k < tile_n ? w[base + k] : 0.0;
  }
  int s = 0;  // first unprocessed element of the tile (uniform)
  while (s < tile_n) {
    int ex;
    (void)frexp(c, &ex);  // c = mant * 2^ex, mant in [0.5,1)
    const bool exact_mode = c >= 0x1p-1000;
    const int e = ex - 1;
    const double C = exact_mode ? ldexp(c, 52 - e) : 0.0;  // integer
    double dl[kWaveItems];
    int my_bad = 1 << 30;
    double tsum = 0.0;
#pragma unroll
    for (int q = 0; q < kWaveItems; ++q) {
      const int k = lane * kWaveItems + q;
      double dq = 0.0;
      bool b = false;
      if (k >= s && k < tile_n) {
        if (!exact_mode || wv[q] < 0.0) {
          b = (c != 0.0) || (wv[q] != 0.0);
        } else {
          const double v = ldexp(wv[q], 52 - e);
          if (!(v < 0x1p53)) {
            b = true;
          } else {
            const double fl = floor(v);
            const double fr = v - fl;
            dq = fl + (fr > 0.5 ? 1.0 : 0.0);
            b = (fr == 0.5);
          }
        }
      }
      tsum += dq;
      dl[q] = tsum;  // inclusive within the lane
      if (b && my_bad == (1 << 30)) my_bad = k;
    }
    const double incl = wave_incl_scan_f64(tsum);
    // exclusive prefix = the previous lane's inclusive one (NOT incl - tsum:
    // a lane past the break may hold a sum above 2^53, inexact in fp64)
    const double excl = wave_shr1_f64(incl);
    // binade exit: C + prefix must stay below 2^53 (one unit margin)
    const double Cx = C + excl;
#pragma unroll
    for (int q = 0; q < kWaveItems; ++q) {
      const int k = lane * kWaveItems + q;
      if (exact_mode && k >= s && k < tile_n && k < my_bad &&
          Cx + dl[q] >= 0x1p53 - 1.0)
        my_bad = k;
    }
    const int b = wave_min_int(my_bad);
#pragma unroll
    for (int q = 0; q < kWaveItems; ++q) {
      const int k = lane * kWaveItems + q;
      if (k >= s && k < tile_n && k < b)
        cdf[base + k] = ldexp(Cx + dl[q], e - 52);
    }
    if (b < tile_n) {
      // the breaking element: the real fp64 add, by its owner lane
      const int owner = b / kWaveItems;
      double cb = 0.0;
      if (lane == owner) {
        const int q0 = b - lane * kWaveItems;
        double prev = c;
        double wb = 0.0;
        double dprev = 0.0;
#pragma unroll
        for (int q = 0; q < kWaveItems; ++q) {
          if (q == q0) wb = wv[q];
          if (q == q0 - 1) dprev = dl[q];
        }
        if (b > s) prev = ldexp(Cx + dprev, e - 52);
        cb = (base + b == 0) ? wb : prev + wb;
        cdf[base + b] = cb;
      }
      c = readlane_f64(cb, owner);
      s = b + 1;
    } else {
      const double total = readlane_f64(incl, 63);
      if (exact_mode) c = ldexp(C + total, e - 52);
      s = tile_n;
    }
  }
}

// The head of the array in numpy's own order, c = fl(c + w_k) (c_0 = w_0):
// the first tile's chain doubles every few elements (a binade exit at ~1,
// 2, 4, ... elements), where the wave walk above pays a full pass per exit
// (~2.7 us each on the MI355X).  Each lane holds 4 consecutive weights; the
// add chain takes them lane by lane through readlane (an SGPR operand), so
// the only dependency per element is the fp64 add itself, and lane l
// catches its own partial sums as they pass.  Raw values written to cdf;
// c out (wave-uniform).
constexpr int kHeadSeq = 256;
constexpr int kHeadPer = kHeadSeq / 64;
__device__ void head_seq_wave(const double* __restrict__ w, int head_n,
                              double& c, double* __restrict__ cdf) {
  const int lane = threadIdx.x & 63;
  double v[kHeadPer], out[kHeadPer];
#pragma unroll
  for (int q = 0; q < kHeadPer; ++q) {
    const int k = lane * kHeadPer + q;
    v[q] = k < head_n ? w[k] : 0.0;
    out[q] = 0.0;
  }
  double cc = 0.0;
#pragma unroll
  for (int l = 0; l < 64; ++l) {
#pragma unroll
    for (int q = 0; q < kHeadPer; ++q) {
      const int k = l * kHeadPer + q;
      if (k < head_n) {  // wave-uniform
        const double s = readlane_f64(v[q], l);
        cc = k == 0 ? s : cc + s;  // numpy: cdf[0] = w[0] (-0.0 stays)
        out[q] = lane == l ? cc : out[q];
      }
    }
  }
  c = cc;
#pragma unroll
  for (int q = 0; q < kHeadPer; ++q) {
    const int k = lane * kHeadPer + q;
    if (k < head_n) cdf[k] = out[q];
  }
}

__global__ __launch_bounds__(kCdfThreads) void cdf_tile_sum_kernel(
    const double* __restrict__ w, int64_t n, double* __restrict__ tsum) {
  __shared__ double red[kCdfThreads / 64];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kCdfTile;
  double v = 0.0;
#pragma unroll
  for (int q = 0; q < kCdfItems; ++q) {
    const int64_t i = base + q * kCdfThreads + threadIdx.x;
    if (i < n) v += w[i];
  }
  v = block_sum<double, kCdfThreads>(v, red);
  if (threadIdx.x == 0) tsum[blockIdx.x] = v;
}

__global__ __launch_bounds__(1024) void cdf_prefix_kernel(
    const double* __restrict__ tsum, int64_t nt, double* __restrict__ pstart) {
  __shared__ double wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double carry = 0.0;
  for (int64_t b0 = 0; b0 < nt; b0 += 1024) {
    const int64_t i = b0 + tid;
    const double v = i < nt ? tsum[i] : 0.0;
    double incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    double woff = 0.0, tot = 0.0;
    for (int q = 0; q < 16; ++q) {
      if (q < wid) woff += wsum[q];
      tot += wsum[q];
    }
    if (i < nt) pstart[i] = carry + woff + incl - v;
    __syncthreads();
    carry += tot;
  }
}

// integer increment of w on the grid of binade e; false if it cannot be
// taken on the fast path (tie, negative, non-finite, too large)
__device__ inline bool grid_increment(double w, int e, long long& dq) {
  const double v = ldexp(w, 52 - e);
  if (!(w >= 0.0) || !(v < 0x1p62)) return false;
  const double fl = floor(v);
  const double fr = v - fl;
  dq = static_cast<long long>(fl) + (fr > 0.5 ? 1 : 0);
  return fr != 0.5;
}

__global__ __launch_bounds__(kCdfThreads) void cdf_tile_plan_kernel(
    const double* __restrict__ w, int64_t n, const double* __restrict__ tsum,
    const double* __restrict__ pstart, double rel, int* __restrict__ e_t,
    long long* __restrict__ T_t) {
  __shared__ long long red[kCdfThreads / 64];
  __shared__ int any_bad;
  const int64_t t = blockIdx.x;
  const int64_t base = t * kCdfTile;
  const double P0 = pstart[t];
  const double P1 = P0 + tsum[t];
  bool slow = !(P0 >= 0x1p-1000) || !(P1 < 0x1p1000) || t == 0;
  int e = 0;
  if (!slow) {
    e = ilogb(P0 * (1.0 - rel));
    slow = e != ilogb(P1 * (1.0 + rel));
  }
  if (slow) {  // block-uniform
    if (threadIdx.x == 0) {
      e_t[t] = kCdfSlow;
      T_t[t] = 0;
    }
    return;
  }
  if (threadIdx.x == 0) any_bad = 0;
  __syncthreads();
  long long sum = 0;
  bool ok = true;
#pragma unroll
  for (int q = 0; q < kCdfItems; ++q) {
    const int64_t i = base + q * kCdfThreads + threadIdx.x;
    if (i < n) {
      long long dq = 0;
      ok &= grid_increment(w[i], e, dq);
      sum += dq;
    }
  }
  if (!ok) any_bad = 1;
  sum = block_sum<long long, kCdfThreads>(sum, red);
  if (threadIdx.x == 0) {
    e_t[t] = any_bad ? kCdfSlow : e;
    T_t[t] = sum;
  }
}

// One wave walks the tile records.  A run of fast tiles of one binade e is
// advanced in parallel: C_in(k) = C_i + (prefix of T over the run), valid up
// to the first tile whose end would leave the binade (found by a wave min);
// the chain value at the run start is checked to lie in binade e.  A tile
// that cannot start a run goes through exact_tile_wave.
constexpr int kChainPer = kChainChunk / 64;

__global__ __launch_bounds__(64) void cdf_chain_kernel(
    const double* __restrict__ w, int64_t n, int64_t nt,
    const int* __restrict__ e_t, const long long* __restrict__ T_t,
    long long* __restrict__ c_start, double* __restrict__ cdf,
    double* __restrict__ last) {
  const int lane = threadIdx.x;
  double c = 0.0;  // chain value (wave-uniform)
  for (int64_t t0 = 0; t0 < nt; t0 += kChainChunk) {
    const int cn = static_cast<int>(nt - t0 < kChainChunk ? nt - t0 : kChainChunk);
    // this lane's records k = lane*kChainPer + q: e, T, exclusive prefix
    int re[kChainPer];
    long long rT[kChainPer], rP[kChainPer];
    long long run = 0;
#pragma unroll
    for (int q = 0; q < kChainPer; ++q) {
      const int k = lane * kChainPer + q;
      re[q] = k < cn ? e_t[t0 + k] : kCdfSlow;
      rT[q] = k < cn ? T_t[t0 + k] : 0;
      rP[q] = run;
      run += rT[q];
    }
    const long long lincl = wave_incl_scan(run);
    const long long lexcl = lincl - run;
#pragma unroll
    for (int q = 0; q < kChainPer; ++q) rP[q] += lexcl;
    int i = 0;
    while (i < cn) {
      const int owner = i / kChainPer, qi = i - owner * kChainPer;
      int e_i = 0;
      long long P_i = 0;
#pragma unroll
      for (int q = 0; q < kChainPer; ++q)
        if (q == qi) {
          e_i = re[q];
          P_i = rP[q];
        }
      e_i = __builtin_amdgcn_readlane(e_i, owner);
      P_i = readlane_i64(P_i, owner);
      int j = i;
      if (e_i != kCdfSlow) {
        const double lo = ldexp(1.0, e_i);
        if (c >= lo && c < 2.0 * lo) {
          const long long Ci = static_cast<long long>(ldexp(c, 52 - e_i));
          // first record >= i that breaks the run
          int my_end = cn;
#pragma unroll
          for (int q = 0; q < kChainPer; ++q) {
            const int k = lane * kChainPer + q;
            if (k >= i && k < cn && k < my_end &&
                (re[q] != e_i || Ci + (rP[q] - P_i) + rT[q] > kBinadeTop))
              my_end = k;
          }
          j = wave_min_int(my_end);
#pragma unroll
          for (int q = 0; q < kChainPer; ++q) {
            const int k = lane * kChainPer + q;
            if (k >= i && k < j) c_start[t0 + k] = Ci + (rP[q] - P_i);
          }
          if (j > i) {
            // chain value after tile j-1 = start of j (or chunk end)
            long long Pj = 0;
            const int oj = (j - 1) / kChainPer, qj = (j - 1) - oj * kChainPer;
#pragma unroll
            for (int q = 0; q < kChainPer; ++q)
              if (q == qj) Pj = rP[q] + rT[q];
            Pj = readlane_i64(Pj, oj);
            c = ldexp(static_cast<double>(Ci + (Pj - P_i)), e_i - 52);
          }
        }
      }
      if (j == i) {  // tile i cannot start a run: exact walk
        const int64_t t = t0 + i;
        const int64_t base = t * kCdfTile;
        const int tile_n = static_cast<int>(n - base < kCdfTile ? n - base : kCdfTile);
        if (t == 0) {  // tile 0 is always slow: its dense binade exits first
          const int h = tile_n < kHeadSeq ? tile_n : kHeadSeq;
          head_seq_wave(w, h, c, cdf);
          if (tile_n > h) exact_tile_wave(w, h, tile_n - h, c, cdf);
        } else {
          exact_tile_wave(w, base, tile_n, c, cdf);
        }
        if (lane == 0) c_start[t] = -1;
        j = i + 1;
      }
      i = j;
    }
  }
  if (lane == 0) *last = c;
}

__global__ __launch_bounds__(kCdfThreads) void cdf_write_kernel(
    const double* __restrict__ w, int64_t n, const int* __restrict__ e_t,
    const long long* __restrict__ c_start, const double* __restrict__ last,
    double* __restrict__ cdf) {
  __shared__ long long wsum[kCdfThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t t = blockIdx.x;
  const int64_t base = t * kCdfTile;
  const double L = *last;
  const long long C0 = c_start[t];
  if (C0 < 0) {  // slow tile: raw values written by the chain kernel
#pragma unroll
    for (int q = 0; q < kCdfItems; ++q) {
      const int64_t i = base + q * kCdfThreads + tid;
      if (i < n) cdf[i] = cdf[i] / L;
    }
    return;
  }
  const int e = e_t[t];
  long long dl[kCdfItems];
  long long tsum = 0;
#pragma unroll
  for (int q = 0; q < kCdfItems; ++q) {
    const int64_t i = base + static_cast<int64_t>(tid) * kCdfItems + q;
    long long dq = 0;
    if (i < n) (void)grid_increment(w[i], e, dq);
    tsum += dq;
    dl[q] = tsum;
  }
  long long incl = tsum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  long long woff = 0;
  for (int q = 0; q < wid; ++q) woff += wsum[q];
  const long long excl = woff + incl - tsum;
#pragma unroll
  for (int q = 0; q < kCdfItems; ++q) {
    const int64_t i = base + static_cast<int64_t>(tid) * kCdfItems + q;
    if (i < n)
      cdf[i] = ldexp(static_cast<double>(C0 + excl + dl[q]), e - 52) / L;
  }
}

static int64_t cdf_tiles(int64_t n) { return ceil_div(n, kCdfTile); }

// first index i with cdf[i] > u (numpy searchsorted side='right'); with a
// bucket table (abc_cdf_index_f64: tab[k] = first i with cdf[i] > k / 2^L)
// the answer lies in [tab[k], tab[k+1]] for k = floor(u 2^L) -- u 2^L is
// exact -- so the dependent-load chain shrinks from log2 N to the log2 of
// one bucket (about log2(N / 2^L) steps for spread weights)
__device__ inline int64_t search_right(const double* __restrict__ cdf, int64_t n,
                                       double u,
                                       const int64_t* __restrict__ tab = nullptr,
                                       int log2k = 0) {
  int64_t lo = 0, hi = n;
  if (tab) {
    const int64_t k = static_cast<int64_t>(ldexp(u, log2k));
    lo = tab[k];
    hi = tab[k + 1];
  }
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cdf[mid] <= u)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// EXACT: d == D, so every loop bound and stride is a compile-time constant
// (the shared factor's rows then load as wide scalar loads instead of one
// dependent s_load per element).  The perturbation is accumulated row of A
// by row (k outer), each component's fma chain in ascending k as before:
// the same bits.
template <int D, bool EXACT = false>
__device__ inline void perturb_one(const double* __restrict__ X, int64_t N,
                                   int d_arg, const double* __restrict__ cdf,
                                   double u, const double (&z)[D],
                                   const double* __restrict__ A,
                                   const double* __restrict__ lo,
                                   const double* __restrict__ scale,
                                   double* __restrict__ theta_row,
                                   int64_t* idx_out, uint8_t* sup_out,
                                   int64_t a_stride = 0,
                                   const int64_t* __restrict__ tab = nullptr,
                                   int log2k = 0) {
  const int d = EXACT ? D : d_arg;
  int64_t idx = search_right(cdf, N, u, tab, log2k);
  const int64_t idx_c = idx < N ? idx : N - 1;  // numpy would raise; u<1 always
  A += idx_c * a_stride;  // per-particle factor (LocalTransition) or shared
  double pl[D];
#pragma unroll
  for (int l = 0; l < D; ++l) pl[l] = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    if (k < d) {
      const double zk = z[k];
      const double* __restrict__ Ak = A + k * d;
#pragma unroll
      for (int l = 0; l < D; ++l)
        if (l < d) pl[l] = fma(zk, Ak[l], pl[l]);
    }
  }
  bool ok = true;
#pragma unroll
  for (int l = 0; l < D; ++l) {
    if (l < d) {
      const double p = pl[l];
      const double th = X[idx_c * d + l] + p;
      theta_row[l] = th;
      if (lo) {
        const double x = (th - lo[l]) / scale[l];
        ok = ok && (x >= 0.0) && (x <= 1.0);
      }
    }
  }
  *idx_out = idx;
  *sup_out = ok ? 1 : 0;
}

// a_stride = 0: one factor A for every draw (MultivariateNormalTransition);
// a_stride = d*d: A[idx] per resampled particle (LocalTransition)
template <int D>
__global__ __launch_bounds__(256) void resample_perturb_kernel(
    const double* __restrict__ X, int64_t N, int d,
    const double* __restrict__ cdf, const double* __restrict__ u,
    const double* __restrict__ z, const double* __restrict__ A,
    const double* __restrict__ lo, const double* __restrict__ scale,
    int64_t B, double* __restrict__ theta, int64_t* __restrict__ idx,
    uint8_t* __restrict__ sup, int64_t a_stride) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double zz[D];
#pragma unroll
  for (int k = 0; k < D; ++k) zz[k] = k < d ? z[b * d + k] : 0.0;
  perturb_one<D>(X, N, d, cdf, u[b], zz, A, lo, scale, theta + b * d, idx + b,
                 sup + b, a_stride);
}

// fp32 storage form (SURVEY 8(b) abc_resample_perturb_f32): X, z, A and
// theta in fp32, the perturbation z A accumulated in fp32 in the same order
// as the fp64 kernel; the CDF search and the support test ((theta - lo) /
// scale in fp64 on the fp32 theta) as in perturb_one.  12d + 25 B/proposal.
template <int D>
__global__ __launch_bounds__(256) void resample_perturb_f32_kernel(
    const float* __restrict__ X, int64_t N, int d,
    const double* __restrict__ cdf, const double* __restrict__ u,
    const float* __restrict__ z, const float* __restrict__ A,
    const double* __restrict__ lo, const double* __restrict__ scale,
    int64_t B, float* __restrict__ theta, int64_t* __restrict__ idx,
    uint8_t* __restrict__ sup) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t i = search_right(cdf, N, u[b]);
  const int64_t ic = i < N ? i : N - 1;
  float zz[D];
#pragma unroll
  for (int k = 0; k < D; ++k) zz[k] = k < d ? z[b * d + k] : 0.0f;
  bool ok = true;
#pragma unroll
  for (int l = 0; l < D; ++l) {
    if (l < d) {
      float p = 0.0f;
#pragma unroll
      for (int k = 0; k < D; ++k)
        if (k < d) p = fmaf(zz[k], A[k * d + l], p);
      const float th = X[ic * d + l] + p;
      theta[b * d + l] = th;
      if (lo) {
        const double x = (static_cast<double>(th) - lo[l]) / scale[l];
        ok = ok && (x >= 0.0) && (x <= 1.0);
      }
    }
  }
  idx[b] = i;
  sup[b] = ok ? 1 : 0;
}

// The production proposal draws as arrays (SURVEY 8(b) abc_philox_fill):
// u[i] = the uniform of proposal offset + i, z[i*dz + k] its k-th normal
// (dz = nz / nu), so abc_resample_perturb_f64 on (u, z) reproduces
// abc_propose_philox_f64 at the same (seed, sid, offset) bit for bit.
template <typename T>
__global__ __launch_bounds__(256) void philox_fill_kernel(
    uint64_t seed, uint64_t sid, uint64_t offset, int64_t nu, int64_t dz,
    int64_t nz, double* __restrict__ u, T* __restrict__ z) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < nu) {
    const uint64_t ui = offset + static_cast<uint64_t>(i);
    const u32x4 b = philox_block(seed, 2 * sid, ui >> 1);
    u[i] = (ui & 1) ? u53(b.z, b.w) : u53(b.x, b.y);
  }
  if (i < nz) {
    const uint64_t zi = offset * static_cast<uint64_t>(dz) + static_cast<uint64_t>(i);
    double c0, c1;
    box_muller(philox_block(seed, 2 * sid + 1, zi >> 1), c0, c1);
    z[i] = static_cast<T>((zi & 1) ? c1 : c0);
  }
}

// Production proposals: u from stream (2*sid), z from stream (2*sid+1).
//   u[b]   = philox_uniform(seed, 2*sid,   offset + b)
//   z[b,k] = philox_normal (seed, 2*sid+1, (offset + b) * d + k)
template <int D, bool EXACT>
__global__ __launch_bounds__(256) void propose_philox_kernel(
    const double* __restrict__ X, int64_t N, int d_arg,
    const double* __restrict__ cdf, const double* __restrict__ A,
    const double* __restrict__ lo, const double* __restrict__ scale,
    uint64_t seed, uint64_t sid, uint64_t offset, int64_t B,
    double* __restrict__ theta, int64_t* __restrict__ idx,
    uint8_t* __restrict__ sup, const int64_t* __restrict__ tab, int log2k) {
  const int d = EXACT ? D : d_arg;
  // the shared factor A through LDS: read directly, the compiler hoists all
  // d*d uniform elements into SGPRs and spills them to VGPR lanes (5344
  // v_readlane per thread at d = 20; the waves waited ~95 % of their time)
  __shared__ double As[D * D];
  for (int i = threadIdx.x; i < d * d; i += blockDim.x) As[i] = A[i];
  __syncthreads();
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t ui = offset + static_cast<uint64_t>(b);
  const u32x4 ub = philox_block(seed, 2 * sid, ui >> 1);
  const double u = (ui & 1) ? u53(ub.z, ub.w) : u53(ub.x, ub.y);
  double zz[D];
  philox_normals<D>(seed, 2 * sid + 1, ui * static_cast<uint64_t>(d), d, zz);
  perturb_one<D, EXACT>(X, N, d, cdf, u, zz, As, lo, scale, theta + b * d, idx + b,
                        sup + b, 0, tab, log2k);
}

// Round 6: four lanes per proposal.  One lane
// per proposal (propose_philox_kernel) keeps d normals and d outputs live
// (108 VGPRs at d = 20: four waves per SIMD) and every load instruction of
// the CDF search and the X row touches 64 unrelated lines; its waves spend
// ~75 % of their life waiting on those loads (PMC, profiles/r06_propose_pmc
// .json).  Here lane q of a proposal's group of four draws Box-Muller pairs
// q, q + 4, ... of the proposal's normal range and owns outputs l = q,
// q + 4, ...; every output's fma chain is perturb_one's (k ascending from
// 0.0), so u, z and theta are the same bits.  The group's four lanes search
// the same CDF addresses (one line request instead of four) and read / write
// the X and theta rows as contiguous 32-byte runs.  OUT = outputs per lane
// (ceil(d / 4)), PR = pairs per lane.
//
// LDS: the factor as At[k][q][m] = A[k][q + 4 m] (zero where q + 4 m >= d),
// so lane q reads its OUT factors of row k as one contiguous run and the
// fma chain runs unmasked (a zero term leaves an unused accumulator at
// +0.0); the group's normals as zb[group][2 pr + br] (component k at
// k + odd), so z_k is one broadcast LDS read.  The first group form picked
// z_k out of registers with a select chain plus a two-dword shuffle and
// guarded every fma with an exec-mask branch: ~36 VALU per k (PMC r06m,
// 1755 VALU per wave at d = 20).
template <int OUT>
constexpr int group_pairs() { return (4 * OUT + 2 + 7) / 8; }
constexpr int kGroupZld(int pr) { return 8 * pr + 1; }  // odd: spreads the banks

template <int OUT>
__global__ __launch_bounds__(256) void propose_group_kernel(
    const double* __restrict__ X, int64_t N, int d,
    const double* __restrict__ cdf, const double* __restrict__ A,
    const double* __restrict__ lo, const double* __restrict__ scale,
    uint64_t seed, uint64_t sid, uint64_t offset, int64_t B,
    double* __restrict__ theta, int64_t* __restrict__ idx,
    uint8_t* __restrict__ sup, const int64_t* __restrict__ tab, int log2k) {
  constexpr int PR = group_pairs<OUT>();
  constexpr int ZLD = kGroupZld(PR);
  constexpr int AW = 4 * OUT;
  extern __shared__ double sh[];
  double* At = sh;              // d * AW
  double* zb = sh + d * AW;     // 64 groups * ZLD
  for (int i = threadIdx.x; i < d * AW; i += blockDim.x) {
    const int k = i / AW, r = i - k * AW;
    const int l = (r % OUT) * 4 + r / OUT;  // r = q * OUT + m -> l = q + 4 m
    At[i] = l < d ? A[k * d + l] : 0.0;
  }
  const int lane = threadIdx.x & 63;
  const int q = lane & 3;
  const int gbase = lane & ~3;
  double* zg = zb + (threadIdx.x >> 2) * ZLD;
  const int64_t b = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 2;
  const bool live = b < B;
  const int64_t bb = live ? b : B - 1;  // padding lanes redo the last proposal
  const uint64_t ui = offset + static_cast<uint64_t>(bb);
  const u32x4 ub = philox_block(seed, 2 * sid, ui >> 1);
  const double u = (ui & 1) ? u53(ub.z, ub.w) : u53(ub.x, ub.y);
  const int64_t i = search_right(cdf, N, u, tab, log2k);
  const int64_t ic = i < N ? i : N - 1;
  const uint64_t zi0 = ui * static_cast<uint64_t>(d);
  const uint64_t p0 = zi0 >> 1;
  const int odd = static_cast<int>(zi0 & 1);
  const int np = (d + odd + 1) >> 1;  // pairs touching components 0 .. d-1
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    const int pr = q + 4 * r;
    if (pr < np) {
      double c0, c1;
      box_muller(philox_block(seed, 2 * sid + 1, p0 + pr), c0, c1);
      zg[2 * pr] = c0;
      zg[2 * pr + 1] = c1;
    }
  }
  // the X row's loads go out before the product (clamped column, masked use)
  double xv[OUT];
#pragma unroll
  for (int m = 0; m < OUT; ++m) {
    const int l = q + 4 * m;
    xv[m] = X[ic * d + (l < d ? l : d - 1)];
  }
  __syncthreads();
  double pl[OUT];
#pragma unroll
  for (int m = 0; m < OUT; ++m) pl[m] = 0.0;
  const double* zk = zg + odd;
  const double* ak = At + q * OUT;
#pragma unroll 2
  for (int k = 0; k < d; ++k) {
    const double z = zk[k];
#pragma unroll
    for (int m = 0; m < OUT; ++m) pl[m] = fma(z, ak[k * AW + m], pl[m]);
  }
  bool ok = true;
#pragma unroll
  for (int m = 0; m < OUT; ++m) {
    const int l = q + 4 * m;
    if (l < d) {
      const double th = xv[m] + pl[m];
      if (live) theta[bb * d + l] = th;
      if (lo) {
        // x = (th - lo) / scale in [0, 1], as perturb_one; the quotient is
        // formed only near the edges: dd > 0 gives x >= 0 (+0 on
        // underflow), and dd < scale (1 - 2^-20) gives x < 1 after rounding
        const double dd = th - lo[l];
        const double sc = scale[l];
        if (!(dd > 0.0 && dd < sc * 0.99999904632568359375)) {
          const double x = dd / sc;
          ok = ok && (x >= 0.0) && (x <= 1.0);
        }
      }
    }
  }
  const uint64_t bad = __ballot(!ok);
  if (live && q == 0) {
    idx[bb] = i;
    sup[bb] = ((bad >> gbase) & 0xFull) ? 0 : 1;
  }
}

// bucket table of the CDF: tab[k] = searchsorted(cdf, k / 2^L, 'right')
__global__ __launch_bounds__(256) void cdf_index_kernel(
    const double* __restrict__ cdf, int64_t n, int log2k,
    int64_t* __restrict__ tab) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (k > (int64_t{1} << log2k)) return;
  tab[k] = search_right(cdf, n, ldexp(static_cast<double>(k), -log2k));
}

// prior sampling at t=0: theta = lo + scale * U  (scipy uniform.rvs)
__global__ __launch_bounds__(256) void prior_uniform_kernel(
    const double* __restrict__ lo, const double* __restrict__ scale, int d,
    uint64_t seed, uint64_t sid, uint64_t offset, int64_t B,
    double* __restrict__ theta) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= B * d) return;
  const int k = static_cast<int>(i % d);
  const uint64_t ui = offset * d + static_cast<uint64_t>(i);
  const u32x4 ub = philox_block(seed, sid, ui >> 1);
  const double u = (ui & 1) ? u53(ub.z, ub.w) : u53(ub.x, ub.y);
  theta[i] = lo[k] + scale[k] * u;
}

// ---------------------------------------------------------------------------
// RNG fills (for tests and for callers that need raw streams)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void philox_uniform_kernel(uint64_t seed,
                                                             uint64_t sid,
                                                             uint64_t offset,
                                                             int64_t n,
                                                             double* __restrict__ u) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ui = offset + static_cast<uint64_t>(i);
  const u32x4 b = philox_block(seed, sid, ui >> 1);
  u[i] = (ui & 1) ? u53(b.z, b.w) : u53(b.x, b.y);
}

__global__ __launch_bounds__(256) void philox_normal_kernel(uint64_t seed,
                                                            uint64_t sid,
                                                            uint64_t offset,
                                                            int64_t n,
                                                            double* __restrict__ z) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t zi = offset + static_cast<uint64_t>(i);
  double c0, c1;
  box_muller(philox_block(seed, sid, zi >> 1), c0, c1);
  z[i] = (zi & 1) ? c1 : c0;
}

// ---------------------------------------------------------------------------
// order-preserving stream compaction of u8 flags -> int64 positions
// ---------------------------------------------------------------------------
constexpr int kCompactBlock = 256;
constexpr int kCompactItems = 16;  // per thread
constexpr int kCompactTile = kCompactBlock * kCompactItems;

__global__ __launch_bounds__(kCompactBlock) void compact_count_kernel(
    const uint8_t* __restrict__ flags, int64_t n, int64_t* __restrict__ counts) {
  __shared__ int64_t red[4];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kCompactTile;
  int64_t c = 0;
  for (int k = 0; k < kCompactItems; ++k) {
    const int64_t i = base + k * kCompactBlock + threadIdx.x;
    if (i < n) c += flags[i] != 0;
  }
  c = block_sum<int64_t, kCompactBlock>(c, red);
  if (threadIdx.x == 0) counts[blockIdx.x] = c;
}

// exclusive scan of the per-tile counts by one block; writes the total
__global__ __launch_bounds__(1024) void compact_scan_kernel(int64_t* __restrict__ counts,
                                                            int64_t ntiles,
                                                            int64_t* __restrict__ total) {
  __shared__ int64_t s[1024];
  int64_t carry = 0;
  for (int64_t base = 0; base < ntiles; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < ntiles ? counts[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int64_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < ntiles) counts[i] = carry + s[threadIdx.x] - v;
    const int64_t tot = s[1023];
    __syncthreads();
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(kCompactBlock) void compact_scatter_kernel(
    const uint8_t* __restrict__ flags, int64_t n,
    const int64_t* __restrict__ offsets, int64_t* __restrict__ out) {
  __shared__ int wsum[4];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kCompactTile;
  int64_t run = offsets[blockIdx.x];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int k = 0; k < kCompactItems; ++k) {
    const int64_t i = base + k * kCompactBlock + threadIdx.x;
    const bool f = i < n && flags[i] != 0;
    const uint64_t m = __ballot(f);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wid] = __popcll(m);
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wid; ++w) woff += wsum[w];
    if (f) out[run + woff + before] = i;
    run += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
}

// gather rows: out[i, :] = src[idx[i], :]   (int64 idx, fp64 rows of width w)
__global__ __launch_bounds__(256) void gather_rows_kernel(
    const double* __restrict__ src, int64_t width, const int64_t* __restrict__ idx,
    int64_t n, double* __restrict__ out) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n * width) return;
  const int64_t i = t / width, k = t % width;
  out[t] = src[idx[i] * width + k];
}

// strided gather of 8-byte words (fp64 or int64 bits; round 6: the accepted
// rows' selection without torch's index_select / cat):
//   out[i * out_ld + k] = src[(idx ? idx[i] : i) * src_ld + k],  k < width
// one thread per word, grid-stride (width is small: d + 1 at most 33)
__global__ __launch_bounds__(256) void gather_words_kernel(
    const uint64_t* __restrict__ src, int64_t src_ld, int64_t width,
    const int64_t* __restrict__ idx, int64_t n, uint64_t* __restrict__ out,
    int64_t out_ld) {
  const int64_t total = n * width;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       t < total; t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t i = t / width, k = t - i * width;
    const int64_t r = idx ? idx[i] : i;
    out[i * out_ld + k] = src[r * src_ld + k];
  }
}

// column gather of a stat-major matrix: out[s * out_ld + i] =
// src[s * src_ld + idx[i]], s < rows (the accepted statistics, [S][B]);
// idx = NULL: a column-block copy
// (one thread per column: its index is read once for all rows; the writes
// of each row stay coalesced across the wave)
__global__ __launch_bounds__(256) void gather_cols_kernel(
    const uint64_t* __restrict__ src, int64_t src_ld, int64_t rows,
    const int64_t* __restrict__ idx, int64_t n, uint64_t* __restrict__ out,
    int64_t out_ld) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t c = idx ? idx[i] : i;
    const uint64_t* __restrict__ sc = src + c;
    uint64_t* __restrict__ oc = out + i;
    int64_t s = 0;
    for (; s + 4 <= rows; s += 4) {  // four independent loads in flight
      const uint64_t v0 = sc[s * src_ld], v1 = sc[(s + 1) * src_ld];
      const uint64_t v2 = sc[(s + 2) * src_ld], v3 = sc[(s + 3) * src_ld];
      oc[s * out_ld] = v0;
      oc[(s + 1) * out_ld] = v1;
      oc[(s + 2) * out_ld] = v2;
      oc[(s + 3) * out_ld] = v3;
    }
    for (; s < rows; ++s) oc[s * out_ld] = sc[s * src_ld];
  }
}

// constant fills and an index ramp (round 6: the calibration / prior
// generations' distances, flags, positions and unit weights without torch
// fill kernels)
__global__ __launch_bounds__(256) void fill_words_kernel(uint64_t* __restrict__ x,
                                                         int64_t n, uint64_t bits) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    x[i] = bits;
}
__global__ __launch_bounds__(256) void fill_u8_kernel(uint8_t* __restrict__ x,
                                                      int64_t n, uint8_t v) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    x[i] = v;
}
__global__ __launch_bounds__(256) void iota_kernel(int64_t* __restrict__ x, int64_t n,
                                                   int64_t start) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       i < n; i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    x[i] = start + i;
}

// ---------------------------------------------------------------------------
static int check_dim(int d) {
  return d >= 1 && d <= 32;
}

#define DISPATCH_D(d, MACRO) \
  if ((d) <= 1) { MACRO(1) } \
  else if ((d) <= 2) { MACRO(2) } \
  else if ((d) <= 4) { MACRO(4) } \
  else if ((d) <= 8) { MACRO(8) } \
  else if ((d) <= 16) { MACRO(16) } \
  else if ((d) <= 24) { MACRO(24) } \
  else { MACRO(32) }

template <typename T>
static int philox_fill_impl(uint64_t seed, uint64_t sid, uint64_t offset,
                            double* u, int64_t nu, T* z, int64_t nz,
                            hipStream_t st) {
  ABC_REQUIRE(nu >= 0 && nz >= 0, "philox_fill: negative size");
  ABC_REQUIRE(nu == 0 || nz % nu == 0,
              "philox_fill: nz must be a multiple of nu (rows of d normals)");
  ABC_REQUIRE((nu == 0 || u) && (nz == 0 || z), "philox_fill: null pointer");
  const int64_t n = nu > nz ? nu : nz;
  if (n == 0) return kOk;
  const int64_t dz = nu ? nz / nu : 1;
  hipLaunchKernelGGL((philox_fill_kernel<T>), dim3(ceil_div(n, 256)), dim3(256),
                     0, st, seed, sid, offset, nu, dz, nz, u, z);
  ABC_LAUNCH_CHECK("philox_fill_kernel");
  return kOk;
}

}  // namespace abc

using namespace abc;

extern "C" {

size_t abc_resample_cdf_workspace_bytes(int64_t n) {
  // tsum, pstart, T_t, c_start (8 B each), e_t (4 B) per tile + last
  return static_cast<size_t>(cdf_tiles(n > 0 ? n : 1)) * 40 + 256;
}

int abc_resample_cdf_f64(const double* w, int64_t n, double* cdf, void* ws,
                         size_t ws_bytes, hipStream_t st) {
  ABC_REQUIRE(n > 0 && w && cdf && ws, "resample_cdf: need n > 0 and buffers");
  ABC_REQUIRE(ws_bytes >= abc_resample_cdf_workspace_bytes(n),
              "resample_cdf: workspace too small");
  const int64_t nt = cdf_tiles(n);
  double* tsum = static_cast<double*>(ws);
  double* pstart = tsum + nt;
  long long* T_t = reinterpret_cast<long long*>(pstart + nt);
  long long* c_start = T_t + nt;
  double* last = reinterpret_cast<double*>(c_start + nt);
  int* e_t = reinterpret_cast<int*>(last + 4);
  // relative margin of the plan's binade test: far above both the chain's
  // accumulated rounding (<= n ulp) and the approximate prefix's
  const double rel = fmax(1e-9, 8.0 * static_cast<double>(n) * 0x1p-53);
  const unsigned g = static_cast<unsigned>(nt);
  hipLaunchKernelGGL(cdf_tile_sum_kernel, dim3(g), dim3(kCdfThreads), 0, st,
                     w, n, tsum);
  hipLaunchKernelGGL(cdf_prefix_kernel, dim3(1), dim3(1024), 0, st, tsum, nt,
                     pstart);
  hipLaunchKernelGGL(cdf_tile_plan_kernel, dim3(g), dim3(kCdfThreads), 0, st,
                     w, n, tsum, pstart, rel, e_t, T_t);
  hipLaunchKernelGGL(cdf_chain_kernel, dim3(1), dim3(64), 0, st, w, n,
                     nt, e_t, T_t, c_start, cdf, last);
  hipLaunchKernelGGL(cdf_write_kernel, dim3(g), dim3(kCdfThreads), 0, st, w, n,
                     e_t, c_start, last, cdf);
  ABC_LAUNCH_CHECK("resample_cdf kernels");
  return kOk;
}

int abc_resample_perturb_f64(const double* X, int64_t N, int d,
                             const double* cdf, const double* u,
                             const double* z, const double* A,
                             const double* lo, const double* scale, int64_t B,
                             double* theta, int64_t* idx, uint8_t* in_support,
                             hipStream_t st) {
  ABC_REQUIRE(check_dim(d), "resample_perturb: unsupported d=%d", d);
  ABC_REQUIRE(N > 0 && B >= 0, "resample_perturb: bad sizes");
  if (B == 0) return kOk;
  ABC_REQUIRE(X && cdf && u && z && A && theta && idx && in_support,
              "resample_perturb: null pointer");
  ABC_REQUIRE((lo == nullptr) == (scale == nullptr),
              "resample_perturb: lo and scale must both be given or NULL");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
#define L(DD)                                                                \
  hipLaunchKernelGGL((resample_perturb_kernel<DD>), dim3(g), dim3(256), 0, st, \
                     X, N, d, cdf, u, z, A, lo, scale, B, theta, idx,         \
                     in_support, int64_t{0});
  DISPATCH_D(d, L)
#undef L
  ABC_LAUNCH_CHECK("resample_perturb_kernel");
  return kOk;
}

int abc_resample_perturb_f32(const float* X, int64_t N, int d,
                             const double* cdf, const double* u,
                             const float* z, const float* A, const double* lo,
                             const double* scale, int64_t B, float* theta,
                             int64_t* idx, uint8_t* in_support,
                             hipStream_t st) {
  ABC_REQUIRE(check_dim(d), "resample_perturb_f32: unsupported d=%d", d);
  ABC_REQUIRE(N > 0 && B >= 0, "resample_perturb_f32: bad sizes");
  if (B == 0) return kOk;
  ABC_REQUIRE(X && cdf && u && z && A && theta && idx && in_support,
              "resample_perturb_f32: null pointer");
  ABC_REQUIRE((lo == nullptr) == (scale == nullptr),
              "resample_perturb_f32: lo and scale must both be given or NULL");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
#define L(DD)                                                                 \
  hipLaunchKernelGGL((resample_perturb_f32_kernel<DD>), dim3(g), dim3(256), 0, \
                     st, X, N, d, cdf, u, z, A, lo, scale, B, theta, idx,      \
                     in_support);
  DISPATCH_D(d, L)
#undef L
  ABC_LAUNCH_CHECK("resample_perturb_f32_kernel");
  return kOk;
}

int abc_philox_fill(uint64_t seed, uint64_t sid, uint64_t offset, double* u,
                    int64_t nu, double* z, int64_t nz, hipStream_t st) {
  return philox_fill_impl<double>(seed, sid, offset, u, nu, z, nz, st);
}

int abc_philox_fill_f32(uint64_t seed, uint64_t sid, uint64_t offset,
                        double* u, int64_t nu, float* z, int64_t nz,
                        hipStream_t st) {
  return philox_fill_impl<float>(seed, sid, offset, u, nu, z, nz, st);
}

int abc_resample_perturb_local_f64(const double* X, int64_t N, int d,
                                   const double* cdf, const double* u,
                                   const double* z, const double* A,
                                   const double* lo, const double* scale,
                                   int64_t B, double* theta, int64_t* idx,
                                   uint8_t* in_support, hipStream_t st) {
  ABC_REQUIRE(check_dim(d), "resample_perturb_local: unsupported d=%d", d);
  ABC_REQUIRE(N > 0 && B >= 0, "resample_perturb_local: bad sizes");
  if (B == 0) return kOk;
  ABC_REQUIRE(X && cdf && u && z && A && theta && idx && in_support,
              "resample_perturb_local: null pointer");
  ABC_REQUIRE((lo == nullptr) == (scale == nullptr),
              "resample_perturb_local: lo and scale must both be given or NULL");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
  const int64_t stride = static_cast<int64_t>(d) * d;
#define L(DD)                                                                \
  hipLaunchKernelGGL((resample_perturb_kernel<DD>), dim3(g), dim3(256), 0, st, \
                     X, N, d, cdf, u, z, A, lo, scale, B, theta, idx,         \
                     in_support, stride);
  DISPATCH_D(d, L)
#undef L
  ABC_LAUNCH_CHECK("resample_perturb_kernel");
  return kOk;
}

int abc_propose_philox_f64(const double* X, int64_t N, int d,
                           const double* cdf, const double* A,
                           const double* lo, const double* scale,
                           uint64_t seed, uint64_t sid, uint64_t offset,
                           int64_t B, double* theta, int64_t* idx,
                           uint8_t* in_support, hipStream_t st) {
  ABC_REQUIRE(check_dim(d), "propose: unsupported d=%d", d);
  ABC_REQUIRE(N > 0 && B >= 0, "propose: bad sizes");
  if (B == 0) return kOk;
  ABC_REQUIRE(X && cdf && A && theta && idx && in_support,
              "propose: null pointer");
  ABC_REQUIRE((lo == nullptr) == (scale == nullptr),
              "propose: lo and scale must both be given or NULL");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
#define LX(DD, EX)                                                              \
  hipLaunchKernelGGL((propose_philox_kernel<DD, EX>), dim3(g), dim3(256), 0, st, \
                     X, N, d, cdf, A, lo, scale, seed, sid, offset, B, theta,    \
                     idx, in_support, nullptr, 0);
#define L(DD)                     \
  if ((DD) <= 8 && d == (DD)) {   \
    LX(DD, (DD) <= 8)             \
  } else {                        \
    LX(DD, false)                 \
  }
  DISPATCH_D(d, L)
#undef L
#undef LX
  ABC_LAUNCH_CHECK("propose_philox_kernel");
  return kOk;
}

int abc_cdf_index_f64(const double* cdf, int64_t n, int log2k, int64_t* tab,
                      hipStream_t st) {
  ABC_REQUIRE(n > 0 && log2k >= 0 && log2k <= 24, "cdf_index: bad sizes");
  ABC_REQUIRE(cdf && tab, "cdf_index: null pointer");
  const int64_t K1 = (int64_t{1} << log2k) + 1;
  hipLaunchKernelGGL(cdf_index_kernel, dim3(ceil_div(K1, 256)), dim3(256), 0,
                     st, cdf, n, log2k, tab);
  ABC_LAUNCH_CHECK("cdf_index_kernel");
  return kOk;
}

int abc_propose_philox_indexed_f64(const double* X, int64_t N, int d,
                                   const double* cdf, const int64_t* tab,
                                   int log2k, const double* A,
                                   const double* lo, const double* scale,
                                   uint64_t seed, uint64_t sid,
                                   uint64_t offset, int64_t B, double* theta,
                                   int64_t* idx, uint8_t* in_support,
                                   hipStream_t st) {
  ABC_REQUIRE(check_dim(d), "propose: unsupported d=%d", d);
  ABC_REQUIRE(N > 0 && B >= 0, "propose: bad sizes");
  ABC_REQUIRE(log2k >= 0 && log2k <= 24, "propose: bad table size");
  if (B == 0) return kOk;
  ABC_REQUIRE(X && cdf && tab && A && theta && idx && in_support,
              "propose: null pointer");
  ABC_REQUIRE((lo == nullptr) == (scale == nullptr),
              "propose: lo and scale must both be given or NULL");
  const unsigned g = static_cast<unsigned>(ceil_div(B, 256));
  if (tuning_knob(kKnobProposeGroup, 1) != 0) {
    // four lanes per proposal (same bits as propose_philox_kernel; N = 1e6,
    // 4.2e6 proposals, tools/propose_group.py, call r06o, one lane -> four:
    // d = 4 0.398 -> 0.219 ms, d = 8 0.375 -> 0.253, d = 12 1.450 -> 0.349,
    // d = 20 1.702 -> 0.538, d = 32 2.099 -> 1.055)
    const unsigned gg = static_cast<unsigned>(ceil_div(B * 4, 256));
#define LG(O)                                                                     \
  {                                                                               \
    const size_t lds = (static_cast<size_t>(d) * 4 * (O) +                       \
                        64 * static_cast<size_t>(kGroupZld(group_pairs<O>()))) * \
                       sizeof(double);                                            \
    hipLaunchKernelGGL((propose_group_kernel<O>), dim3(gg), dim3(256), lds, st,   \
                       X, N, d, cdf, A, lo, scale, seed, sid, offset, B, theta,   \
                       idx, in_support, tab, log2k);                              \
  }
    switch ((d + 3) / 4) {
      case 1: LG(1) break;
      case 2: LG(2) break;
      case 3: LG(3) break;
      case 4: LG(4) break;
      case 5: LG(5) break;
      case 6: LG(6) break;
      case 7: LG(7) break;
      default: LG(8) break;
    }
#undef LG
    ABC_LAUNCH_CHECK("propose_group_kernel");
    return kOk;
  }
#define LX(DD, EX)                                                              \
  hipLaunchKernelGGL((propose_philox_kernel<DD, EX>), dim3(g), dim3(256), 0, st, \
                     X, N, d, cdf, A, lo, scale, seed, sid, offset, B, theta,    \
                     idx, in_support, tab, log2k);
#define L(DD)                     \
  if ((DD) <= 8 && d == (DD)) {   \
    LX(DD, (DD) <= 8)             \
  } else {                        \
    LX(DD, false)                 \
  }
  // exact instantiations (compile-time d) for d <= 8; above, a
  // compile-time d lets the scheduler interleave all d/2 Box-Muller pairs
  // (512 VGPRs and scratch at d >= 16), so d > 8 keeps the runtime-d form
  DISPATCH_D(d, L)
#undef L
#undef LX
  ABC_LAUNCH_CHECK("propose_philox_kernel");
  return kOk;
}

int abc_prior_uniform_f64(const double* lo, const double* scale, int d,
                          uint64_t seed, uint64_t sid, uint64_t offset,
                          int64_t B, double* theta, hipStream_t st) {
  ABC_REQUIRE(d >= 1 && B >= 0, "prior_uniform: bad sizes");
  if (B == 0) return kOk;
  hipLaunchKernelGGL(prior_uniform_kernel, dim3(ceil_div(B * d, 256)),
                     dim3(256), 0, st, lo, scale, d, seed, sid, offset, B,
                     theta);
  ABC_LAUNCH_CHECK("prior_uniform_kernel");
  return kOk;
}

int abc_philox_uniform_f64(uint64_t seed, uint64_t sid, uint64_t offset,
                           int64_t n, double* u, hipStream_t st) {
  ABC_REQUIRE(n >= 0, "philox_uniform: n < 0");
  if (n == 0) return kOk;
  hipLaunchKernelGGL(philox_uniform_kernel, dim3(ceil_div(n, 256)), dim3(256),
                     0, st, seed, sid, offset, n, u);
  ABC_LAUNCH_CHECK("philox_uniform_kernel");
  return kOk;
}

int abc_philox_normal_f64(uint64_t seed, uint64_t sid, uint64_t offset,
                          int64_t n, double* z, hipStream_t st) {
  ABC_REQUIRE(n >= 0, "philox_normal: n < 0");
  if (n == 0) return kOk;
  hipLaunchKernelGGL(philox_normal_kernel, dim3(ceil_div(n, 256)), dim3(256),
                     0, st, seed, sid, offset, n, z);
  ABC_LAUNCH_CHECK("philox_normal_kernel");
  return kOk;
}

size_t abc_compact_workspace_bytes(int64_t n) {
  return static_cast<size_t>(ceil_div(n > 0 ? n : 1, kCompactTile)) * 8 + 64;
}

int abc_compact_flags(const uint8_t* flags, int64_t n, int64_t* out_idx,
                      int64_t* out_count, void* ws, size_t ws_bytes,
                      hipStream_t st) {
  ABC_REQUIRE(n >= 0, "compact: n < 0");
  if (n == 0) {
    ABC_HIP(hipMemsetAsync(out_count, 0, 8, st));
    return kOk;
  }
  const int64_t tiles = ceil_div(n, kCompactTile);
  ABC_REQUIRE(ws_bytes >= static_cast<size_t>(tiles) * 8,
              "compact: workspace too small");
  int64_t* counts = static_cast<int64_t*>(ws);
  hipLaunchKernelGGL(compact_count_kernel, dim3(tiles), dim3(kCompactBlock), 0,
                     st, flags, n, counts);
  ABC_LAUNCH_CHECK("compact_count_kernel");
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, st, counts,
                     tiles, out_count);
  ABC_LAUNCH_CHECK("compact_scan_kernel");
  hipLaunchKernelGGL(compact_scatter_kernel, dim3(tiles), dim3(kCompactBlock),
                     0, st, flags, n, counts, out_idx);
  ABC_LAUNCH_CHECK("compact_scatter_kernel");
  return kOk;
}

int abc_gather_rows_f64(const double* src, int64_t width, const int64_t* idx,
                        int64_t n, double* out, hipStream_t st) {
  ABC_REQUIRE(width > 0 && n >= 0, "gather_rows: bad sizes");
  if (n == 0) return kOk;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(ceil_div(n * width, 256)),
                     dim3(256), 0, st, src, width, idx, n, out);
  ABC_LAUNCH_CHECK("gather_rows_kernel");
  return kOk;
}

// Accepted-row selection (round 6; replaces torch index_select / cat on the
// hot path).  The first-n-by-id population of the reference's samplers
// (sampler/multicore_evaluation_parallel.py:131-132, singlecore.py:19-38):
// rows src[idx[i]] (8-byte words: fp64 parameters, distances, weights, int64
// parent indices) written at out + i * out_ld, so several columns and
// several sampling rounds land in one preallocated buffer.  idx = NULL:
// the identity (a strided row copy).
int abc_gather_words(const void* src, int64_t src_ld, int64_t width,
                     const int64_t* idx, int64_t n, void* out, int64_t out_ld,
                     hipStream_t st) {
  ABC_REQUIRE(width > 0 && n >= 0 && src_ld >= width && out_ld >= width,
              "gather_words: bad sizes (width %lld, ld %lld / %lld)",
              static_cast<long long>(width), static_cast<long long>(src_ld),
              static_cast<long long>(out_ld));
  if (n == 0) return kOk;
  ABC_REQUIRE(src && out, "gather_words: null pointer");
  hipLaunchKernelGGL(gather_words_kernel, dim3(stream_grid(n * width, 256, 4096)),
                     dim3(256), 0, st, static_cast<const uint64_t*>(src), src_ld,
                     width, idx, n, static_cast<uint64_t*>(out), out_ld);
  ABC_LAUNCH_CHECK("gather_words_kernel");
  return kOk;
}

// x[i] = bits (8-byte words: an fp64 or int64 constant), i < n
int abc_fill_words(void* x, int64_t n, uint64_t bits, hipStream_t st) {
  ABC_REQUIRE(n >= 0, "fill_words: n < 0");
  if (n == 0) return kOk;
  ABC_REQUIRE(x, "fill_words: null pointer");
  hipLaunchKernelGGL(fill_words_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256),
                     0, st, static_cast<uint64_t*>(x), n, bits);
  ABC_LAUNCH_CHECK("fill_words_kernel");
  return kOk;
}
// x[i] = v (flags), i < n
int abc_fill_u8(uint8_t* x, int64_t n, int v, hipStream_t st) {
  ABC_REQUIRE(n >= 0 && v >= 0 && v < 256, "fill_u8: bad arguments");
  if (n == 0) return kOk;
  ABC_REQUIRE(x, "fill_u8: null pointer");
  hipLaunchKernelGGL(fill_u8_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0,
                     st, x, n, static_cast<uint8_t>(v));
  ABC_LAUNCH_CHECK("fill_u8_kernel");
  return kOk;
}
// x[i] = start + i, i < n (positions of an all-accepted round)
int abc_iota_i64(int64_t* x, int64_t n, int64_t start, hipStream_t st) {
  ABC_REQUIRE(n >= 0, "iota: n < 0");
  if (n == 0) return kOk;
  ABC_REQUIRE(x, "iota: null pointer");
  hipLaunchKernelGGL(iota_kernel, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, st,
                     x, n, start);
  ABC_LAUNCH_CHECK("iota_kernel");
  return kOk;
}

// Column selection of a stat-major [rows][*] matrix (the accepted
// statistics kept for adaptive distances, sampler/base.py:119-141):
// out[s * out_ld + i] = src[s * src_ld + idx[i]] (idx = NULL: idx[i] = i).
int abc_gather_cols_words(const void* src, int64_t src_ld, int64_t rows,
                          const int64_t* idx, int64_t n, void* out,
                          int64_t out_ld, hipStream_t st) {
  ABC_REQUIRE(rows >= 0 && n >= 0 && out_ld >= n, "gather_cols_words: bad sizes");
  if (n == 0 || rows == 0) return kOk;
  ABC_REQUIRE(src && out, "gather_cols_words: null pointer");
  hipLaunchKernelGGL(gather_cols_kernel, dim3(stream_grid(n, 256, 8192)), dim3(256),
                     0, st, static_cast<const uint64_t*>(src), src_ld, rows, idx, n,
                     static_cast<uint64_t*>(out), out_ld);
  ABC_LAUNCH_CHECK("gather_cols_kernel");
  return kOk;
}

}  // extern "C"

namespace abc {
// Loads this translation unit's code object (HIP loads each one lazily, at
// the first launch of one of its kernels: ~4 ms for local_mfma's inside
// C4's first weighted generation); abc_preload calls every unit's hook.
int preload_propose() { return preload_kernel(cdf_tile_sum_kernel); }
}  // namespace abc
