/*
 * libabc_hip — C-ABI of the MI355X (gfx950) per-generation ABC-SMC particle
 * update.  The host side is Python (pyabc_amd/_native.py binds this file with
 * ctypes); any other FFI can bind the same symbols.
 *
 * Every entry point replaces a numpy/scipy expression of the reference
 * chrhck/pyABC 0.10.1 (paths relative to the reference checkout):
 *
 *   conventions
 *   -----------
 *   * all array pointers are DEVICE pointers owned by the caller;
 *   * row-major; statistics are stat-major [S][ld] (one column per particle);
 *   * the last argument is the hipStream_t the work is enqueued on; calls are
 *     asynchronous and never allocate or synchronise (graph-capturable);
 *   * scratch memory is passed as (ws, ws_bytes), sized by the matching
 *     abc_*_workspace_bytes() query;
 *   * return 0 on success, < 0 on error (-1 invalid argument, -2 HIP error,
 *     -3 unsupported dimension); abc_last_error() describes the last failure
 *     of the calling thread.
 */
#ifndef ABC_HIP_H_
#define ABC_HIP_H_

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* abc_last_error(void);
int abc_version(void);
/* Re-read the launch-shape tuning knobs (ABC_KDE_MFMA_SPLIT / _IB / _PIPE /
 * _LDS2 / _SMAJOR, ABC_KDE_TIER, ABC_LZ_IB / _TPB, ABC_KNN_ROWS) from the
 * environment.
 * The library reads them once, at the first launch that consults them; the
 * knobs only change how work maps to the chip, never a result bit
 * (tests/test_gpu_kernels.py knob tests).  No reference counterpart. */
void abc_tuning_reload(void);
/* Load the library's code objects on the current device now (HIP loads each
 * translation unit's code object at the first launch of one of its kernels,
 * which otherwise lands inside the first generation that uses it: ~4 ms for
 * the LocalTransition density pass).  Returns the number of units that did
 * not resolve (0 on a GPU).  Idempotent.  No reference counterpart. */
int abc_preload(void);

/* ---------------- (a1) MultivariateNormalTransition.fit ------------------
 * Replaces smart_cov = np.cov(X, aweights=w)        transition/util.py:4-15
 * and the weight sums of fit_cov                     multivariatenormal.py:67-73
 * out = [sum w, sum w^2, mu[d], C[d*d]] with C = sum w (x-mu)(x-mu)^T; the host
 * finishes cov = C / (sum w - sum w^2 / sum w) * bw(ESS)^2 * scaling. */
size_t abc_moments_workspace_bytes(int d);
int abc_weighted_moments_f64(const double* X, const double* w, int64_t n,
                             int d, double* out, void* ws, size_t ws_bytes,
                             hipStream_t stream);
/* fp32 storage of X and w (SURVEY 8(b) minimum set), the same fp64 sums */
int abc_weighted_moments_f32(const float* X, const float* w, int64_t n,
                             int d, double* out, void* ws, size_t ws_bytes,
                             hipStream_t stream);

/* ---------------- (a2) MultivariateNormalTransition.rvs + prior support ----
 * Replaces np.random.choice(p=w) (cumsum, /= cdf[-1], searchsorted 'right')
 * + np.random.multivariate_normal (z @ sqrt(s)V)     multivariatenormal.py:87-95
 * and the support test prior.pdf(theta) > 0         smc.py:643-645,
 *                                                    random_variables.py:425-452
 * lo/scale may be NULL (no support test). */
size_t abc_resample_cdf_workspace_bytes(int64_t n);
int abc_resample_cdf_f64(const double* w, int64_t n, double* cdf, void* ws,
                         size_t ws_bytes, hipStream_t stream);
int abc_resample_perturb_f64(const double* X, int64_t N, int d,
                             const double* cdf, const double* u,
                             const double* z, const double* A,
                             const double* lo, const double* scale, int64_t B,
                             double* theta, int64_t* idx, uint8_t* in_support,
                             hipStream_t stream);
/* fp32 storage form (X, z, A, theta fp32; z A accumulated in fp32; the CDF
 * search and the support test in fp64): 12d + 25 B per proposal
 *                                                    multivariatenormal.py:87-95 */
int abc_resample_perturb_f32(const float* X, int64_t N, int d,
                             const double* cdf, const double* u,
                             const float* z, const float* A,
                             const double* lo, const double* scale, int64_t B,
                             float* theta, int64_t* idx, uint8_t* in_support,
                             hipStream_t stream);
/* production variant: u, z drawn from Philox4x32-10 (seed, streams 2*sid and
 * 2*sid+1, counter offset) inside the kernel */
int abc_propose_philox_f64(const double* X, int64_t N, int d,
                           const double* cdf, const double* A,
                           const double* lo, const double* scale,
                           uint64_t seed, uint64_t sid, uint64_t offset,
                           int64_t B, double* theta, int64_t* idx,
                           uint8_t* in_support, hipStream_t stream);
/* t = 0 prior draws, RV('uniform', lo, scale).rvs()  random_variables.py:434 */
/* Bucket table of a CDF for the proposal search: tab[k] = searchsorted(cdf,
 * k / 2^log2k, 'right') for k = 0 .. 2^log2k (tab has 2^log2k + 1 entries).
 * abc_propose_philox_indexed_f64 = abc_propose_philox_f64 with the search
 * of u bracketed by tab[floor(u 2^log2k)] .. tab[.. + 1]: identical
 * indices, ~log2(N / 2^log2k) dependent loads instead of log2 N.
 *                                   multivariatenormal.py:89 (choice p=w) */
int abc_cdf_index_f64(const double* cdf, int64_t n, int log2k, int64_t* tab,
                      hipStream_t stream);
int abc_propose_philox_indexed_f64(const double* X, int64_t N, int d,
                                   const double* cdf, const int64_t* tab,
                                   int log2k, const double* A,
                                   const double* lo, const double* scale,
                                   uint64_t seed, uint64_t sid,
                                   uint64_t offset, int64_t B, double* theta,
                                   int64_t* idx, uint8_t* in_support,
                                   hipStream_t stream);
int abc_prior_uniform_f64(const double* lo, const double* scale, int d,
                          uint64_t seed, uint64_t sid, uint64_t offset,
                          int64_t B, double* theta, hipStream_t stream);
int abc_philox_uniform_f64(uint64_t seed, uint64_t sid, uint64_t offset,
                           int64_t n, double* u, hipStream_t stream);
int abc_philox_normal_f64(uint64_t seed, uint64_t sid, uint64_t offset,
                          int64_t n, double* z, hipStream_t stream);
/* The draws of proposals offset .. offset + nu - 1 as arrays (SURVEY 8(b)
 * abc_philox_fill): u[i] from stream 2*sid, z[i*dz + k] (dz = nz / nu) from
 * stream 2*sid+1 -- exactly what abc_propose_philox_f64 draws in-kernel,
 * so abc_resample_perturb_f64(u, z) reproduces it bit for bit. Replaces the
 * numpy draws u = random_sample(), z = standard_normal(d)
 *                                                    multivariatenormal.py:89-94 */
int abc_philox_fill(uint64_t seed, uint64_t sid, uint64_t offset, double* u,
                    int64_t nu, double* z, int64_t nz, hipStream_t stream);
int abc_philox_fill_f32(uint64_t seed, uint64_t sid, uint64_t offset,
                        double* u, int64_t nu, float* z, int64_t nz,
                        hipStream_t stream);
/* order-preserving compaction: proposal ids for in-support draws only
 * (out-of-support redraws are not evaluations, smc.py:629-645) */
size_t abc_compact_workspace_bytes(int64_t n);
int abc_compact_flags(const uint8_t* flags, int64_t n, int64_t* out_idx,
                      int64_t* out_count, void* ws, size_t ws_bytes,
                      hipStream_t stream);
int abc_gather_rows_f64(const double* src, int64_t width, const int64_t* idx,
                        int64_t n, double* out, hipStream_t stream);
/* The accepted population's rows, first n by evaluation id
 *   (sampler/multicore_evaluation_parallel.py:131-132, singlecore.py:19-38):
 * out[i*out_ld + k] = src[(idx ? idx[i] : i)*src_ld + k], k < width, over
 * 8-byte words (fp64 values or int64 indices), so several columns and
 * sampling rounds land in one buffer; idx = NULL is a strided row copy. */
int abc_gather_words(const void* src, int64_t src_ld, int64_t width,
                     const int64_t* idx, int64_t n, void* out, int64_t out_ld,
                     hipStream_t stream);
/* The same selection on a stat-major [rows][ld] matrix (the accepted sum
 * stats, sampler/base.py:119-141): out[s*out_ld + i] = src[s*src_ld + idx[i]]
 * (idx = NULL: a column-block copy) */
int abc_gather_cols_words(const void* src, int64_t src_ld, int64_t rows,
                          const int64_t* idx, int64_t n, void* out,
                          int64_t out_ld, hipStream_t stream);
/* Constant fills and an index ramp for the calibration / prior
 * generations (smc.py:486-534: every proposal accepted, distance inf, weight
 * 1): x[i] = bits (8-byte words), x[i] = v (bytes), x[i] = start + i. */
int abc_fill_words(void* x, int64_t n, uint64_t bits, hipStream_t stream);
int abc_fill_u8(uint8_t* x, int64_t n, int v, hipStream_t stream);
int abc_iota_i64(int64_t* x, int64_t n, int64_t start, hipStream_t stream);
/* Stable LSD radix sort of (key, int32 value) pairs by the low end_bit key
 * bits -- the spatial index's Hilbert-key sort, in place of cKDTree's build
 *                                                 local_transition.py:82-83
 * keys / vals are overwritten (ping-pong); the result goes to keys_out /
 * vals_out. */
size_t abc_radix_sort_workspace_bytes(int64_t n);
int abc_radix_sort_pairs_u64(uint64_t* keys, int32_t* vals, int64_t n,
                             int end_bit, uint64_t* keys_out, int32_t* vals_out,
                             void* ws, size_t ws_bytes, hipStream_t stream);

/* ---------------- (a3) KDE importance-weight pass ------------------------
 * Replaces MultivariateNormalTransition.pdf / pdf_static
 *   sum_j w_j N(theta; X_j, cov) (scipy multivariate_normal(allow_singular))
 *                                                    multivariatenormal.py:102-125
 * called once per accepted particle by transition_pdf smc.py:722-733.
 * Us = U * sqrt(log2(e)/2) with U the scipy _PSD pseudo-inverse root of cov;
 * P is the packed previous population [npad][D+1], D = abc_kde_padded_dim(d),
 * npad a multiple of abc_kde_row_pad(); Ynew is [M][D].
 * out_logpd[i] = log pdf(theta_i) when log_const = -(rank ln 2pi + log_pdet)/2. */
int abc_kde_padded_dim(int d);
int abc_kde_row_pad(void);
/* Number of fixed j-segments of the KDE pass (a function of npad only:
   every row is the fixed-order sum of its segment partials, so results do
   not depend on M or on the number of ranks sharing the rows). */
int abc_kde_segments(int64_t npad);
int abc_kde_split(int64_t M, int64_t npad, int d);
size_t abc_kde_workspace_bytes(int64_t M, int64_t npad, int d);
int abc_whiten_f32(const double* X, int64_t n, int d, const double* mu,
                   const double* Us, float* Y, hipStream_t stream);
int abc_whiten_f64(const double* X, int64_t n, int d, const double* mu,
                   const double* Us, double* Y, hipStream_t stream);
int abc_kde_pack_prev_f32(const double* X, const double* w, int64_t n, int d,
                          const double* mu, const double* Us, float* P,
                          int64_t npad, double* lw2max, void* ws,
                          hipStream_t stream);
int abc_kde_pack_prev_f64(const double* X, const double* w, int64_t n, int d,
                          const double* mu, const double* Us, double* P,
                          int64_t npad, double* lw2max, void* ws,
                          hipStream_t stream);
int abc_kde_logpdf_f32(const float* Ynew, int64_t M, const float* P,
                       int64_t npad, int d, const double* lw2max,
                       double log_const, double* out_logpd, void* ws,
                       size_t ws_bytes, hipStream_t stream);
int abc_kde_logpdf_f64(const double* Ynew, int64_t M, const double* P,
                       int64_t npad, int d, const double* lw2max,
                       double log_const, double* out_logpd, void* ws,
                       size_t ws_bytes, hipStream_t stream);
/* SURVEY 8(b) form on rows already whitened with scipy's U:
 *   out[i] = log_offset + log sum_j exp(logw[j] - |Ynew_i - Yprev_j|^2 / 2)
 * (the host adds -(rank log 2pi + log_pdet)/2 and the prior); Ynew [M*d],
 * Yprev [N*d], logw [N] in T, the same fixed-segment pass as above.
 *                                  multivariatenormal.py:102-125 (scipy _PSD) */
size_t abc_kde_logsum_workspace_bytes_f32(int64_t M, int64_t N, int d);
size_t abc_kde_logsum_workspace_bytes_f64(int64_t M, int64_t N, int d);
int abc_kde_logsum_f32(const float* Ynew, const float* Yprev, const float* logw,
                       int64_t M, int64_t N, int d, float log_offset,
                       float* out_log_sum, void* ws, size_t ws_bytes,
                       hipStream_t stream);
int abc_kde_logsum_f64(const double* Ynew, const double* Yprev,
                       const double* logw, int64_t M, int64_t N, int d,
                       double log_offset, double* out_log_sum, void* ws,
                       size_t ws_bytes, hipStream_t stream);
/* Same density on the matrix cores (v_mfma_f32_32x32x16_f16): the
 * exponent lw2_j - |y_i - y_j|^2 is expanded as a_j + b_i + 2 y_i.y_j with
 * every operand split into f16 pieces on a power-of-two grid so that the
 * large part of the sum is EXACT in the fp32 accumulator (the
 * piece scheme per dimension class is kde_mfma.hip's Mk<D>::SCH).
 * Afr: population fragments (abc_kde_mfma_prev_bytes), built with the
 * fp64 whitened population P [npad][D+1] by abc_kde_pack_prev_mfma (which
 * also writes lw2max and the grid g to gscale; ws >= 128 B).  Bfr: new-row
 * fragments (abc_kde_mfma_new_bytes, abc_kde_mfma_new_rows padded rows) and
 * the fp64 whitened rows Ynew [M][D], built by abc_kde_pack_new_mfma from
 * theta.  Rows whose fp32-exponent sum falls below 2^-32 (of the largest
 * weight's scale) and rows beyond the grid range are re-evaluated exactly in
 * fp64 from Ynew and P; their count is the int32 at byte
 * abc_kde_segments(npad) * M * 8 of the workspace after the call.
 * Workspace: abc_kde_workspace_bytes.
 *
 * The _rows forms (round 5) evaluate each row relative to its own offset
 * row_off[i] (log2 units, <= 0; NULL = 0 for every row):
 * abc_kde_pack_new_mfma_rows writes row_off from the rows' parents
 * (parent[i] = the index into the previous population the proposal was
 * resampled from, smc.py:602-645; NULL: no parents, row_off = 0) using the
 * fp64 population P; abc_kde_logpdf_mfma_rows (which also takes the grid
 * gscale) re-evaluates rows whose sum leaves the folded scheme's routing
 * range on the matrix cores with their own offsets
 * and only the rest exactly in fp64; the int32 after the fixup count is the
 * number of rows re-evaluated.  Same result contract (1e-5 relative).
 *                                          multivariatenormal.py:102-125 */
size_t abc_kde_mfma_prev_bytes(int64_t npad, int d);
int64_t abc_kde_mfma_new_rows(int64_t M, int d);
size_t abc_kde_mfma_new_bytes(int64_t M, int d);
int abc_kde_pack_prev_mfma(const double* X, const double* w, int64_t n, int d,
                           const double* mu, const double* Us, double* P,
                           void* Afr, int64_t npad, double* lw2max,
                           double* gscale, void* ws, hipStream_t stream);
int abc_kde_pack_new_mfma(const double* theta, int64_t M, int d,
                          const double* mu, const double* Us,
                          const double* gscale, double* Ynew, void* Bfr,
                          hipStream_t stream);
int abc_kde_logpdf_mfma(const void* Bfr, const double* Ynew, int64_t M,
                        const void* Afr, const double* P, int64_t npad, int d,
                        const double* lw2max, double log_const,
                        double* out_logpd, void* ws, size_t ws_bytes,
                        hipStream_t stream);
int abc_kde_pack_new_mfma_rows(const double* theta, int64_t M, int d,
                               const double* mu, const double* Us,
                               const double* gscale, const double* P,
                               int64_t npad, const int64_t* parent,
                               double* Ynew, void* Bfr, double* row_off,
                               hipStream_t stream);
int abc_kde_logpdf_mfma_rows(const void* Bfr, const double* Ynew,
                             const double* row_off, int64_t M, const void* Afr,
                             const double* P, int64_t npad, int d,
                             const double* lw2max, const double* gscale,
                             double log_const, double* out_logpd, void* ws,
                             size_t ws_bytes, hipStream_t stream);
/* w = prior_pd / exp(logpd)                          smc.py:776-792
 * prior may be NULL (then prior_const is used for every row) */
int abc_importance_weights_f64(const double* logpd, const double* prior,
                               double prior_const, int64_t M, double* w,
                               hipStream_t stream);

/* ---------------- (a4) weight normalisation / ESS ------------------------
 * Replaces Population._normalize_weights            population.py:120-142
 * and effective_sample_size                         weighted_statistics.py:73-83 */
size_t abc_reduce_workspace_bytes(void);
int abc_sum_f64(const double* x, int64_t n, int squares, double* out,
                void* ws, hipStream_t stream);
int abc_scale_inplace_f64(double* x, int64_t n, const double* divisor,
                          hipStream_t stream);

/* ---------------- (a5) PNormDistance + UniformAcceptor -------------------
 * Replaces PNormDistance.__call__                   distance/distance.py:76-102
 * and accept_use_current_time (d <= eps)            acceptor/acceptor.py:235-244
 * stats_T is [S][ld]; fw = factors * weights in x_0 key order. */
int abc_pnorm_distance_f64(const double* stats_T, int64_t ld,
                           const double* x0, const double* fw, int64_t B,
                           int S, double p, double eps, double* d_out,
                           uint8_t* accept, uint8_t* guard,
                           hipStream_t stream);

/* ---------------- (a6) AdaptivePNormDistance scale functions -------------
 * Replaces median_absolute_deviation / standard_deviation per statistic
 *                                                    distance/scale.py:38-65
 * as gathered by AdaptivePNormDistance._update      distance/distance.py:253-297 */
size_t abc_column_select_workspace_bytes(int S);
/* Median (and MAD when mad_out != NULL) of every column of data_T [S][ld],
 * np.median semantics, bit-exact.  From n = 500000 rows on it synchronises
 * `stream` once per order statistic (a 4-byte read-back of the
 * settled-column count, which skips the radix passes when the sampled
 * bracket settled every column); below that it is the radix select alone,
 * fully asynchronous. */
int abc_column_median_mad_f64(const double* data_T, int64_t ld, int64_t n,
                              int S, double* median_out, double* mad_out,
                              void* ws, size_t ws_bytes, hipStream_t stream);
int abc_column_std_f64(const double* data_T, int64_t ld, int64_t n, int S,
                       double* mean_out, double* std_out, hipStream_t stream);
/* the same over S * bps blocks (one block per column leaves most CUs idle
 * at S = 100): fixed-order partials in ws; mean_out may be NULL */
size_t abc_column_std_workspace_bytes(int64_t n, int S);
int abc_column_std_ws_f64(const double* data_T, int64_t ld, int64_t n, int S,
                          double* mean_out, double* std_out, void* ws,
                          size_t ws_bytes, hipStream_t stream);

/* ---------------- (a7) weighted-quantile epsilon -------------------------
 * Replaces weighted_quantile                        weighted_statistics.py:26-43
 * used by QuantileEpsilon._update                   epsilon/epsilon.py:202-228
 * w may be NULL (uniform weights).  out4 = [eps, p_k, cs_{k-1}, w_k].
 * Tied points form one block of knots at the same p: alpha between the
 * block's first and last knot gives p exactly; the block's end knots take
 * its smallest weight (numpy's unstable argsort leaves their order open). */
size_t abc_wquantile_workspace_bytes(void);
int abc_wquantile_f64(const double* d, const double* w, int64_t n,
                      double alpha, double* out4, void* ws, size_t ws_bytes,
                      hipStream_t stream);
/* The same select as exchangeable steps, for a population sharded over
 * ranks ("the multi-GPU variant exposes its histogram pass so
 * RCCL can all-reduce between passes"; 8(e) epsilon).  Each rank runs the
 * step sequence 0, 1, 2, 3, 10, 20, 11, 21, ..., 17, 27, 30, 31, 33, 32 on its
 * rows (n_local of n_total); after a step, abc_wquantile_exchange names the
 * words of ws to all-reduce across ranks before the next step (offset in
 * bytes, count of int64 words, op 1 = sum, 2 = max, 3 = min, 4 = max of the
 * first word and min of the second).  Every exchanged word is an integer
 * (fixed-point masses, keys), so the result is bit-identical for any rank
 * count and equals abc_wquantile_f64 on the whole population. */
int abc_wquantile_step_f64(int step, const double* d, const double* w,
                           int64_t n_local, int64_t n_total, double alpha,
                           double* out4, void* ws, size_t ws_bytes,
                           hipStream_t stream);
int abc_wquantile_exchange(int step, int64_t* offset_bytes, int64_t* count,
                           int* op);

/* ---------------- (a8) LocalTransition -----------------------------------
 * Replaces cKDTree(X).query(X, k+1)                 local_transition.py:82-83
 * _cov_and_inv / _cov per particle                  local_transition.py:112-139
 * and _pdf_single                                   local_transition.py:103-110 */
size_t abc_knn_workspace_bytes(int64_t N, int k);
int abc_knn_f64(const double* X, int64_t N, int d, int k, int32_t* nbr,
                double* nbr_d2, void* ws, size_t ws_bytes, hipStream_t stream);
int abc_local_cov_f64(const double* X, const double* w, int64_t N, int d,
                      const int32_t* nbr, int k, double scaling,
                      double* covs, double* inv_covs, double* dets,
                      hipStream_t stream);
/* fp32 storage forms (SURVEY 8(b) abc_knn_topk_f32 / abc_local_cov_f32):
 * the fp32 points are widened (exactly) and the fp64 kernels run on them;
 * neighbour sets are those of the fp32 points, results rounded to fp32.
 *                              local_transition.py:82-83, 112-139 */
size_t abc_knn_topk_f32_workspace_bytes(int64_t N, int d, int k);
int abc_knn_topk_f32(const float* X, int64_t N, int d, int k, int32_t* nbr,
                     float* nbr_d2, void* ws, size_t ws_bytes,
                     hipStream_t stream);
size_t abc_local_cov_f32_workspace_bytes(int64_t N, int d);
int abc_local_cov_f32(const float* X, const float* w, int64_t N, int d,
                      const int32_t* nbr, int k, double scaling, float* covs,
                      float* inv_covs, float* dets, void* ws, size_t ws_bytes,
                      hipStream_t stream);
/* The same for the particles [row0, row0 + nrows) only (one rank's share of
 * the fit): nbr / nbr_d2 / covs / inv_covs / dets hold those
 * rows, indexed from row0; every row's result equals the full call's.
 *                                                   local_transition.py:77-96 */
int abc_knn_rows_f64(const double* X, int64_t N, int d, int k, int64_t row0,
                     int64_t nrows, int32_t* nbr, double* nbr_d2, void* ws,
                     size_t ws_bytes, hipStream_t stream);
int abc_local_cov_rows_f64(const double* X, const double* w, int64_t N, int d,
                           const int32_t* nbr, int k, int64_t row0,
                           int64_t nrows, double scaling, double* covs,
                           double* inv_covs, double* dets, hipStream_t stream);
int abc_local_logpdf_f64(const double* pts, int64_t M, const double* X,
                         const double* w, const double* inv_covs,
                         const double* dets, int64_t N, int d,
                         double* out_logpdf, void* ws, size_t ws_bytes,
                         hipStream_t stream);
size_t abc_local_logpdf_workspace_bytes(int64_t M, int64_t N);
/* the same density with the pair loop in fp32 (1e-5 relative; rows whose
 * sum falls below 2^-60 are re-evaluated exactly in fp64) */
int abc_local_logpdf_f32(const double* pts, int64_t M, const double* X,
                         const double* w, const double* inv_covs,
                         const double* dets, int64_t N, int d,
                         double* out_logpdf, void* ws, size_t ws_bytes,
                         hipStream_t stream);
size_t abc_local_logpdf_f32_workspace_bytes(int64_t M, int64_t N);
/* the same density on the f16 matrix cores ("z form": q = |L^T (theta - X_n)|^2
 * with inv_n = L L^T, the GEMM on exact-grid f16 pieces, local_mfma.hip;
 * rows whose sum falls below 2^-32 are re-evaluated exactly in fp64) */
int abc_local_logpdf_mfma(const double* pts, int64_t M, const double* X,
                          const double* w, const double* inv_covs,
                          const double* dets, int64_t N, int d,
                          double* out_logpdf, void* ws, size_t ws_bytes,
                          hipStream_t stream);
size_t abc_local_logpdf_mfma_workspace_bytes(int64_t M, int64_t N, int d);
/* LocalTransition.rvs_single                        local_transition.py:141-145
 * (CDF index as abc_propose_philox_f64; Cholesky factor of C[idx]) */
int abc_propose_local_philox_f64(const double* X, int64_t N, int d,
                                 const double* cdf, const double* covs,
                                 const double* lo, const double* scale,
                                 uint64_t seed, uint64_t sid, uint64_t offset,
                                 int64_t B, double* theta, int64_t* idx,
                                 uint8_t* in_support, hipStream_t stream);
/* Parity form of the same draw with the caller's uniforms u[B] and normals
 * z[B*d] and the reference's own factor: A[N][d][d] = sqrt(s)[:,None] * V
 * from numpy svd(C_n) (legacy multivariate_normal), theta = X[idx] +
 * z @ A[idx], idx = searchsorted(cdf, u, 'right').
 *                                                   local_transition.py:141-145 */
int abc_resample_perturb_local_f64(const double* X, int64_t N, int d,
                                   const double* cdf, const double* u,
                                   const double* z, const double* A,
                                   const double* lo, const double* scale,
                                   int64_t B, double* theta, int64_t* idx,
                                   uint8_t* in_support, hipStream_t stream);

/* ---------------- synthetic batch simulators (benchmark models) ----------
 * linear-Gaussian y = A theta + c + sigma eps (SURVEY configs C2/C5) and the
 * quickstart Gaussian mean model (doc/examples/parameter_inference.ipynb). */
int abc_sim_linear_gaussian_f64(const double* theta, int64_t B, int d,
                                const double* A, const double* c, int S,
                                double sigma, uint64_t seed, uint64_t sid,
                                uint64_t offset, double* out_T, int64_t ld,
                                hipStream_t stream);
/* Fused simulation + p-norm distance + uniform acceptance for rounds whose
 * statistics are not kept: per proposal the column of
 * abc_sim_linear_gaussian_f64 (same arithmetic, same Philox noise) goes
 * straight into the abc_pnorm_distance_f64 chain without being stored;
 * d_out / accept / guard are bit-identical to the two calls.
 * Replaces model(par) + distance(x, x_0) + acceptor  smc.py:650-700,
 *                                 distance/distance.py:76-102,
 *                                 acceptor/acceptor.py:235-244 */
int abc_sim_linear_gaussian_pnorm_f64(const double* theta, int64_t B, int d,
                                      const double* A, const double* c, int S,
                                      double sigma, uint64_t seed, uint64_t sid,
                                      uint64_t offset, const double* x0,
                                      const double* fw, double p, double eps,
                                      double* d_out, uint8_t* accept,
                                      uint8_t* guard, hipStream_t stream);
/* The same pass for rounds whose statistics ARE kept (stored population,
 * recorded evaluations, adaptive distances): the columns are also written
 * to out_T (stat-major [S][ld], ld >= B) as abc_sim_linear_gaussian_f64
 * writes them, so the distance pass does not read them back. */
int abc_sim_linear_gaussian_pnorm_stats_f64(
    const double* theta, int64_t B, int d, const double* A, const double* c,
    int S, double sigma, uint64_t seed, uint64_t sid, uint64_t offset,
    const double* x0, const double* fw, double p, double eps, double* d_out,
    uint8_t* accept, uint8_t* guard, double* out_T, int64_t ld,
    hipStream_t stream);
int abc_sim_gaussian_mean_f64(const double* theta, int64_t B, double sigma,
                              uint64_t seed, uint64_t sid, uint64_t offset,
                              double* out, hipStream_t stream);

/* ---------------- (f3) exact inference: stochastic acceptance -------------
 * SURVEY 8(f) rank 3.  Replaces, per evaluation b (stat-major stats_T):
 *   IndependentNormalKernel.__call__  (kind 0, prm = var)  distance/kernel.py:256-282
 *     pd = -0.5 * (c + np.sum(diff**2 / var))
 *   IndependentLaplaceKernel.__call__ (kind 1, prm = b)    distance/kernel.py:332-357
 *     pd = -(c + np.sum(|diff| / b))
 * with c the kernel's constant np.sum(log 2 [+ log pi] + log prm) (host) and
 * numpy's pairwise summation order (bit-identical); S <= 4096.  When accept
 * is non-NULL the StochasticAcceptor decision is fused (SCALE_LOG):
 *   StochasticAcceptor.__call__                            acceptor/acceptor.py:440-473
 *     acc = exp((pd - pdf_norm) * inv_temp); accept = acc >= u;
 *     accw = acc == 0 ? 0 : (apply_iw ? acc / min(1, acc) : 1)
 * u[b] is injected (u != NULL) or Philox stream (seed, stream) counter
 * offset + b; guard[b] flags |acc - u| <= 4 ulp. */
int abc_stochastic_kernel_f64(const double* stats_T, int64_t ld,
                              const double* x0, const double* prm, int S,
                              int kind, double c, int64_t B, double* pd,
                              double pdf_norm, double inv_temp, int apply_iw,
                              const double* u, uint64_t seed, uint64_t stream,
                              uint64_t offset, uint8_t* accept, double* accw,
                              uint8_t* guard, hipStream_t stream_);
/* StochasticAcceptor decision for given densities, SCALE_LOG (log_scale=1)
 * or SCALE_LIN: acc = (pd / pdf_norm) ** inv_temp.   acceptor/acceptor.py:456-473 */
int abc_stochastic_accept_f64(const double* pd, int64_t B, double pdf_norm,
                              double inv_temp, int log_scale, int apply_iw,
                              const double* u, uint64_t seed, uint64_t stream,
                              uint64_t offset, uint8_t* accept, double* accw,
                              uint8_t* guard, hipStream_t stream_);
/* weight = prior_pd * acceptance_weight * 1 / transition_pd  smc.py:776-792
 * (logpd == NULL at t = 0: prior_const * s_i,                smc.py:762-770) */
int abc_importance_weights_scaled_f64(const double* logpd, const double* s,
                                      double prior_const, int64_t M, double* w,
                                      hipStream_t stream);
/* Temperature-scheme sums (epsilon/temperature.py:306-345 AcceptanceRateScheme
 * objective with weights t_pd / t_pd_prev, :695-742 EssScheme):
 *   w_i = (w ? w_i : 1) * (logw_num ? exp(logw_num_i - (logw_den ? logw_den_i : 0)) : 1)
 *   v = exp((pd - c) beta_k) [log] or (pd / c)^beta_k [lin], min(v, 1) if clamp
 *   out[0] = sum w, out[1] = sum w^2, out[2+2k] = sum w v, out[3+2k] = sum (w v)^2
 * for k < K (<= 16).  Deterministic fixed-order reduction. */
size_t abc_tempered_sums_workspace_bytes(int K);
int abc_tempered_sums_f64(const double* pd, const double* w,
                          const double* logw_num, const double* logw_den,
                          int64_t n, double c, int log_scale,
                          const double* betas, int K, int clamp, double* out,
                          void* ws, size_t ws_bytes, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* ABC_HIP_H_ */
