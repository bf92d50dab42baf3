// Internal interface between kde.hip (direct fp32/fp64 pass) and
// kde_mfma.hip (exact-grid f16-piece MFMA pass): both share the fixed j-segment
// plan, the direct packed population (P[npad][D+1], fp64 for the MFMA
// pass's fixup) and the finalize/underflow-fixup kernels.  Not part of the
// C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace abc {
int kde_padded_dim(int d);
int kde_num_segments(int64_t npad);
constexpr int kKdeRowPad = 64;
int kde_pack_direct_f64(const double* X, const double* w, int64_t n, int d,
                        const double* mu, const double* Us, double* P,
                        int64_t npad, double* lw2max, void* ws,
                        hipStream_t st);
// the exact two-pass fixup (fp64 rows, v_exp_f32 on each term's fraction)
// of the MFMA pass's listed rows: (*n_fix, fix_rows)
int kde_fixup_rows_mfma(const double* Ynew, const double* P, int64_t npad,
                        int d, const double* lw2max, double log_const,
                        const int* n_fix, const int* fix_rows,
                        double* out_logpd, hipStream_t stream);
// workspace of abc_kde_logpdf_mfma[_rows] (partials, refine lists and
// fragments)
size_t kde_mfma_ws_bytes(int64_t M, int64_t npad, int d);
}  // namespace abc
