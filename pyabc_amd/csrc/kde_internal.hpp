// Internal interface between kde.hip (direct fp32/fp64 pass) and
// kde_mfma.hip (exact-grid bf16 MFMA pass): both share the fixed j-segment
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
int kde_finish_mfma(const double* partial, int64_t M, int nseg,
                    const double* Ynew, const double* P, int64_t npad, int d,
                    const double* lw2max, double log_const, double* out_logpd,
                    int* n_fix, int* fix_rows, hipStream_t stream);
}  // namespace abc
