"""ctypes binding of ``libabc_hip.so`` (declared in ``include/abc_hip.h``).

The library is built in-tree (``make -C pyabc_amd/csrc``) for gfx950 and is
the ONLY compute path of this package: if it is missing or fails to load, every
device operation raises ``NativeLibraryError``; nothing falls back to the CPU.

torch is imported first so that the HIP runtime torch ships with is the one
the library's ``libamdhip64.so.7`` dependency resolves to (one runtime per
process; streams from ``torch.cuda.current_stream()`` are valid handles).
"""
import ctypes
import os

import torch  # noqa: F401  (loads the process-wide HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libabc_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "abc_hip.h")


class NativeLibraryError(RuntimeError):
    """The HIP library is missing, failed to load, or a call failed."""


c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int
c_dbl = ctypes.c_double
c_size = ctypes.c_size_t
c_ptr = ctypes.c_void_p

# name -> (restype, argtypes)
_SIGS = {
    "abc_last_error": (ctypes.c_char_p, []),
    "abc_version": (c_int, []),
    "abc_tuning_reload": (None, []),
    "abc_preload": (c_int, []),
    # (a1)
    "abc_moments_workspace_bytes": (c_size, [c_int]),
    "abc_weighted_moments_f64": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr,
                                         c_ptr, c_size, c_ptr]),
    # (a2)
    "abc_resample_cdf_workspace_bytes": (c_size, [c_i64]),
    "abc_resample_cdf_f64": (c_int, [c_ptr, c_i64, c_ptr, c_ptr, c_size,
                                     c_ptr]),
    "abc_resample_perturb_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                         c_ptr, c_ptr, c_ptr, c_ptr, c_i64,
                                         c_ptr, c_ptr, c_ptr, c_ptr]),
    "abc_propose_philox_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                       c_ptr, c_ptr, c_u64, c_u64, c_u64,
                                       c_i64, c_ptr, c_ptr, c_ptr, c_ptr]),
    "abc_cdf_index_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr]),
    "abc_propose_philox_indexed_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr,
                                               c_ptr, c_int, c_ptr, c_ptr,
                                               c_ptr, c_u64, c_u64, c_u64,
                                               c_i64, c_ptr, c_ptr, c_ptr,
                                               c_ptr]),
    "abc_prior_uniform_f64": (c_int, [c_ptr, c_ptr, c_int, c_u64, c_u64,
                                      c_u64, c_i64, c_ptr, c_ptr]),
    "abc_philox_uniform_f64": (c_int, [c_u64, c_u64, c_u64, c_i64, c_ptr,
                                       c_ptr]),
    "abc_philox_normal_f64": (c_int, [c_u64, c_u64, c_u64, c_i64, c_ptr,
                                      c_ptr]),
    "abc_compact_workspace_bytes": (c_size, [c_i64]),
    "abc_compact_flags": (c_int, [c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_size,
                                  c_ptr]),
    "abc_gather_rows_f64": (c_int, [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr]),
    "abc_gather_words": (c_int, [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr,
                                 c_i64, c_ptr]),
    "abc_gather_cols_words": (c_int, [c_ptr, c_i64, c_i64, c_ptr, c_i64,
                                      c_ptr, c_i64, c_ptr]),
    "abc_fill_words": (c_int, [c_ptr, c_i64, c_u64, c_ptr]),
    "abc_fill_u8": (c_int, [c_ptr, c_i64, c_int, c_ptr]),
    "abc_iota_i64": (c_int, [c_ptr, c_i64, c_i64, c_ptr]),
    "abc_radix_sort_workspace_bytes": (c_size, [c_i64]),
    "abc_radix_sort_pairs_u64": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr,
                                         c_ptr, c_ptr, c_size, c_ptr]),
    # (a3)
    "abc_kde_padded_dim": (c_int, [c_int]),
    "abc_kde_row_pad": (c_int, []),
    "abc_kde_segments": (c_int, [c_i64]),
    "abc_kde_split": (c_int, [c_i64, c_i64, c_int]),
    "abc_kde_workspace_bytes": (c_size, [c_i64, c_i64, c_int]),
    "abc_whiten_f32": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr, c_ptr,
                               c_ptr]),
    "abc_whiten_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr, c_ptr,
                               c_ptr]),
    "abc_kde_pack_prev_f32": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr,
                                      c_ptr, c_ptr, c_i64, c_ptr, c_ptr,
                                      c_ptr]),
    "abc_kde_pack_prev_f64": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr,
                                      c_ptr, c_ptr, c_i64, c_ptr, c_ptr,
                                      c_ptr]),
    "abc_kde_logpdf_f32": (c_int, [c_ptr, c_i64, c_ptr, c_i64, c_int, c_ptr,
                                   c_dbl, c_ptr, c_ptr, c_size, c_ptr]),
    "abc_kde_logpdf_f64": (c_int, [c_ptr, c_i64, c_ptr, c_i64, c_int, c_ptr,
                                   c_dbl, c_ptr, c_ptr, c_size, c_ptr]),
    "abc_kde_mfma_prev_bytes": (c_size, [c_i64, c_int]),
    "abc_kde_mfma_new_rows": (c_i64, [c_i64, c_int]),
    "abc_kde_mfma_new_bytes": (c_size, [c_i64, c_int]),
    "abc_kde_pack_prev_mfma": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr,
                                       c_ptr, c_ptr, c_ptr, c_i64, c_ptr,
                                       c_ptr, c_ptr, c_ptr]),
    "abc_kde_pack_new_mfma": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                      c_ptr, c_ptr, c_ptr, c_ptr]),
    "abc_kde_logpdf_mfma": (c_int, [c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                    c_int, c_ptr, c_dbl, c_ptr, c_ptr, c_size,
                                    c_ptr]),
    "abc_kde_pack_new_mfma_rows": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                           c_ptr, c_ptr, c_i64, c_ptr, c_ptr,
                                           c_ptr, c_ptr, c_ptr]),
    "abc_kde_logpdf_mfma_rows": (c_int, [c_ptr, c_ptr, c_ptr, c_i64, c_ptr,
                                         c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                         c_dbl, c_ptr, c_ptr, c_size, c_ptr]),
    "abc_importance_weights_f64": (c_int, [c_ptr, c_ptr, c_dbl, c_i64, c_ptr,
                                           c_ptr]),
    # (a4)
    "abc_reduce_workspace_bytes": (c_size, []),
    "abc_sum_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr, c_ptr]),
    "abc_scale_inplace_f64": (c_int, [c_ptr, c_i64, c_ptr, c_ptr]),
    # (a5)
    "abc_pnorm_distance_f64": (c_int, [c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                       c_int, c_dbl, c_dbl, c_ptr, c_ptr,
                                       c_ptr, c_ptr]),
    # (a6)
    "abc_column_select_workspace_bytes": (c_size, [c_int]),
    "abc_column_median_mad_f64": (c_int, [c_ptr, c_i64, c_i64, c_int, c_ptr,
                                          c_ptr, c_ptr, c_size, c_ptr]),
    "abc_column_std_f64": (c_int, [c_ptr, c_i64, c_i64, c_int, c_ptr, c_ptr,
                                   c_ptr]),
    "abc_column_std_workspace_bytes": (c_size, [c_i64, c_int]),
    "abc_column_std_ws_f64": (c_int, [c_ptr, c_i64, c_i64, c_int, c_ptr,
                                      c_ptr, c_ptr, c_size, c_ptr]),
    # SURVEY 8(b) fp32-storage and logsum forms
    "abc_weighted_moments_f32": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr,
                                         c_ptr, c_size, c_ptr]),
    "abc_resample_perturb_f32": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                         c_ptr, c_ptr, c_ptr, c_ptr, c_i64,
                                         c_ptr, c_ptr, c_ptr, c_ptr]),
    "abc_philox_fill": (c_int, [c_u64, c_u64, c_u64, c_ptr, c_i64, c_ptr,
                                c_i64, c_ptr]),
    "abc_philox_fill_f32": (c_int, [c_u64, c_u64, c_u64, c_ptr, c_i64, c_ptr,
                                    c_i64, c_ptr]),
    "abc_kde_logsum_workspace_bytes_f32": (c_size, [c_i64, c_i64, c_int]),
    "abc_kde_logsum_workspace_bytes_f64": (c_size, [c_i64, c_i64, c_int]),
    "abc_kde_logsum_f32": (c_int, [c_ptr, c_ptr, c_ptr, c_i64, c_i64, c_int,
                                   ctypes.c_float, c_ptr, c_ptr, c_size,
                                   c_ptr]),
    "abc_kde_logsum_f64": (c_int, [c_ptr, c_ptr, c_ptr, c_i64, c_i64, c_int,
                                   c_dbl, c_ptr, c_ptr, c_size, c_ptr]),
    "abc_knn_topk_f32_workspace_bytes": (c_size, [c_i64, c_int, c_int]),
    "abc_knn_topk_f32": (c_int, [c_ptr, c_i64, c_int, c_int, c_ptr, c_ptr,
                                 c_ptr, c_size, c_ptr]),
    "abc_local_cov_f32_workspace_bytes": (c_size, [c_i64, c_int]),
    "abc_local_cov_f32": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr, c_int,
                                  c_dbl, c_ptr, c_ptr, c_ptr, c_ptr, c_size,
                                  c_ptr]),
    # (a7)
    "abc_wquantile_workspace_bytes": (c_size, []),
    "abc_wquantile_f64": (c_int, [c_ptr, c_ptr, c_i64, c_dbl, c_ptr, c_ptr,
                                  c_size, c_ptr]),
    "abc_wquantile_step_f64": (c_int, [c_int, c_ptr, c_ptr, c_i64, c_i64,
                                       c_dbl, c_ptr, c_ptr, c_size, c_ptr]),
    "abc_wquantile_exchange": (c_int, [c_int, c_ptr, c_ptr, c_ptr]),
    # (a8)
    "abc_knn_workspace_bytes": (c_size, [c_i64, c_int]),
    "abc_knn_f64": (c_int, [c_ptr, c_i64, c_int, c_int, c_ptr, c_ptr, c_ptr,
                            c_size, c_ptr]),
    "abc_local_cov_f64": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr, c_int,
                                  c_dbl, c_ptr, c_ptr, c_ptr, c_ptr]),
    "abc_knn_rows_f64": (c_int, [c_ptr, c_i64, c_int, c_int, c_i64, c_i64,
                                 c_ptr, c_ptr, c_ptr, c_size, c_ptr]),
    "abc_local_cov_rows_f64": (c_int, [c_ptr, c_ptr, c_i64, c_int, c_ptr,
                                       c_int, c_i64, c_i64, c_dbl, c_ptr,
                                       c_ptr, c_ptr, c_ptr]),
    "abc_local_logpdf_workspace_bytes": (c_size, [c_i64, c_i64]),
    "abc_local_logpdf_f64": (c_int, [c_ptr, c_i64, c_ptr, c_ptr, c_ptr,
                                     c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                     c_size, c_ptr]),
    "abc_local_logpdf_f32": (c_int, [c_ptr, c_i64, c_ptr, c_ptr, c_ptr,
                                     c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                     c_size, c_ptr]),
    "abc_local_logpdf_f32_workspace_bytes": (c_size, [c_i64, c_i64]),
    "abc_local_logpdf_mfma": (c_int, [c_ptr, c_i64, c_ptr, c_ptr, c_ptr,
                                      c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                      c_size, c_ptr]),
    "abc_local_logpdf_mfma_workspace_bytes": (c_size, [c_i64, c_i64, c_int]),
    "abc_propose_local_philox_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr,
                                             c_ptr, c_ptr, c_ptr, c_u64,
                                             c_u64, c_u64, c_i64, c_ptr,
                                             c_ptr, c_ptr, c_ptr]),
    "abc_resample_perturb_local_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr,
                                               c_ptr, c_ptr, c_ptr, c_ptr,
                                               c_ptr, c_i64, c_ptr, c_ptr,
                                               c_ptr, c_ptr]),
    # (f3) exact inference: stochastic kernels / acceptor / temperatures
    "abc_stochastic_kernel_f64": (c_int, [c_ptr, c_i64, c_ptr, c_ptr, c_int,
                                          c_int, c_dbl, c_i64, c_ptr, c_dbl,
                                          c_dbl, c_int, c_ptr, c_u64, c_u64,
                                          c_u64, c_ptr, c_ptr, c_ptr, c_ptr]),
    "abc_stochastic_accept_f64": (c_int, [c_ptr, c_i64, c_dbl, c_dbl, c_int,
                                          c_int, c_ptr, c_u64, c_u64, c_u64,
                                          c_ptr, c_ptr, c_ptr, c_ptr]),
    "abc_importance_weights_scaled_f64": (c_int, [c_ptr, c_ptr, c_dbl, c_i64,
                                                  c_ptr, c_ptr]),
    "abc_tempered_sums_workspace_bytes": (c_size, [c_int]),
    "abc_tempered_sums_f64": (c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64,
                                      c_dbl, c_int, c_ptr, c_int, c_int,
                                      c_ptr, c_ptr, c_size, c_ptr]),
    # simulators
    "abc_sim_linear_gaussian_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr,
                                            c_int, c_dbl, c_u64, c_u64, c_u64,
                                            c_ptr, c_i64, c_ptr]),
    "abc_sim_linear_gaussian_pnorm_f64": (c_int, [c_ptr, c_i64, c_int, c_ptr,
                                                  c_ptr, c_int, c_dbl, c_u64,
                                                  c_u64, c_u64, c_ptr, c_ptr,
                                                  c_dbl, c_dbl, c_ptr, c_ptr,
                                                  c_ptr, c_ptr]),
    "abc_sim_linear_gaussian_pnorm_stats_f64": (
        c_int, [c_ptr, c_i64, c_int, c_ptr, c_ptr, c_int, c_dbl, c_u64, c_u64,
                c_u64, c_ptr, c_ptr, c_dbl, c_dbl, c_ptr, c_ptr, c_ptr, c_ptr,
                c_i64, c_ptr]),
    "abc_sim_gaussian_mean_f64": (c_int, [c_ptr, c_i64, c_dbl, c_u64, c_u64,
                                          c_u64, c_ptr, c_ptr]),
}

_lib = None
_load_error = None


def _load():
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise NativeLibraryError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"{LIB_PATH} not found: build it with "
                       f"`make -C pyabc_amd/csrc` (hipcc --offload-arch=gfx950)")
        raise NativeLibraryError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:
        _load_error = f"failed to load {LIB_PATH}: {e}"
        raise NativeLibraryError(_load_error) from e
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib():
    """The loaded library (raises NativeLibraryError when unavailable)."""
    return _load()


def available():
    try:
        _load()
        return True
    except NativeLibraryError:
        return False


def exported_symbols():
    return list(_SIGS)


def check(rc, what=""):
    if rc != 0:
        msg = _load().abc_last_error().decode(errors="replace")
        raise NativeLibraryError(f"{what or 'abc call'} failed ({rc}): {msg}")


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise NativeLibraryError(
            "libabc_hip takes device tensors; got a host tensor "
            "(no CPU fallback exists)")
    return ctypes.c_void_p(t.data_ptr())


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream():
    """The current HIP stream of the current device, as a void pointer
    (torch's raw accessor when it has one: torch.cuda.current_stream()
    builds a Stream object, a few microseconds per launch)."""
    if _raw_stream is not None:
        return ctypes.c_void_p(_raw_stream(torch.cuda.current_device()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def call(name, *args):
    fn = getattr(_load(), name)
    check(fn(*args), name)
