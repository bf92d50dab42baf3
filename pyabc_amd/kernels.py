"""Typed torch-tensor wrappers over the libabc_hip C-ABI.

Every function here enqueues HIP kernels on torch's current stream through
``_native`` and returns device tensors.  Inputs must already be device
tensors of the stated dtype and layout; there is no host/CPU path.  Small
d x d linear algebra (eigh/svd of the KDE covariance) is done by the callers on
the host, exactly where the reference calls numpy/scipy on d x d matrices.
"""
import ctypes
import math

import numpy as np
import torch

from . import _native as nat
from ._native import ptr, call

F64 = torch.float64
F32 = torch.float32


def _dev():
    return torch.device("cuda", torch.cuda.current_device())


class Workspace:
    """Grow-only scratch buffer per device (no allocation in steady state)."""

    def __init__(self):
        self._buf = {}

    def get(self, nbytes, tag="default"):
        nbytes = max(int(nbytes), 256)
        key = (torch.cuda.current_device(), tag)
        b = self._buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.empty(nbytes + (nbytes >> 3), dtype=torch.uint8,
                            device=_dev())
            self._buf[key] = b
        return b


WS = Workspace()


def _contig(t, dtype):
    if t.dtype != dtype:
        raise TypeError(f"expected {dtype}, got {t.dtype}")
    return t.contiguous()


def _stat_major(stats_T):
    """(tensor, ld, n) of a stat-major [S, n] fp64 matrix for the kernels'
    (pointer, ld) convention: a column slice of a larger matrix (rows
    contiguous, row stride ld >= n) is passed as is -- no copy -- and
    anything else is made contiguous."""
    if stats_T.dtype != F64:
        raise TypeError(f"expected {F64}, got {stats_T.dtype}")
    S, n = stats_T.shape
    if S > 1 and stats_T.stride(1) == 1 and stats_T.stride(0) >= n:
        return stats_T, stats_T.stride(0), n
    t = stats_T.contiguous()
    return t, max(n, 1), n


# ---------------------------------------------------------------------------
# RNG / proposals (a2)
# ---------------------------------------------------------------------------
def philox_uniform(seed, sid, offset, n):
    out = torch.empty(n, dtype=F64, device=_dev())
    call("abc_philox_uniform_f64", seed, sid, offset, n, ptr(out), nat.stream())
    return out


def philox_normal(seed, sid, offset, n):
    out = torch.empty(n, dtype=F64, device=_dev())
    call("abc_philox_normal_f64", seed, sid, offset, n, ptr(out), nat.stream())
    return out


def resample_cdf(w, ws_tag="cdf"):
    """The resampling CDF of w; ``ws_tag`` names the scratch buffer (callers
    on another stream pass their own, engine.start_cdf: "cdf_side")."""
    w = _contig(w, F64)
    cdf = torch.empty_like(w)
    wsb = nat.lib().abc_resample_cdf_workspace_bytes(w.numel())
    ws = WS.get(wsb, ws_tag)
    call("abc_resample_cdf_f64", ptr(w), w.numel(), ptr(cdf), ptr(ws), wsb,
         nat.stream())
    return cdf


def resample_perturb(X, cdf, u, z, A, lo=None, scale=None):
    X = _contig(X, F64)
    N, d = X.shape
    B = u.numel()
    theta = torch.empty((B, d), dtype=F64, device=_dev())
    idx = torch.empty(B, dtype=torch.int64, device=_dev())
    sup = torch.empty(B, dtype=torch.uint8, device=_dev())
    call("abc_resample_perturb_f64", ptr(X), N, d, ptr(_contig(cdf, F64)),
         ptr(_contig(u, F64)), ptr(_contig(z, F64)), ptr(_contig(A, F64)),
         ptr(lo), ptr(scale), B, ptr(theta), ptr(idx), ptr(sup), nat.stream())
    return theta, idx, sup


CDF_INDEX_LOG2 = 16


def cdf_index_log2(n):
    """Bucket-table size for an n-particle CDF: about four buckets per
    particle (2^22 at n = 1e6), so the proposal's search is the two table
    reads plus ~1 CDF read.  Round 6 (tools/propose_tab.py, N = 1e6, 4.2e6
    proposals): 2^16 -> 2^22 buckets cut the proposal kernel 0.451 -> 0.359
    ms at d = 8 and 1.85 -> 1.69 ms at d = 20 (indices identical); the table
    costs 8 B per bucket and one search per bucket, on the side stream."""
    L = max(int(n) - 1, 1).bit_length() + 2
    return min(22, max(CDF_INDEX_LOG2, L))


def cdf_index(cdf, log2k=None):
    """Bucket table tab[k] = searchsorted(cdf, k / 2^log2k, 'right')
    (log2k None: :func:`cdf_index_log2` of the CDF's length)."""
    if log2k is None:
        log2k = cdf_index_log2(cdf.numel())
    tab = torch.empty((1 << log2k) + 1, dtype=torch.int64, device=_dev())
    call("abc_cdf_index_f64", ptr(_contig(cdf, F64)), cdf.numel(), log2k,
         ptr(tab), nat.stream())
    return tab


def propose_philox(X, cdf, A, lo, scale, seed, sid, offset, B, out=None,
                   tab=None):
    """Resample + perturb + support flag for B Philox proposals; ``tab``
    (:func:`cdf_index`) brackets the CDF search (same indices)."""
    X = _contig(X, F64)
    N, d = X.shape
    if out is None:
        theta = torch.empty((B, d), dtype=F64, device=_dev())
        idx = torch.empty(B, dtype=torch.int64, device=_dev())
        sup = torch.empty(B, dtype=torch.uint8, device=_dev())
    else:
        theta, idx, sup = out
    if tab is not None:
        log2k = (tab.numel() - 1).bit_length() - 1
        call("abc_propose_philox_indexed_f64", ptr(X), N, d, ptr(cdf),
             ptr(tab), log2k, ptr(A), ptr(lo), ptr(scale), seed, sid, offset,
             B, ptr(theta), ptr(idx), ptr(sup), nat.stream())
        return theta, idx, sup
    call("abc_propose_philox_f64", ptr(X), N, d, ptr(cdf), ptr(A), ptr(lo),
         ptr(scale), seed, sid, offset, B, ptr(theta), ptr(idx), ptr(sup),
         nat.stream())
    return theta, idx, sup


def prior_uniform(lo, scale, seed, sid, offset, B):
    d = lo.numel()
    theta = torch.empty((B, d), dtype=F64, device=_dev())
    call("abc_prior_uniform_f64", ptr(lo), ptr(scale), d, seed, sid, offset,
         B, ptr(theta), nat.stream())
    return theta


def compact(flags, out_idx=None, count=None):
    """Order-preserving positions of nonzero u8 flags; returns (idx,
    count_dev).  ``count``: an int64 device slot to write the count into
    (several counts in one buffer come back in one host read)."""
    n = flags.numel()
    if out_idx is None:
        out_idx = torch.empty(max(n, 1), dtype=torch.int64, device=_dev())
    if count is None:
        count = torch.empty(1, dtype=torch.int64, device=_dev())
    wsb = nat.lib().abc_compact_workspace_bytes(n)
    ws = WS.get(wsb, "compact")
    call("abc_compact_flags", ptr(flags), n, ptr(out_idx), ptr(count), ptr(ws),
         wsb, nat.stream())
    return out_idx, count


def gather_rows(src, idx, n=None):
    src = _contig(src, F64)
    width = src.shape[1] if src.dim() == 2 else 1
    n = idx.numel() if n is None else n
    out = torch.empty((n, width), dtype=F64, device=_dev())
    call("abc_gather_rows_f64", ptr(src), width, ptr(idx), n, ptr(out),
         nat.stream())
    return out if src.dim() == 2 else out.view(-1)


def full(n, value, dtype=F64):
    """A device vector of n copies of ``value`` (fp64 / int64: abc_fill_words;
    uint8: abc_fill_u8) -- torch.full without torch's fill kernel."""
    out = torch.empty(n, dtype=dtype, device=_dev())
    if dtype == torch.uint8:
        call("abc_fill_u8", ptr(out), n, int(value), nat.stream())
        return out
    if dtype == F64:
        bits = int(np.array(value, dtype=np.float64).view(np.uint64))
    elif dtype == torch.int64:
        bits = int(np.array(value, dtype=np.int64).view(np.uint64))
    else:
        raise TypeError(f"full: unsupported dtype {dtype}")
    call("abc_fill_words", ptr(out), n, bits, nat.stream())
    return out


def arange(n, start=0):
    """int64 start .. start + n - 1 on the device (abc_iota_i64)."""
    out = torch.empty(n, dtype=torch.int64, device=_dev())
    call("abc_iota_i64", ptr(out), n, int(start), nat.stream())
    return out


def radix_sort_pairs(keys, vals, end_bit=64):
    """Stable sort of (uint64 key as int64 bits, int32 value) pairs by the
    low ``end_bit`` key bits (abc_radix_sort_pairs_u64, the spatial index's
    sort); returns (keys_sorted, vals_sorted).  The inputs are copied."""
    n = keys.numel()
    kin = keys.clone() if keys.dtype == torch.int64 else None
    if kin is None or vals.dtype != torch.int32:
        raise TypeError("keys int64 (uint64 bits), vals int32")
    vin = vals.clone()
    ko = torch.empty_like(kin)
    vo = torch.empty_like(vin)
    wsb = nat.lib().abc_radix_sort_workspace_bytes(n)
    ws = WS.get(wsb, "sort")
    call("abc_radix_sort_pairs_u64", ptr(kin), ptr(vin), n, end_bit, ptr(ko),
         ptr(vo), ptr(ws), wsb, nat.stream())
    return ko, vo


def _words(t):
    """(tensor, row stride, width) of an 8-byte-element 1-D / 2-D view with
    unit column stride (a column block of a wider buffer is fine)."""
    if t.element_size() != 8:
        raise TypeError(f"8-byte elements expected, got {t.dtype}")
    if t.dim() == 1:
        if t.numel() > 1 and t.stride(0) != 1:
            raise ValueError("1-D view must be contiguous")
        return 1, 1
    if t.dim() != 2 or (t.shape[1] > 1 and t.stride(1) != 1):
        raise ValueError("2-D view with unit column stride expected")
    return max(t.stride(0), t.shape[1]), t.shape[1]


def gather_words(src, idx, n, out):
    """out[i, :] = src[idx[i], :] for i < n (idx None: src[i, :]) over
    8-byte words -- fp64 values or int64 indices, bit copies
    (abc_gather_words).  ``out`` may be a row / column block of a larger
    buffer: the accepted rows of several rounds and columns land in place.
    Returns ``out``."""
    src_ld, w = _words(src)
    out_ld, wo = _words(out)
    if w != wo or out.shape[0] < n:
        raise ValueError(f"gather_words: widths {w} / {wo}, rows {out.shape[0]} < {n}")
    if n:
        call("abc_gather_words", ptr(src), src_ld, w,
             ptr(idx) if idx is not None else None, n, ptr(out), out_ld,
             nat.stream())
    return out


def gather_cols(src, idx, n, out):
    """out[s, i] = src[s, idx[i]] for i < n (idx None: src[s, i]) over
    8-byte words of a stat-major [S, *] matrix (abc_gather_cols_words);
    ``out`` may be a column block of a wider [S, *] buffer."""
    if src.element_size() != 8 or out.element_size() != 8:
        raise TypeError("8-byte elements expected")
    S = src.shape[0]
    if out.shape[0] != S or out.shape[1] < n or src.stride(1) != 1 \
            or (out.shape[1] > 1 and out.stride(1) != 1):
        raise ValueError("gather_cols: shapes")
    if n and S:
        call("abc_gather_cols_words", ptr(src), src.stride(0), S,
             ptr(idx) if idx is not None else None, n, ptr(out),
             out.stride(0), nat.stream())
    return out


# ---------------------------------------------------------------------------
# fit (a1)
# ---------------------------------------------------------------------------
def weighted_moments(X, w):
    """Device [sw, sw2, mu(d), C(d*d)] (C un-normalised centred products)."""
    X = _contig(X, F64)
    n, d = X.shape
    out = torch.empty(2 + d + d * d, dtype=F64, device=_dev())
    wsb = nat.lib().abc_moments_workspace_bytes(d)
    ws = WS.get(wsb, "moments")
    call("abc_weighted_moments_f64", ptr(X), ptr(_contig(w, F64)), n, d,
         ptr(out), ptr(ws), wsb, nat.stream())
    return out


# ---------------------------------------------------------------------------
# KDE (a3)
# ---------------------------------------------------------------------------
LOG2E = 1.4426950408889634
LOG_2PI = math.log(2 * math.pi)


def padded_dim(d):
    D = nat.lib().abc_kde_padded_dim(d)
    if D < 0:
        raise nat.NativeLibraryError(f"KDE: unsupported dimension d={d}")
    return D


def row_pad():
    return nat.lib().abc_kde_row_pad()


def reload_tuning():
    """Re-read the launch-shape tuning knobs (ABC_KDE_MFMA_*, ABC_KDE_TIER,
    ABC_LZ_*) from os.environ; the library reads them once per process
    (abc_tuning_reload).  They never change a result bit."""
    nat.lib().abc_tuning_reload()


_PRELOADED = set()


def preload():
    """Load every translation unit's code object on the current device
    (abc_preload; HIP otherwise loads one at its first kernel launch, e.g.
    ~4 ms for the LocalTransition density pass inside C4's first weighted
    generation).  Once per device."""
    dev = torch.cuda.current_device()
    if dev in _PRELOADED:
        return
    rc = nat.lib().abc_preload()
    if rc:
        raise RuntimeError(f"abc_preload: {rc} code objects did not load")
    _PRELOADED.add(dev)


def psd_whitening(cov):
    """scipy _PSD semantics on the host (d x d): U, rank, log_pdet."""
    cov = np.asarray(cov, dtype=np.float64)
    s, u = np.linalg.eigh(cov)
    eps = 1e6 * np.finfo(np.float64).eps * np.max(np.abs(s))
    keep = s > eps
    s_pinv = np.where(keep, 1.0 / np.where(keep, s, 1.0), 0.0)
    U = u * np.sqrt(s_pinv)
    return U, int(keep.sum()), float(np.sum(np.log(s[keep])))


class WhitenedRows:
    """New rows prepared for the MFMA KDE pass: direct fp64 whitened rows
    (refine and exact fixup), the f16 piece fragments of the B operand and
    each row's exponent offset (log2 units; 0, or the parent's term)."""

    def __init__(self, Y, frags, M, row_off=None):
        self.Y, self.frags, self.M = Y, frags, M
        self.row_off = row_off
        self.shape = (M, Y.shape[1])


class PackedPopulation:
    """The previous population packed for the KDE pass (built once per fit).

    precision: "mfma" (default: exact-grid f16 pieces on the matrix cores,
    kde_mfma.hip), "f32" (direct fp32 VALU pass) or "f64" (fp64 VALU pass).
    """

    def __init__(self, X, w, mu, Us, rank, log_pdet, precision="mfma",
                 ws_tag="pack"):
        X = _contig(X, F64)
        n, d = X.shape
        self.n, self.d = n, d
        self.D = padded_dim(d)
        rp = row_pad()
        self.npad = ((n + rp - 1) // rp) * rp
        if precision not in ("mfma", "f32", "f64"):
            raise ValueError(f"unknown KDE precision {precision!r}")
        self.precision = precision
        # the MFMA pass keeps an fp64 direct copy for its exact fixup rows
        dt = F32 if precision == "f32" else F64
        self.P = torch.empty((self.npad, self.D + 1), dtype=dt, device=_dev())
        self.lw2max = torch.empty(1, dtype=F64, device=_dev())
        self.mu = mu
        self.Us = Us
        self.log_const = -0.5 * (rank * LOG_2PI + log_pdet)
        ws = WS.get(256, ws_tag)   # "pack_side" on the engine's side stream
        w = _contig(w, F64)
        if precision == "mfma":
            nb = nat.lib().abc_kde_mfma_prev_bytes(self.npad, d)
            self.A = torch.empty(nb, dtype=torch.uint8, device=_dev())
            self.gscale = torch.empty(1, dtype=F64, device=_dev())
            call("abc_kde_pack_prev_mfma", ptr(X), ptr(w), n, d, ptr(mu),
                 ptr(Us), ptr(self.P), ptr(self.A), self.npad,
                 ptr(self.lw2max), ptr(self.gscale), ptr(ws), nat.stream())
            return
        fn = "abc_kde_pack_prev_f32" if precision == "f32" else \
            "abc_kde_pack_prev_f64"
        call(fn, ptr(X), ptr(w), n, d, ptr(mu), ptr(Us),
             ptr(self.P), self.npad, ptr(self.lw2max), ptr(ws), nat.stream())

    def whiten(self, theta, parent=None):
        """Rows for :meth:`logpdf_whitened`.  ``parent`` (MFMA pass only,
        optional): per row the index into this population its proposal was
        resampled from; the row's exponents are then taken relative to the
        parent's term (the density is the same; the folded pass rounds at
        the row's own scale, kde_mfma.hip)."""
        theta = _contig(theta, F64)
        M = theta.shape[0]
        if self.precision == "mfma":
            # every column written by the pack (zeros beyond d)
            Y = torch.empty((M, self.D), dtype=F64, device=_dev())
            nb = nat.lib().abc_kde_mfma_new_bytes(M, self.d)
            B = torch.empty(max(nb, 16), dtype=torch.uint8, device=_dev())
            off = torch.empty(max(M, 1), dtype=F64, device=_dev())
            par = None
            if parent is not None:
                par = _contig(parent, torch.int64)
                if par.shape[0] != M:
                    raise ValueError("parent: one index per row")
            call("abc_kde_pack_new_mfma_rows", ptr(theta), M, self.d,
                 ptr(self.mu), ptr(self.Us), ptr(self.gscale), ptr(self.P),
                 self.npad, ptr(par) if par is not None else None, ptr(Y),
                 ptr(B), ptr(off), nat.stream())
            return WhitenedRows(Y, B, M, off[:M])
        dt = F32 if self.precision == "f32" else F64
        Y = torch.zeros((M, self.D), dtype=dt, device=_dev())
        fn = "abc_whiten_f32" if self.precision == "f32" else "abc_whiten_f64"
        call(fn, ptr(theta), M, self.d, ptr(self.mu), ptr(self.Us), ptr(Y),
             nat.stream())
        return Y

    def logpdf_whitened(self, Y, out=None):
        M = Y.shape[0]
        if out is None:
            out = torch.empty(M, dtype=F64, device=_dev())
        if M == 0:
            return out
        wsb = nat.lib().abc_kde_workspace_bytes(M, self.npad, self.d)
        ws = WS.get(wsb, "kde")
        # the fixup-row counter follows the [nseg][M] fp64 partials
        self._fix_at = (ws, nat.lib().abc_kde_segments(self.npad) * M * 8)
        if self.precision == "mfma":
            if not isinstance(Y, WhitenedRows):
                raise TypeError("mfma KDE pass takes rows from whiten()")
            call("abc_kde_logpdf_mfma_rows", ptr(Y.frags), ptr(Y.Y),
                 ptr(Y.row_off) if Y.row_off is not None else None, M,
                 ptr(self.A), ptr(self.P), self.npad, self.d,
                 ptr(self.lw2max), ptr(self.gscale), self.log_const,
                 ptr(out), ptr(ws), wsb, nat.stream())
            return out
        fn = "abc_kde_logpdf_f32" if self.precision == "f32" else \
            "abc_kde_logpdf_f64"
        call(fn, ptr(Y), M, ptr(self.P), self.npad, self.d, ptr(self.lw2max),
             self.log_const, ptr(out), ptr(ws), wsb, nat.stream())
        return out

    def logpdf(self, theta, parent=None):
        return self.logpdf_whitened(self.whiten(theta, parent))

    def fixup_rows(self):
        """Rows the last pass of this population handed to the two-pass
        fixup (sum below the pass's threshold, or beyond the grid);
        synchronises with the stream.  Valid until the next KDE call reuses
        the workspace."""
        ws, off = getattr(self, "_fix_at", (None, 0))
        if ws is None:
            return 0
        return int(ws[off:off + 4].view(torch.int32).item())

    def refined_rows(self):
        """Rows the last MFMA pass re-evaluated with their own offset (sum
        outside the folded scheme's routing range, kde_mfma.hip Route; the
        fixup rows among them are counted by :meth:`fixup_rows`)."""
        ws, off = getattr(self, "_fix_at", (None, 0))
        if ws is None or self.precision != "mfma":
            return 0
        return int(ws[off + 4:off + 8].view(torch.int32).item())


def importance_weights(logpd, prior=None, prior_const=1.0):
    M = logpd.numel()
    w = torch.empty(M, dtype=F64, device=_dev())
    call("abc_importance_weights_f64", ptr(logpd), ptr(prior), prior_const, M,
         ptr(w), nat.stream())
    return w


# ---------------------------------------------------------------------------
# reductions (a4)
# ---------------------------------------------------------------------------
def dsum(x, squares=False):
    out = torch.empty(1, dtype=F64, device=_dev())
    ws = WS.get(nat.lib().abc_reduce_workspace_bytes(), "reduce")
    call("abc_sum_f64", ptr(_contig(x, F64)), x.numel(), 1 if squares else 0,
         ptr(out), ptr(ws), nat.stream())
    return out


def scale_inplace(x, divisor_dev):
    call("abc_scale_inplace_f64", ptr(x), x.numel(), ptr(divisor_dev),
         nat.stream())
    return x


# ---------------------------------------------------------------------------
# distances (a5), scales (a6), quantile (a7)
# ---------------------------------------------------------------------------
def pnorm_distance(stats_T, x0, fw, p, eps=math.inf, B=None, with_accept=True,
                   d_out=None, acc_out=None, guard_out=None):
    S = stats_T.shape[0]
    stats_T, ld, n = _stat_major(stats_T)
    B = n if B is None else B
    d = torch.empty(B, dtype=F64, device=_dev()) if d_out is None else d_out
    acc = guard = None
    if with_accept:
        acc = torch.empty(B, dtype=torch.uint8, device=_dev()) \
            if acc_out is None else acc_out
        guard = torch.empty(B, dtype=torch.uint8, device=_dev()) \
            if guard_out is None else guard_out
    call("abc_pnorm_distance_f64", ptr(stats_T), ld, ptr(x0), ptr(fw), B, S,
         float(p), float(eps), ptr(d), ptr(acc), ptr(guard), nat.stream())
    return d, acc, guard


def column_median_mad(data_T, n=None, mad=True):
    S = data_T.shape[0]
    data_T, ld, n0 = _stat_major(data_T)
    n = n0 if n is None else n
    med = torch.empty(S, dtype=F64, device=_dev())
    madv = torch.empty(S, dtype=F64, device=_dev()) if mad else None
    wsb = nat.lib().abc_column_select_workspace_bytes(S)
    ws = WS.get(wsb, "colsel")
    call("abc_column_median_mad_f64", ptr(data_T), ld, n, S, ptr(med),
         ptr(madv), ptr(ws), wsb, nat.stream())
    return med, madv


def column_std(data_T, n=None):
    S = data_T.shape[0]
    data_T, ld, n0 = _stat_major(data_T)
    n = n0 if n is None else n
    mean = torch.empty(S, dtype=F64, device=_dev())
    std = torch.empty(S, dtype=F64, device=_dev())
    wsb = nat.lib().abc_column_std_workspace_bytes(n, S)
    ws = WS.get(wsb, "colstd")
    call("abc_column_std_ws_f64", ptr(data_T), ld, n, S, ptr(mean), ptr(std),
         ptr(ws), wsb, nat.stream())
    return mean, std


_WQ_SEQ = [0, 1, 2, 3] + [s for p in range(8) for s in (10 + p, 20 + p)] \
    + [30, 31, 33, 32]


def weighted_quantile(d, w, alpha, comm=None, shard=False):
    """Device [eps, p_k, cs_{k-1}, w_k] for interp(alpha, cs - w/2, sort d).

    With ``comm`` over several ranks every rank holds the same global
    population.  By default each rank evaluates the quantile on its own
    copy: no exchange, the same bits on every rank (the sharded protocol's
    13 collectives cost more than the N/R histogram work they split: 13 x
    ~25 us against 0.12 ms for the whole N = 1e6 select, DESIGN.md section
    5).  ``shard=True``: each rank histograms only its row_range of (d, w)
    and the integer histograms / key bounds are all-reduced between the
    radix passes; bit-identical to one rank's."""
    n = d.numel()
    out = torch.empty(4, dtype=F64, device=_dev())
    wsb = nat.lib().abc_wquantile_workspace_bytes()
    ws = WS.get(wsb, "wq")
    d = _contig(d, F64)
    w = None if w is None else _contig(w, F64)
    if comm is None or not comm.active or not shard:
        call("abc_wquantile_f64", ptr(d), ptr(w), n, float(alpha), ptr(out),
             ptr(ws), wsb, nat.stream())
        return out
    q, m = divmod(n, comm.world)
    lo = comm.rank * q + min(comm.rank, m)
    hi = lo + q + (1 if comm.rank < m else 0)
    dl = d[lo:hi]
    wl = None if w is None else w[lo:hi]
    words = ws[:(wsb // 8) * 8].view(torch.int64)
    off, cnt, op = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
    for step in _WQ_SEQ:
        call("abc_wquantile_step_f64", step, ptr(dl) if hi > lo else None,
             ptr(wl) if (wl is not None and hi > lo) else None, hi - lo, n,
             float(alpha), ptr(out), ptr(ws), wsb, nat.stream())
        call("abc_wquantile_exchange", step, ctypes.byref(off),
             ctypes.byref(cnt), ctypes.byref(op))
        if op.value:
            a = off.value // 8
            comm.all_reduce_words(words[a:a + cnt.value], op.value)
    return out


# ---------------------------------------------------------------------------
# LocalTransition (a8)
# ---------------------------------------------------------------------------
def knn(X, k):
    X = _contig(X, F64)
    N, d = X.shape
    nbr = torch.empty((N, k), dtype=torch.int32, device=_dev())
    d2 = torch.empty((N, k), dtype=F64, device=_dev())
    wsb = nat.lib().abc_knn_workspace_bytes(N, k)
    ws = WS.get(wsb, "knn")
    call("abc_knn_f64", ptr(X), N, d, k, ptr(nbr), ptr(d2), ptr(ws), wsb,
         nat.stream())
    return nbr, d2


def knn_rows(X, k, row0, nrows):
    """kNN of the particles [row0, row0 + nrows) against all N."""
    X = _contig(X, F64)
    N, d = X.shape
    nbr = torch.empty((nrows, k), dtype=torch.int32, device=_dev())
    d2 = torch.empty((nrows, k), dtype=F64, device=_dev())
    wsb = nat.lib().abc_knn_workspace_bytes(N, k)
    ws = WS.get(wsb, "knn")
    call("abc_knn_rows_f64", ptr(X), N, d, k, row0, nrows, ptr(nbr), ptr(d2),
         ptr(ws), wsb, nat.stream())
    return nbr, d2


def local_cov_rows(X, w, nbr, row0, scaling=1.0):
    """Local covariances of the particles [row0, row0 + len(nbr))."""
    X = _contig(X, F64)
    N, d = X.shape
    nrows, k = nbr.shape
    covs = torch.empty((nrows, d, d), dtype=F64, device=_dev())
    invs = torch.empty((nrows, d, d), dtype=F64, device=_dev())
    dets = torch.empty(nrows, dtype=F64, device=_dev())
    call("abc_local_cov_rows_f64", ptr(X), ptr(_contig(w, F64)), N, d,
         ptr(nbr.contiguous()), k, row0, nrows, float(scaling), ptr(covs),
         ptr(invs), ptr(dets), nat.stream())
    return covs, invs, dets


def local_cov(X, w, nbr, scaling=1.0):
    X = _contig(X, F64)
    N, d = X.shape
    k = nbr.shape[1]
    covs = torch.empty((N, d, d), dtype=F64, device=_dev())
    invs = torch.empty((N, d, d), dtype=F64, device=_dev())
    dets = torch.empty(N, dtype=F64, device=_dev())
    call("abc_local_cov_f64", ptr(X), ptr(_contig(w, F64)), N, d,
         ptr(nbr.contiguous()), k, float(scaling), ptr(covs), ptr(invs),
         ptr(dets), nat.stream())
    return covs, invs, dets


def local_logpdf(pts, X, w, invs, dets, precision="f64"):
    """log LocalTransition density; ``precision`` "f64" (1e-12), "f32"
    (pair loop in fp32, 1e-5 relative) or "mfma" (z form on the f16 matrix
    cores, 1e-5 relative)."""
    if precision not in ("f64", "f32", "mfma"):
        raise ValueError(f"unknown LocalTransition precision {precision!r}")
    pts = _contig(pts, F64)
    M, d = pts.shape
    N = X.shape[0]
    out = torch.empty(M, dtype=F64, device=_dev())
    if precision == "mfma":
        wsb = nat.lib().abc_local_logpdf_mfma_workspace_bytes(M, N, d)
    else:
        wsb = getattr(nat.lib(), f"abc_local_logpdf{'_f32' if precision == 'f32' else ''}"
                      "_workspace_bytes")(M, N)
    ws = WS.get(wsb, "localpdf")
    call(f"abc_local_logpdf_{precision}", ptr(pts), M, ptr(_contig(X, F64)),
         ptr(_contig(w, F64)), ptr(invs), ptr(dets), N, d, ptr(out), ptr(ws),
         wsb, nat.stream())
    return out


def resample_perturb_local(X, cdf, u, z, A, lo=None, scale=None):
    """LocalTransition draws from given uniforms / normals with the per-
    particle factors A [N, d, d] (parity form, local_transition.py:141-145)."""
    X = _contig(X, F64)
    N, d = X.shape
    B = u.numel()
    theta = torch.empty((B, d), dtype=F64, device=_dev())
    idx = torch.empty(B, dtype=torch.int64, device=_dev())
    sup = torch.empty(B, dtype=torch.uint8, device=_dev())
    call("abc_resample_perturb_local_f64", ptr(X), N, d,
         ptr(_contig(cdf, F64)), ptr(_contig(u, F64)), ptr(_contig(z, F64)),
         ptr(_contig(A, F64)), ptr(lo), ptr(scale), B, ptr(theta), ptr(idx),
         ptr(sup), nat.stream())
    return theta, idx, sup


def propose_local(X, cdf, covs, seed, sid, offset, B, lo=None, scale=None):
    X = _contig(X, F64)
    N, d = X.shape
    theta = torch.empty((B, d), dtype=F64, device=_dev())
    idx = torch.empty(B, dtype=torch.int64, device=_dev())
    sup = torch.empty(B, dtype=torch.uint8, device=_dev())
    call("abc_propose_local_philox_f64", ptr(X), N, d, ptr(cdf),
         ptr(covs.contiguous()), ptr(lo), ptr(scale), seed, sid, offset, B,
         ptr(theta), ptr(idx), ptr(sup), nat.stream())
    return theta, idx, sup


# ---------------------------------------------------------------------------
# synthetic simulators
# ---------------------------------------------------------------------------
def sim_linear_gaussian(theta, A, c, sigma, seed, sid, offset, out_T=None,
                        B=None):
    theta = _contig(theta, F64)
    B = theta.shape[0] if B is None else B
    S, d = A.shape
    if out_T is None:
        out_T = torch.empty((S, max(B, 1)), dtype=F64, device=_dev())
    call("abc_sim_linear_gaussian_f64", ptr(theta), B, d, ptr(A), ptr(c), S,
         float(sigma), seed, sid, offset, ptr(out_T), out_T.shape[1],
         nat.stream())
    return out_T


def sim_linear_gaussian_pnorm(theta, A, c, sigma, seed, sid, offset, x0, fw,
                              p, eps=math.inf, B=None, keep_stats=False):
    """Fused simulation + p-norm distance + acceptance: (d, accept, guard),
    bit-identical to sim_linear_gaussian followed by pnorm_distance; with
    ``keep_stats`` the statistics are written too (stat-major [S, B]) and
    returned as a fourth item."""
    theta = _contig(theta, F64)
    B = theta.shape[0] if B is None else B
    S, d = A.shape
    dist = torch.empty(B, dtype=F64, device=_dev())
    acc = torch.empty(B, dtype=torch.uint8, device=_dev())
    guard = torch.empty(B, dtype=torch.uint8, device=_dev())
    if keep_stats:
        out_T = torch.empty((S, max(B, 1)), dtype=F64, device=_dev())
        call("abc_sim_linear_gaussian_pnorm_stats_f64", ptr(theta), B, d,
             ptr(A), ptr(c), S, float(sigma), seed, sid, offset,
             ptr(_contig(x0, F64)), ptr(_contig(fw, F64)), float(p),
             float(eps), ptr(dist), ptr(acc), ptr(guard), ptr(out_T),
             out_T.shape[1], nat.stream())
        return dist, acc, guard, out_T
    call("abc_sim_linear_gaussian_pnorm_f64", ptr(theta), B, d, ptr(A), ptr(c),
         S, float(sigma), seed, sid, offset, ptr(_contig(x0, F64)),
         ptr(_contig(fw, F64)), float(p), float(eps), ptr(dist), ptr(acc),
         ptr(guard), nat.stream())
    return dist, acc, guard


def sim_gaussian_mean(theta, sigma, seed, sid, offset, out=None, B=None):
    B = theta.shape[0] if B is None else B
    if out is None:
        out = torch.empty(B, dtype=F64, device=_dev())
    call("abc_sim_gaussian_mean_f64", ptr(_contig(theta, F64)), B,
         float(sigma), seed, sid, offset, ptr(out), nat.stream())
    return out


# ---------------------------------------------------------------------------
# exact inference: stochastic kernels and acceptance
# ---------------------------------------------------------------------------
KERNEL_NORMAL = 0
KERNEL_LAPLACE = 1


def stochastic_kernel(stats_T, x0, prm, kind, c, B=None, pdf_norm=None,
                      inv_temp=1.0, apply_iw=True, u=None, seed=0, stream=0,
                      offset=0):
    """Log-densities of an independent normal / Laplace kernel per column of
    stat-major ``stats_T`` ([S, ld]); with ``pdf_norm`` also the fused
    stochastic acceptance.  Returns (pd, accept, accw, guard)."""
    S = stats_T.shape[0]
    stats_T, ld, n = _stat_major(stats_T)
    B = n if B is None else B
    pd = torch.empty(B, dtype=F64, device=_dev())
    acc = accw = guard = None
    if pdf_norm is not None:
        acc = torch.empty(B, dtype=torch.uint8, device=_dev())
        accw = torch.empty(B, dtype=F64, device=_dev())
        guard = torch.empty(B, dtype=torch.uint8, device=_dev())
    call("abc_stochastic_kernel_f64", ptr(stats_T), ld, ptr(_contig(x0, F64)),
         ptr(_contig(prm, F64)), S, int(kind), float(c), B, ptr(pd),
         float(pdf_norm if pdf_norm is not None else 0.0), float(inv_temp),
         1 if apply_iw else 0, ptr(None if u is None else _contig(u, F64)),
         int(seed), int(stream), int(offset), ptr(acc), ptr(accw), ptr(guard),
         nat.stream())
    return pd, acc, accw, guard


def stochastic_accept(pd, pdf_norm, inv_temp, log_scale=True, apply_iw=True,
                      u=None, seed=0, stream=0, offset=0):
    """StochasticAcceptor decisions for given densities: (accept, accw, guard)."""
    pd = _contig(pd, F64)
    B = pd.numel()
    acc = torch.empty(B, dtype=torch.uint8, device=_dev())
    accw = torch.empty(B, dtype=F64, device=_dev())
    guard = torch.empty(B, dtype=torch.uint8, device=_dev())
    call("abc_stochastic_accept_f64", ptr(pd), B, float(pdf_norm),
         float(inv_temp), 1 if log_scale else 0, 1 if apply_iw else 0,
         ptr(None if u is None else _contig(u, F64)), int(seed), int(stream),
         int(offset), ptr(acc), ptr(accw), ptr(guard), nat.stream())
    return acc, accw, guard


def importance_weights_scaled(logpd, s, prior_const=1.0, M=None):
    """(prior_const * s_i) / exp(logpd_i); logpd None -> prior_const * s_i."""
    M = (s if logpd is None else logpd).numel() if M is None else M
    w = torch.empty(M, dtype=F64, device=_dev())
    call("abc_importance_weights_scaled_f64",
         ptr(None if logpd is None else _contig(logpd, F64)),
         ptr(None if s is None else _contig(s, F64)), float(prior_const), M,
         ptr(w), nat.stream())
    return w


def tempered_sums(pd, c, betas, w=None, logw_num=None, logw_den=None,
                  log_scale=True, clamp=True):
    """Device [K+1, 2]: row 0 = (sum w, sum w^2), row 1+k = (sum w v_k,
    sum (w v_k)^2) for v_k = exp((pd-c) beta_k) [log] or (pd/c)^beta_k [lin]
    (clamped at 1 when ``clamp``); w = w * exp(logw_num - logw_den)."""
    pd = _contig(pd, F64)
    b = np.asarray(betas, dtype=np.float64).ravel()
    K = b.size
    bt = torch.as_tensor(b, device=_dev()) if K else None
    out = torch.empty((K + 1, 2), dtype=F64, device=_dev())
    wsb = nat.lib().abc_tempered_sums_workspace_bytes(K)
    ws = WS.get(wsb, "tempered")
    opt = lambda t: ptr(None if t is None else _contig(t, F64))  # noqa: E731
    call("abc_tempered_sums_f64", ptr(pd), opt(w), opt(logw_num),
         opt(logw_den), pd.numel(), float(c), 1 if log_scale else 0, ptr(bt),
         K, 1 if clamp else 0, ptr(out), ptr(ws), wsb, nat.stream())
    return out
