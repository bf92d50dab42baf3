"""Derived accuracy bound of the folded MFMA KDE pass, row by row
("Accuracy of the folded accumulation"); shared by
tests/test_gpu_kde_band.py and tests/test_gpu_fullsize.py.  Not a test
module (no test functions): torch on the GPU evaluates every pair's fp64
exponent of the rows it is given."""
import ctypes
import math
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ulp32(x):
    """ulp of fp32 at |x| (x > 0; normal range)."""
    _, E = torch.frexp(x)
    return torch.ldexp(torch.ones_like(x), (E - 24).to(torch.int32))


def row_stats(Yp, lw, Y, off, KL, D, g, chunk=128):
    """Per row: the largest exponent (relative to the global offset), the
    term-share entropy H (bits), log2 of the sum, and the derived bound
    under the row offset ``off`` (log2 units).  The folded accumulator of
    pair (i, j) starts at the exact hi_ij = 2 y1_i.y1_j + aH_j + bH_i
    (multiples of G = g^2; bH carries the offset) and each lo MFMA rounds
    at most at |hi_ij| + |lo_ij|, lo_ij = e'_ij - hi_ij."""
    G = g * g
    n2p = (Yp * Yp).sum(1)
    y1p = g * torch.round(Yp / g)
    aH = G * torch.round((lw - n2p) / G)
    out = {k: [] for k in ("emax", "H", "log2S", "bound")}
    for i0 in range(0, Y.shape[0], chunk):
        y = Y[i0:i0 + chunk]
        m = off[i0:i0 + chunk]
        n2 = (y * y).sum(1)
        e = lw[None, :] - (n2[:, None] + n2p[None, :] - 2.0 * y @ Yp.T)
        emax = e.max(1).values
        t = torch.exp2(e - emax[:, None])
        s = t.sum(1)
        p = t / s[:, None]
        H = -(p * torch.log2(torch.where(p > 0, p, torch.ones_like(p)))).sum(1)
        bH = G * torch.round((-n2 - m) / G)
        hi = 2.0 * (g * torch.round(y / g)) @ y1p.T + aH[None, :] + bH[:, None]
        lo = (e - m[:, None]) - hi
        u = (p * ulp32(hi.abs() + lo.abs())).sum(1)
        b = math.log(2) * (1.5 * KL * u + D * G * 2.0 ** -12) \
            + 2.0 ** -23 + 6 * 2.0 ** -24
        out["emax"].append(emax)
        out["H"].append(H)
        out["log2S"].append(emax + torch.log2(s))
        out["bound"].append(b)
    return {k: torch.cat(v).cpu().numpy() for k, v in out.items()}


PARENT_WIN = 7   # kde_mfma.hip kParentWin (log2 of the parent rows' window)


def pass_offsets(log2S, emax, m1, D, lo=None, win=PARENT_WIN):
    """The offset each row ends up with in kde_mfma.hip: the pass-1 offset
    m1 while the sum relative to it lies in the routing range (Route for
    rows without an offset, [2^-win, 2^win] for rows with a parent offset),
    otherwise m1 + floor(log2 S') (S' in the normal range) or the max
    pass's m1 + floor(max e')."""
    KL = (5 * D + 4 + 15) // 16
    if lo is None:  # kde_mfma.hip Route<D>::lo
        lo = 2.0 ** -26 if KL <= 2 else (2.0 ** -12 if KL <= 3 else 2.0 ** -4)
    lS = log2S - m1
    keep = np.where(m1 == 0, lS >= math.log2(lo), (lS >= -win) & (lS <= win))
    normal = (lS > -100) & (lS < 100)
    m2 = np.where(normal, m1 + np.floor(lS), m1 + np.floor(emax - m1))
    return np.where(keep, m1, m2), ~keep


_PROBE = {}


def _probe():
    if "lib" not in _PROBE:
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probes",
                                       "libabc_probe.so"))
        f = lib.abc_probe_kde_bound
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                      ctypes.c_double, ctypes.c_int, ctypes.c_void_p,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _PROBE["lib"] = lib
    return _PROBE["lib"]


def row_stats_all(packed, Y, off, KL):
    """:func:`row_stats` on EVERY row, in fp64 on the GPU
    (tools/probes/kde_bound.hip): ``packed`` the MFMA PackedPopulation,
    ``Y`` the whitened rows [M][D] (WhitenedRows.Y), ``off`` their offsets.
    Returns numpy arrays bound, log2S_rel (the sum relative to the row's
    offset) and H."""
    M, D = Y.shape
    n = int(packed.n)
    g = float(packed.gscale.item())
    out = torch.empty((3, M), dtype=torch.float64, device=Y.device)
    off = off.contiguous()
    rc = _probe().abc_probe_kde_bound(
        packed.P.data_ptr(), n, D, Y.contiguous().data_ptr(), off.data_ptr(),
        M, g, KL, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
        torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    o = out.cpu().numpy()
    return {"bound": o[0], "log2S_rel": o[1], "H": o[2]}
