"""Tolerance of the weighted-quantile epsilon (a7) and the record of the
achieved errors (test infrastructure).

The reference computes ``interp(alpha, cumsum(w[argsort p]) - w / 2,
sort p)`` (pyabc/weighted_statistics.py:26-43).  The device sums the
weights exactly in fixed point; numpy's sequential cumsum is off the exact
sum by at most ~N ulp, and that shift of the knots moves the result along
the bracketing segment.  SURVEY 8(a7)'s LOCAL bound, from the bracketing
knots k, k+1 of the stable-sorted array:

    |eps_gpu - eps_ref| <= 1e-12 |eps| + (p_{k+1} - p_k) * 4 N 2^-53
                                          / (0.5 (w_k + w_{k+1}))

(the adjacent segment is taken too when alpha lies within that shift of a
knot).  With equal weights the device restates numpy's cumsum itself and
the result is required bit for bit; inside a tie block (p_k = p_{k+1}) the
bound is 0 and equality is required too.
"""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def local_bound(points, weights, alpha):
    """(bound, exact): the SURVEY 8(a7) tolerance at ``alpha`` (without the
    1e-12 relative term) and whether the bracketing segments are all inside
    tie blocks (bound 0: equality required)."""
    p = np.asarray(points, dtype=np.float64)
    n = p.size
    w = np.full(n, 1.0 / n) if weights is None else \
        np.asarray(weights, dtype=np.float64)
    order = np.argsort(p, kind="stable")
    ps, ws = p[order], w[order]
    x = np.cumsum(ws) - 0.5 * ws
    delta = 2.0 * n * 2.0 ** -53          # knot shift, cumsum vs exact
    j = int(np.searchsorted(x, alpha, side="right")) - 1
    segs = {j}
    if 0 <= j < n and abs(alpha - x[j]) <= delta:
        segs.add(j - 1)
    if j + 1 < n and abs(x[j + 1] - alpha) <= delta:
        segs.add(j + 1)
    bound = 0.0
    for s in segs:
        if s < 0 or s >= n - 1:
            continue                      # clamped: the end point itself
        gap = ps[s + 1] - ps[s]
        if gap == 0.0:
            continue
        dx = 0.5 * (ws[s] + ws[s + 1])
        bound = max(bound, gap if dx == 0.0 else gap * 2.0 * delta / dx)
    return bound, bound == 0.0


def record(name, rows):
    """Append measured errors to gpurun_out/quantile_parity.json when that
    directory exists (DESIGN.md quotes them; profiles/ keeps a copy)."""
    out = os.path.join(ROOT, "gpurun_out")
    if not os.path.isdir(out):
        return
    path = os.path.join(out, "quantile_parity.json")
    old = {}
    if os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
    old[name] = rows
    with open(path, "w") as f:
        json.dump(old, f, indent=1)
