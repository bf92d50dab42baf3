"""How many (32-proposal, 32-particle) tile pairs of the d = 8 KDE pass could
be skipped by a bounding-box test (CPU estimate, numpy): N = 1e6 standard
normal particles (whitened coordinates), proposals = parents + h-scaled noise
(Scott h = N^(-1/(d+4))), both Morton-ordered, 32-point boxes; a pair is
prunable when its smallest possible term is 2^-bits below a parent-like
term (q = 16).

    python tools/prune_estimate.py [bits ...]"""
import sys

import numpy as np


def morton_order(A, bits=4):
    lo, hi = A.min(0), A.max(0)
    q = np.clip(((A - lo) / (hi - lo) * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
    code = np.zeros(len(A), np.int64)
    for b in range(bits - 1, -1, -1):
        for k in range(A.shape[1]):
            code = (code << 1) | ((q[:, k] >> b) & 1)
    return np.argsort(code, kind="stable")


def main():
    rng = np.random.default_rng(0)
    N, d = 1_000_000, 8
    X = rng.standard_normal((N, d)).astype(np.float32)
    h = N ** (-1 / (d + 4))
    P = X[rng.integers(0, N, N)] + h * rng.standard_normal((N, d)).astype(np.float32)
    Xs, Ps = X[morton_order(X)], P[morton_order(P)]
    xt, pt = Xs.reshape(-1, 32, d), Ps.reshape(-1, 32, d)
    xl, xh, pl, ph = xt.min(1), xt.max(1), pt.min(1), pt.max(1)
    rows = rng.integers(0, len(pl), 300)
    for bits in [int(b) for b in sys.argv[1:]] or [40, 60]:
        frac = []
        for i in rows:
            gap = np.maximum(0, np.maximum(pl[i] - xh, xl - ph[i]))
            qmin = (gap ** 2).sum(1) / h ** 2
            frac.append(np.mean(qmin / 2 - 8 > bits * np.log(2)))
        print(f"h={h:.4f} bits={bits}: prunable tile pairs {np.mean(frac):.3f}")


if __name__ == "__main__":
    main()
