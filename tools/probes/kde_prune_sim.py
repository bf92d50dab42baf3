"""How much of the MVN KDE pass could pair pruning skip?  (VERDICT r03
weak item 3; DESIGN.md section 4 "Pair pruning".)

numpy simulation of the headline workload's geometry: a Gaussian population
of N particles in d = 8, whitened by the Silverman-bandwidth kernel
covariance exactly as the KDE pass does (kernel standard deviation 1 in the
whitened units), log-normal importance weights, and M = N new rows drawn
from the KDE itself (resample + perturb, the proposals of the next
generation).  Rows and particles are put in Morton order and cut into the
pass's 32 x 32 MFMA tiles.  A tile pair (I, J) may be skipped when even the
nearest corners of the two bounding boxes give a term below the cut:

    32 * max_j w_j * exp(-boxdist(I, J)^2 / 2) <= cut * min_{i in I} S_i

with S_i a lower bound of row i's sum (its exact sum over the 8 nearest
particle tiles).  Reported per cut: the fraction of PAIRS that matter
(exact per pair), of 32-particle tiles that survive per ROW, and of 32 x 32
tile pairs that survive (what an MFMA pass could skip).

    python tools/probes/kde_prune_sim.py [log2 N ...]     (default 14 16)
"""
import json
import sys

import numpy as np


def morton_order(y, bits=8):
    lo, hi = y.min(0), y.max(0)
    q = ((y - lo) / (hi - lo + 1e-12) * ((1 << bits) - 1)).astype(np.uint64)
    key = np.zeros(len(y), dtype=np.uint64)
    d = y.shape[1]
    for b in range(bits):
        for k in range(d):
            key |= ((q[:, k] >> np.uint64(b)) & np.uint64(1)) << np.uint64(b * d + k)
    return np.argsort(key, kind="stable")


def boxes(y, t=32):
    n = len(y) // t * t
    yt = y[:n].reshape(-1, t, y.shape[1])
    return yt.min(1), yt.max(1)


def run(log2n, d=8, seed=0, cuts=(2.0 ** -40, 2.0 ** -60)):
    rng = np.random.default_rng(seed)
    N = 1 << log2n
    h = (4.0 / (N * (d + 2))) ** (1.0 / (d + 4))     # Silverman
    x = rng.normal(size=(N, d))                      # population ~ N(0, I)
    y = x / h                                        # whitened: kernel sd 1
    logw = rng.normal(scale=0.5, size=N)
    w = np.exp(logw - logw.max())
    w /= w.sum()
    par = rng.choice(N, size=N, p=w)
    q = y[par] + rng.normal(size=(N, d))             # new rows from the KDE
    py, pq = morton_order(y), morton_order(q)
    y, w, q = y[py], w[py], q[pq]
    T = 32
    ylo, yhi = boxes(y, T)
    qlo, qhi = boxes(q, T)
    wt = w[:len(ylo) * T].reshape(-1, T).max(1)
    nT = len(ylo)
    # lower bound of each row's sum: exact over the 8 nearest particle tiles
    cen = 0.5 * (ylo + yhi)
    S = np.empty(nT * T)
    for I in range(len(qlo)):
        rows = q[I * T:(I + 1) * T]
        c = 0.5 * (qlo[I] + qhi[I])
        near = np.argsort(((cen - c) ** 2).sum(1))[:8]
        idx = (near[:, None] * T + np.arange(T)).ravel()
        d2 = ((rows[:, None, :] - y[idx][None]) ** 2).sum(-1)
        S[I * T:(I + 1) * T] = (w[idx][None] * np.exp(-0.5 * d2)).sum(1)
    out = {"log2N": log2n, "N": N, "d": d, "bandwidth": h, "tile": T}
    for cut in cuts:
        surv_pairs = 0
        surv_row_tiles = 0
        pairs_matter = 0
        sample = set(rng.choice(len(qlo), size=min(len(qlo), 64),
                                replace=False).tolist())
        for I in range(len(qlo)):
            gap = np.maximum(0.0, np.maximum(ylo - qhi[I], qlo[I] - yhi))
            bd2 = (gap ** 2).sum(1)
            smin = S[I * T:(I + 1) * T].min()
            surv_pairs += np.count_nonzero(
                T * wt * np.exp(-0.5 * bd2) > cut * smin)
            if I in sample:
                rows = q[I * T:(I + 1) * T]
                for r in range(T):
                    g = np.maximum(0.0, np.maximum(ylo - rows[r], rows[r] - yhi))
                    rb = (g ** 2).sum(1)
                    surv_row_tiles += np.count_nonzero(
                        T * wt * np.exp(-0.5 * rb) > cut * S[I * T + r])
                    d2 = ((y - rows[r]) ** 2).sum(1)
                    pairs_matter += np.count_nonzero(
                        w * np.exp(-0.5 * d2) > cut * S[I * T + r] / N)
        k = len(sample) * T
        out[f"cut_2^{int(np.log2(cut))}"] = {
            "tile_pairs_surviving": surv_pairs / (len(qlo) * nT),
            "row_tiles_surviving": surv_row_tiles / (k * nT),
            "pairs_mattering": pairs_matter / (k * len(y)),
        }
    return out


if __name__ == "__main__":
    sizes = [int(a) for a in sys.argv[1:]] or [14, 16]
    for s in sizes:
        print(json.dumps(run(s)), flush=True)
