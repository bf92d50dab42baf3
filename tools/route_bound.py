"""Derived bound of the folded MFMA KDE pass against the routing threshold
(rows whose pass-1 sum falls below it are refined with their own offset):
for constructed rows whose largest exponent lies in [-EMIN, -16] (log2,
few dominant terms: tests/test_gpu_kde_band.py's construction), the largest
per-row bound and the refined fraction for each candidate threshold.

    python tools/route_bound.py d [EMIN]"""
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_cpu as ref  # noqa: E402
from pyabc_amd import kernels as K  # noqa: E402
from tests.kde_bound import row_stats, pass_offsets  # noqa: E402


def band_rows(Yp, lw, n_want, rng, d, emin):
    Yh, lh = Yp.cpu().numpy(), lw.cpu().numpy()
    rows = []
    while sum(len(r) for r in rows) < n_want:
        m = 4096
        j = rng.integers(0, len(Yh), m)
        t = rng.uniform(16.0, emin, m)
        u = rng.normal(size=(m, Yh.shape[1]))
        u[:, d:] = 0.0
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        y = Yh[j] + np.sqrt(lh[j] + t)[:, None] * u
        st = row_stats(Yp, lw, torch.as_tensor(y, device="cuda"),
                       torch.zeros(m, dtype=torch.float64, device="cuda"),
                       1, Yp.shape[1], 1.0)
        keep = (st["emax"] >= -emin) & (st["emax"] <= -16) & (st["H"] <= 3.0)
        rows.append(y[keep])
    return np.concatenate(rows)[:n_want]


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    emin = float(sys.argv[2]) if len(sys.argv) > 2 else 40.0
    torch.cuda.set_device(0)
    rng = np.random.default_rng(700 + d)
    N = 65536
    X = rng.normal(size=(N, d)) * rng.uniform(0.5, 2.0, d)
    w = rng.uniform(0.5, 1.5, N)
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    U, rank, log_pdet = K.psd_whitening(cov)
    Us = U * math.sqrt(0.5 * K.LOG2E)
    mu = (X * w[:, None]).sum(0) / w.sum()
    dv = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda")
    pp = K.PackedPopulation(dv(X), dv(w), dv(mu), dv(Us), rank, log_pdet, "mfma")
    D = pp.D
    Yp = pp.P[:N, :D].contiguous()
    lw = pp.P[:N, D].contiguous()
    g = float(pp.gscale.item())
    KL = (5 * D + 4 + 15) // 16
    Yc = band_rows(Yp, lw, 12000, rng, d, emin)
    theta = mu + Yc[:, :d] @ np.linalg.pinv(Us)
    Wr = pp.whiten(dv(theta))
    z = torch.zeros(len(Yc), dtype=torch.float64, device="cuda")
    st0 = row_stats(Yp, lw, Wr.Y, z, KL, D, g)
    out = []
    for e in (24, 26, 28, 30, 32):
        m_fin, routed = pass_offsets(st0["log2S"], st0["emax"],
                                     np.zeros(len(Yc)), D, lo=2.0 ** -e)
        st = row_stats(Yp, lw, Wr.Y, torch.as_tensor(m_fin, device="cuda"),
                       KL, D, g)
        out.append(dict(d=d, D=D, KL=KL, threshold_log2=-e, rows=len(Yc),
                        emax_min=-emin, refined_frac=float(routed.mean()),
                        bound_max=float(st["bound"].max()),
                        bound_p999=float(np.quantile(st["bound"], 0.999))))
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
