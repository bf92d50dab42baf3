"""Where the MFMA KDE pass's per-row offsets leave the rows of a bench
generation: log2 of each row's sum relative to its offset (parent term or
the global one), the rows the routing range sends to the refine, and the
launch time either way.

    python tools/kde_offsets.py d [N] [gens]"""
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pyabc_amd import kernels as K  # noqa: E402
from tests.test_gpu_fullsize import _bench_population  # noqa: E402


def timed(pp, theta, parent, reps=3):
    Y = pp.whiten(theta, parent)
    pp.logpdf_whitened(Y)
    ts = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        lp = pp.logpdf_whitened(Y)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return lp, Y, min(ts), pp.refined_rows(), pp.fixup_rows()


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1_000_000
    gens = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    torch.cuda.set_device(0)
    fit, res = _bench_population(d, N, gens)
    pp = fit.packed
    pp64 = K.PackedPopulation(fit.X, fit.w, pp.mu, pp.Us, fit.rank,
                              fit.log_pdet, "f64")
    lp64 = pp64.logpdf(res.theta).cpu().numpy()
    off = math.log(2) * float(pp.lw2max.item()) + pp.log_const
    l2s = (lp64 - off) / math.log(2)
    out = dict(d=d, N=N, gens=gens)
    q = [0.0, 0.001, 0.01, 0.5, 0.99, 0.999, 1.0]
    for name, par in (("global", None), ("parent", res.parent)):
        lp, Y, ms, nref, nfix = timed(pp, res.theta, par)
        m = Y.row_off.cpu().numpy()
        rel = l2s - m
        err = np.abs(np.expm1(lp.cpu().numpy() - lp64))
        out[name] = dict(ms=ms, refined=nref, fixup=nfix,
                         max_err=float(err.max()),
                         log2S_rel_quantiles=np.quantile(rel, q).tolist(),
                         m_quantiles=np.quantile(m, q).tolist())
        for T in (4, 8, 12, 16, 24):
            out[name][f"outside_{T}"] = int(np.sum((rel < -T) | ((rel > T) & (m < 0))))
        print(json.dumps(out[name]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
