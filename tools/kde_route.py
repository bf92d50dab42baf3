"""Routing experiment of the folded MFMA KDE pass at d > 8 (VERDICT r05
item 1): for each (parent shift c, window U) the pass evaluates a parent
row relative to m = floor(e_parent) + c and refines it when its sum S''
leaves [2^-U, 2^U] (kde_mfma.hip, ABC_KDE_PARENT_SHIFT / _WIN).  Per
setting: the launch time, the refined rows, the error of every row against
the fp64 pass, and the derived bound (tests/kde_bound.py) on the rows most
at risk (largest / smallest S'' inside the window, the worst rows) plus a
random sample.

    python tools/kde_route.py d N gens  c:U [c:U ...]"""
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pyabc_amd import kernels as K  # noqa: E402
from tests.test_gpu_fullsize import _bench_population  # noqa: E402
from tests.kde_bound import row_stats, row_stats_all  # noqa: E402


def set_route(c, U):
    os.environ["ABC_KDE_PARENT_SHIFT"] = str(c)
    os.environ["ABC_KDE_PARENT_WIN"] = str(U)
    K.reload_tuning()


def main():
    d = int(sys.argv[1])
    N = int(float(sys.argv[2]))
    gens = int(sys.argv[3])
    settings = [tuple(int(v) for v in a.split(":")) for a in sys.argv[4:]]
    torch.cuda.set_device(0)
    fit, res = _bench_population(d, N, gens)
    pp = fit.packed
    pp64 = K.PackedPopulation(fit.X, fit.w, pp.mu, pp.Us, fit.rank,
                              fit.log_pdet, "f64")
    lp64 = pp64.logpdf(res.theta).cpu().numpy()
    off = math.log(2) * float(pp.lw2max.item()) + pp.log_const
    l2s = (lp64 - off) / math.log(2)
    D = pp.D
    KL = (5 * D + 4 + 15) // 16
    g = float(pp.gscale.item())
    n = int(fit.n)
    Yp = pp.P[:n, :D].contiguous()
    lw = pp.P[:n, D].contiguous()
    rng = np.random.default_rng(7)
    M = res.theta.shape[0]
    for c, U in settings:
        set_route(c, U)
        Y = pp.whiten(res.theta, res.parent)
        pp.logpdf_whitened(Y)
        ts = []
        for _ in range(3):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            lp = pp.logpdf_whitened(Y)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        nref, nfix = pp.refined_rows(), pp.fixup_rows()
        err = np.abs(np.expm1(lp.cpu().numpy() - lp64))
        m1 = Y.row_off.cpu().numpy()
        rel = l2s - m1
        keep = np.where(m1 == 0, rel >= -4, (rel >= -U) & (rel <= U))
        # the final offsets: refined rows get m1 + floor(log2 S'')
        m_fin = np.where(keep, m1, m1 + np.floor(rel))
        relf = l2s - m_fin
        kept = np.nonzero(keep)[0]
        order = kept[np.argsort(relf[kept])]
        pick = np.union1d(rng.choice(M, 8192, replace=False),
                          np.concatenate([order[:2048], order[-4096:],
                                          np.argsort(err)[-512:]]))
        pb = torch.as_tensor(pick, device="cuda")
        st = row_stats(Yp, lw, Y.Y.index_select(0, pb),
                       torch.as_tensor(m_fin[pick], device="cuda"), KL, D, g)
        torch.cuda.synchronize()
        tb = time.perf_counter()
        sa = row_stats_all(pp, Y.Y, torch.as_tensor(m_fin, device="cuda"), KL)
        tb = time.perf_counter() - tb
        cmp = np.abs(sa["bound"][pick] / st["bound"] - 1).max()
        q = [0.0, 0.001, 0.01, 0.1, 0.5, 0.9, 0.99, 0.999, 1.0]
        out = dict(d=d, N=N, shift=c, win=U, ms_min=min(ts), ms=ts,
                   refined=nref, fixup=nfix, max_err=float(err.max()),
                   p99_err=float(np.quantile(err, 0.99)),
                   rel_quantiles=np.quantile(rel, q).tolist(),
                   frac_routed=float(1 - keep.mean()),
                   bound_rows=int(len(pick)),
                   bound_max=float(st["bound"].max()),
                   bound_p99=float(np.quantile(st["bound"], 0.99)),
                   bound_median=float(np.median(st["bound"])),
                   H_quantiles=np.quantile(st["H"], q).tolist(),
                   err_over_bound_max=float((err[pick] / st["bound"]).max()),
                   worst_bound_row_rel=float(relf[pick][np.argmax(st["bound"])]),
                   worst_bound_row_H=float(st["H"][np.argmax(st["bound"])]),
                   all_rows_bound_s=tb,
                   all_rows_vs_sample_bound_maxrel=float(cmp),
                   all_rows_bound_max=float(sa["bound"].max()),
                   all_rows_bound_p999=float(np.quantile(sa["bound"], 0.999)),
                   all_rows_err_over_bound_max=float((err / sa["bound"]).max()),
                   all_rows_n_over=int(np.sum(sa["bound"] > 1e-5 / 1.5)),
                   all_rows_H_max=float(sa["H"].max()),
                   all_rows_worst=dict(
                       rel=float(sa["log2S_rel"][np.argmax(sa["bound"])]),
                       H=float(sa["H"][np.argmax(sa["bound"])])))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
