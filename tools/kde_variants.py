"""Launch-shape variants of the MFMA KDE pass: time at one size and check
that every variant's rows are bit-identical to the default's.

    python tools/kde_variants.py d N [name=ENV:VAL,ENV:VAL ...]

Without variant arguments the tuning knobs of kde_mfma.hip launch_mfma are
swept (IB / PIPE / SPLIT / LDS2); each must leave every row unchanged."""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402
from oracle import ref_cpu as ref  # noqa: E402

KEYS = ("ABC_KDE_MFMA_IB", "ABC_KDE_MFMA_PIPE", "ABC_KDE_MFMA_SPLIT",
        "ABC_KDE_MFMA_LDS2", "ABC_KDE_MFMA_FOLD", "ABC_KDE_MFMA_SMAJOR")

SWEEP = [
    ("default", {}),
    ("pipe0", {"ABC_KDE_MFMA_PIPE": "0"}),
    ("ib2", {"ABC_KDE_MFMA_IB": "2"}),
    ("ib1", {"ABC_KDE_MFMA_IB": "1"}),
    ("lds2_1", {"ABC_KDE_MFMA_LDS2": "1"}),
    ("lds2_0", {"ABC_KDE_MFMA_LDS2": "0"}),
    ("split8", {"ABC_KDE_MFMA_SPLIT": "8"}),
]


def population(N, d, seed, prec="mfma"):
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
    w /= w.sum()
    cov = ref.mvn_fit_cov(X.cpu().numpy(), w.cpu().numpy())
    U, rank, lpd = K.psd_whitening(cov)
    Us = torch.as_tensor(U * math.sqrt(0.5 * K.LOG2E), device="cuda")
    mu = torch.zeros(d, dtype=torch.float64, device="cuda")
    return X, K.PackedPopulation(X, w, mu, Us, rank, lpd, prec), (w, mu, Us,
                                                                  rank, lpd)


def set_env(env):
    for k in KEYS:
        os.environ.pop(k, None)
    os.environ.update(env)
    K.reload_tuning()


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1000000
    variants = SWEEP
    if len(sys.argv) > 3:
        variants = []
        for a in sys.argv[3:]:
            name, _, spec = a.partition("=")
            env = dict(kv.split(":") for kv in spec.split(",") if kv)
            variants.append((name, env))
    Xs, pps, (ws, mus, Uss, rk, lpd) = population(20000, d, 1)
    # near rows and spread-out (low-density) rows
    th = torch.cat([Xs[:5000] + 0.05, Xs[5000:8000] * 1.8])
    Ys = pps.whiten(th)
    p64 = K.PackedPopulation(Xs, ws, mus, Uss, rk, lpd, "f64")
    exact = p64.logpdf(th).cpu().numpy()
    X, pp, _ = population(N, d, 0)
    Y = pp.whiten(X + 0.1)
    base = None
    for name, env in variants:
        set_env(env)
        rows = pps.logpdf_whitened(Ys).cpu().numpy()
        if base is None:
            base = rows
        same = np.array_equal(rows, base)
        dev = float(np.max(np.abs(np.expm1(rows - base))))
        e64 = float(np.max(np.abs(np.expm1(rows - exact))))
        pp.logpdf_whitened(Y)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            pp.logpdf_whitened(Y)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        t = min(ts)
        print(f"{name:14s} d={d} N=M={N}: {t:8.2f} ms  "
              f"{N * pp.npad / t / 1e9:.3e} pairs/s  bit-identical={same} "
              f"max-rel-vs-default={dev:.2e} vs-f64={e64:.2e}",
              flush=True)
    set_env({})


if __name__ == "__main__":
    main()
