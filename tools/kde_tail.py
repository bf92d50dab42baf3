"""The MFMA KDE launch at a rank's share of the rows (M = N / R) against the
full population (N = 1e6, d = 8): ms per launch and the excess over
R x (M = N)'s time / R -- the 'tail' of the rank-slice model (DESIGN.md
section 5) -- for the launch-order knobs (ABC_KDE_MFMA_SMAJOR, _SPLIT):

    python tools/kde_tail.py [d]"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402
from oracle import ref_cpu as ref  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = 1_000_000
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
w /= w.sum()
cov = ref.mvn_fit_cov(X.cpu().numpy(), w.cpu().numpy())
U, rank, lpd = K.psd_whitening(cov)
Us = torch.as_tensor(U * math.sqrt(0.5 * K.LOG2E), device="cuda")
mu = torch.zeros(d, dtype=torch.float64, device="cuda")
pp = K.PackedPopulation(X, w, mu, Us, rank, lpd, "mfma")
Yall = X + 0.1


def launch_ms(Y, reps):
    ts = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        pp.logpdf_whitened(Y)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    launch_ms.mean = sum(ts[1:]) / max(len(ts) - 1, 1)
    return min(ts)


variants = [("default", {})] if os.environ.get("KDE_TAIL_DEFAULT_ONLY") \
    else [("default", {}), ("row_major", {"ABC_KDE_MFMA_SMAJOR": "0"})]
base = None
for name, env in variants:
    for k in ("ABC_KDE_MFMA_SMAJOR", "ABC_KDE_MFMA_SPLIT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    K.reload_tuning()
    for R in (1, 2, 4, 8, 16):
        M = N // R
        Y = pp.whiten(Yall[:M])
        ms = launch_ms(Y, 3 if R == 1 else 6)
        if name == "default" and R == 1:
            base = ms
        print(json.dumps({"variant": name, "R": R, "M": M, "ms": ms,
                          "ms_mean": launch_ms.mean,
                          "excess_ms": ms - base / R}), flush=True)
