"""Is the density pass slower on the bench's own rows than on synthetic
ones?  Runs bench-like generations (N = 1e6, d = 8, S = 100) through the
engine, then times the KDE launch of the last generation's population
against its own accepted rows, back to back, beside a synthetic population
of the same shape (tools/kde_time.py's data) -- same process, same box:

    python tools/kde_inloop.py [generations]"""
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd.batch_models import LinearGaussianModel  # noqa: E402
from pyabc_amd.engine import (DeviceMVNFit, GenerationEngine,  # noqa: E402
                              next_generation_inputs)
from oracle import ref_cpu as ref  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 6
N, d, S = 1_000_000, 8, 100
torch.cuda.set_device(0)
model = LinearGaussianModel.benchmark(d, S)
x0 = torch.as_tensor(model._x0, device="cuda")
fw = K.full(S, 1.0)
eng = GenerationEngine(model, np.full(d, -5.0), np.full(d, 10.0),
                       distance_p=2.0, seed=2024)
r0 = eng.sample_prior(0, N)
d0, _, _ = K.pnorm_distance(r0.stats_T, x0, fw, 2.0, math.inf,
                            with_accept=False)
w = K.full(N, 1.0 / N)
eps = float(K.weighted_quantile(d0, w, 0.5)[0].item())
fit = DeviceMVNFit(r0.theta, w)
eng.kde_events = []
for t in range(1, G + 1):
    res = eng.sample_generation(t, N, fit, x0, fw, eps)
    th, dd, ww, _, _ = eng.gather_population(res)
    last_fit, last_theta = fit, res.theta
    eps, fit = next_generation_inputs(th, dd, ww, 0.5)
torch.cuda.synchronize()
inloop = [e0.elapsed_time(e1) for (e0, e1, _, _) in eng.kde_events]


def time_launches(pp, Y, reps=6):
    ts = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        pp.logpdf_whitened(Y)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return ts


# the last generation's population against its own accepted rows
pp = last_fit.packed
Y = pp.whiten(last_theta)
real = time_launches(pp, Y)
# synthetic rows of the same shape (tools/kde_time.py)
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
ws = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
ws /= ws.sum()
cov = ref.mvn_fit_cov(X.cpu().numpy(), ws.cpu().numpy())
U, rank, lpd = K.psd_whitening(cov)
Us = torch.as_tensor(U * math.sqrt(0.5 * K.LOG2E), device="cuda")
ps = K.PackedPopulation(X, ws, torch.zeros(d, dtype=torch.float64,
                                           device="cuda"), Us, rank, lpd, "mfma")
Ys = ps.whiten(X + 0.1)
synth = time_launches(ps, Ys)
real2 = time_launches(pp, Y)
print(json.dumps({"inloop_ms": inloop, "real_rows_standalone_ms": real,
                  "synthetic_standalone_ms": synth,
                  "real_rows_again_ms": real2}), flush=True)
