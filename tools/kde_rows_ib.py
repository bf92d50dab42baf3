"""KDE launch time at M = N / R rows (one rank's share of an R-GPU job)
for each i-tiles-per-wave choice (ABC_KDE_MFMA_IB 3 / 2 / 1: finer row
blocks fill the launch's last wave of blocks better), interleaved, rows
checked bit-identical across the choices:

    python tools/kde_rows_ib.py N d R [R ...]"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402
from oracle import ref_cpu as ref  # noqa: E402

N, d = int(float(sys.argv[1])), int(sys.argv[2])
Rs = [int(r) for r in sys.argv[3:]] or [1, 2, 4, 8]
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
for R in Rs:
    M = -(-N // R)
    Y = pp.whiten(X[:M] + 0.1)
    res = {}
    outs = {}
    for rep in range(4):
        for ib in ("3", "2", "1"):
            os.environ["ABC_KDE_MFMA_IB"] = ib
            K.reload_tuning()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            out = pp.logpdf_whitened(Y)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                res.setdefault(ib, []).append(e0.elapsed_time(e1))
            outs[ib] = out.clone()
    same = all(torch.equal(outs[k], outs["3"]) for k in outs)
    print(json.dumps(dict(N=N, d=d, R=R, M=M, identical=same,
                          ms={k: min(v) for k, v in res.items()},
                          all_ms=res)), flush=True)
os.environ.pop("ABC_KDE_MFMA_IB", None)
