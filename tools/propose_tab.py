"""Proposal kernel time against the CDF bucket table's size (the search's
dependent loads: ~log2(N / 2^L) of them after the two table reads), rows
checked bit-identical across table sizes, at config 5's and the headline's
shapes:

    python tools/propose_tab.py [N] [B]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd.engine import DeviceMVNFit  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
B = int(float(sys.argv[2])) if len(sys.argv) > 2 else 4_194_304
torch.cuda.set_device(0)
for d in (8, 20):
    g = torch.Generator(device="cuda").manual_seed(d)
    X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
    w /= w.sum()
    fit = DeviceMVNFit(X, w)
    cdf = fit.cdf
    lo = torch.full((d,), -5.0, dtype=torch.float64, device="cuda")
    sc = torch.full((d,), 10.0, dtype=torch.float64, device="cuda")
    tabs = {L: K.cdf_index(cdf, L) for L in (12, 16, 18, 20, 22)}
    ts = {L: [] for L in tabs}
    outs = {}
    for rep in range(5):
        for L, tab in tabs.items():
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            o = K.propose_philox(fit.X, cdf, fit.A, lo, sc, 1, 2, 0, B, tab=tab)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                ts[L].append(e0.elapsed_time(e1))
            outs[L] = o
    same = all(torch.equal(a, b) for L in outs for a, b in zip(outs[L], outs[16]))
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for L in (20,):
        K.cdf_index(cdf, L)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps(dict(N=N, d=d, B=B, identical=same,
                          ms={L: min(v) for L, v in ts.items()},
                          table_build_ms_L20=e0.elapsed_time(e1))), flush=True)
