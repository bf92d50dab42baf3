"""Interleaved timing of the d > 8 proposal kernel forms (ABC_PROPOSE_FORM
0 round 5, 1 chunked exact-d, 2 chunked runtime-d) at config 5's shape,
plus the HBM rate at 16d + 17 algorithmic bytes per proposal:

    python tools/propose_forms.py [N] [d] [B] [rounds]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd.engine import DeviceMVNFit  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B = int(float(sys.argv[3])) if len(sys.argv) > 3 else 4_194_304
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
w /= w.sum()
fit = DeviceMVNFit(X, w)
lo = torch.full((d,), -5.0, dtype=torch.float64, device="cuda")
sc = torch.full((d,), 10.0, dtype=torch.float64, device="cuda")
ts = {f: [] for f in ("0", "1", "2")}
outs = {}
for r in range(rounds + 1):
    for f in ts:
        os.environ["ABC_PROPOSE_FORM"] = f
        K.reload_tuning()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        o = fit.propose(lo, sc, 1, 2, 0, B)
        e1.record()
        torch.cuda.synchronize()
        if r:
            ts[f].append(e0.elapsed_time(e1))
        outs[f] = o
same = all(torch.equal(a, b) for f in ("1", "2")
           for a, b in zip(outs[f], outs["0"]))
res = {f: dict(ms_min=min(v), ms=v,
               tb_per_s=(16 * d + 17) * B / (min(v) * 1e-3) / 1e12)
       for f, v in ts.items()}
print(json.dumps(dict(N=N, d=d, B=B, bit_identical=same, forms=res)))
