"""A few production proposal launches (resample + perturb + prior-box flag,
Philox) at config 5's shape, for rocprofv3 PMC passes and timing:

    python tools/propose_one.py [N] [d] [B] [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd.engine import DeviceMVNFit  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B = int(float(sys.argv[3])) if len(sys.argv) > 3 else 4_194_304
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
w /= w.sum()
fit = DeviceMVNFit(X, w)
lo = torch.full((d,), -5.0, dtype=torch.float64, device="cuda")
sc = torch.full((d,), 10.0, dtype=torch.float64, device="cuda")
fit.propose(lo, sc, 1, 2, 0, B)
ts = []
for r in range(reps):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    th, idx, sup = fit.propose(lo, sc, 1, 2, r * B, B)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
print(f"propose N={N} d={d} B={B}: min {min(ts):.3f} ms, "
      f"{min(ts) * 1e6 / B:.3f} ns per proposal, "
      f"in support {float(sup.float().mean()):.3f}", flush=True)
