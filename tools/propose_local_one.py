"""LocalTransition production proposals (resample + Cholesky perturb + prior
box flag, Philox) at config 4's shape: launch time and a checksum of the
draws, for same-box A/B runs of library builds through tools/lib_ab.py:

    python tools/lib_ab.py LIB tools/propose_local_one.py [N] [d] [B] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import _native  # noqa: E402
from pyabc_amd import kernels as K  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 6
B = int(float(sys.argv[3])) if len(sys.argv) > 3 else 400_000
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
w /= w.sum()
A = torch.randn((N, d, d), dtype=torch.float64, device="cuda", generator=g) * 0.1
covs = (A @ A.transpose(1, 2) + 0.05 * torch.eye(d, dtype=torch.float64,
                                                 device="cuda")).contiguous()
cdf = K.resample_cdf(w)
lo = torch.full((d,), -3.0, dtype=torch.float64, device="cuda")
sc = torch.full((d,), 6.0, dtype=torch.float64, device="cuda")
th0, idx0, sup0 = K.propose_local(X, cdf, covs, 11, 0, 0, B, lo, sc)
ts = []
for r in range(reps):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    th, idx, sup = K.propose_local(X, cdf, covs, 11, 0, 0, B, lo, sc)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
same = bool(torch.equal(th, th0) and torch.equal(idx, idx0) and torch.equal(sup, sup0))
print(f"{_native.LIB_PATH}: propose_local N={N} d={d} B={B}: min {ts[0]:.3f} ms "
      f"median {ts[len(ts) // 2]:.3f} ms checksum {float(th0.sum()):.17g} "
      f"{int(idx0.sum())} {int(sup0.sum())} repeat_identical={same}", flush=True)
