"""Launch time of the LocalTransition z-form density pass (mfma) at config
4's shape, for same-box A/B runs of compile-time variants:

    python tools/lib_ab.py LIB tools/lz_time.py [N] [d] [reps]"""
import sys

import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd import _native  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 6
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(3)
X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g)
w /= w.sum()
nbr, _ = K.knn(X, 50)
covs, invs, dets = K.local_cov(X, w, nbr)
pts, _, _ = K.propose_local(X, K.resample_cdf(w), covs, 11, 0, 0, N)
out0 = K.local_logpdf(pts, X, w, invs, dets, precision="mfma").clone()
ts = []
for _ in range(reps):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    out = K.local_logpdf(pts, X, w, invs, dets, precision="mfma")
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
print(f"{_native.LIB_PATH}: N={N} d={d} min {ts[0]:.2f} ms median "
      f"{ts[len(ts) // 2]:.2f} ms identical={bool(torch.equal(out, out0))} "
      f"checksum {float(out0.sum()):.17g}", flush=True)
