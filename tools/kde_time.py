"""Launch time of the MFMA KDE pass at N = M, dimension d (min and median of
HIP-event-timed launches after one warm-up), for same-box A/B runs of
compile-time variants through tools/lib_ab.py:

    python tools/lib_ab.py LIB tools/kde_time.py N d [reps]"""
import math
import sys

import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd import _native  # noqa: E402
from oracle import ref_cpu as ref  # noqa: E402

N, d = int(float(sys.argv[1])), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
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
Y = pp.whiten(X + 0.1)
out0 = pp.logpdf_whitened(Y).clone()
ts = []
for _ in range(reps):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    out = pp.logpdf_whitened(Y)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
print(f"{_native.LIB_PATH}: N={N} d={d} min {ts[0]:.2f} ms median "
      f"{ts[len(ts) // 2]:.2f} ms  checksum {float(out0.sum()):.17g} "
      f"identical={bool(torch.equal(out, out0))}", flush=True)
