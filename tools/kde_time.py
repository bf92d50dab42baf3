"""Launch time of the MFMA KDE pass at one shape (for same-box A/B of
library builds through tools/lib_ab.py), with a checksum of the rows:

    python tools/kde_time.py N d [reps] [tag] [M]   (M new rows, default N)"""
import hashlib
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd import _native as nat  # noqa: E402
from oracle import ref_cpu as ref  # noqa: E402

N, d = int(float(sys.argv[1])), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
tag = sys.argv[4] if len(sys.argv) > 4 and sys.argv[4] != "-" else \
    os.path.basename(nat.LIB_PATH)
M = int(float(sys.argv[5])) if len(sys.argv) > 5 else N
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
Y = pp.whiten(X[:M] + 0.1)
ts = []
for _ in range(reps):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    out = pp.logpdf_whitened(Y)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps({"lib": tag, "N": N, "M": M, "d": d, "ms_min": min(ts),
                  "ms_median": sorted(ts)[len(ts) // 2], "sha1": h}),
      flush=True)
