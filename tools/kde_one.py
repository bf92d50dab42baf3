"""One MFMA KDE configuration, a few launches (for rocprofv3 --pmc runs):
    python tools/kde_one.py N d [reps]   (variant via ABC_KDE_MFMA_* env)"""
import math
import sys

import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402
from oracle import ref_cpu as ref  # noqa: E402

N, d = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
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
for _ in range(reps):
    pp.logpdf_whitened(Y)
torch.cuda.synchronize()
print("ok", flush=True)
