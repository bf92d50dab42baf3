"""Launch time and checksum of the previous population's pack
(`abc_kde_pack_prev_f64` / `_f32`: max-weight key + whitened rows with log2
weights) at N rows, dimension d, for same-box A/B runs of library builds:

    python tools/lib_ab.py LIB tools/pack_time.py N d [f64|f32] [reps]"""
import hashlib
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import _native  # noqa: E402
from pyabc_amd import kernels as K  # noqa: E402

N, d = int(float(sys.argv[1])), int(sys.argv[2])
prec = sys.argv[3] if len(sys.argv) > 3 else "f64"
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
w[::97] = 0.0
w /= w.sum()
A = torch.randn((d, d), dtype=torch.float64, device="cuda", generator=g)
Us = (A / math.sqrt(d)).contiguous()
mu = X.mean(0).contiguous()
pp0 = K.PackedPopulation(X, w, mu, Us, d, 0.0, prec)
P0 = pp0.P.clone()
ts = []
for _ in range(reps):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    pp = K.PackedPopulation(X, w, mu, Us, d, 0.0, prec)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
print(f"{_native.LIB_PATH}: pack {prec} N={N} d={d}: min {ts[0]:.3f} ms "
      f"median {ts[len(ts) // 2]:.3f} ms sha1 "
      f"{hashlib.sha1(P0.cpu().numpy().tobytes()).hexdigest()[:16]} "
      f"{float(pp0.lw2max):.17g} identical={bool(torch.equal(pp.P, P0))}",
      flush=True)
