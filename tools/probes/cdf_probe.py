"""Times the tiled exact CDF on the bench's weight shapes (run under
rocprofv3 --kernel-trace --stats for the per-kernel split)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from pyabc_amd import kernels as K  # noqa: E402

torch.cuda.set_device(0)
rng = np.random.default_rng(0)
for n in [100_000, 1_000_000]:
    for kind in ["uniform", "equal", "lognormal1", "lognormal3"]:
        if kind == "uniform":
            w = rng.uniform(0.5, 1.5, n)
        elif kind == "equal":
            w = np.ones(n)
        else:  # importance-weight-like spread
            w = rng.lognormal(0.0, float(kind[-1]), n)
        w = torch.as_tensor(w / w.sum(), device="cuda")
        K.resample_cdf(w)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            K.resample_cdf(w)
        e1.record()
        torch.cuda.synchronize()
        print(f"n={n} {kind}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us",
              flush=True)
