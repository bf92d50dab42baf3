"""Host time of the between-generation fit (engine.DeviceMVNFit and
next_generation_inputs) at the bench's shape, with the device idle before
each call, so only the host's own work is measured (DESIGN.md section 5:
the repeated full-population stages that do not shrink with R):

    python tools/fit_host_time.py [N] [d]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd import engine as E  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 8
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
w /= w.sum()
dist = torch.rand(N, dtype=torch.float64, device="cuda", generator=g)
side = E._side_stream()
mom = K.weighted_moments(X, w).cpu().numpy()


def host_ms(fn, reps=20):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
    return float(np.median(ts[2:]))


out = {"N": N, "d": d}
out["svd_eigh_ms"] = host_ms(lambda: (np.linalg.svd(np.eye(d) + 0.1),
                                      K.psd_whitening(np.eye(d) * 2.0)))
out["fit_no_pack_stream_ms"] = host_ms(
    lambda: E.DeviceMVNFit(X, w, moments=mom.copy()))
out["fit_side_pack_ms"] = host_ms(
    lambda: E.DeviceMVNFit(X, w, moments=mom.copy(), pack_stream=side))
out["packed_population_ms"] = host_ms(
    lambda: K.PackedPopulation(X, w, torch.zeros(d, dtype=torch.float64,
                                                 device="cuda"),
                               torch.eye(d, dtype=torch.float64,
                                         device="cuda"), d, 0.0, "mfma"))
out["next_generation_inputs_ms"] = host_ms(
    lambda: E.next_generation_inputs(X, dist, w, 0.5))
out["weighted_quantile_ms"] = host_ms(lambda: K.weighted_quantile(dist, w, 0.5))
out["start_cdf_ms"] = host_ms(lambda: E.start_cdf(w))
print(json.dumps(out))
