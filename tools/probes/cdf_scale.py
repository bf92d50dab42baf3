"""Exact-CDF chain cost against the number of binade exits: equal weights
at n = 2^k (an exit at every doubling of the chain), one call per n, run
under rocprofv3 --kernel-trace to read cdf_chain_kernel's duration per n."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
from pyabc_amd import kernels as K  # noqa: E402

torch.cuda.set_device(0)
ns = [256, 1024, 2048, 4096, 8192, 16384, 32768, 65536, 131072, 1 << 20]
for rep in range(3):
    for n in ns:
        w = torch.full((n,), 1.0 / n, dtype=torch.float64, device="cuda")
        K.resample_cdf(w)
        torch.cuda.synchronize()
print("ns", ns, flush=True)
