"""A few weighted-quantile calls at N = 1e6 (for rocprofv3 kernel traces)."""
import sys

import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
g = torch.Generator(device="cuda").manual_seed(0)
d = torch.rand(n, dtype=torch.float64, device="cuda", generator=g) * 3 + 1
w = torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
w /= w.sum()
for _ in range(5):
    K.weighted_quantile(d, w, 0.5)
torch.cuda.synchronize()
print("ok")
