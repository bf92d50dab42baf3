"""Column median / MAD at n = 2e5 and 2e6, S = 100 (for rocprofv3 traces):
normal columns, and columns of three values (the radix fallback)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(1)
    for n in (200_000, 2_000_000):
        data = torch.randn((100, n), dtype=torch.float64, device="cuda", generator=g)
        for _ in range(3):
            med, mad = K.column_median_mad(data)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            K.column_median_mad(data)
        e1.record()
        torch.cuda.synchronize()
        print(f"n={n} normal: {e0.elapsed_time(e1) / 5:.3f} ms", flush=True)
    data = torch.randint(0, 3, (100, 200_000), device="cuda", generator=g).double()
    K.column_median_mad(data)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
