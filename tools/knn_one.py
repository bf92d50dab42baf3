"""Two kNN calls at config 4's shape (N = 2e5, d = 6, k = 50) for
rocprofv3 PMC passes of knn_kernel.

    python tools/knn_one.py [N] [d] [k]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402


def main():
    N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
    X *= torch.linspace(0.5, 2.0, d, dtype=torch.float64, device="cuda")
    for _ in range(2):
        K.knn(X, k)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
