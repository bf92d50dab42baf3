"""Interleaved timing of the kNN kernel's rows-per-wave choices (tuning knob
ABC_KNN_ROWS) at config 4's shape; every variant must return the same
neighbour sets and distances.

    python tools/knn_ab.py [N] [d] [k]"""
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
    base = None
    for rnd in range(3):
        for rpw in ("4", "8"):
            os.environ["ABC_KNN_ROWS"] = rpw
            K.reload_tuning()
            nbr, d2 = K.knn(X, k)
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                K.knn(X, k)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            if base is None:
                base = (nbr.clone(), d2.clone())
            same = bool(torch.equal(nbr, base[0]) and torch.equal(d2, base[1]))
            print(f"round {rnd} rows/wave {rpw:>2}: {min(ts):7.3f} ms  "
                  f"identical={same}", flush=True)
    os.environ.pop("ABC_KNN_ROWS", None)
    K.reload_tuning()


if __name__ == "__main__":
    main()
