"""Host profile of engine.next_generation_inputs (epsilon + fit + pack +
CDF of the next generation) on the bench's population: wall time per call
(synchronised), and cProfile's cumulative breakdown of 20 calls.

    python tools/next_inputs_prof.py [d] [N]"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pyabc_amd.engine import next_generation_inputs  # noqa: E402
from tests.test_gpu_fullsize import _bench_population  # noqa: E402


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1_000_000
    torch.cuda.set_device(0)
    fit, res = _bench_population(d, N, 2)
    th, dd = res.theta, res.d
    ww = res.w / res.w.sum()
    for _ in range(3):
        next_generation_inputs(th, dd, ww, 0.5)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        eps, f = next_generation_inputs(th, dd, ww, 0.5)
        f.cdf
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"next_generation_inputs d={d} N={N}: min {min(ts):.3f} ms, "
          f"median {sorted(ts)[10]:.3f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        eps, f = next_generation_inputs(th, dd, ww, 0.5)
        f.cdf
        torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
