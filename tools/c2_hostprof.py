"""Host-side profile of config 2's generations (torch.profiler): where the
sampler's wall time goes besides the kernels."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tools.bench_configs as bc  # noqa: E402


def main():
    torch.cuda.set_device(0)
    bc.c2(gens=3)                      # warm-up (allocations, JIT)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as p:
        bc.c2(gens=4)
    print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))


if __name__ == "__main__":
    main()
