"""Host profile (cProfile, cumulative time) of one tools/bench_configs.py
config: where a generation's host time goes between the device stages.

    python tools/prof_configs.py x1 [TOP]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "x1"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 45
    import torch
    torch.cuda.set_device(0)
    getattr(bench_configs, name)()          # warm-up (compiles, caches)
    pr = cProfile.Profile()
    pr.enable()
    getattr(bench_configs, name)()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(top)


if __name__ == "__main__":
    main()
