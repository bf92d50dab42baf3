"""Host-side profile of config 2's generations (torch.profiler): where the
sampler's wall time goes besides the kernels, and the Python call sites of
every synchronous copy (hipMemcpyWithStream) and device synchronisation.

    python tools/c2_hostprof.py [c2|c4|c5]"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tools.bench_configs as bc  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    torch.cuda.set_device(0)
    fn = getattr(bc, name)
    fn(gens=3)                      # warm-up (allocations, JIT)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 with_stack=True) as p:
        fn(gens=4)
    print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
    # call sites of the synchronous copies / syncs (innermost repo frames)
    sites = {}
    for ev in p.events():
        if ev.name not in ("aten::_local_scalar_dense", "aten::_to_copy",
                           "aten::synchronize", "cudaDeviceSynchronize",
                           "hipDeviceSynchronize"):
            continue
        stack = [s for s in (ev.stack or [])
                 if "repo" in s and "profiler" not in s][:5]
        key = (ev.name, " <- ".join(stack))
        n, t = sites.get(key, (0, 0.0))
        sites[key] = (n + 1, t + ev.cpu_time_total)
    for (nm, st), (n, t) in sorted(sites.items(), key=lambda kv: -kv[1][1]):
        print(f"{nm:22s} n={n:3d} {t / 1e3:8.3f} ms  {st}")


if __name__ == "__main__":
    main()
