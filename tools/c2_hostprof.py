"""Host-side profile of a tools/bench_configs.py config's generations:
where the wall time goes between the device stages, and which Python call
sites issue the synchronous device reads / copies (.item(), .cpu(),
torch.as_tensor of host data, torch.cuda.synchronize).

    python tools/c2_hostprof.py [c2|c4|c5] [gens]"""
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tools.bench_configs as bc  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    gens = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    torch.cuda.set_device(0)
    fn = getattr(bc, name)
    fn(gens=3)                      # warm-up (allocations, JIT)
    pr = cProfile.Profile()
    pr.enable()
    fn(gens=gens)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(30)
    st.sort_stats("tottime").print_stats(30)
    out = io.StringIO()
    st2 = pstats.Stats(pr, stream=out)
    st2.sort_stats("tottime").print_callers(
        r"method 'item'|method 'cpu'|as_tensor|_cuda_synchronize|method 'tolist'")
    print(out.getvalue())


if __name__ == "__main__":
    main()
