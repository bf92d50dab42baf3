"""The spatial index's key sort (abc_radix_sort_pairs_u64): time per sort of
n random 60-bit keys with int32 indices, min over repeats, HIP events on the
library's stream:

    python tools/sort_time.py [n ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402

torch.cuda.set_device(0)
for n in [int(float(a)) for a in sys.argv[1:]] or [200_000, 1_000_000]:
    g = torch.Generator(device="cuda").manual_seed(n)
    keys = torch.randint(0, 2 ** 60, (n,), dtype=torch.int64, device="cuda",
                         generator=g)
    vals = torch.arange(n, dtype=torch.int32, device="cuda")
    ts = []
    for rep in range(12):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        ko, vo = K.radix_sort_pairs(keys, vals, 60)
        e1.record()
        torch.cuda.synchronize()
        if rep >= 2:
            ts.append(e0.elapsed_time(e1))
    ok = bool(torch.equal(ko, torch.sort(keys, stable=True).values))
    print(json.dumps({"n": n, "end_bit": 60, "ms_min": min(ts),
                      "ms_median": sorted(ts)[len(ts) // 2], "sorted": ok}))
