"""Proposal kernel: one lane per proposal (ABC_PROPOSE_GROUP=0) against
four lanes per proposal (1, the default; 2 = 1 since the group form became
the default for every d), interleaved, at N = 1e6, B = 4.2e6,
with the adaptive CDF bucket table; draws checked bit-identical:

    python tools/propose_group.py [d ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd.engine import DeviceMVNFit  # noqa: E402

N, B = 1_000_000, 4_194_304
torch.cuda.set_device(0)
for d in [int(a) for a in sys.argv[1:]] or [12, 20, 24, 32]:
    g = torch.Generator(device="cuda").manual_seed(d)
    X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
    w /= w.sum()
    fit = DeviceMVNFit(X, w)
    lo = torch.full((d,), -5.0, dtype=torch.float64, device="cuda")
    sc = torch.full((d,), 10.0, dtype=torch.float64, device="cuda")
    ts, outs = {}, {}
    for rep in range(6):
        for form in ("0", "1", "2"):
            os.environ["ABC_PROPOSE_GROUP"] = form
            K.reload_tuning()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            o = fit.propose(lo, sc, 1, 2, 0, B)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                ts.setdefault(form, []).append(e0.elapsed_time(e1))
            outs[form] = o
    same = all(torch.equal(a, b) for f in ("1", "2")
               for a, b in zip(outs["0"], outs[f]))
    ms = {f: min(v) for f, v in ts.items()}
    print(json.dumps(dict(N=N, d=d, B=B, identical=same, ms=ms,
                          tb_per_s={f: (16 * d + 17) * B / (v * 1e-3) / 1e12
                                    for f, v in ms.items()},
                          log2k=K.cdf_index_log2(N))), flush=True)
os.environ.pop("ABC_PROPOSE_GROUP", None)
