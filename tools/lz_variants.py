"""Launch-shape variants of the z-form local density (local_mfma.hip) at C4
(N = M = 2e5, d = 6, k = 50): time each and check that its rows are
bit-identical to the default's.

    python tools/lz_variants.py [N] [d] [name=ENV:VAL,ENV:VAL ...]"""
import os
import sys

import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402

KEYS = ("ABC_LZ_IB", "ABC_LZ_TPB")
SWEEP = [("default", {}), ("ib2", {"ABC_LZ_IB": "2"}), ("ib1", {"ABC_LZ_IB": "1"}),
         ("tpb4", {"ABC_LZ_TPB": "4"}), ("ib2_tpb4", {"ABC_LZ_IB": "2", "ABC_LZ_TPB": "4"})]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    variants = SWEEP
    if len(sys.argv) > 3:
        variants = []
        for a in sys.argv[3:]:
            name, _, spec = a.partition("=")
            variants.append((name, dict(kv.split(":") for kv in spec.split(",") if kv)))
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g)
    w /= w.sum()
    nbr, _ = K.knn(X, 50)
    covs, invs, dets = K.local_cov(X, w, nbr)
    pts, _, _ = K.propose_local(X, K.resample_cdf(w), covs, 11, 0, 0, N)
    ref = K.local_logpdf(pts, X, w, invs, dets, precision="f64")
    base = None
    for name, env in variants:
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        K.reload_tuning()
        out = K.local_logpdf(pts, X, w, invs, dets, precision="mfma")
        if base is None:
            base = out.clone()
        same = bool(torch.equal(out, base))
        err = float(torch.expm1(out - ref).abs().max())
        ts = []
        for _ in range(3):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            K.local_logpdf(pts, X, w, invs, dets, precision="mfma")
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"{name:10s} N=M={N} d={d}: {min(ts):7.2f} ms  bit-identical={same} "
              f"vs-f64={err:.2e}", flush=True)
    for k in KEYS:
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
