"""LocalTransition device passes at C4 (N = 2e5, d = 6, k = 50): kNN,
local covariances, density (f16 MFMA z form, fp32, fp64) -- ms per call,
HIP events."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts)


def main(N=200_000, d=6, k=50, scale=1.0):
    g = torch.Generator(device="cuda").manual_seed(3)
    X = scale * torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g)
    w /= w.sum()
    nbr, _ = K.knn(X, k)
    covs, invs, dets = K.local_cov(X, w, nbr)
    # evaluation points as the C4 generation draws them: the production
    # LocalTransition proposal (X[idx] + Cholesky(C_idx) z, Philox)
    cdf = K.resample_cdf(w)
    pts, _, _ = K.propose_local(X, cdf, covs, 11, 0, 0, N)
    out = {"knn_ms": timed(lambda: K.knn(X, k)),
           "local_cov_ms": timed(lambda: K.local_cov(X, w, nbr))}
    for prec in ("mfma", "f32", "f64"):
        out[f"pdf_{prec}_ms"] = timed(
            lambda: K.local_logpdf(pts, X, w, invs, dets, precision=prec))
    b = K.local_logpdf(pts, X, w, invs, dets, precision="f64")
    for prec in ("f32", "mfma"):
        a = K.local_logpdf(pts, X, w, invs, dets, precision=prec)
        out[f"max_rel_{prec}_vs_f64"] = float(torch.expm1(a - b).abs().max())
    print({k_: (f"{v:.3e}" if k_.startswith("max_rel") else round(v, 4))
           if isinstance(v, float) else v for k_, v in out.items()}, flush=True)


def prof(N=200_000, d=6, k=50, reps=5):
    """the z-form pass alone at C4 (for rocprofv3 kernel stats / PMC)"""
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g)
    w /= w.sum()
    nbr, _ = K.knn(X, k)
    covs, invs, dets = K.local_cov(X, w, nbr)
    pts, _, _ = K.propose_local(X, K.resample_cdf(w), covs, 11, 0, 0, N)
    for _ in range(reps):
        K.local_logpdf(pts, X, w, invs, dets, precision="mfma")
    torch.cuda.synchronize()


if __name__ == "__main__":
    if sys.argv[1:] == ["prof"]:
        prof()
        sys.exit(0)
    main()
    main(N=200_000, d=4, k=50)
    main(N=50_000, d=8, k=50)
