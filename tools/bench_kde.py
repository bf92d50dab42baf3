"""KDE kernel micro-benchmark on the GPU: pairs/s and FP32 roofline fraction."""
import math
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from pyabc_amd import kernels as K  # noqa: E402


def run(N, M, d, prec="f32", reps=3):
    K.reload_tuning()   # the callers below set the knobs in os.environ
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn((N, d), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand(N, dtype=torch.float64, device="cuda", generator=g) + 0.5
    w /= w.sum()
    Xh = X.cpu().numpy()
    wh = w.cpu().numpy()
    from oracle import ref_cpu as ref
    cov = ref.mvn_fit_cov(Xh, wh)
    U, rank, lpd = K.psd_whitening(cov)
    Us = torch.as_tensor(U * math.sqrt(0.5 * K.LOG2E), device="cuda")
    mu = torch.zeros(d, dtype=torch.float64, device="cuda")
    pp = K.PackedPopulation(X, w, mu, Us, rank, lpd, prec)
    theta = X[:M] + 0.1
    Y = pp.whiten(theta)
    pp.logpdf_whitened(Y)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        pp.logpdf_whitened(Y)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    t = min(ts)
    pairs = M * pp.npad
    fl = (3 * d + 4) * pairs / t
    print(f"N={N} M={M} d={d} {prec}: {t*1e3:.2f} ms  {pairs/t:.3e} pairs/s "
          f"{fl/1e12:.1f} TFLOP/s  frac={fl/157.3e12:.3f}  split="
          f"{K.nat.lib().abc_kde_split(M, pp.npad, d)}", flush=True)


if __name__ == "__main__":
    import os
    if len(sys.argv) > 1 and sys.argv[1] == "tiers":
        # per-rank shapes of the N=1e6 bench at 1/2/4/8 GPUs, every tier
        for M in [1000000, 500000, 250000, 125000]:
            for tier in ["0", "1", "2"]:
                os.environ["ABC_KDE_TIER"] = tier
                print(f"tier {tier}:", end=" ")
                run(1000000, M, 8, "f32", reps=2)
        for M in [100000]:
            for tier in ["0", "1", "2"]:
                os.environ["ABC_KDE_TIER"] = tier
                print(f"tier {tier}:", end=" ")
                run(100000, M, 4, "f32", reps=3)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "msplit":
        for sp in ["1", "2", "4", "8", "16", "32"]:
            os.environ["ABC_KDE_MFMA_SPLIT"] = sp
            print(f"split {sp}:", end=" ")
            run(1000000, 1000000, 8, "mfma", reps=2)
        os.environ.pop("ABC_KDE_MFMA_SPLIT")
        for ib in ["3", "1"]:
            os.environ["ABC_KDE_MFMA_IB"] = ib
            print(f"ib {ib}:", end=" ")
            run(100000, 100000, 4, "mfma", reps=3)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "lds":
        # LDS-shared A fragments vs the register version: bits and time
        def rows(N, M, d):
            g = torch.Generator(device="cuda").manual_seed(1)
            X = torch.randn((N, d), dtype=torch.float64, device="cuda",
                            generator=g)
            w = torch.rand(N, dtype=torch.float64, device="cuda",
                           generator=g) + 0.5
            w /= w.sum()
            from oracle import ref_cpu as ref
            cov = ref.mvn_fit_cov(X.cpu().numpy(), w.cpu().numpy())
            U, rank, lpd = K.psd_whitening(cov)
            Us = torch.as_tensor(U * math.sqrt(0.5 * K.LOG2E), device="cuda")
            mu = torch.zeros(d, dtype=torch.float64, device="cuda")
            pp = K.PackedPopulation(X, w, mu, Us, rank, lpd, "mfma")
            return pp.logpdf(X[:M] + 0.05)
        for d in (20, 8, 4):
            outs = {}
            for lds in ("0", "1"):
                for ib in (["2", "1"] if d == 20 else ["3", "1"] if d <= 8
                           else ["2"]):
                    os.environ["ABC_KDE_MFMA_LDS"] = lds
                    os.environ["ABC_KDE_MFMA_IB"] = ib
                    outs[(lds, ib)] = rows(20000, 5000, d).cpu().numpy()
                    print(f"d {d} lds {lds} ib {ib}:", end=" ")
                    run(262144 if d != 8 else 1000000,
                        262144 if d != 8 else 1000000, d, "mfma", reps=2)
            ref0 = outs[("0", "2" if d == 20 else "3")]
            for k, v in outs.items():
                print(f"  d {d} {k} bit-identical: {np.array_equal(v, ref0)}",
                      flush=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "sw":
        # software-pipelined / sched_group_barrier variants: bits and time
        def rows(N, M, d):
            g = torch.Generator(device="cuda").manual_seed(1)
            X = torch.randn((N, d), dtype=torch.float64, device="cuda",
                            generator=g)
            w = torch.rand(N, dtype=torch.float64, device="cuda",
                           generator=g) + 0.5
            w /= w.sum()
            from oracle import ref_cpu as ref
            cov = ref.mvn_fit_cov(X.cpu().numpy(), w.cpu().numpy())
            U, rank, lpd = K.psd_whitening(cov)
            Us = torch.as_tensor(U * math.sqrt(0.5 * K.LOG2E), device="cuda")
            mu = torch.zeros(d, dtype=torch.float64, device="cuda")
            pp = K.PackedPopulation(X, w, mu, Us, rank, lpd, "mfma")
            return pp.logpdf(X[:M] + 0.05)
        variants = [("base", {}), ("nosched", {"ABC_KDE_MFMA_SCHED": "0"}),
                    ("dma", {"ABC_KDE_MFMA_DMA": "1"})]
        dims = [int(x) for x in sys.argv[2:]] or [8, 20, 4]
        for d in dims:
            ib = {8: "1", 20: "1", 4: "1"}.get(d, "1")
            outs = {}
            for name, env in variants:
                for k in ("ABC_KDE_MFMA_SCHED", "ABC_KDE_MFMA_SW",
                          "ABC_KDE_MFMA_IB", "ABC_KDE_MFMA_DMA"):
                    os.environ.pop(k, None)
                for k, v in env.items():
                    os.environ[k] = ib if v == "h" else v
                outs[name] = rows(20000, 5000, d).cpu().numpy()
                print(f"d {d} {name}:", end=" ")
                N = {8: 1000000, 20: 262144, 4: 100000}.get(d, 262144)
                if os.environ.get("KDE_QUICK"):
                    N = min(N, 262144)
                run(N, N, d, "mfma", reps=3)
            for k, v in outs.items():
                print(f"  d {d} {k} bit-identical: "
                      f"{np.array_equal(v, outs['base'])}", flush=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "d20":
        # launch-shape sweep of the MFMA pass at d = 20 (config 5)
        for pipe in ["0", "1"]:
            for ib in ["2", "1"]:
                os.environ["ABC_KDE_MFMA_PIPE"] = pipe
                os.environ["ABC_KDE_MFMA_IB"] = ib
                print(f"pipe {pipe} ib {ib}:", end=" ")
                run(262144, 262144, 20, "mfma", reps=3)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "mfma":
        for (N, M, d) in [(1000000, 1000000, 8), (262144, 262144, 8),
                          (1000000, 500000, 8), (1000000, 125000, 8),
                          (262144, 262144, 20), (100000, 100000, 4)]:
            run(N, M, d, "mfma")
            if len(sys.argv) > 2:
                run(N, M, d, "f32")
        if len(sys.argv) > 2 and sys.argv[2] == "split":
            for sp in ["1", "2", "4", "8", "16"]:
                os.environ["ABC_KDE_MFMA_SPLIT"] = sp
                print(f"split {sp}:", end=" ")
                run(1000000, 1000000, 8, "mfma", reps=2)
        sys.exit(0)
    for (N, M, d, p) in [(262144, 262144, 8, "f32"), (1000000, 1000000, 8, "f32"),
                         (262144, 262144, 4, "f32"), (262144, 262144, 20, "f32"),
                         (65536, 65536, 8, "f64")]:
        run(N, M, d, p)
