"""Per-kernel roofline table on the GPU (one MI355X).

Times every hot-path entry point of libabc_hip at the BASELINE.json config
sizes with HIP events on the stream the kernels are launched on (torch's
current stream), and prices each against its roofline with the algorithmic
bytes / flops per unit of SURVEY.md 8(d) (DESIGN.md restates them):

  HBM-bound kernels:  frac = (units * bytes_per_unit / t) / 8.0 TB/s
  VALU-bound kernels: frac = (units * flops_per_unit / t) / 157.3 TF (f32)
                      or / 78.6 TF (f64)

    python tools/bench_kernels.py [--quick] > gpurun_out/kernels.jsonl
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd.engine import DeviceMVNFit  # noqa: E402

HBM = 8.0e12
FP32 = 157.3e12
FP64 = 78.6e12
F64 = torch.float64


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = math.inf
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 1e3)
    return best


def report(name, t, units, unit, per_unit, bound, extra=None):
    if bound == "hbm":
        ach = units * per_unit / t
        peak = HBM
        u = "GB/s"
        scale = 1e9
    else:
        ach = units * per_unit / t
        peak = FP32 if bound == "valu_f32" else FP64
        u = "TFLOP/s"
        scale = 1e12
    row = {"kernel": name, "ms": t * 1e3, "units": units, "unit": unit,
           "per_unit": per_unit, "bound": bound,
           "achieved": ach / scale, "peak": peak / scale, "ach_unit": u,
           "frac": ach / peak, "units_per_s": units / t}
    if extra:
        row.update(extra)
    print(json.dumps(row), flush=True)
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(0)
    q = 4 if args.quick else 1

    # ---------------- (a3) KDE weight pass -------------------------------
    for (N, d, prec) in [(1_000_000 // q, 8, "mfma"), (1_000_000 // q, 8, "f32"),
                         (1_000_000 // q, 20, "mfma"), (100_000, 4, "mfma"),
                         (200_000 // q, 8, "f64")]:
        X = torch.randn((N, d), dtype=F64, device="cuda", generator=g)
        w = torch.rand(N, dtype=F64, device="cuda", generator=g) + 0.5
        w /= w.sum()
        fit = DeviceMVNFit(X, w, precision=prec)
        theta = X + 0.05 * torch.randn((N, d), dtype=F64, device="cuda",
                                       generator=g)
        Y = fit.packed.whiten(theta)
        t = timed(lambda: fit.packed.logpdf_whitened(Y), reps=3)
        pairs = N * fit.packed.npad
        if prec == "mfma":
            # priced against its own SIMD issue ceiling (bench.py
            # kde_roofline: PMC per-tile counts at d = 8, static otherwise)
            import bench
            tiles = (K.nat.lib().abc_kde_mfma_new_rows(N, d) // 32) * \
                (fit.packed.npad // 32)
            ach = (3 * d + 4) * pairs / t / 1e12
            rl = bench.kde_roofline(d, ach, None, None, t, pairs, tiles)
            print(json.dumps({
                "kernel": "kde_logpdf_mfma", "ms": t * 1e3, "units": pairs,
                "unit": "pairs", "per_unit": 3 * d + 4, "bound": "valu_issue",
                "achieved": ach, "peak": rl["peak"], "ach_unit": "TFLOP/s",
                "frac": rl["frac"], "units_per_s": pairs / t,
                "ceiling_ms": rl["ceiling_ms"],
                "probe_ns_per_tile_per_simd": rl["probe_ns_per_tile_per_simd"],
                "static_cycles_per_tile": rl["static_issue"]["cycles_per_tile"],
                "valu_equiv_frac_fp32": rl["valu_equiv"]["frac"],
                "mfma_f16_frac": rl["mfma_f16"]["frac"],
                "N": N, "M": N, "d": d}), flush=True)
            continue
        report(f"kde_logpdf_{prec}", t, pairs, "pairs", 3 * d + 4,
               "valu_f64" if prec == "f64" else "valu_f32",
               {"N": N, "M": N, "d": d})

    # ---------------- (a1) fit: weighted moments -------------------------
    N, d = 1_000_000, 8
    X = torch.randn((N, d), dtype=F64, device="cuda", generator=g)
    w = torch.rand(N, dtype=F64, device="cuda", generator=g)
    t = timed(lambda: K.weighted_moments(X, w))
    report("weighted_moments_f64", t, N, "particles", 8 * (d + 1), "hbm",
           {"d": d})

    # ---------------- (a2) resample + perturb -----------------------------
    cdf = K.resample_cdf(w)
    t = timed(lambda: K.resample_cdf(w))
    report("resample_cdf_f64", t, N, "weights", 16, "hbm")
    fit = DeviceMVNFit(X, w / w.sum())
    lo = torch.full((d,), -5.0, dtype=F64, device="cuda")
    sc = torch.full((d,), 10.0, dtype=F64, device="cuda")
    B = 1 << 21
    out = (torch.empty((B, d), dtype=F64, device="cuda"),
           torch.empty(B, dtype=torch.int64, device="cuda"),
           torch.empty(B, dtype=torch.uint8, device="cuda"))
    t = timed(lambda: K.propose_philox(fit.X, cdf, fit.A, lo, sc, 1, 2, 0, B,
                                       out=out))
    # in-kernel Philox: cdf hit 8 + X[idx] 8d + theta 8d + idx 8 + flag 1
    report("propose_philox_f64", t, B, "proposals", 16 * d + 17, "hbm",
           {"N": N, "d": d})
    tab = K.cdf_index(cdf)
    t = timed(lambda: K.propose_philox(fit.X, cdf, fit.A, lo, sc, 1, 2, 0, B,
                                       out=out, tab=tab))
    report("propose_philox_indexed_f64", t, B, "proposals", 16 * d + 17,
           "hbm", {"N": N, "d": d, "log2k": K.CDF_INDEX_LOG2})
    vpos, _ = K.compact(out[2])
    t = timed(lambda: K.compact(out[2], vpos))
    report("compact_flags", t, B, "flags", 1 + 8, "hbm")

    # ---------------- batch model + (a5) distance -------------------------
    S = 100
    from pyabc_amd.batch_models import LinearGaussianModel
    model = LinearGaussianModel.benchmark(d, S)
    theta = out[0]
    stats = model.simulate(theta, 1, 3, 0)
    t = timed(lambda: model.simulate(theta, 1, 3, 0))
    report("sim_linear_gaussian_f64", t, B, "proposals", 8 * d + 8 * S, "hbm",
           {"S": S})
    x0 = torch.as_tensor(model._x0, device="cuda")
    fw = torch.ones(S, dtype=F64, device="cuda")
    dd, acc, guard = K.pnorm_distance(stats, x0, fw, 2.0, 20.0)
    t = timed(lambda: K.pnorm_distance(stats, x0, fw, 2.0, 20.0, d_out=dd,
                                       acc_out=acc, guard_out=guard))
    report("pnorm_distance_f64", t, B, "particles", 8 * S + 10, "hbm",
           {"S": S})

    # ------- (f3) exact inference: kernel density + stochastic acceptance --
    var = torch.full((S,), 0.25, dtype=F64, device="cuda")
    c = float(np.sum(np.log(2) + np.log(np.pi) + np.log(np.full(S, 0.25))))
    t = timed(lambda: K.stochastic_kernel(stats, x0, var, K.KERNEL_NORMAL, c,
                                          pdf_norm=-50.0, inv_temp=0.1,
                                          seed=1, stream=9))
    # stats 8S + pd 8 + accept 1 + weight 8 + guard 1 (u is in-kernel Philox)
    report("stochastic_kernel_accept_f64", t, B, "evaluations", 8 * S + 18,
           "hbm", {"S": S})
    pdv = dd.clone()
    lnum = torch.randn(B, dtype=F64, device="cuda", generator=g)
    lden = torch.randn(B, dtype=F64, device="cuda", generator=g)
    t = timed(lambda: K.tempered_sums(pdv, 30.0, [0.5], logw_num=lnum,
                                      logw_den=lden))
    report("tempered_sums_f64", t, B, "records", 24, "hbm", {"K": 1})

    # ---------------- (a6) adaptive scales --------------------------------
    for n in (200_000, 2_000_000 // q):
        data = stats[:, :n].contiguous() if n <= B else torch.randn(
            (S, n), dtype=F64, device="cuda", generator=g)
        t = timed(lambda: K.column_median_mad(data), reps=3)
        report("column_median_mad_f64", t, S * n, "values", 16, "hbm",
               {"S": S, "n": n})
        t = timed(lambda: K.column_std(data), reps=3)
        report("column_std_f64", t, S * n, "values", 8, "hbm",
               {"S": S, "n": n})

    # ---------------- (a4) normalisation + (a7) quantile -------------------
    dist = torch.rand(N, dtype=F64, device="cuda", generator=g)
    t = timed(lambda: K.dsum(w))
    report("sum_f64", t, N, "weights", 8, "hbm")
    t = timed(lambda: K.weighted_quantile(dist, w / w.sum(), 0.5))
    report("weighted_quantile_f64", t, N, "particles", 16, "hbm")

    # ---------------- (a8) LocalTransition (config 4) ----------------------
    N4, d4, k4 = 200_000 // q, 6, 50
    X4 = torch.randn((N4, d4), dtype=F64, device="cuda", generator=g)
    w4 = torch.rand(N4, dtype=F64, device="cuda", generator=g)
    w4 /= w4.sum()
    nbr, _ = K.knn(X4, k4)
    t = timed(lambda: K.knn(X4, k4), reps=2)
    report("knn_f64", t, N4 * N4, "pairs", 3 * d4, "valu_f32",
           {"N": N4, "d": d4, "k": k4})
    covs, invs, dets = K.local_cov(X4, w4, nbr)
    t = timed(lambda: K.local_cov(X4, w4, nbr))
    report("local_cov_f64", t, N4, "particles", 8 * (k4 * (d4 + 1) + 2 * d4 * d4 + 1)
           + 4 * k4, "hbm", {"N": N4, "d": d4, "k": k4})
    pts = X4 + 0.01
    t = timed(lambda: K.local_logpdf(pts, X4, w4, invs, dets), reps=2)
    report("local_logpdf_f64", t, N4 * N4, "pairs",
           3 * d4 + 2 * d4 * d4 + 4, "valu_f64", {"N": N4, "d": d4})
    t = timed(lambda: K.local_logpdf(pts, X4, w4, invs, dets, "f32"), reps=2)
    report("local_logpdf_f32", t, N4 * N4, "pairs",
           3 * d4 + 2 * d4 * d4 + 4, "valu_f32", {"N": N4, "d": d4})


if __name__ == "__main__":
    main()
