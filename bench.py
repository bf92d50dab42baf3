"""Headline benchmark: one ABC-SMC generation (t >= 1) at N = 1e6, d = 8.

metric (BASELINE.json): accepted particles/s per generation + KDE weight
pairs/s, N=1e6, d=8, 1-8 GPUs.

One step = one full generation of the per-generation particle update on the
device (pyabc_amd.engine): Philox proposals (resample + perturb + prior
support), batch simulation of the S=100 linear-Gaussian model, p-norm
distances + acceptance until N particles are accepted, the O(N^2 d) KDE
importance-weight pass, weight normalisation, the all-gather of the new
population (N > 1 GPUs), the transition refit and the quantile epsilon.
Strong scaling: N is the whole population whatever the GPU count; ranks
split the proposals and new particles.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from pyabc_amd import kernels as K  # noqa: E402
from pyabc_amd.batch_models import LinearGaussianModel  # noqa: E402
from pyabc_amd.distributed import Comm  # noqa: E402
from pyabc_amd.engine import (GenerationEngine, DeviceMVNFit,  # noqa: E402
                              next_generation_inputs)

FP32_PEAK_TFLOPS = 157.3   # MI355X vector FP32 (MI355X_MICROARCH.md)
MFMA16_PEAK_TFLOPS = 2500.0  # dense f16 / bf16 MFMA (no sparsity)
CLOCK_HZ = 2.4e9
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(gens, model, x0, d, seconds):
    """The reference's per-particle CPU path (restated by the oracle) on the
    host cores, MulticoreEvalParallelSampler-style (oracle/cpu_baseline.py),
    over the same generations (previous population, fit, epsilon) the GPU
    timed."""
    from oracle import cpu_baseline as cb
    return cb.run(gens, model.A_host, x0.cpu().numpy(), np.full(d, -5.0),
                  np.full(d, 10.0), model.sigma, 2.0, seconds=seconds,
                  kde_dims=sorted({d, 20}))


def kde_traffic():
    """HBM bytes per launch of the KDE kernel from the committed rocprofv3
    PMC passes (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE;
    tools/pmc_traffic.py writes the file)."""
    path = os.path.join(ROOT, "profiles", "kde_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        t = json.load(f)
    return t.get("hbm_bytes_per_launch"), t.get("source")


def kde_pmc(d):
    """Per-tile instruction counts of the MFMA KDE kernel from the NEWEST
    committed rocprofv3 PMC file taken at this d (tools/kde_pmc.py writes
    ``profiles/rNN_kde_pmc.json`` with a ``d`` key; the d > 8 passes are
    ``profiles/rNN_kde_dDD_pmc.json``).  Files are ranked by their round
    tag, never by a fixed list, so a new round's profile supersedes the
    old one as soon as it is committed."""
    import glob
    import re
    best = None
    for path in glob.glob(os.path.join(ROOT, "profiles", "r*_kde*_pmc.json")):
        m = re.match(r"r(\d+)_kde(?:_d(\d+))?_pmc\.json$",
                     os.path.basename(path))
        if not m:
            continue
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        fd = t.get("d", int(m.group(2)) if m.group(2) else None)
        pt = t.get("per_tile", {})
        if fd != d or "SQ_INSTS_VALU" not in pt or "SQ_INSTS_MFMA" not in pt:
            continue
        key = int(m.group(1))
        if best is None or key > best[0]:
            best = (key, t, path)
    return (best[1], best[2]) if best else (None, None)


# tools/probes/issue_probe.hip variants holding the kernel's PMC-counted
# per-tile mix (MFMA, v_exp_f32, other VALU); a non-integer VALU count is
# the mean of two variants
# (round 6: SQ_INSTS_VALU counts the MFMAs too -- the issue probe's own mix
# under --pmc, 4 MFMA + 16 exp + 22 adds per step, reads 42.0 VALU -- so
# the kernel's other VALU per tile is VALU - TRANS - MFMA: 17.5 at d = 8,
# 18.0 at d = 20; rounds 2-5 priced 21.5 / 28 and over-stated the probe's
# ceiling)
PROBE_MIX = {8: (22, 23),  # 4 MFMA, 16 exp, 17 / 18 other (PMC 17.5)
             20: (24,)}    # 9 MFMA, 16 exp, 18 other (PMC 18.0)
PROBE_WAVES = {8: 4, 20: 2}  # the KDE kernel's occupancy (waves per SIMD)

# MI355X_MICROARCH.md per-instruction constants (cycles per wave64
# instruction on one SIMD): the guide's hardware floor prices plain VALU at
# its SIMD-32 throughput (2), the single-wave static pricing at the issue
# cost one wave's stream sees (4); transcendentals 8, an MFMA holds vector
# issue 8 of its 32 matrix-pipe cycles
GUIDE_CYC = {"valu": 2.0, "trans": 8.0, "mfma_issue": 8.0, "mfma_pipe": 32.0}
STATIC_CYC = {"valu": 4.0, "trans": 8.0, "mfma_issue": 8.0, "mfma_pipe": 32.0}


def mix_cycles(V, T, F, c):
    """Cycles per 32x32 tile per SIMD of the mix (V VALU incl. T
    transcendentals, F MFMAs) at the cost table c: the larger of the SIMD's
    vector issue and the matrix pipe."""
    return max(c["valu"] * (V - T) + c["trans"] * T + c["mfma_issue"] * F,
               c["mfma_pipe"] * F)


def issue_probe(d, waves_per_simd=None):
    """Live ceiling of the KDE kernel's per-tile instruction mix on THIS GPU
    (tools/probes/issue_probe.hip: the mix with no memory traffic, VALU in
    the MFMA gaps, at the kernel's own waves per SIMD): ns per tile and
    SIMD, or None when the probe library is not built or has no mix for d."""
    if waves_per_simd is None:
        waves_per_simd = PROBE_WAVES.get(d, 2)
    import ctypes
    path = os.path.join(ROOT, "tools", "probes", "libabc_probe.so")
    vs = PROBE_MIX.get(d)
    if vs is None or not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.abc_probe_kde_mix.restype = ctypes.c_double
    lib.abc_probe_kde_mix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    torch.cuda.synchronize()
    ns = [lib.abc_probe_kde_mix(v, waves_per_simd, 100000) for v in vs]
    return sum(ns) / len(ns) if min(ns) > 0 else None


def kde_roofline(d, achieved_tf, traffic, traffic_src, avg_launch_s,
                 pairs_per_launch, tiles_per_launch):
    """Roofline of the dominant kernel (the MFMA KDE pass).

    The pass is bound by the SIMD's instruction issue: per 32x32 tile of
    pairs a wave issues MFMAs (the d-dimensional exponent on the matrix
    cores) and VALU (v_exp_f32, row-sum tree; plus the hi+lo add when the
    accumulation is split, d > 8).  The ceiling is MEASURED live: the probe
    (tools/probes/issue_probe.hip) runs that per-tile mix -- PMC-counted,
    profiles/r0*_kde_pmc.json -- with no memory traffic and the VALU spread
    over the MFMA gaps, at the kernel's own occupancy (PROBE_WAVES) on
    every SIMD of this GPU, so clock and dual-wave issue are those the chip
    really sustains:

        t_ceiling = tiles / 1024 SIMDs * t_probe(per tile per SIMD)

    frac = t_ceiling / t_launch.  achieved / peak are the same ratio in
    SURVEY 8(d)'s algorithmic unit (3d+4 FLOP per pair).  The static
    pricing of the same mix at the guide's single-wave issue costs and
    2.4 GHz is kept beside it (``static_issue``), the same mix priced at
    the guide's hardware floor (plain VALU 2 cycles at SIMD-32 throughput,
    ``guide_floor`` / ``frac_guide_floor``), and the FP32 vector-peak
    figure of a VALU-only pass as ``valu_equiv`` (it exceeds 1: the MFMA
    does the d-dimensional part)."""
    pmc, pmc_path = kde_pmc(d)
    pairs_per_s = pairs_per_launch / avg_launch_s
    fpp = 3 * d + 4
    D = K.padded_dim(d)
    # f16 piece schemes (kde_mfma.hip Mk<D>): folded up to D = 24, split above
    KH, KL = (D + 4 + 15) // 16, (5 * D + 4 + 15) // 16
    if pmc is not None:
        pt = pmc["per_tile"]
        # SQ_INSTS_VALU includes the MFMAs (measured on the issue probe):
        # V below is the VALU excluding them
        F = pt["SQ_INSTS_MFMA"]
        V, T = (pt["SQ_INSTS_VALU"] - F, pt.get("SQ_INSTS_VALU_TRANS_F32", 0.0))
        src = f"{os.path.relpath(pmc_path, ROOT)} (rocprofv3 --pmc, per-tile)"
    else:   # static count of the kernel's per-tile code
        F = KH + KL
        # folded accumulation (D <= 24): no hi + lo add (kde_mfma.hip)
        V, T = (32.0 if D <= 24 else 48.0), 16.0
        src = "static per-tile instruction count (no PMC file for this d)"
    cyc = mix_cycles(V, T, F, STATIC_CYC)
    t_static = tiles_per_launch * cyc / (1024 * CLOCK_HZ)
    # the guide's hardware floor: plain VALU at its SIMD-32 throughput
    cyc_floor = mix_cycles(V, T, F, GUIDE_CYC)
    t_floor = tiles_per_launch * cyc_floor / (1024 * CLOCK_HZ)
    ns_probe = issue_probe(d)
    if ns_probe is not None:
        t_ceil = tiles_per_launch * ns_probe * 1e-9 / 1024
        basis = ("live issue probe on this GPU (tools/probes/issue_probe.hip: "
                 "the kernel's per-tile mix, no memory traffic, VALU in the "
                 f"MFMA gaps, {PROBE_WAVES.get(d, 2)} waves per SIMD) x tiles / 1024 SIMDs; "
                 f"mix counts: {src}; algorithmic {fpp} FLOP/pair")
    else:
        t_ceil = t_static
        basis = ("SIMD issue ceiling of the instruction mix (VALU 4, TRANS 8, "
                 "MFMA 8 issue / 32 pipe cycles per wave64 instruction, 1024 "
                 f"SIMDs at 2.4 GHz; probe library not built); {src}; "
                 f"algorithmic {fpp} FLOP/pair")
    frac = t_ceil / avg_launch_s
    peak_tf = achieved_tf / frac
    mfma_tf = 32768 * F * tiles_per_launch / avg_launch_s / 1e12
    return {
        "bound": "issue (MFMA + VALU)",
        "kernel": "MFMA KDE pass (exact-grid f16 pieces: "
                  "v_mfma_f32_32x32x16_f16 for the d-dim exponent, hi and "
                  "lo in one accumulator up to d = 24 -- then v_exp_f32 + "
                  "the row-sum add per pair on the VALU)",
        "achieved": achieved_tf,
        "peak": peak_tf,
        "unit": "TFLOP/s",
        "frac": frac,
        "frac_static_issue": t_static / avg_launch_s,
        "frac_guide_floor": t_floor / avg_launch_s,
        "ceiling_note": "frac divides by a SELF-MEASURED ceiling (this "
                        "repo's tools/probes/issue_probe.hip run live on "
                        "this GPU); frac_static_issue prices the same "
                        "PMC-counted mix at one wave's issue costs (VALU 4, "
                        "TRANS 8, MFMA 8 of 32 cycles), frac_guide_floor at "
                        "MI355X_MICROARCH.md's hardware floor (VALU 2 at "
                        "SIMD-32 throughput, TRANS 8, MFMA 8 issue / 32 "
                        "pipe), both at 2.4 GHz on 1024 SIMDs",
        "traffic": traffic,
        "traffic_source": traffic_src,
        "peak_basis": basis,
        "probe_ns_per_tile_per_simd": ns_probe,
        "ceiling_ms": t_ceil * 1e3,
        "static_issue": {"cycles_per_tile": cyc,
                         "ceiling_ms": t_static * 1e3,
                         "frac": t_static / avg_launch_s},
        "guide_floor": {"cycles_per_tile": cyc_floor,
                        "ceiling_ms": t_floor * 1e3,
                        "frac": t_floor / avg_launch_s,
                        "cycles": GUIDE_CYC},
        "mix_per_tile": {"mfma": F, "trans": T, "other_valu": V - T,
                         "source": src},
        "flops_per_pair": fpp,
        "avg_launch_ms": avg_launch_s * 1e3,
        "pairs_per_launch": pairs_per_launch,
        "pairs_per_s": pairs_per_s,
        "valu_equiv": {"achieved": achieved_tf, "peak": FP32_PEAK_TFLOPS,
                       "unit": "TFLOP/s", "frac": achieved_tf / FP32_PEAK_TFLOPS},
        "mfma_f16": {"achieved": mfma_tf, "peak": MFMA16_PEAK_TFLOPS,
                      "unit": "TFLOP/s",
                      "frac": mfma_tf / MFMA16_PEAK_TFLOPS},
    }


# xGMI model for the rank-slice prediction: ASSUMED
# constants, not measured here (no multi-GPU box): one link per GPU pair,
# 153 GB/s nominal per link (the task's figure) at an assumed 50 % RCCL
# efficiency, and a fixed latency per collective call.
XGMI_LINK_GBS = 153.0 * 0.5
RCCL_LATENCY_US = 25.0


def rank_slice_report(args, comm, N, d, S, ms_step, stages, kde_ms,
                      kde_pairs, coll, state):
    """One line per R: rank 0's measured share of a generation, its stage
    breakdown, the collectives it would issue (calls, bytes) and the
    predicted whole-job time with the xGMI model added."""
    R = comm.world
    steps = len(stages)
    keys = sorted({k for tm in stages for k in tm})
    avg = {k: sum(tm.get(k, 0.0) for tm in stages) / steps for k in keys}
    per_step = {k: [v[0] / steps, v[1] / steps, v[2] / steps]
                for k, v in coll.items()}
    # latency per call; all-gathers: the largest piece over one link (each
    # peer sends its own piece on its own link, in parallel)
    xgmi_ms = 0.0
    for kind, (calls, sent, recv) in per_step.items():
        if kind == "barrier" and R == 1:
            continue
        xgmi_ms += calls * RCCL_LATENCY_US * 1e-3 if R > 1 else 0.0
        if kind == "all_gather_rows" and R > 1:
            xgmi_ms += recv / (R - 1) / (XGMI_LINK_GBS * 1e9) * 1e3
    kde_avg = sum(kde_ms) / max(len(kde_ms), 1)
    scaling = ("sample_generation", "engine_kde")
    fixed = {k: v for k, v in avg.items()
             if k in ("cdf", "normalise", "quantile", "fit_pack",
                      "next_inputs")}
    pred_ms = ms_step + xgmi_ms
    return {
        "kind": "rank-slice (predicted, unmeasured on multi-GPU hardware)",
        "R": R, "N": N, "d": d, "S": S, "steps": steps,
        "rank0_ms_per_step": ms_step,
        "stage_ms": avg,
        "stage_timing": "rank0_ms_per_step: the timed steps, unsynchronised "
                        "as in the real job (side-stream work overlaps); "
                        "stage_ms: as many further steps with the launching "
                        "stream synchronised after every stage (side-stream "
                        "work is charged where it is waited for)",
        "kde_launch_ms": kde_avg,
        "kde_rows_per_launch": (sum(kde_pairs) / max(len(kde_pairs), 1)) / N,
        "repeated_full_population_ms": sum(fixed.values()),
        "largest_non_scaling_term": max(fixed, key=fixed.get) if fixed
        else None,
        "collectives_per_step": {k: {"calls": v[0], "bytes_sent": v[1],
                                     "bytes_received": v[2]}
                                 for k, v in per_step.items()},
        "xgmi_model_ms": xgmi_ms,
        "xgmi_model": f"{RCCL_LATENCY_US} us per collective call + the "
                      f"largest all-gather piece / {XGMI_LINK_GBS} GB/s "
                      f"(one link per GPU pair; assumed constants)",
        "predicted_ms_per_step": pred_ms,
        "predicted_value": N / (pred_ms * 1e-3),
        "unit": "accepted particles/s",
        "eps_last": state["eps"],
        "scaling_terms": list(scaling),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--particles", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=8)
    ap.add_argument("--n-stats", type=int, default=100)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rank-slice", type=int, default=0, metavar="R",
                    help="one GPU runs rank 0's share of an R-GPU job "
                         "(pyabc_amd.distributed.RankSliceComm): B/R "
                         "proposals per round, M/R KDE rows, every "
                         "full-population stage; prints the stage times, "
                         "the collectives' byte counts and the xGMI-model "
                         "prediction instead of the contract line")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="multi-rank rehearsal on a one-GPU box: every rank "
                         "on cuda:0, gloo collectives staged through host")
    args = ap.parse_args()

    if args.rank_slice:
        from pyabc_amd.distributed import RankSliceComm
        comm = RankSliceComm(args.rank_slice)
        torch.cuda.set_device(0)
    elif args.rehearse_gloo:
        comm = Comm.from_env("gloo", device=0)
    else:
        comm = Comm.from_env("nccl")
    if comm.world == 1 and not args.rank_slice:
        torch.cuda.set_device(0)
    R = comm.world
    N, d, S = args.particles, args.dim, args.n_stats
    model = LinearGaussianModel.benchmark(d, S)
    x0 = torch.as_tensor(model._x0, device="cuda")
    fw = K.full(S, 1.0)
    eng = GenerationEngine(model, np.full(d, -5.0), np.full(d, 10.0),
                           distance_p=2.0, comm=comm, seed=args.seed)

    # population 0: prior sample, uniform weights; eps from the sample
    # (QuantileEpsilon 'from_sample', epsilon.py:138-155)
    r0 = eng.sample_prior(0, N)
    d0, _, _ = K.pnorm_distance(r0.stats_T, x0, fw, 2.0, math.inf,
                                with_accept=False)
    theta = comm.all_gather_rows(r0.theta)
    dist = comm.all_gather_rows(d0)
    w = K.full(theta.shape[0], 1.0 / theta.shape[0])
    eps = float(K.weighted_quantile(dist, w, 0.5, comm=comm)[0].item())
    fit = DeviceMVNFit(theta, w)

    # the CPU leg reruns up to 4 evenly spaced timed generations; their fits
    # are kept by reference (no copy inside the timed region)
    K_ = args.steps
    pick = sorted({round(i * (K_ - 1) / 3) for i in range(4)}) if K_ > 4 \
        else list(range(K_))
    state = {"fit": fit, "eps": eps, "n_eval": 0, "t": 1, "sched": {},
             "k": None}

    stages = []     # --rank-slice: synchronised stage times per step
    sync_marks = {"on": False}

    def mark(tm, key, t0):
        if sync_marks["on"]:
            # the launching stream only: side-stream work that overlaps the
            # next stages (the CDF, the KDE pack) is charged where it is
            # waited for (the next step's "cdf", the density pass)
            torch.cuda.current_stream().synchronize()
            t1 = time.perf_counter()
            tm[key] = tm.get(key, 0.0) + (t1 - t0) * 1e3
            return t1
        return t0

    def step():
        t = state["t"]
        if state["k"] is not None:
            if state["k"] in pick:
                state["sched"][state["k"]] = (state["fit"], state["eps"])
            state["k"] += 1
        tm, t0 = {}, time.perf_counter()
        if sync_marks["on"]:
            state["fit"].cdf          # the side stream's CDF, if still running
            t0 = mark(tm, "cdf", t0)
        res = eng.sample_generation(t, N, state["fit"], x0, fw, state["eps"])
        t0 = mark(tm, "sample_generation", t0)
        th, dd, ww, n_eval, _ = eng.gather_population(res)
        t0 = mark(tm, "normalise", t0)
        # epsilon, fit + pack and the resampling CDF of the next generation,
        # overlapped (engine.next_generation_inputs)
        state["eps"], state["fit"] = next_generation_inputs(th, dd, ww, 0.5,
                                                            comm=comm)
        t0 = mark(tm, "next_inputs", t0)
        if sync_marks["on"]:
            tm.update({f"engine_{k}": v * 1e3 for k, v in eng.timers.items()})
            stages.append(tm)
        state["n_eval"] = n_eval
        state["t"] = t + 1
        return res

    for _ in range(args.warmup):
        step()
    state["k"] = 0
    stages.clear()
    eng.kde_events = []
    log0 = len(comm.log) if args.rank_slice else 0
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    phases = []
    for _ in range(args.steps):
        step()
        phases.append(dict(eng.timers))
    coll = comm.summary(log0) if args.rank_slice else None
    torch.cuda.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = comm.all_reduce_max_float(elapsed)
    kde_ms = [e0.elapsed_time(e1) for (e0, e1, _, _) in eng.kde_events]
    kde_pairs = [M * Np for (_, _, M, Np) in eng.kde_events]
    rp = K.row_pad()
    kde_tiles = [(K.nat.lib().abc_kde_mfma_new_rows(M, d) // 32)
                 * (-(-Np // rp) * rp // 32) for (_, _, M, Np) in eng.kde_events]
    kde_t = sum(kde_ms) / 1e3
    pairs_local = sum(kde_pairs)
    kde_t_max = comm.all_reduce_max_float(kde_t)
    pairs_total = comm.all_reduce_int(pairs_local)
    ms_step = elapsed / args.steps * 1e3
    value = N * args.steps / elapsed
    flops_per_pair = 3 * d + 4
    traffic, traffic_src = kde_traffic()
    # per-launch roofline of the dominant kernel on this rank
    avg_launch_s = kde_t / max(len(kde_ms), 1)
    pairs_per_launch = pairs_local / max(len(kde_ms), 1)
    tiles_per_launch = sum(kde_tiles) / max(len(kde_ms), 1)
    achieved_tf = flops_per_pair * pairs_per_launch / avg_launch_s / 1e12
    log(f"[rank {comm.rank}] steps={args.steps} elapsed={elapsed:.3f}s "
        f"ms/step={ms_step:.1f} kde avg launch {avg_launch_s*1e3:.1f} ms "
        f"({achieved_tf:.1f} TF/s) eps={state['eps']:.4g} "
        f"n_eval={state['n_eval']} phases={phases[-1]}")

    if args.rank_slice:
        # the stage breakdown: as many steps again, synchronised after each
        # stage (the timed steps above ran unsynchronised, as the real job)
        sync_marks["on"] = True
        for _ in range(args.steps):
            step()
        sync_marks["on"] = False
    if comm.rank != 0:
        return
    if args.rank_slice:
        print(json.dumps(rank_slice_report(
            args, comm, N, d, S, ms_step, stages, kde_ms, kde_pairs,
            coll, state)), flush=True)
        return
    out = {
        "metric": "accepted particles/s per generation + KDE weight pairs/s, "
                  "N=1e6 d=8",
        "value": value,
        "unit": "accepted particles/s",
        "n_gpus": R,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32 (KDE exponent from exact-grid f16-piece MFMA, fp64 "
                 "row sums) / f64 (all other stages)",
        "data": "synthetic",
        "config": {
            "workload": "one ABC-SMC generation t>=1: MVN transition, "
                        "N=1e6, d=8, S=100 linear-Gaussian batch model, "
                        "PNormDistance p=2, QuantileEpsilon alpha=0.5, "
                        "Uniform(-5,5)^8 prior",
            "N": N, "d": d, "S": S,
            "parallelism": f"dp{R} (proposals + new particles sharded, "
                           f"population all-gathered per generation)"},
        "kde_pairs_per_s": pairs_total / kde_t_max,
        "roofline": kde_roofline(d, achieved_tf, traffic, traffic_src,
                                 avg_launch_s, pairs_per_launch,
                                 tiles_per_launch),
    }
    if R == 1 and not args.no_cpu_baseline:
        # the timed generations themselves, up to 4 evenly spaced ones
        sched = state["sched"]
        gens = [(sched[i][0].X.cpu().numpy(), sched[i][0].w.cpu().numpy(),
                 sched[i][0].cov, sched[i][1]) for i in pick]
        cb = cpu_baseline(gens, model, x0, d, args.cpu_seconds)
        out["cpu_baseline"] = {
            "value": cb["rate"], "unit": "accepted particles/s",
            "cores": cb["workers"], "kind": "port",
            "cpu_model": cb["cpu_model"], "host_cpus": cb["host_cpus"],
            "physical_cores": cb["physical_cores"],
            "cpu_share": cb["cpu_share"],
            "value_all_physical_cores_ideal": cb[
                "rate_all_physical_cores_ideal"],
            "kde_pairs_per_s": cb.get("kde_pairs_per_s_1core"),
            "kde_pairs_per_s_ideal_all_cores": cb.get(
                "kde_pairs_per_s_ideal_all_cores"),
            "kde_pairs_basis": f"one core, the reference's MVN.pdf of one "
                               f"particle against N_prev="
                               f"{cb.get('kde_n_prev')} (eigh + whitening + "
                               f"exp-sum, multivariatenormal.py:102-125); "
                               f"ideal = x physical cores",
            "tN_fit": cb.get("tN_fit"),
            "per_generation": cb["per_generation"],
            "eps": [g[3] for g in gens],
            "sample": f"the timed schedule's generations {pick} (of "
                      f"{K_}; eps {[round(g[3], 3) for g in gens]}), "
                      f"{cb['seconds_per_generation']:.1f} s each on "
                      f"{cb['workers']} spawned workers (min of the "
                      f"{cb['physical_cores']} physical cores and this "
                      f"process's {cb['cpu_share']}-CPU share; 1 BLAS thread "
                      f"each; "
                      f"{cb['accepted']} accepted of {cb['evaluations']} "
                      f"evaluations); value = harmonic mean of the "
                      f"per-generation rates (N_prev={N}, d={d}, S={S}): the "
                      f"reference's per-particle algorithm "
                      f"(MulticoreEvalParallelSampler layout; O(N) CDF per "
                      f"proposal, O(N d) KDE per acceptance) restated by "
                      f"the numpy oracle"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
