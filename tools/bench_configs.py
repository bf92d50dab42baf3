"""End-to-end runs of BASELINE.json's configs through the drop-in API
(pyabc_amd.ABCSMC + GPUBatchSampler) on one MI355X.

    python tools/bench_configs.py [--only c1 c2 c4 c5] > gpurun_out/configs.jsonl

One JSON line per config: per-generation sampling wall time (the metric's
"accepted particles/s per generation" = N / sample_until_n_accepted wall,
generations t >= 1), the whole-generation wall time (start to next start:
sampling plus the refits between generations), acceptance, epsilon
trajectory, total wall time and the posterior mean.  Config 3 (the KDE pass at N = 1e6, d = 8) is bench.py.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import pyabc_amd as pa  # noqa: E402


def linear_problem(d, S, A_scale):
    A = np.random.RandomState(42).randn(S, d) / A_scale
    theta_true = np.linspace(-1, 1, d) if d != 4 else np.array(
        [0.5, -1.0, 1.5, 0.0])
    x0 = A @ theta_true + 0.5 * np.random.RandomState(7).randn(S)
    keys = [f"y{k:03d}" for k in range(S)]
    names = [f"p{k:02d}" for k in range(d)]
    return A, theta_true, x0, keys, names


def run(name, abc, x0, names, theta_true=None, db=None, **run_kw):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    abc.new(db or f"mem://{name}", x0)
    if db is not None:
        # the reference's timing runs store no statistics
        abc.history.stores_sum_stats = False
    h = abc.run(**run_kw)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    store_s = None
    if db is not None:
        t1 = time.perf_counter()
        h._sql.flush()          # writes still queued after the last one
        store_s = time.perf_counter() - t1
        wall += store_s
    log = abc.generation_log
    N = abc.population_size(0) if callable(getattr(abc, "population_size",
                                                   None)) else None
    df, w = h.distribution_numpy(0, h.max_t)
    w = w / w.sum()
    mean = (df[names].values * w[:, None]).sum(0)
    tl = getattr(abc.sampler, "timer_log", [])
    tl = tl[-len(log):] if len(tl) >= len(log) else [{}] * len(log)
    gens = [dict(t=e["t"], eps=float(e["eps"]), n_sim=int(e["n_sim"]),
                 sample_s=float(e["sample_seconds"]), batch=e["batch"],
                 timers={k: round(v * 1e3, 4) for k, v in tm.items()})
            for e, tm in zip(log, tl)]
    # whole generation: from one generation's start to the next's (sampling,
    # History append, the transition / distance / epsilon refit between them)
    for g, e, e1 in zip(gens, log, log[1:]):
        g["generation_s"] = float(e1["started"] - e["started"])
    n_pop = int(len(w))
    rates = [n_pop / g["sample_s"] for g in gens if g["t"] >= 1]
    whole = [g["generation_s"] for g in gens if g["t"] >= 1 and "generation_s" in g]
    out = dict(config=name, N=n_pop, generations=len(gens), wall_s=wall,
               accepted_per_s_median_t_ge_1=float(np.median(rates))
               if rates else None,
               generation_ms_median_t_ge_1=float(np.median(whole)) * 1e3
               if whole else None,
               all_batch=all(g["batch"] for g in gens), gens=gens,
               posterior_mean=mean.tolist())
    if db is not None:
        out["db"] = db
        out["store_wait_after_run_s"] = store_s
    if theta_true is not None:
        out["theta_true"] = list(map(float, theta_true))
    print(json.dumps(out), flush=True)
    return out


def c1(gens=10):
    np.random.seed(0)
    prior = pa.Distribution(mean=pa.RV("uniform", 0, 5))
    abc = pa.ABCSMC(pa.GaussianMeanModel(), prior, pa.PNormDistance(p=2),
                    population_size=1000, eps=pa.MedianEpsilon(),
                    sampler=pa.GPUBatchSampler(seed=1))
    run("c1_quickstart_N1000", abc, {"data": 2.5}, ["mean"], [2.5],
        minimum_epsilon=0.1, max_nr_populations=gens)


def c2(N=100_000, gens=6):
    A, th, x0, keys, names = linear_problem(4, 100, 2.0)
    model = pa.LinearGaussianModel(A, None, 0.5, keys=keys)
    prior = pa.Distribution(**{n: pa.RV("uniform", -5, 10) for n in names})
    abc = pa.ABCSMC(model, prior, pa.AdaptivePNormDistance(
        p=2, scale_function=pa.median_absolute_deviation),
        population_size=N, eps=pa.QuantileEpsilon(alpha=0.5),
        sampler=pa.GPUBatchSampler(seed=2))
    run("c2_adaptive_mad_N1e5_d4_S100", abc, dict(zip(keys, x0)), names, th,
        max_nr_populations=gens)


def c2_file(N=100_000, gens=6):
    """C2 with its History in a sqlite file (the reference's schema,
    SURVEY 8(f) rank 1): the population writes overlap the generations."""
    import tempfile
    A, th, x0, keys, names = linear_problem(4, 100, 2.0)
    model = pa.LinearGaussianModel(A, None, 0.5, keys=keys)
    prior = pa.Distribution(**{n: pa.RV("uniform", -5, 10) for n in names})
    abc = pa.ABCSMC(model, prior, pa.AdaptivePNormDistance(
        p=2, scale_function=pa.median_absolute_deviation),
        population_size=N, eps=pa.QuantileEpsilon(alpha=0.5),
        sampler=pa.GPUBatchSampler(seed=2))
    db = pa.create_sqlite_db_id(tempfile.mkdtemp(), "c2.db")
    run("c2_file_history_N1e5_d4_S100", abc, dict(zip(keys, x0)), names, th,
        db=db, max_nr_populations=gens)


def c4(N=200_000, gens=4):
    A, th, x0, keys, names = linear_problem(6, 100, np.sqrt(6))
    model = pa.LinearGaussianModel(A, None, 0.5, keys=keys)
    prior = pa.Distribution(**{n: pa.RV("uniform", -5, 10) for n in names})
    abc = pa.ABCSMC(model, prior, pa.PNormDistance(p=2),
                    population_size=N,
                    transitions=pa.LocalTransition(k=50, k_fraction=None),
                    eps=pa.QuantileEpsilon(alpha=0.5),
                    sampler=pa.GPUBatchSampler(seed=4))
    run("c4_local_k50_N2e5_d6", abc, dict(zip(keys, x0)), names, th,
        max_nr_populations=gens)


def c5(N=1_000_000, gens=10):
    A, th, x0, keys, names = linear_problem(20, 100, np.sqrt(20))
    model = pa.LinearGaussianModel(A, None, 0.5, keys=keys)
    prior = pa.Distribution(**{n: pa.RV("uniform", -5, 10) for n in names})
    abc = pa.ABCSMC(model, prior, pa.PNormDistance(p=2),
                    population_size=N, eps=pa.QuantileEpsilon(alpha=0.5),
                    sampler=pa.GPUBatchSampler(seed=5))
    run("c5_10gen_N1e6_d20_S100", abc, dict(zip(keys, x0)), names, th,
        max_nr_populations=gens)


def x1(N=100_000, gens=6):
    """Exact inference: noise-free C2 model, Gaussian
    likelihood IndependentNormalKernel(var=0.25), StochasticAcceptor,
    Temperature() (AcceptanceRateScheme over all recorded evaluations:
    two device KDE passes per generation)."""
    A, th, x0, keys, names = linear_problem(4, 100, 2.0)
    model = pa.LinearGaussianModel(A, None, 0.0, keys=keys)
    prior = pa.Distribution(**{n: pa.RV("uniform", -5, 10) for n in names})
    abc = pa.ABCSMC(model, prior, pa.IndependentNormalKernel(var=0.25),
                    population_size=N, eps=pa.Temperature(),
                    acceptor=pa.StochasticAcceptor(),
                    sampler=pa.GPUBatchSampler(seed=6))
    out = run("x1_exact_inference_N1e5_d4_S100", abc, dict(zip(keys, x0)),
              names, th, max_nr_populations=gens)
    P = A.T @ A / 0.25
    post = np.linalg.solve(P, A.T @ x0 / 0.25)
    print(json.dumps({"config": "x1_exact_posterior_mean",
                      "analytic": post.tolist(),
                      "abc": out["posterior_mean"]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*",
                    default=["c1", "c2", "c4", "c5", "x1"])
    args = ap.parse_args()
    torch.cuda.set_device(0)
    for c in args.only:
        globals()[c]()


if __name__ == "__main__":
    main()
