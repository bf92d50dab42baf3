"""CPU baseline leg of bench.py: the reference's per-particle generation path,
restated by the numpy oracle, timed on the host cores.

TEST INFRASTRUCTURE ONLY (``bench.py``'s ``cpu_baseline`` leg).  It mirrors
what pyABC's ``MulticoreEvalParallelSampler``
(sampler/multicore_evaluation_parallel.py:12-48, 92-146) does on a node:
C forked workers, each running the ``simulate_one`` closure
(smc.py:580-645) until the shared target is met, per proposal

  * ``MultivariateNormalTransition.rvs``: ``np.random.choice(p=w)`` rebuilds
    and searches the O(N) CDF on every call (multivariatenormal.py:87-95),
    then ``x + z @ A``;
  * the prior-support redraw loop (smc.py:629-645);
  * the batch model and ``PNormDistance`` (distance.py:76-102), ``d <= eps``;

and per accepted particle the O(N d) KDE density ``transition_pdf``
(smc.py:722-733, multivariatenormal.py:102-125).

Workers are started with the ``spawn`` method (fresh interpreters that
import numpy and this module only; they never touch the GPU) and pinned to
one BLAS thread each.  They run the SAME generations the GPU timed (each
generation's previous population, fit and epsilon), an equal wall slice per
generation; a generation's rate is the sum over workers of accepted
particles / busy time, and the baseline is their harmonic mean -- the rate
of running each generation to the same population size, as the GPU's value
is measured.
"""
import multiprocessing as mp
import os
import time

import numpy as np


def _worker(paths, seconds, seed, out_q):
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import ref_cpu as ref
    rng = np.random.default_rng(seed)
    res = []
    for path in paths:     # one slice per generation of the GPU's schedule
        with np.load(path, allow_pickle=False) as f:
            X, w, cov = f["X"], f["w"], f["cov"]
            A_model, x0, lo, sc = f["A_model"], f["x0"], f["lo"], f["sc"]
            eps, sigma, p = float(f["eps"]), float(f["sigma"]), float(f["p"])
        A = ref.svd_factor(cov)
        fw = np.ones_like(x0)
        d = X.shape[1]
        acc = evals = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            cdf = ref.resample_cdf(w)                      # O(N) per proposal
            idx = ref.resample_indices(cdf, rng.random())
            th = X[idx] + rng.standard_normal(d) @ A
            if not ref.uniform_box_support(th[None], lo, sc)[0]:
                continue
            y = th @ A_model.T + sigma * rng.standard_normal(A_model.shape[0])
            dist = ref.pnorm_distance(y[None], x0, fw, p)[0]
            evals += 1
            if dist <= eps:
                acc += 1
                ref.kde_transition_pd(th[None], X, w, cov)  # O(N d)
        res.append((acc, evals, time.perf_counter() - t0))
    out_q.put(res)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def run(gens, A_model, x0, lo, sc, sigma, p=2.0, workers=None, seconds=8.0,
        tmpdir="/tmp"):
    """The CPU path over the GPU's own generations: ``gens`` is a list of
    (X, w, cov, eps) -- previous population, its fitted covariance and the
    generation's epsilon -- each run for seconds / len(gens) on every
    worker.  Returns a dict: per-generation accepted/s summed over workers,
    their schedule rate (the harmonic mean: the rate of running every
    generation to the same population size, as the GPU value is), workers,
    accepted, evaluations, wall seconds."""
    if workers is None:
        workers = min(16, os.cpu_count() or 1)
    paths = []
    for g, (X, w, cov, eps) in enumerate(gens):
        path = os.path.join(tmpdir, f"abc_cpu_baseline_{os.getpid()}_{g}.npz")
        np.savez(path, X=X, w=w, cov=cov, A_model=A_model, x0=x0, lo=lo,
                 sc=sc, eps=eps, sigma=sigma, p=p)
        paths.append(path)
    per = seconds / len(gens)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(paths, per, 1000 + i, q))
             for i in range(workers)]
    t0 = time.perf_counter()
    for pr in procs:
        pr.start()
    res = [q.get() for _ in procs]
    for pr in procs:
        pr.join()
    wall = time.perf_counter() - t0
    for path in paths:
        os.remove(path)
    rates = [sum(r[g][0] / r[g][2] for r in res) for g in range(len(gens))]
    acc = [sum(r[g][0] for r in res) for g in range(len(gens))]
    ev = [sum(r[g][1] for r in res) for g in range(len(gens))]
    sched = len(rates) / sum(1.0 / max(r, 1e-12) for r in rates)
    return dict(rate=sched, per_generation=rates, workers=workers,
                accepted=acc, evaluations=ev, wall=wall,
                seconds_per_generation=per, cpu_model=cpu_model(),
                host_cpus=os.cpu_count())
