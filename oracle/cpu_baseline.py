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
one BLAS thread each.  Each runs for a fixed wall budget; the baseline is the
sum over workers of accepted particles / that worker's busy time.
"""
import multiprocessing as mp
import os
import time

import numpy as np


def _worker(path, seconds, seed, out_q):
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import ref_cpu as ref
    with np.load(path, allow_pickle=False) as f:
        X, w, cov = f["X"], f["w"], f["cov"]
        A_model, x0, lo, sc = f["A_model"], f["x0"], f["lo"], f["sc"]
        eps, sigma, p = float(f["eps"]), float(f["sigma"]), float(f["p"])
    A = ref.svd_factor(cov)
    fw = np.ones_like(x0)
    d = X.shape[1]
    rng = np.random.default_rng(seed)
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
    out_q.put((acc, evals, time.perf_counter() - t0))


def run(X, w, cov, A_model, x0, lo, sc, eps, sigma, p=2.0, workers=None,
        seconds=8.0, tmpdir="/tmp"):
    """Returns (accepted/s over all workers, workers, accepted, evaluations,
    wall seconds)."""
    if workers is None:
        workers = min(16, os.cpu_count() or 1)
    path = os.path.join(tmpdir, f"abc_cpu_baseline_{os.getpid()}.npz")
    np.savez(path, X=X, w=w, cov=cov, A_model=A_model, x0=x0, lo=lo, sc=sc,
             eps=eps, sigma=sigma, p=p)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(path, seconds, 1000 + i, q))
             for i in range(workers)]
    t0 = time.perf_counter()
    for pr in procs:
        pr.start()
    res = [q.get() for _ in procs]
    for pr in procs:
        pr.join()
    wall = time.perf_counter() - t0
    os.remove(path)
    acc = sum(r[0] for r in res)
    ev = sum(r[1] for r in res)
    rate = sum(r[0] / r[2] for r in res)
    return rate, workers, acc, ev, wall
