"""Fixture generator for the a9 parity pin (runs in THIS container only).

The reference's own generation closure -- ``ABCSMC._create_simulate_function``
(``pyabc/smc.py:543-598``: ``_generate_valid_proposal`` ``:602-645`` with the
prior support test, ``_evaluate_proposal`` ``:647-705``, the weight function
``:750-794``) -- is driven by the reference's ``SingleCoreSampler``
(``pyabc/sampler/singlecore.py:19-38``) over the DEVICE's random numbers:

* the transition's ``rvs`` returns the device proposal sequence raw id by raw
  id: resample index and perturbation from Philox counters ``p`` of streams
  ``2*sid`` / ``2*sid + 1`` (``sid = 8 t``), restated by the oracle;
* the model's ``sample`` returns ``A theta + c + sigma z_e`` with the noise of
  evaluation ``e`` (Philox stream ``2*(8 t + 1)``), again the oracle's
  restatement of the device simulator;
* everything else -- the prior support test, evaluation counting, the
  distance, the acceptance, the weights, the Sample bookkeeping with
  ``record_rejected`` and ``check_max_eval`` -- is the reference's code.

The GPU test (``tests/test_gpu_api.py::test_singlecore_parity_same_draws``)
runs the device engine with the same seed and checks the population, its
order, ``nr_evaluations_``, the recorded evaluations and the max_eval cut.
epsilon is placed in a wide gap of the distances so the oracle's fp32-noise
restatement (a few fp32 ulps from the device's) cannot flip a decision.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_singlecore_replay.py
"""
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ref_stub  # noqa: E402

pyabc = ref_stub.import_pyabc()
from pyabc.sampler import SingleCoreSampler  # noqa: E402
from oracle import ref_cpu as ref  # noqa: E402

SEED, T = 20240611, 1
D, S, N_PREV, N = 3, 6, 400, 150
P_RAW = 6000


def problem():
    rng = np.random.default_rng(91)
    X = rng.normal(size=(N_PREV, D)) * 0.8 + np.array([0.5, -0.3, 1.2])
    w = rng.uniform(0.5, 1.5, N_PREV)
    w /= w.sum()
    lo = np.array([-2.0, -2.0, -1.0])
    sc = np.array([4.0, 4.0, 3.0])
    A = rng.normal(size=(S, D))
    c = rng.normal(size=S) * 0.1
    sigma = 0.5
    x0 = A @ np.array([0.4, -0.2, 1.0]) + c + sigma * rng.normal(size=S)
    return X, w, lo, sc, A, c, sigma, x0


def replay(X, w, cov, lo, sc, A, c, sigma):
    """The device's raw proposal sequence and the noise per evaluation."""
    sid = 8 * T
    u = ref.philox_uniform(SEED, 2 * sid, P_RAW)
    z = ref.philox_normal(SEED, 2 * sid + 1, P_RAW * D).reshape(P_RAW, D)
    idx, th = ref.resample_perturb(X, w, cov, u, z)
    sup = ref.uniform_box_support(th, lo, sc)
    E = int(sup.sum())
    noise = ref.philox_normal4_f32(SEED, 2 * (8 * T + 1), E * S).reshape(E, S)
    stats = th[sup] @ A.T + c + sigma * noise.astype(np.float64)
    return th, sup, stats


def run_reference(X, w, lo, sc, A, c, sigma, x0, eps, th, sup,
                  check_max_eval=False, max_eval=np.inf):
    names = [f"p{k:02d}" for k in range(D)]
    keys = [f"y{k:03d}" for k in range(S)]
    cnt = {"raw": 0, "eval": 0}
    valid = th[sup]

    def sample(par):
        e = cnt["eval"]
        cnt["eval"] += 1
        theta = np.array([par[nm] for nm in names])
        # the device restated: same theta (replayed), same noise
        np.testing.assert_allclose(theta, valid[e], rtol=0, atol=0)
        y = A @ theta + c + sigma * NOISE[e]
        return dict(zip(keys, y))

    prior = pyabc.Distribution(**{nm: pyabc.RV("uniform", lo[k], sc[k])
                                  for k, nm in enumerate(names)})
    abc = pyabc.ABCSMC(sample, prior, pyabc.PNormDistance(p=2),
                       population_size=N,
                       eps=pyabc.ConstantEpsilon(eps),
                       sampler=SingleCoreSampler(check_max_eval))
    abc.new("sqlite://", dict(zip(keys, x0)))
    tr = abc.transitions[0]
    tr.fit(pd.DataFrame(X, columns=names), w)

    def rvs(size=None):
        p = cnt["raw"]
        cnt["raw"] += 1
        return pd.Series(th[p], index=names)
    tr.rvs = rvs
    abc.history.get_model_probabilities = \
        lambda t=None: pd.DataFrame({"p": [1.0]}, index=[0])
    simulate_one = abc._create_simulate_function(T)
    sampler = abc.sampler
    sampler.sample_factory.record_rejected = True
    sample = sampler.sample_until_n_accepted(N, simulate_one, max_eval)
    return sample, sampler.nr_evaluations_, tr, names, keys


def main():
    global NOISE
    X, w, lo, sc, A, c, sigma, x0 = problem()
    # the transition's own covariance (the device refits it from X, w)
    names = [f"p{k:02d}" for k in range(D)]
    tr0 = pyabc.MultivariateNormalTransition()
    tr0.fit(pd.DataFrame(X, columns=names), w)
    th, sup, stats = replay(X, w, tr0.cov, lo, sc, A, c, sigma)
    E = stats.shape[0]
    sid = 8 * T
    NOISE = ref.philox_normal4_f32(SEED, 2 * (sid + 1), E * S).reshape(
        E, S).astype(np.float64)
    dist = np.sqrt(((stats - x0) ** 2).sum(1))
    # eps: the widest gap among the first evaluations near the 35 % quantile
    head = np.sort(dist[:1200])
    lo_i, hi_i = int(0.30 * len(head)), int(0.40 * len(head))
    gaps = np.diff(head[lo_i:hi_i])
    g = int(np.argmax(gaps))
    eps = 0.5 * (head[lo_i + g] + head[lo_i + g + 1])
    print(f"eps {eps:.6f}, gap {gaps[g]:.2e}, in-support "
          f"{sup[:2000].mean():.3f}")
    assert gaps[g] > 1e-4 * eps
    # no proposal within 1e-9 of the prior box (the device refits cov)
    rel = (th - lo) / sc
    assert np.min(np.abs(rel)) > 1e-9 and np.min(np.abs(rel - 1)) > 1e-9

    sample, nr_eval, tr, names, keys = run_reference(
        X, w, lo, sc, A, c, sigma, x0, eps, th, sup)
    pop = sample.get_accepted_population()
    parts = pop.get_list()
    theta_acc = np.array([[p.parameter[nm] for nm in names] for p in parts])
    d_acc = np.array([p.accepted_distances[0] for p in parts])
    w_acc = np.array([p.weight for p in parts])
    rec = np.array([[s[k] for k in keys] for s in sample.all_sum_stats])
    rec_acc = np.array([p.accepted for p in sample._particles])
    assert len(parts) == N and rec.shape[0] == nr_eval
    print(f"nr_evaluations_ {nr_eval}, accepted {len(parts)}")
    out = dict(X=X, w=w, lo=lo, sc=sc, A=A, c=c, sigma=sigma, x0=x0,
               eps=eps, seed=SEED, t=T, n=N, cov=tr.cov,
               theta=theta_acc, d=d_acc, weight=w_acc,
               nr_evaluations=nr_eval, rec_stats=rec, rec_acc=rec_acc)
    # check_max_eval: the cut at, just below and half below the n-th
    # acceptance's evaluation count (singlecore.py:24-35)
    cuts = np.array([nr_eval - 1, nr_eval - 0.5, nr_eval, nr_eval // 2])
    oks, nrs = [], []
    for me in cuts:
        s2, nr2, *_ = run_reference(X, w, lo, sc, A, c, sigma, x0, eps, th,
                                    sup, check_max_eval=True, max_eval=me)
        oks.append(bool(s2.ok))
        nrs.append(int(nr2))
        print(f"  max_eval {me}: ok {s2.ok}, nr_evaluations_ {nr2}")
    out.update(cut_max_eval=cuts, cut_ok=np.array(oks),
               cut_nr_evaluations=np.array(nrs))
    out["_ref"] = np.array(
        "pyabc/sampler/singlecore.py:19-38 driving ABCSMC."
        "_create_simulate_function (smc.py:543-705, weights :750-794) over "
        "the device's Philox proposals and simulator noise "
        "(tests/golden/gen_singlecore_replay.py)")
    path = os.path.join(HERE, "singlecore_replay.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


if __name__ == "__main__":
    main()
