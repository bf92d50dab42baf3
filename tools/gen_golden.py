"""Generate golden input/output vectors from the reference (THIS container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [--only NAME ...]

Imports pyabc 0.10.1 from /root/reference through ``tools/ref_stub.py`` and
writes small ``.npz`` fixtures under ``tests/golden/``.  Only arrays (inputs and
the reference's outputs) are written; no reference source travels.  The GPU box
never runs this script: the committed fixtures are what the tests read there.

Every fixture records the call site it pins (reference file:line) in the
``_ref`` string entry.
"""
import argparse
import os
import sys
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(__file__))
import ref_stub  # noqa: E402

pyabc = ref_stub.import_pyabc()
from pyabc.transition import (MultivariateNormalTransition,  # noqa: E402
                              LocalTransition)
from pyabc.distance import (PNormDistance, AdaptivePNormDistance,  # noqa: E402
                            median_absolute_deviation, standard_deviation)
from pyabc.weighted_statistics import weighted_quantile  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))), "tests", "golden")


def pnames(d):
    # zero-padded so pandas' name-sorted columns equal the natural order
    # (history.py:307 pivots -> columns sorted by name)
    return [f"p{k:02d}" for k in range(d)]


def save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    print(f"  wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


def make_population(rng, n, d, offset=3.0):
    """Correlated, offset population with non-uniform weights."""
    L = np.tril(rng.normal(size=(d, d)) * 0.3) + np.eye(d)
    X = rng.normal(size=(n, d)) @ L.T + offset * rng.uniform(-1, 1, size=d)
    w = rng.uniform(0.5, 1.5, size=n)
    w = w / w.sum()
    return X, w


# --------------------------------------------------------------------------
# (a1) + (a3): MVN fit and KDE transition density / importance weight
# --------------------------------------------------------------------------
def gen_kde():
    cases = [(4096, 1024, 8, 0), (2048, 512, 20, 1), (1024, 1024, 1, 2),
             (2048, 512, 4, 3), (1, 16, 3, 4), (2, 16, 2, 5)]
    for N, M, d, seed in cases:
        rng = np.random.default_rng(100 + seed)
        X, w = make_population(rng, N, d)
        cols = pnames(d)
        tr = MultivariateNormalTransition()
        df = pd.DataFrame(X, columns=cols)
        w_in = w.copy()
        tr.fit(df, w_in)                      # transitionmeta.py:9-20
        np.random.seed(1000 + seed)
        theta = tr.rvs(size=M).values         # multivariatenormal.py:87-95
        pd_df = tr.pdf(pd.DataFrame(theta, columns=cols))   # :102-125
        pd_df = np.atleast_1d(np.asarray(pd_df, dtype=float))
        # single-row Series path (smc.py:726-727) on a few rows
        k = min(8, M)
        pd_series = np.array([tr.pdf(pd.Series(dict(zip(cols, theta[i]))))
                              for i in range(k)])
        # prior U(-10, 20)^d (box containing the data); weight = prior/transition
        lo = np.full(d, -10.0)
        sc = np.full(d, 30.0)
        prior = pyabc.Distribution(**{c: pyabc.RV("uniform", lo[j], sc[j])
                                      for j, c in enumerate(cols)})
        prior_pd = np.array([prior.pdf(pd.Series(dict(zip(cols, th))))
                             for th in theta])
        weight = prior_pd / pd_df            # smc.py:776-792
        wsum = sum(weight)                   # population.py:127-128 (sequential)
        weight_norm = weight / wsum
        save(f"kde_N{N}_M{M}_d{d}",
             X=X, w=w, theta=theta, cov=tr.cov, transition_pd=pd_df,
             transition_pd_series=pd_series, prior_lo=lo, prior_scale=sc,
             prior_pd=prior_pd, weight=weight, weight_norm=weight_norm,
             _ref=np.array("pyabc/transition/multivariatenormal.py:67-125; "
                           "pyabc/smc.py:709-792; pyabc/population.py:120-142"))


# --------------------------------------------------------------------------
# (a2): resample + perturb + prior-support test
# --------------------------------------------------------------------------
def gen_resample():
    for N, d, B, seed in [(4096, 8, 3000, 0), (1000, 3, 2000, 1),
                          (50, 1, 500, 2), (2048, 20, 1000, 3)]:
        rng = np.random.default_rng(200 + seed)
        X, w = make_population(rng, N, d, offset=1.0)
        # make a few weights tiny / zero-ish to exercise the CDF plateaus
        w[:5] = 0.0
        w = w / w.sum()
        cols = pnames(d)
        tr = MultivariateNormalTransition(scaling=1.3)
        tr.fit(pd.DataFrame(X, columns=cols), w.copy())
        s = 5000 + seed
        np.random.seed(s)
        theta_batch = tr.rvs(size=B).values
        np.random.seed(s)
        u = np.random.random_sample(B)
        z = np.random.standard_normal((B, d))
        # scalar path: u then z(d) per call
        np.random.seed(s + 1)
        theta_single = np.array([np.asarray(tr.rvs(), dtype=float)
                                 for _ in range(8)])
        np.random.seed(s + 1)
        u_single, z_single = [], []
        for _ in range(8):
            u_single.append(np.random.random_sample())
            z_single.append(np.random.standard_normal(d))
        cdf = np.cumsum(tr.w)
        cdf /= cdf[-1]
        idx = cdf.searchsorted(u, side="right")
        # prior box: centred at the population mean, narrow enough that
        # a fraction of proposals falls outside; plus exact-boundary probes
        lo = X.mean(0) - 2.0 * X.std(0)
        sc = 4.0 * X.std(0)
        prior = pyabc.Distribution(**{c: pyabc.RV("uniform", lo[j], sc[j])
                                      for j, c in enumerate(cols)})
        probes = np.repeat(X.mean(0)[None, :], 4 * d, axis=0)
        for j in range(d):
            hi = lo[j] + sc[j]
            probes[4 * j + 0, j] = lo[j]
            probes[4 * j + 1, j] = np.nextafter(lo[j], -np.inf)
            probes[4 * j + 2, j] = hi
            probes[4 * j + 3, j] = np.nextafter(hi, np.inf)
        all_theta = np.concatenate([theta_batch, probes])
        in_support = np.array([
            prior.pdf(pd.Series(dict(zip(cols, th)))) > 0
            for th in all_theta])
        save(f"resample_N{N}_d{d}_B{B}",
             X=X, w=tr.w, cov=tr.cov, u=u, z=z, idx=idx,
             theta=theta_batch, u_single=np.array(u_single),
             z_single=np.array(z_single), theta_single=theta_single,
             prior_lo=lo, prior_scale=sc, probes=probes,
             in_support=in_support.astype(np.uint8),
             _ref=np.array("pyabc/transition/multivariatenormal.py:87-95; "
                           "pyabc/smc.py:629-645; "
                           "pyabc/random_variables.py:425-452"))


# --------------------------------------------------------------------------
# (a5) + (a6): p-norm distances, accept mask, adaptive MAD / std weights
# --------------------------------------------------------------------------
def gen_distance():
    rng = np.random.default_rng(300)
    S = 100
    keys = [f"s{k:03d}" for k in range(S)]
    order = rng.permutation(S)           # x_0 insertion order != sorted
    keys = [keys[k] for k in order]
    x0 = {k: float(v) for k, v in zip(keys, rng.normal(size=S))}
    for n_rec, tag in [(1000, "even"), (999, "odd")]:
        scale = np.exp(rng.normal(size=S))
        data = rng.normal(size=(n_rec, S)) * scale + rng.normal(size=S)
        # a constant column -> isclose(scale, 0) -> weight 0 (distance.py:272)
        data[:, 7] = 1.25
        recs = [dict(zip(keys, row)) for row in data]
        out = {}
        for name, sf in [("mad", median_absolute_deviation),
                         ("std", None)]:
            dist = AdaptivePNormDistance(p=2, scale_function=sf)
            dist.initialize(0, lambda: recs, x0)   # distance.py:216-235
            out["w_" + name] = np.array([dist.weights[0][k] for k in keys])
        save(f"adaptive_{tag}_n{n_rec}_S{S}", data=data,
             x0=np.array([x0[k] for k in keys]), **out,
             _ref=np.array("pyabc/distance/distance.py:216-338; "
                           "pyabc/distance/scale.py:38-65"))
    # distances for B particles under several p, with adaptive weights
    B = 1500
    data = rng.normal(size=(B, S)) * 1.5 + np.array(list(x0.values()))
    recs = [dict(zip(keys, row)) for row in data]
    dist = AdaptivePNormDistance(p=2, scale_function=median_absolute_deviation)
    dist.initialize(0, lambda: recs[:1000], x0)
    wvec = np.array([dist.weights[0][k] for k in keys])
    res = {"stats": data, "x0": np.array([x0[k] for k in keys]),
           "fw": wvec}
    for p in [1, 2, 3, np.inf]:
        dp = PNormDistance(p=p, weights={0: dist.weights[0]})
        dp.initialize(0, lambda: recs, x0)
        dvals = np.array([dp(r, x0, 0) for r in recs])   # distance.py:76-102
        tag = "inf" if p == np.inf else str(p)
        res["d_p" + tag] = dvals
    eps = weighted_quantile(res["d_p2"], np.ones(B) / B, alpha=0.5)
    res["eps_p2"] = np.array(eps)
    res["accept_p2"] = (res["d_p2"] <= eps).astype(np.uint8)  # acceptor.py:241
    # python-pow semantics check: how often pow(a,2) != a*a here
    save(f"pnorm_B{B}_S{S}", **res,
         _ref=np.array("pyabc/distance/distance.py:76-102; "
                       "pyabc/acceptor/acceptor.py:235-244"))


# --------------------------------------------------------------------------
# (a7): weighted quantile epsilon
# --------------------------------------------------------------------------
def gen_quantile():
    rng = np.random.default_rng(400)
    res = {}
    alphas = np.array([0.1, 0.5, 0.9, 1.0, 0.25, 0.01])
    for N in [3, 4, 1000, 100000]:
        d = np.abs(rng.normal(size=N)) * 3 + rng.uniform(0, 1e-3, size=N)
        assert len(np.unique(d)) == N
        w = rng.uniform(0.1, 2.0, size=N)
        w = w / w.sum()
        q = np.array([weighted_quantile(d, w, alpha=a) for a in alphas])
        qu = np.array([weighted_quantile(d, None, alpha=a) for a in alphas])
        res[f"d_{N}"] = d
        res[f"w_{N}"] = w
        res[f"q_{N}"] = q
        res[f"qu_{N}"] = qu
    # QuantileEpsilon semantics incl. multiplier (epsilon.py:202-228)
    eps = pyabc.QuantileEpsilon(alpha=0.5, quantile_multiplier=1.1,
                                weighted=True)
    df = pd.DataFrame({"distance": res["d_1000"], "w": res["w_1000"] * 7.0})
    eps.initialize(0, lambda: df, lambda: None, None, None)
    res["eps_mult"] = np.array(eps(0))
    save("quantile", alphas=alphas, **res,
         _ref=np.array("pyabc/weighted_statistics.py:26-43; "
                       "pyabc/epsilon/epsilon.py:138-228"))


# --------------------------------------------------------------------------
# (a8): LocalTransition kNN covariances and density
# --------------------------------------------------------------------------
def gen_local():
    for N, d, k, seed in [(2000, 6, 50, 0), (300, 3, 10, 1), (500, 2, 20, 2)]:
        rng = np.random.default_rng(500 + seed)
        X = rng.normal(size=(N, d)) * rng.uniform(0.5, 2.0, size=d)
        w = rng.uniform(0.0, 1.0, size=N)
        w = w / w.sum()
        cols = pnames(d)
        tr = LocalTransition(k=k, k_fraction=None, scaling=1.0)
        t0 = time.time()
        tr.fit(pd.DataFrame(X, columns=cols), w.copy())   # :77-96
        from scipy.spatial import cKDTree
        _, nbr = cKDTree(X).query(X, k=min(tr.k + 1, N))
        pts = X[rng.integers(0, N, 64)] + rng.normal(size=(64, d)) * 0.2
        pdf = tr.pdf(pd.DataFrame(pts, columns=cols))     # :98-110
        save(f"local_N{N}_d{d}_k{k}", X=X, w=w, k=np.array(tr.k),
             nbr=np.sort(nbr[:, 1:], axis=1).astype(np.int32),
             covs=tr.covs, inv_covs=tr.inv_covs, dets=tr.determinants,
             pts=pts, pdf=np.asarray(pdf, dtype=float),
             _ref=np.array("pyabc/transition/local_transition.py:50-145"))
        print(f"    local fit {time.time() - t0:.2f}s")


def gen_local_rvs():
    """LocalTransition.rvs_single (local_transition.py:141-145): B calls
    after np.random.seed; the uniforms and normals each call consumes
    (choice: one random_sample; multivariate_normal: standard_normal(d)) are
    replayed from the same seed and stored with the outputs."""
    for N, d, k, seed, B in [(2000, 6, 50, 0, 400), (300, 3, 10, 1, 200)]:
        rng = np.random.default_rng(700 + seed)
        X = rng.normal(size=(N, d)) * rng.uniform(0.5, 2.0, size=d)
        w = rng.uniform(0.0, 1.0, size=N)
        w = w / w.sum()
        cols = pnames(d)
        tr = LocalTransition(k=k, k_fraction=None, scaling=1.0)
        tr.fit(pd.DataFrame(X, columns=cols), w.copy())
        np.random.seed(4242 + seed)
        theta = np.array([tr.rvs_single().values for _ in range(B)])
        rs = np.random.RandomState(4242 + seed)
        u = np.empty(B)
        z = np.empty((B, d))
        for b in range(B):
            u[b] = rs.random_sample()
            z[b] = rs.standard_normal(d)
        cdf = np.cumsum(tr.w)
        cdf /= cdf[-1]
        idx = cdf.searchsorted(u, side="right")
        # replay check: the reference's own factor (svd of C_idx)
        rep = np.empty_like(theta)
        for b in range(B):
            _, s, v = np.linalg.svd(tr.covs[idx[b]])
            rep[b] = z[b] @ (np.sqrt(s)[:, None] * v) + X[idx[b]]
        assert np.array_equal(rep, theta), np.abs(rep - theta).max()
        save(f"local_rvs_N{N}_d{d}_k{k}", X=X, w=w, k=np.array(tr.k),
             covs=tr.covs, u=u, z=z, idx=idx.astype(np.int64), theta=theta,
             _ref=np.array("pyabc/transition/local_transition.py:141-145 "
                           "(np.random.choice + multivariate_normal)"))


GENS = {"kde": gen_kde, "resample": gen_resample, "distance": gen_distance,
        "quantile": gen_quantile, "local": gen_local,
        "local_rvs": gen_local_rvs}

def _main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    args = ap.parse_args()
    for name, fn in GENS.items():
        if args.only and name not in args.only:
            continue
        print(f"[{name}]")
        fn()


# --------------------------------------------------------------------------
# end-to-end statistics (Monte-Carlo pins): reference runs over seeds
# --------------------------------------------------------------------------
def _run_stats(history, names):
    out = []
    for t in range(history.max_t + 1):
        df, w = history.get_distribution(m=0, t=t)
        X = df[names].values
        w = w / w.sum()
        mean = (X * w[:, None]).sum(0)
        std = np.sqrt(((X - mean) ** 2 * w[:, None]).sum(0))
        ess = 1.0 / np.sum(w ** 2)
        out.append((mean, std, ess))
    pops = history.get_all_populations()
    eps = pops[pops.t >= 0].epsilon.values
    nsim = pops[pops.t >= 0].samples.values
    return out, eps, nsim


def gen_e2e():
    from pyabc.sampler import SingleCoreSampler
    # C1: quickstart Gaussian mean (doc/examples/parameter_inference.ipynb)
    res = {}
    R, T = 5, 4
    for r in range(R):
        np.random.seed(100 + r)

        def model(parameter):
            return {"data": parameter["mean"] + 0.5 * np.random.randn()}
        prior = pyabc.Distribution(mean=pyabc.RV("uniform", 0, 5))
        abc = pyabc.ABCSMC(model, prior, PNormDistance(p=2),
                           population_size=1000,
                           eps=pyabc.MedianEpsilon(),
                           sampler=SingleCoreSampler())
        abc.new("sqlite://", {"data": 2.5})
        h = abc.run(minimum_epsilon=0.1, max_nr_populations=T)
        st, eps, nsim = _run_stats(h, ["mean"])
        res[f"c1_mean_{r}"] = np.array([s[0] for s in st])
        res[f"c1_std_{r}"] = np.array([s[1] for s in st])
        res[f"c1_ess_{r}"] = np.array([s[2] for s in st])
        res[f"c1_eps_{r}"] = eps
        res[f"c1_nsim_{r}"] = nsim
        print(f"    c1 seed {r}: eps {eps} mean {st[-1][0]}")
    # C2 (reduced N): 4-param linear Gaussian, S=100, AdaptivePNorm(MAD)
    d, S = 4, 100
    A = np.random.RandomState(42).randn(S, d) / 2
    th_true = np.array([0.5, -1.0, 1.5, 0.0])
    x0v = A @ th_true + 0.5 * np.random.RandomState(7).randn(S)
    keys = [f"y{k:03d}" for k in range(S)]
    names = [f"p{k}" for k in range(d)]
    x0 = dict(zip(keys, x0v))
    for r in range(3):
        np.random.seed(200 + r)

        def model2(par):
            th = np.array([par[n] for n in names])
            y = A @ th + 0.5 * np.random.randn(S)
            return dict(zip(keys, y))
        prior = pyabc.Distribution(**{n: pyabc.RV("uniform", -5, 10)
                                      for n in names})
        abc = pyabc.ABCSMC(
            model2, prior,
            AdaptivePNormDistance(p=2,
                                  scale_function=median_absolute_deviation),
            population_size=1000, eps=pyabc.QuantileEpsilon(alpha=0.5),
            sampler=SingleCoreSampler())
        abc.new("sqlite://", x0)
        h = abc.run(max_nr_populations=4)
        st, eps, nsim = _run_stats(h, names)
        res[f"c2_mean_{r}"] = np.array([s[0] for s in st])
        res[f"c2_std_{r}"] = np.array([s[1] for s in st])
        res[f"c2_eps_{r}"] = eps
        res[f"c2_nsim_{r}"] = nsim
        print(f"    c2 seed {r}: eps {eps} mean {st[-1][0]}")
    save("e2e_stats", A2=A, x0_2=x0v, theta_true_2=th_true, **res,
         _ref=np.array("pyabc/smc.py:796-1022 (ABCSMC.run) with "
                       "SingleCoreSampler; C1 doc/examples/"
                       "parameter_inference.ipynb; C2 SURVEY 8(d)"))


GENS["e2e"] = gen_e2e


# --------------------------------------------------------------------------
# (f3) exact inference: stochastic kernels, acceptor, temperature schemes
# --------------------------------------------------------------------------
def gen_stochastic():
    from pyabc.distance import (IndependentNormalKernel,
                                IndependentLaplaceKernel, NormalKernel,
                                SimpleFunctionKernel, SCALE_LIN, SCALE_LOG)
    from pyabc.acceptor import StochasticAcceptor, pdf_norm_from_kernel
    rng = np.random.default_rng(31)
    for S, B in [(100, 400), (300, 120), (5, 200)]:
        keys = [f"s{k:03d}" for k in range(S)]
        x0v = rng.normal(size=S)
        X = x0v[None, :] + rng.normal(size=(B, S)) * rng.uniform(0.2, 3, S)
        var = rng.uniform(0.1, 4.0, S)
        scale = rng.uniform(0.1, 4.0, S)
        x0 = dict(zip(keys, x0v))
        kn = IndependentNormalKernel(var=var)
        kn.initialize(0, None, x0)
        kl = IndependentLaplaceKernel(scale=scale)
        kl.initialize(0, None, x0)
        rows = [dict(zip(keys, r)) for r in X]
        ln = np.array([kn(x, x0) for x in rows])
        ll = np.array([kl(x, x0) for x in rows])
        save(f"stoch_kernel_S{S}", X=X, x0=x0v, var=var, scale=scale,
             normal=ln, laplace=ll, normal_pdf_max=kn.pdf_max,
             laplace_pdf_max=kl.pdf_max,
             _ref=np.array("distance/kernel.py:256-282 "
                           "(IndependentNormalKernel), :332-357 "
                           "(IndependentLaplaceKernel); keys sorted"))
    # NormalKernel (full covariance, scipy multivariate_normal), S=6
    S, B = 6, 200
    keys = [f"s{k}" for k in range(S)]
    L = np.tril(rng.normal(size=(S, S))) + 2 * np.eye(S)
    cov = L @ L.T
    x0v = rng.normal(size=S)
    X = x0v[None, :] + rng.normal(size=(B, S)) * 2
    x0 = dict(zip(keys, x0v))
    out = {}
    for scale_name in ["log", "lin"]:
        k = NormalKernel(cov=cov, ret_scale=SCALE_LOG if scale_name == "log"
                         else SCALE_LIN)
        k.initialize(0, None, x0)
        out[f"normal_full_{scale_name}"] = np.array(
            [k(dict(zip(keys, r)), x0) for r in X])
        out[f"pdf_max_{scale_name}"] = k.pdf_max
    save("stoch_kernel_full", X=X, x0=x0v, cov=cov, **out,
         _ref=np.array("distance/kernel.py:108-187 (NormalKernel)"))
    # StochasticAcceptor.__call__ on given densities, both scales
    B = 3000
    res = {}
    for scale_name, sc in [("log", SCALE_LOG), ("lin", SCALE_LIN)]:
        if scale_name == "log":
            pdv = rng.normal(-5, 3, size=B)
            pdf_max = -1.0
        else:
            pdv = np.exp(rng.normal(-2, 1.5, size=B))
            pdf_max = 0.4
        kern = SimpleFunctionKernel(lambda x, x_0, t, par: x["pd"],
                                    ret_scale=sc, pdf_max=pdf_max)
        for temp in [1.0, 3.7]:
            for iw in [True, False]:
                acc = StochasticAcceptor(pdf_norm_method=pdf_norm_from_kernel,
                                         apply_importance_weighting=iw)
                acc.initialize(0, lambda: None, kern, {})
                np.random.seed(77)
                r = [acc(kern, lambda t: temp, {"pd": p}, {}, 0, None)
                     for p in pdv]
                np.random.seed(77)
                u = np.random.uniform(0, 1, size=B)
                tag = f"{scale_name}_T{temp}_iw{int(iw)}"
                res[f"accept_{tag}"] = np.array([x.accept for x in r])
                res[f"weight_{tag}"] = np.array([x.weight for x in r])
                res[f"u_{tag}"] = u
        res[f"pd_{scale_name}"] = pdv
        res[f"pdf_max_{scale_name}"] = pdf_max
    save("stoch_accept", **res,
         _ref=np.array("acceptor/acceptor.py:440-473 "
                       "(StochasticAcceptor.__call__), pdf_norm.py:6-14"))


def gen_temperature():
    import pyabc.epsilon as E
    from pyabc.distance import SCALE_LOG, SCALE_LIN
    from pyabc.acceptor import pdf_norm_max_found, ScaledPDFNorm
    rng = np.random.default_rng(41)
    n = 5000
    pds = rng.normal(-20, 6, size=n)
    tpp = np.exp(rng.normal(0, 1, size=n))
    tp = tpp * np.exp(rng.normal(0, 0.3, size=n))
    acc_flag = rng.random(n) < 0.3
    records = [dict(distance=a, transition_pd_prev=b, transition_pd=c,
                    accepted=bool(f)) for a, b, c, f in
               zip(pds, tpp, tp, acc_flag)]
    wd = pd.DataFrame({"distance": pds[:2000],
                       "w": rng.uniform(0.2, 1.0, 2000)})
    out = dict(pds=pds, tpp=tpp, tp=tp, wd_d=wd.distance.values,
               wd_w=wd.w.values)
    pdf_norm = float(np.max(pds))
    for rate in [0.3, 0.05, 0.9]:
        for sc in ["log", "lin"]:
            if sc == "log":
                args = dict(pdf_norm=pdf_norm, kernel_scale=SCALE_LOG)
                recs = records
            else:
                lin = np.exp(pds / 10)
                recs = [dict(r, distance=v) for r, v in zip(records, lin)]
                args = dict(pdf_norm=float(lin.max()), kernel_scale=SCALE_LIN)
            s = E.AcceptanceRateScheme(target_rate=rate)
            out[f"accrate_{rate}_{sc}"] = s(
                t=1, get_weighted_distances=lambda: wd,
                get_all_records=lambda: recs, max_nr_populations=10,
                prev_temperature=50., acceptance_rate=0.3, **args)
    # obj(0) > 0 (T = 1) and the numerics-limit branch
    s = E.AcceptanceRateScheme(target_rate=0.3)
    out["accrate_norm_min"] = s(
        t=1, get_weighted_distances=lambda: wd,
        get_all_records=lambda: records, max_nr_populations=10,
        pdf_norm=float(np.min(pds)), kernel_scale=SCALE_LOG,
        prev_temperature=50., acceptance_rate=0.3)
    base = dict(get_weighted_distances=lambda: wd,
                get_all_records=lambda: records, pdf_norm=pdf_norm,
                kernel_scale=SCALE_LOG)
    for t, prev, rate in [(1, 50., 0.4), (3, 12.5, 1e-5), (2, 7.3, 0.7)]:
        for name, sch in [("expiter", E.ExpDecayFixedIterScheme()),
                          ("expratio", E.ExpDecayFixedRatioScheme()),
                          ("poly", E.PolynomialDecayFixedIterScheme()),
                          ("daly", E.DalyScheme()),
                          ("friel", E.FrielPettittScheme()),
                          ("ess", E.EssScheme())]:
            out[f"{name}_t{t}"] = sch(t=t, max_nr_populations=6,
                                      prev_temperature=prev,
                                      acceptance_rate=rate, **base)
    # a full Temperature sequence (default schemes) over 5 generations
    temp = E.Temperature()
    cfg = dict(pdf_norm=pdf_norm, kernel_scale=SCALE_LOG)
    temp.initialize(0, lambda: wd, lambda: records, 5, cfg)
    seq = [temp(0)]
    for t, rate in zip(range(1, 5), [0.5, 0.2, 0.1, 0.05]):
        temp.update(t, lambda: wd, lambda: records, rate, cfg)
        seq.append(temp(t))
    out["temperature_seq"] = np.array(seq)
    # pdf norms
    out["pdfnorm_maxfound"] = pdf_norm_max_found(
        prev_pdf_norm=-3.0, get_weighted_distances=lambda: wd)
    sp_ = ScaledPDFNorm()
    out["pdfnorm_scaled_hi"] = sp_(prev_pdf_norm=-30.0,
                                   get_weighted_distances=lambda: wd,
                                   prev_temp=5.0, acceptance_rate=0.5)
    out["pdfnorm_scaled_lo"] = sp_(prev_pdf_norm=-30.0,
                                   get_weighted_distances=lambda: wd,
                                   prev_temp=5.0, acceptance_rate=0.01)
    save("temperature", **out,
         _ref=np.array("epsilon/temperature.py:45-742, "
                       "acceptor/pdf_norm.py:17-110"))


GENS["stochastic"] = gen_stochastic
GENS["temperature"] = gen_temperature


def gen_e2e_stochastic():
    """Exact-inference run: noise-free linear model y = A theta, Gaussian
    likelihood via IndependentNormalKernel(var), StochasticAcceptor,
    Temperature (smc.py:796-1022 with acceptor/acceptor.py:309-473,
    epsilon/temperature.py:45-345)."""
    from pyabc.sampler import SingleCoreSampler
    from pyabc.distance import IndependentNormalKernel
    from pyabc.acceptor import StochasticAcceptor
    from pyabc.epsilon import Temperature
    d, S, var = 2, 10, 0.25
    A = np.random.RandomState(11).randn(S, d)
    th_true = np.array([0.8, -0.4])
    x0v = A @ th_true + np.sqrt(var) * np.random.RandomState(12).randn(S)
    keys = [f"y{k:02d}" for k in range(S)]
    names = [f"p{k}" for k in range(d)]
    x0 = dict(zip(keys, x0v))
    res = {}
    for r in range(3):
        np.random.seed(300 + r)

        def model(par):
            th = np.array([par[n] for n in names])
            return dict(zip(keys, A @ th))
        prior = pyabc.Distribution(**{n: pyabc.RV("uniform", -5, 10)
                                      for n in names})
        abc = pyabc.ABCSMC(model, prior, IndependentNormalKernel(var=var),
                           population_size=1000, eps=Temperature(),
                           acceptor=StochasticAcceptor(),
                           sampler=SingleCoreSampler())
        abc.new("sqlite://", x0)
        h = abc.run(max_nr_populations=6)
        st, eps, nsim = _run_stats(h, names)
        res[f"mean_{r}"] = np.array([s_[0] for s_ in st])
        res[f"std_{r}"] = np.array([s_[1] for s_ in st])
        res[f"ess_{r}"] = np.array([s_[2] for s_ in st])
        res[f"temp_{r}"] = eps
        res[f"nsim_{r}"] = nsim
        print(f"    seed {r}: T {eps} mean {st[-1][0]} std {st[-1][1]}")
    save("e2e_stochastic", A=A, x0=x0v, var=var, theta_true=th_true, **res,
         _ref=np.array("pyabc/smc.py:796-1022 with StochasticAcceptor + "
                       "Temperature + IndependentNormalKernel, "
                       "SingleCoreSampler"))


GENS["e2e_stochastic"] = gen_e2e_stochastic


def gen_cv():
    """AdaptivePopulationSize pieces (populationstrategy.py:318-345):
    bootstrap KDE fit (fit_cov, multivariatenormal.py:67-73) + pdf_static
    (:114-126) at the test points, cv/bootstrap.py calc_variation (:12-32)
    and cv/powerlaw.py fitpowerlaw (:13-18)."""
    from pyabc.cv.bootstrap import calc_variation
    from pyabc.cv.powerlaw import fitpowerlaw
    rng = np.random.default_rng(41)
    d, N, n, B = 3, 500, 200, 5
    test_X = np.asarray(make_population(rng, N, d)[0])
    test_w = rng.uniform(0.5, 1.5, N)
    test_w /= test_w.sum()
    tr = MultivariateNormalTransition(scaling=1)
    boots = np.stack([test_X[rng.integers(0, N, n)]
                      + 0.3 * rng.normal(size=(n, d)) for _ in range(B)])
    w0 = np.ones(n) / n
    dens, covs = [], []
    for b in range(B):
        cov = tr.fit_cov(boots[b], w0)
        covs.append(cov)
        dens.append(tr.pdf_static(test_X, boots[b], cov, w0))
    dens = np.stack(dens)
    cv = calc_variation([dens], np.array([n]), test_w[None, :])
    # a second model with a different share
    dens2 = dens[::-1] * rng.uniform(0.9, 1.1, dens.shape)
    cv2 = calc_variation([dens, dens2], np.array([n, 3 * n]),
                         np.vstack([test_w, test_w[::-1]]))
    xs = np.arange(100, 2000, 190)
    ys = 0.8 * xs ** -0.45 * (1 + 0.01 * np.sin(xs))
    popt, _, finv = fitpowerlaw(xs, ys)
    save("cv_bootstrap", test_X=test_X, test_w=test_w, boots=boots,
         covs=np.stack(covs), dens=dens, cv=np.float64(cv), dens2=dens2,
         cv2=np.float64(cv2), xs=xs, ys=ys, popt=popt,
         n_at_005=np.float64(finv(0.05)),
         _ref="pyabc/populationstrategy.py:318-345, "
              "transition/multivariatenormal.py:67-73,114-126, "
              "cv/bootstrap.py:12-32, cv/powerlaw.py:13-18")


GENS["cv"] = gen_cv


def gen_vis():
    """visualization/kde.py:19-75 kde_1d and :173-247 kde_2d."""
    from pyabc.visualization.kde import kde_1d, kde_2d
    rng = np.random.default_rng(43)
    N = 800
    df = pd.DataFrame({"a": rng.normal(1, 0.5, N),
                       "b": rng.gamma(2.0, 1.0, N)})
    w = rng.uniform(0.2, 1.0, N)
    w /= w.sum()
    x1, pdf1 = kde_1d(df, w, "a", numx=40)
    x1l, pdf1l = kde_1d(df, w, "b", xmin=-1, xmax=9, numx=33)
    X, Y, PDF = kde_2d(df, w, "a", "b", numx=20, numy=15)
    save("vis_kde", a=df["a"].values, b=df["b"].values, w=w, x1=x1,
         pdf1=pdf1, x1l=x1l, pdf1l=pdf1l, X=X, Y=Y, PDF=PDF,
         _ref="pyabc/visualization/kde.py:19-75, 173-247")


GENS["vis"] = gen_vis


C5_D, C5_S, C5_N, C5_T, C5_R = 20, 100, 10_000, 4, 5


def _c5_problem():
    """y = A theta + 0.5 eps, A = RandomState(42).randn(100,
    20)/sqrt(20), theta_true = linspace(-1, 1, 20), x0 from RandomState(7)."""
    A = np.random.RandomState(42).randn(C5_S, C5_D) / np.sqrt(C5_D)
    th_true = np.linspace(-1, 1, C5_D)
    x0v = A @ th_true + 0.5 * np.random.RandomState(7).randn(C5_S)
    return A, th_true, x0v


def _c5_seed(r):
    A, th_true, x0v = _c5_problem()
    keys = [f"y{k:03d}" for k in range(C5_S)]
    names = pnames(C5_D)
    x0 = dict(zip(keys, x0v))
    np.random.seed(500 + r)

    def model(par):
        th = np.array([par[n] for n in names])
        return dict(zip(keys, A @ th + 0.5 * np.random.randn(C5_S)))
    from pyabc.sampler import SingleCoreSampler
    prior = pyabc.Distribution(**{n: pyabc.RV("uniform", -5, 10)
                                  for n in names})
    abc = pyabc.ABCSMC(model, prior, PNormDistance(p=2),
                       population_size=C5_N,
                       eps=pyabc.QuantileEpsilon(alpha=0.5),
                       sampler=SingleCoreSampler())
    abc.new("sqlite://", x0)
    abc.history.stores_sum_stats = False      # storage only; not the algorithm
    t0 = time.time()
    h = abc.run(max_nr_populations=C5_T)
    st, eps, nsim = _run_stats(h, names)
    print(f"    c5 seed {r}: {time.time() - t0:.0f} s eps {eps}", flush=True)
    return r, st, eps, nsim


def gen_e2e_c5():
    """C5 at reduced N (SURVEY 8(c) 'a d=20 variant at N=1e4'): 20-param
    linear Gaussian, S=100, PNormDistance(p=2), QuantileEpsilon(0.5),
    SingleCoreSampler, R seeds in parallel processes."""
    import multiprocessing as mp
    with mp.get_context("fork").Pool(C5_R) as pool:
        outs = pool.map(_c5_seed, range(C5_R))
    A, th_true, x0v = _c5_problem()
    res = {}
    for r, st, eps, nsim in outs:
        res[f"c5_mean_{r}"] = np.array([s[0] for s in st])
        res[f"c5_std_{r}"] = np.array([s[1] for s in st])
        res[f"c5_ess_{r}"] = np.array([s[2] for s in st])
        res[f"c5_eps_{r}"] = eps
        res[f"c5_nsim_{r}"] = nsim
    save("e2e_c5", A=A, x0=x0v, theta_true=th_true, N=np.array(C5_N),
         T=np.array(C5_T), R=np.array(C5_R), **res,
         _ref=np.array("pyabc/smc.py:796-1022 (ABCSMC.run), "
                       "SingleCoreSampler, PNormDistance(p=2), "
                       "QuantileEpsilon(alpha=0.5); SURVEY 8(d) C5 at "
                       "N=1e4"))


GENS["e2e_c5"] = gen_e2e_c5


if __name__ == "__main__":
    _main()
