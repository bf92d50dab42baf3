"""Exact-inference path on the MI355X, through the
C-ABI: stochastic kernel densities and acceptance against the reference's
golden vectors, the temperature schemes' device objectives, and end-to-end
StochasticAcceptor + Temperature runs against reference runs
(``tests/golden/e2e_stochastic.npz``) and the analytic posterior.

Tolerances: kernel log-densities bit-exact (numpy pairwise order restated);
accept masks bit-exact (guard band asserted empty); acceptance weights
<= 4 ulp (device exp vs numpy exp); temperatures from the AcceptanceRateScheme
<= 1e-9 relative (the reference's own bisection stops at xtol 2e-12 in log
beta), EssScheme <= 1e-4 relative (scipy L-BFGS-B tolerance on a
finite-difference gradient); posterior moments within Monte-Carlo error.
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch

from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pyabc_amd import kernels
    return kernels


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda")


def host(t):
    return t.detach().cpu().numpy()


def _const(kind, prm):
    if kind == 0:
        return float(np.sum(np.log(2) + np.log(np.pi) + np.log(prm)))
    return float(np.sum(np.log(2) + np.log(prm)))


# ------------------------------------------------------------ kernels
@pytest.mark.parametrize("S", [5, 100, 300])
def test_independent_kernels_bit_exact(K, S):
    g = load_golden(f"stoch_kernel_S{S}")
    stats_T = dev(g["X"].T)
    for kind, prm, want in [(0, g["var"], g["normal"]),
                            (1, g["scale"], g["laplace"])]:
        pd_, _, _, _ = K.stochastic_kernel(stats_T, dev(g["x0"]), dev(prm),
                                           kind, _const(kind, prm))
        np.testing.assert_array_equal(host(pd_), want)


def test_fused_acceptance_matches_reference(K):
    """Kernel density + acceptance in one launch with the reference's
    uniforms injected: same decisions and weights as
    StochasticAcceptor.__call__ on the same densities."""
    import pyabc_amd as pa
    g = load_golden("stoch_kernel_S100")
    rng = np.random.default_rng(3)
    B = g["X"].shape[0]
    u = rng.random(B)
    stats_T = dev(g["X"].T)
    c = _const(0, g["var"])
    norm = float(np.max(g["normal"])) - 3.0
    for temp in [1.0, 5.5]:
        pd_, acc, accw, guard = K.stochastic_kernel(
            stats_T, dev(g["x0"]), dev(g["var"]), 0, c, pdf_norm=norm,
            inv_temp=1 / temp, u=dev(u))
        assert host(guard).sum() == 0
        acc_prob = np.exp((g["normal"] - norm) * (1 / temp))
        np.testing.assert_array_equal(host(acc).astype(bool), acc_prob >= u)
        want = np.where(acc_prob == 0, 0.0, acc_prob / np.minimum(1, acc_prob))
        np.testing.assert_allclose(host(accw), want, rtol=4 * 2.0 ** -52)
        # the API class gives the same single-call density
        k = pa.IndependentNormalKernel(var=g["var"])
        x0 = {f"s{i:03d}": v for i, v in enumerate(g["x0"])}
        k.initialize(0, None, x0)
        x = {f"s{i:03d}": v for i, v in enumerate(g["X"][7])}
        assert k(x, x0) == g["normal"][7]


@pytest.mark.parametrize("scale", ["log", "lin"])
@pytest.mark.parametrize("temp", [1.0, 3.7])
@pytest.mark.parametrize("iw", [1, 0])
def test_stochastic_accept_golden(K, scale, temp, iw):
    g = load_golden("stoch_accept")
    tag = f"{scale}_T{temp}_iw{iw}"
    acc, accw, guard = K.stochastic_accept(
        dev(g["pd_" + scale]), float(g["pdf_max_" + scale]), 1 / temp,
        log_scale=scale == "log", apply_iw=bool(iw), u=dev(g["u_" + tag]))
    assert host(guard).sum() == 0
    np.testing.assert_array_equal(host(acc).astype(bool), g["accept_" + tag])
    np.testing.assert_allclose(host(accw), g["weight_" + tag],
                               rtol=4 * 2.0 ** -52)


def test_philox_uniforms_keyed_by_evaluation_id(K):
    """The production acceptance draws u from Philox counter (offset + b):
    one launch over [0, B) equals two launches over the halves."""
    rng = np.random.default_rng(9)
    pdv = dev(rng.normal(-3, 1, 5000))
    a1, w1, _ = K.stochastic_accept(pdv, -1.0, 1.0, seed=7, stream=40,
                                    offset=100)
    a2, _, _ = K.stochastic_accept(pdv[:2000], -1.0, 1.0, seed=7, stream=40,
                                   offset=100)
    a3, _, _ = K.stochastic_accept(pdv[2000:], -1.0, 1.0, seed=7, stream=40,
                                   offset=2100)
    np.testing.assert_array_equal(host(a1), np.concatenate([host(a2),
                                                            host(a3)]))
    from oracle import ref_cpu as ref
    u = ref.philox_uniform(7, 40, 5100)[100:]
    acc = np.exp(host(pdv) + 1.0) >= u
    np.testing.assert_array_equal(host(a1).astype(bool), acc)


def test_tempered_sums_vs_numpy(K):
    rng = np.random.default_rng(2)
    n = 100003
    pdv = rng.normal(-10, 4, n)
    lnum, lden = rng.normal(0, 1, n), rng.normal(0, 1, n)
    betas = [1e-3, 0.1, 0.5, 1.0]
    for log_scale in [True, False]:
        p = pdv if log_scale else np.exp(pdv / 8)
        c = float(p.max())
        out = host(K.tempered_sums(dev(p), c, betas, logw_num=dev(lnum),
                                   logw_den=dev(lden), log_scale=log_scale,
                                   clamp=True))
        w = np.exp(lnum - lden)
        np.testing.assert_allclose(out[0], [w.sum(), (w * w).sum()],
                                   rtol=1e-12)
        for k, b in enumerate(betas):
            v = np.exp((p - c) * b) if log_scale else (p / c) ** b
            v = np.minimum(v, 1)
            np.testing.assert_allclose(out[k + 1], [(w * v).sum(),
                                                    ((w * v) ** 2).sum()],
                                       rtol=1e-12)
    # deterministic: same bits on a second call
    a = host(K.tempered_sums(dev(pdv), -1.0, [0.3], w=dev(np.exp(lnum))))
    b = host(K.tempered_sums(dev(pdv), -1.0, [0.3], w=dev(np.exp(lnum))))
    np.testing.assert_array_equal(a, b)


# ------------------------------------------------------------ schemes
def _records(g, lin=False):
    d = np.exp(g["pds"] / 10) if lin else g["pds"]
    return [dict(distance=a, transition_pd_prev=b, transition_pd=c,
                 accepted=True) for a, b, c in zip(d, g["tpp"], g["tp"])]


@pytest.mark.parametrize("rate", [0.3, 0.05, 0.9])
def test_acceptance_rate_scheme_matches_reference(K, rate):
    import pyabc_amd as pa
    from pyabc_amd.temperature import DeviceRecords
    g = load_golden("temperature")
    for sc in ["log", "lin"]:
        recs = _records(g, lin=sc == "lin")
        norm = float(max(r["distance"] for r in recs))
        s = pa.AcceptanceRateScheme(target_rate=rate)
        args = dict(t=1, get_weighted_distances=None, max_nr_populations=10,
                    pdf_norm=norm, kernel_scale=pa.SCALE_LOG if sc == "log"
                    else pa.SCALE_LIN, prev_temperature=50.,
                    acceptance_rate=0.3)
        got = s(get_all_records=lambda: recs, **args)
        want = float(g[f"accrate_{rate}_{sc}"])
        assert abs(got / want - 1) <= 1e-9, (sc, got, want)
        # device records (log transition densities) give the same value
        drec = DeviceRecords(dev([r["distance"] for r in recs]),
                             dev(np.log(g["tpp"])), dev(np.log(g["tp"])),
                             dev(np.ones(len(recs))))
        got2 = s(get_all_records=lambda: drec, **args)
        assert abs(got2 / want - 1) <= 1e-9, (sc, got2, want)


def test_acceptance_rate_scheme_limits(K):
    """obj(0) > 0 gives T = 1 (test/test_epsilon.py:135-147)."""
    import pyabc_amd as pa
    g = load_golden("temperature")
    recs = _records(g)
    s = pa.AcceptanceRateScheme(target_rate=0.3)
    got = s(t=1, get_weighted_distances=None, get_all_records=lambda: recs,
            max_nr_populations=10, pdf_norm=float(np.min(g["pds"])),
            kernel_scale=pa.SCALE_LOG, prev_temperature=50.,
            acceptance_rate=0.3)
    assert got == 1.0 == g["accrate_norm_min"]
    s = pa.AcceptanceRateScheme(target_rate=0.3, min_rate=0.5)
    assert s(t=1, get_weighted_distances=None, get_all_records=lambda: recs,
             max_nr_populations=10, pdf_norm=0.0, kernel_scale=pa.SCALE_LOG,
             prev_temperature=50., acceptance_rate=0.3) == np.inf


def test_ess_scheme_matches_reference(K):
    import pyabc_amd as pa
    g = load_golden("temperature")
    df = pd.DataFrame({"distance": g["wd_d"], "w": g["wd_w"]})
    norm = float(np.max(g["pds"]))
    for t, prev, rate in [(1, 50., 0.4), (3, 12.5, 1e-5), (2, 7.3, 0.7)]:
        got = pa.EssScheme()(t=t, get_weighted_distances=lambda: df,
                             get_all_records=None, max_nr_populations=6,
                             pdf_norm=norm, kernel_scale=pa.SCALE_LOG,
                             prev_temperature=prev, acceptance_rate=rate)
        want = float(np.ravel(g[f"ess_t{t}"])[0])
        assert abs(got / want - 1) <= 1e-4, (t, got, want)


def test_temperature_sequence_matches_reference(K):
    import pyabc_amd as pa
    g = load_golden("temperature")
    recs = _records(g)
    df = pd.DataFrame({"distance": g["wd_d"], "w": g["wd_w"]})
    cfg = dict(pdf_norm=float(np.max(g["pds"])), kernel_scale=pa.SCALE_LOG)
    temp = pa.Temperature()
    temp.initialize(0, lambda: df, lambda: recs, 5, cfg)
    seq = [temp(0)]
    for t, rate in zip(range(1, 5), [0.5, 0.2, 0.1, 0.05]):
        temp.update(t, lambda: df, lambda: recs, rate, cfg)
        seq.append(temp(t))
    np.testing.assert_allclose(seq, g["temperature_seq"], rtol=1e-9)


def test_reference_scheme_kats(K):
    """test/test_epsilon.py:94-132: every scheme proposes 1 < T < inf."""
    import pyabc_amd as pa
    wd = pd.DataFrame({"distance": [1, 2, 3, 4], "w": [2, 1, 1, 0]})
    recs = [dict(distance=d, transition_pd_prev=p, transition_pd=q,
                 accepted=True) for d, p, q in
            zip([1, 2, 3, 4], [1, 2, 3, 4], [2, 2, 2, 2])]
    args = dict(get_weighted_distances=lambda: wd,
                get_all_records=lambda: recs, max_nr_populations=3,
                pdf_norm=10, kernel_scale=pa.SCALE_LOG,
                prev_temperature=7.53, acceptance_rate=0.4)
    for s in [pa.AcceptanceRateScheme(), pa.ExpDecayFixedIterScheme(),
              pa.ExpDecayFixedRatioScheme(),
              pa.PolynomialDecayFixedIterScheme(), pa.DalyScheme(),
              pa.FrielPettittScheme(), pa.EssScheme()]:
        temp = s(t=0, **args)
        assert 1.0 < temp < np.inf, s


def test_kernel_kats(K):
    """test/test_distance_function.py:250-330 known answers."""
    import pyabc_amd as pa
    import scipy.stats as st
    x0 = {"y0": np.array([1, 2]), "y1": 2.5}
    x = {"y0": np.array([0, 0]), "y1": 7}
    k = pa.IndependentNormalKernel()
    k.initialize(0, None, x0)
    assert np.isclose(k(x, x0),
                      -0.5 * (3 * np.log(2 * np.pi) + 1 + 4 + 4.5 ** 2))
    k = pa.IndependentNormalKernel([1, 2, 3])
    k.initialize(0, None, x0)
    exp_ = -0.5 * (3 * np.log(2 * np.pi) + np.log(1) + np.log(2) + np.log(3)
                   + 1 / 1 + 4 / 2 + 4.5 ** 2 / 3)
    assert np.isclose(k(x, x0), exp_)
    nk = pa.NormalKernel(cov=np.diag([1, 2, 3]))
    nk.initialize(0, None, x0)
    assert np.isclose(nk(x, x0), exp_)
    k = pa.IndependentNormalKernel(lambda p: np.array([p["th0"], p["th1"], 3]))
    k.initialize(0, None, x0)
    assert np.isclose(k(x, x0, par={"th0": 1, "th1": 2}), exp_)
    k = pa.IndependentLaplaceKernel([1, 2, 3])
    k.initialize(0, None, x0)
    want = np.log(np.prod([st.laplace.pdf(x=v, loc=0, scale=s)
                           for v, s in zip([1, 2, 4.5], [1, 2, 3])]))
    assert np.isclose(k(x, x0), want)


def test_normal_kernel_golden(K):
    import pyabc_amd as pa
    g = load_golden("stoch_kernel_full")
    keys = [f"s{i}" for i in range(g["X"].shape[1])]
    x0 = dict(zip(keys, g["x0"]))
    for sc, scale in [("log", pa.SCALE_LOG), ("lin", pa.SCALE_LIN)]:
        k = pa.NormalKernel(cov=g["cov"], ret_scale=scale)
        k.initialize(0, None, x0)
        got = np.array([k(dict(zip(keys, r)), x0) for r in g["X"]])
        np.testing.assert_allclose(got, g[f"normal_full_{sc}"], rtol=1e-12)
        np.testing.assert_allclose(k.pdf_max, g[f"pdf_max_{sc}"], rtol=1e-12)


# ------------------------------------------------------------ end to end
def _stochastic_problem():
    g = load_golden("e2e_stochastic")
    A, x0v, var = g["A"], g["x0"], float(g["var"])
    S, d = A.shape
    keys = [f"y{k:02d}" for k in range(S)]
    names = [f"p{k}" for k in range(d)]
    # exact posterior of the uniform-prior Gaussian-likelihood problem
    P = A.T @ A / var
    cov = np.linalg.inv(P)
    mean = cov @ (A.T @ x0v / var)
    return g, A, x0v, var, keys, names, mean, np.sqrt(np.diag(cov))


def test_e2e_stochastic_batch_path(K):
    """StochasticAcceptor + Temperature through the GPU batch sampler: the
    final (T = 1) population matches the exact posterior and the reference
    runs within Monte-Carlo error."""
    import pyabc_amd as pa
    g, A, x0v, var, keys, names, mean, std = _stochastic_problem()
    model = pa.LinearGaussianModel(A, sigma=0.0, keys=keys)
    prior = pa.Distribution(**{n: pa.RV("uniform", -5, 10) for n in names})
    sampler = pa.GPUBatchSampler(seed=2024)
    abc = pa.ABCSMC(model, prior, pa.IndependentNormalKernel(var=var),
                    population_size=4000, eps=pa.Temperature(),
                    acceptor=pa.StochasticAcceptor(), sampler=sampler)
    abc.new(pa.create_sqlite_db_id(), dict(zip(keys, x0v)))
    h = abc.run(max_nr_populations=6)
    assert sampler.fallback_reason is None
    pops = h.get_all_populations()
    pops = pops[pops.t >= 0]
    temps = pops.epsilon.values
    assert temps[-1] == 1.0
    assert np.all(np.diff(temps) <= 0)
    df, w = h.distribution_numpy(0, h.max_t)
    X = df[names].values
    w = w / w.sum()
    m = (X * w[:, None]).sum(0)
    s = np.sqrt(((X - m) ** 2 * w[:, None]).sum(0))
    ess = 1 / np.sum(w ** 2)
    # analytic posterior: mean within 5 MC standard errors, std within 10 %
    assert np.all(np.abs(m - mean) < 5 * std / np.sqrt(ess)), (m, mean)
    np.testing.assert_allclose(s, std, rtol=0.1)
    # reference runs (N = 1000): same posterior
    ref_m = np.mean([g[f"mean_{r}"][-1] for r in range(3)], axis=0)
    ref_s = np.mean([g[f"std_{r}"][-1] for r in range(3)], axis=0)
    assert np.all(np.abs(m - ref_m) < 5 * std / np.sqrt(800)), (m, ref_m)
    np.testing.assert_allclose(s, ref_s, rtol=0.15)
    # first temperature (AcceptanceRateScheme on the calibration sample) is
    # in the reference's range
    ref_t0 = [g[f"temp_{r}"][0] for r in range(3)]
    assert 0.8 * min(ref_t0) < temps[0] < 1.25 * max(ref_t0)


def test_e2e_stochastic_closure_path(K):
    """test/test_acceptor.py:67-114: a Python model (closure sampler path)
    with the StochasticAcceptor, every pdf norm method."""
    import pyabc_amd as pa

    def model(par):
        return {"s0": par["p0"] + np.array([0.3, 0.7])}
    x_0 = {"s0": np.array([0.4, -0.6])}
    for pdf_norm in [pa.pdf_norm_max_found, pa.pdf_norm_from_kernel,
                     pa.ScaledPDFNorm()]:
        abc = pa.ABCSMC(model, pa.Distribution(p0=pa.RV("uniform", -1, 2)),
                        pa.IndependentNormalKernel(var=np.array([1, 1])),
                        eps=pa.Temperature(),
                        acceptor=pa.StochasticAcceptor(
                            pdf_norm_method=pdf_norm),
                        population_size=20)
        abc.new(pa.create_sqlite_db_id(), x_0)
        h = abc.run(max_nr_populations=3)
        assert h.n_populations >= 1
        wd = h.get_weighted_distances()
        assert np.isfinite(wd["distance"]).all()


def test_stochastic_acceptor_log_file(K):
    """test/test_acceptor.py:67-92: pdf norms stored per t."""
    import tempfile
    import pyabc_amd as pa
    pnorm_file = tempfile.mkstemp(suffix=".json")[1]

    def model(par):
        return {"s0": par["p0"] + np.array([0.3, 0.7])}
    x_0 = {"s0": np.array([0.4, -0.6])}
    abc = pa.ABCSMC(model, pa.Distribution(p0=pa.RV("uniform", -1, 2)),
                    pa.IndependentNormalKernel(var=np.array([1, 1])),
                    eps=pa.Temperature(initial_temperature=1),
                    acceptor=pa.StochasticAcceptor(
                        pdf_norm_method=pa.pdf_norm_max_found,
                        log_file=pnorm_file), population_size=10)
    abc.new(pa.create_sqlite_db_id(), x_0)
    h = abc.run(max_nr_populations=1, minimum_epsilon=1.)
    pnorms = pa.storage.load_dict_from_json(pnorm_file)
    assert len(pnorms) == h.max_t + 2
    assert isinstance(list(pnorms.keys())[0], int)
    assert isinstance(pnorms[0], float)
    os.remove(pnorm_file)


def test_device_records_parents_d12(K, monkeypatch):
    """get_all_records at d > 8: the records' transition
    log-densities come from the MFMA pass WITH parents -- the previous
    population's resample index, and cumsum(acc) - 1 in the new population
    (smc.py _device_records).  Every record's density must match the fp64
    pass on the same fit within 1e-5 (multivariatenormal.py:102-125), and
    so must the pass with wrong (shuffled, out-of-range) parents: a wrong
    parent only moves the row's offset, which the routing window catches."""
    import pyabc_amd as pa
    from pyabc_amd import smc as smc_mod
    rng = np.random.default_rng(12)
    d, S = 12, 40
    A = rng.normal(size=(S, d)) / np.sqrt(d)
    th0 = np.linspace(-1, 1, d)
    var = 0.5
    x0v = A @ th0 + np.sqrt(var) * rng.normal(size=S)
    keys = [f"y{k:02d}" for k in range(S)]
    names = [f"p{k:02d}" for k in range(d)]
    seen = []
    orig = smc_mod.ABCSMC._device_records

    def spy(self, t, sample, prev_transitions):
        rec = orig(self, t, sample, prev_transitions)
        theta = sample.rec_particles[0]
        m = rec.distance.numel()
        fits = (prev_transitions[0].device_fit if t > 1 else None,
                self.transitions[0].device_fit)
        par = sample.rec_particles[3] if len(sample.rec_particles) > 3 \
            else None
        seen.append((t, theta[:m].clone(), rec.log_transition_pd_prev.clone(),
                     rec.log_transition_pd.clone(), fits,
                     None if par is None else par[:m].clone()))
        return rec

    monkeypatch.setattr(smc_mod.ABCSMC, "_device_records", spy)
    model = pa.LinearGaussianModel(A, sigma=0.0, keys=keys)
    prior = pa.Distribution(**{n: pa.RV("uniform", -5, 10) for n in names})
    sampler = pa.GPUBatchSampler(seed=77)
    abc = pa.ABCSMC(model, prior, pa.IndependentNormalKernel(var=var * np.ones(S)),
                    population_size=3000, eps=pa.Temperature(),
                    acceptor=pa.StochasticAcceptor(), sampler=sampler)
    abc.new(pa.create_sqlite_db_id(), dict(zip(keys, x0v)))
    abc.run(max_nr_populations=4)
    assert sampler.fallback_reason is None
    checked = 0
    for t, theta, lp_prev, lp_cur, fits, par in seen:
        for fit, lp in zip(fits, (lp_prev, lp_cur)):
            if fit is None:
                continue
            pp64 = K.PackedPopulation(fit.X, fit.w, fit.packed.mu,
                                      fit.packed.Us, fit.rank, fit.log_pdet,
                                      "f64")
            ref64 = pp64.logpdf(theta).cpu().numpy()
            err = np.abs(np.expm1(lp.cpu().numpy() - ref64))
            assert err.max() < 1e-5, (t, err.max())
            # wrong parents: shuffled and out of range
            n = fit.n
            bad = torch.as_tensor(rng.integers(-5, n + 5, theta.shape[0]),
                                  device="cuda")
            lpb = fit.logpdf(theta, bad).cpu().numpy()
            errb = np.abs(np.expm1(lpb - ref64))
            assert errb.max() < 1e-5, (t, errb.max())
            checked += 1
    assert checked >= 3, checked
