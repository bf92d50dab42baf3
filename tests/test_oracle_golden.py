"""The CPU oracle against the reference's golden vectors and its own KATs.

Pins ``oracle/ref_cpu.py`` before anything is compared with it.  Fixtures come
from ``tools/gen_golden.py`` (reference pyabc 0.10.1 run in the build
container); KATs restate ``test/test_weighted_statistics.py:6-39``,
``test/test_epsilon.py:25-47`` and ``test/test_distance_function.py:75-150``.
"""
import numpy as np
import pytest

from oracle import ref_cpu as ref
from tests.conftest import load_golden, golden_names


@pytest.mark.parametrize("name", golden_names("kde_"))
def test_kde_fit_and_density(name):
    g = load_golden(name)
    w = ref.fit_normalize_weights(g["w"])
    cov = ref.mvn_fit_cov(g["X"], w)
    np.testing.assert_allclose(cov, g["cov"], rtol=1e-13, atol=1e-15)
    pd_ = ref.kde_transition_pd(g["theta"], g["X"], w, g["cov"])
    if g["X"].shape[0] == 1:
        # reference quirk: pdf_static squeezes the [M,1] density matrix, so
        # pdf(DataFrame) with ONE previous particle returns the SUM over the
        # M rows (multivariatenormal.py:119-125); the per-row Series path
        # used by the weight function (smc.py:726) is the semantics we keep.
        np.testing.assert_allclose(pd_.sum(), g["transition_pd"][0],
                                   rtol=1e-12)
    else:
        np.testing.assert_allclose(pd_, g["transition_pd"], rtol=1e-12)
    k = len(g["transition_pd_series"])
    np.testing.assert_allclose(pd_[:k], g["transition_pd_series"], rtol=1e-12)
    prior = ref.uniform_box_pdf(g["theta"], g["prior_lo"], g["prior_scale"])
    np.testing.assert_allclose(prior, g["prior_pd"], rtol=1e-15)
    if g["X"].shape[0] > 1:
        wt = ref.importance_weight(prior, pd_)
        np.testing.assert_allclose(wt, g["weight"], rtol=1e-12)
        wn, _ = ref.normalize_population_weights(wt)
        np.testing.assert_allclose(wn, g["weight_norm"], rtol=1e-12)


@pytest.mark.parametrize("name", golden_names("kde_"))
def test_kde_logsum_contract(name):
    """log-sum contract of the device pass reproduces the scipy density."""
    g = load_golden(name)
    w = ref.fit_normalize_weights(g["w"])
    U, rank, log_pdet = ref.psd_whitening(g["cov"])
    ls = ref.kde_logsum(g["theta"] @ U, g["X"] @ U, np.log(w))
    dens = np.exp(ls - 0.5 * (rank * ref.LOG_2PI + log_pdet))
    k = len(g["transition_pd_series"])
    np.testing.assert_allclose(dens[:k], g["transition_pd_series"], rtol=1e-12)
    if g["X"].shape[0] > 1:
        np.testing.assert_allclose(dens, g["transition_pd"], rtol=1e-12)


@pytest.mark.parametrize("name", golden_names("resample_"))
def test_resample_perturb(name):
    g = load_golden(name)
    idx, theta = ref.resample_perturb(g["X"], g["w"], g["cov"], g["u"], g["z"])
    np.testing.assert_array_equal(idx, g["idx"])
    np.testing.assert_allclose(theta, g["theta"], rtol=1e-13, atol=1e-13)
    # scalar path: u then z[d] per call
    idx1, th1 = ref.resample_perturb(g["X"], g["w"], g["cov"], g["u_single"],
                                     g["z_single"])
    np.testing.assert_allclose(th1, g["theta_single"], rtol=1e-13, atol=1e-13)
    allth = np.concatenate([g["theta"], g["probes"]])
    sup = ref.uniform_box_support(allth, g["prior_lo"], g["prior_scale"])
    np.testing.assert_array_equal(sup.astype(np.uint8), g["in_support"])


@pytest.mark.parametrize("name", golden_names("adaptive_"))
def test_adaptive_weights(name):
    g = load_golden(name)
    w_mad = ref.adaptive_pnorm_weights(g["data"], "mad")
    np.testing.assert_array_equal(w_mad, g["w_mad"])      # order statistics: exact
    w_std = ref.adaptive_pnorm_weights(g["data"], "std")
    np.testing.assert_allclose(w_std, g["w_std"], rtol=1e-12)


def test_pnorm_distances():
    g = load_golden("pnorm_B1500_S100")
    for tag, p in [("1", 1), ("2", 2), ("3", 3), ("inf", np.inf)]:
        d = ref.pnorm_distance(g["stats"], g["x0"], g["fw"], p)
        np.testing.assert_array_equal(d, g["d_p" + tag])
    acc = ref.accept(g["d_p2"], float(g["eps_p2"]))
    np.testing.assert_array_equal(acc.astype(np.uint8), g["accept_p2"])


def test_weighted_quantile_golden():
    g = load_golden("quantile")
    for N in [3, 4, 1000, 100000]:
        for j, a in enumerate(g["alphas"]):
            assert ref.weighted_quantile(g[f"d_{N}"], g[f"w_{N}"], a) == \
                g[f"q_{N}"][j]
            assert ref.weighted_quantile(g[f"d_{N}"], None, a) == \
                g[f"qu_{N}"][j]
    eps = ref.quantile_epsilon(g["d_1000"], g["w_1000"] * 7.0, 0.5, 1.1)
    assert eps == float(g["eps_mult"])


def test_weighted_statistics_kat():
    """test/test_weighted_statistics.py:6-39."""
    points = np.array([1, 5, 2.5])
    weights = np.array([0.5, 0.2, 0.3])
    q = ref.weighted_quantile(points, weights)
    assert 1 < q < 2.5
    assert ref.weighted_quantile(points, weights, alpha=0.2) == 1
    q = ref.weighted_quantile(points, weights, alpha=0.8)
    assert 2.5 < q < 5
    assert ref.weighted_quantile(points, weights, alpha=0.9) == 5
    assert ref.weighted_quantile(points, weights, alpha=1.0) == 5


def test_quantile_epsilon_kat():
    """test/test_epsilon.py:25-47."""
    d = np.array([1, 2, 3, 4], dtype=float)
    w = np.array([2, 1, 1, 1], dtype=float)
    assert np.isclose(ref.quantile_epsilon(d, w, 0.5, 1.1, weighted=False),
                      1.1 * 2.5)
    e = ref.quantile_epsilon(d, w, 0.9, 1.0, weighted=True)
    assert 3 <= e <= 4


def test_pnorm_kat():
    """test/test_distance_function.py:75-91 and 132-150."""
    x = np.array([[-1, -1, -1]], dtype=float)
    x0 = np.array([-1, 0, 1], dtype=float)
    assert ref.pnorm_distance(x, x0, np.ones(3), 2)[0] == pow(1 ** 2 + 2 ** 2, .5)
    fw = np.array([1, 2, 3], dtype=float)
    assert ref.pnorm_distance(x, x0, fw, 2)[0] == \
        pow(sum([(2 * 1) ** 2, (3 * 2) ** 2]), 1 / 2)


@pytest.mark.parametrize("name", [n for n in golden_names("local_")
                                  if not n.startswith("local_rvs")])
def test_local_transition(name):
    g = load_golden(name)
    X, w, k = g["X"], g["w"], int(g["k"])
    nbr = ref.knn_indices(X, k)
    np.testing.assert_array_equal(np.sort(nbr, axis=1), g["nbr"])
    covs, invs, dets = ref.local_covs(X, w, nbr)
    np.testing.assert_allclose(covs, g["covs"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(dets, g["dets"], rtol=1e-11)
    np.testing.assert_allclose(invs, g["inv_covs"], rtol=1e-10, atol=1e-12)
    pdf = ref.local_pdf(g["pts"], X, w, g["inv_covs"], g["dets"])
    np.testing.assert_allclose(pdf, g["pdf"], rtol=1e-12)


@pytest.mark.parametrize("name", golden_names("local_rvs"))
def test_local_rvs(name):
    """LocalTransition.rvs_single from the reference's replayed random
    numbers: indices and draws bit-exact (local_transition.py:141-145)."""
    g = load_golden(name)
    idx, theta = ref.local_rvs(g["X"], g["w"], g["covs"], g["u"], g["z"])
    np.testing.assert_array_equal(idx, g["idx"])
    np.testing.assert_array_equal(theta, g["theta"])


def test_philox_kat():
    """Published Philox4x32-10 known-answer vectors (Random123 kat_vectors)."""
    out = ref.philox4x32_10(np.array([0, 0, 0, 0]), np.array([0, 0]))
    assert [hex(int(v)) for v in out] == \
        ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]
    out = ref.philox4x32_10(np.array([0xffffffff] * 4),
                            np.array([0xffffffff] * 2))
    assert [hex(int(v)) for v in out] == \
        ["0x408f276d", "0x41c83b0e", "0xa20bc7c6", "0x6d5451fd"]
    out = ref.philox4x32_10(
        np.array([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344]),
        np.array([0xa4093822, 0x299f31d0]))
    assert [hex(int(v)) for v in out] == \
        ["0xd16cfe09", "0x94fdcceb", "0x5001e420", "0x24126ea1"]


def test_philox_streams_statistics():
    u = ref.philox_uniform(1234, 7, 200000)
    assert 0.0 <= u.min() and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 5e-3
    z = ref.philox_normal(1234, 7, 200000)
    assert abs(z.mean()) < 1e-2 and abs(z.std() - 1) < 1e-2


def test_philox_normal4_f32_distribution():
    """The synthetic simulators' fp32 Box-Muller stream is standard normal
    (moments, tails, pairwise independence of the members of one block)."""
    z = ref.philox_normal4_f32(99, 4, 400_000)
    assert abs(z.mean()) < 0.005 and abs(z.std() - 1) < 0.005
    assert np.abs(z).max() <= 5.8
    q = z.reshape(-1, 4)
    c = np.corrcoef(q.T)
    assert np.all(np.abs(c - np.eye(4)) < 0.01)


def test_singlecore_replay_fixture():
    """The a9 fixture (tests/golden/gen_singlecore_replay.py): the oracle's
    restatement of the device draws, decided by the oracle's distance and
    acceptance and cut at the n-th acceptance, gives the reference's
    population, evaluation count, recorded set and weights."""
    g = load_golden("singlecore_replay")
    X, w, cov = g["X"], g["w"], g["cov"]
    d, S, n, seed, t = X.shape[1], g["A"].shape[0], int(g["n"]), \
        int(g["seed"]), int(g["t"])
    np.testing.assert_allclose(ref.mvn_fit_cov(X, w), cov, rtol=1e-13)
    P = 3000
    sid = 8 * t
    u = ref.philox_uniform(seed, 2 * sid, P)
    z = ref.philox_normal(seed, 2 * sid + 1, P * d).reshape(P, d)
    _, th = ref.resample_perturb(X, w, cov, u, z)
    valid = th[ref.uniform_box_support(th, g["lo"], g["sc"])]
    E = valid.shape[0]
    noise = ref.philox_normal4_f32(seed, 2 * (sid + 1), E * S).reshape(E, S)
    stats = valid @ g["A"].T + g["c"] + g["sigma"] * noise.astype(np.float64)
    dist = ref.pnorm_distance(stats, g["x0"], np.ones(S), 2.0)
    acc = ref.accept(dist, float(g["eps"]))
    n_eval = int(np.flatnonzero(acc)[n - 1]) + 1
    assert n_eval == int(g["nr_evaluations"])
    np.testing.assert_array_equal(acc[:n_eval], g["rec_acc"])
    np.testing.assert_allclose(stats[:n_eval], g["rec_stats"], rtol=1e-15,
                               atol=1e-15)
    np.testing.assert_array_equal(valid[acc][:n], g["theta"])
    np.testing.assert_allclose(dist[acc][:n], g["d"], rtol=1e-13)
    prior = ref.uniform_box_pdf(g["theta"], g["lo"], g["sc"])
    wt = ref.importance_weight(prior, ref.kde_transition_pd(g["theta"], X, w,
                                                            cov))
    # the accepted Population normalises its weights (population.py:120-142)
    wn, _ = ref.normalize_population_weights(wt)
    np.testing.assert_allclose(wn, g["weight"], rtol=1e-12)
