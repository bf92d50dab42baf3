"""HIP kernels through the C-ABI vs the oracle and the reference's golden vectors.

Tolerances (BASELINE north star): resampled indices, support masks, accept
masks and order statistics bit-exact; weights / densities / distances /
covariances / epsilon within 1e-5 relative for the fp32 KDE kernel and
1e-12 for fp64.
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu as ref
from tests.conftest import load_golden, golden_names

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


# ---------------------------------------------------------------- (a3) KDE
def _packed(K, X, w, cov, precision):
    U, rank, log_pdet = K.psd_whitening(cov)
    Us = U * math.sqrt(0.5 * K.LOG2E)
    mu = (X * w[:, None]).sum(0) / w.sum()
    return K.PackedPopulation(dev(X), dev(w), dev(mu), dev(Us), rank,
                              log_pdet, precision)


@pytest.mark.parametrize("precision,rtol", [("mfma", 1e-5), ("f32", 1e-5),
                                            ("f64", 1e-12)])
@pytest.mark.parametrize("name", golden_names("kde_"))
def test_kde_density_vs_reference(K, name, precision, rtol):
    g = load_golden(name)
    w = ref.fit_normalize_weights(g["w"])
    pp = _packed(K, g["X"], w, g["cov"], precision)
    logpd = pp.logpdf(dev(g["theta"]))
    dens = np.exp(host(logpd))
    k = len(g["transition_pd_series"])
    np.testing.assert_allclose(dens[:k], g["transition_pd_series"], rtol=rtol)
    if g["X"].shape[0] > 1:
        np.testing.assert_allclose(dens, g["transition_pd"], rtol=rtol)
        prior = dev(ref.uniform_box_pdf(g["theta"], g["prior_lo"],
                                        g["prior_scale"]))
        wt = K.importance_weights(logpd, prior)
        np.testing.assert_allclose(host(wt), g["weight"], rtol=rtol)
        s = K.dsum(wt)
        K.scale_inplace(wt, s)
        np.testing.assert_allclose(host(wt), g["weight_norm"], rtol=rtol)


@pytest.mark.parametrize("precision", ["mfma", "f32", "f64"])
def test_kde_underflow_rows_fixup(K, precision):
    """Rows far from every previous particle underflow the fixed offset;
    the fixup pass must still return the exact log density.  f64: rows
    whose density lies below 1e-280 (every fp64 term underflows) keep the
    fp64 pass's 1e-12 contract through the fixup (fp64 exp2 there)."""
    rng = np.random.default_rng(7)
    X = rng.normal(size=(3000, 4))
    w = rng.uniform(0.5, 1.5, 3000)
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    far = 40.0 if precision == "f64" else 6.0
    theta = np.concatenate([X[:50] + 0.01, X[:20] + far])   # far rows
    pp = _packed(K, X, w, cov, precision)
    lp = host(pp.logpdf(dev(theta)))
    if precision == "mfma":
        # the 20 far rows (and no near row) were re-evaluated with their own
        # offsets on the matrix cores (kde_mfma.hip refine)
        assert pp.refined_rows() == 20
    else:
        # the 20 far rows (and no near row) went through the exact fixup
        assert pp.fixup_rows() == 20
    U, rank, log_pdet = ref.psd_whitening(cov)
    ls = ref.kde_logsum(theta @ U, X @ U, np.log(w))
    expect = ls - 0.5 * (rank * ref.LOG_2PI + log_pdet)
    if precision == "f64":
        assert np.all(expect[50:] < math.log(1e-280))
        # density relative error = |log difference|; the far rows' exponents
        # are ~3e3, whose fp64 evaluation itself carries ~1e-12 absolute
        np.testing.assert_allclose(lp[:50], expect[:50], rtol=0, atol=1e-12)
        np.testing.assert_allclose(lp[50:], expect[50:], rtol=0, atol=1e-10)
    else:
        np.testing.assert_allclose(lp, expect, rtol=2e-6, atol=1e-5)


def test_kde_large_random_vs_oracle(K):
    rng = np.random.default_rng(11)
    N, M, d = 20000, 777, 8
    X = rng.normal(size=(N, d)) * 2 + 5
    w = rng.uniform(0.2, 2, N)
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    theta = X[rng.integers(0, N, M)] + rng.normal(size=(M, d)) * 0.3
    expect = ref.kde_transition_pd(theta, X, w, cov)
    for prec, rtol in [("mfma", 1e-5), ("f32", 1e-5), ("f64", 1e-12)]:
        pp = _packed(K, X, w, cov, prec)
        got = np.exp(host(pp.logpdf(dev(theta))))
        np.testing.assert_allclose(got, expect, rtol=rtol)


@pytest.mark.parametrize("d", [1, 2, 3, 5, 8, 12, 20, 32])
def test_kde_mfma_all_dims_vs_oracle(K, d):
    """Exact-grid f16 MFMA pass at every padded-dimension instance (folded
    up to d = 24, split above), including ragged N / M (tails of 32-row
    tiles and 64-row chunks)."""
    rng = np.random.default_rng(100 + d)
    N, M = 3001 + 7 * d, 517
    X = rng.normal(size=(N, d)) * rng.uniform(0.5, 3, d) + 1.0
    w = rng.uniform(0.1, 2, N)
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    theta = X[rng.integers(0, N, M)] + rng.normal(size=(M, d)) * 0.2
    expect = ref.kde_transition_pd(theta, X, w, cov)
    pp = _packed(K, X, w, cov, "mfma")
    got = np.exp(host(pp.logpdf(dev(theta))))
    np.testing.assert_allclose(got, expect, rtol=1e-5)


@pytest.mark.parametrize("d", [2, 4, 6, 8, 16])
def test_kde_mfma_anisotropic_heavy_weights(K, d):
    """A strongly correlated population (condition number ~1e4), log-normal
    weights over eight decades, rows near and far (1.5x outward), ragged
    sizes: every row against the oracle at north_star's 1e-5."""
    rng = np.random.default_rng(300 + d)
    N, M = 6007, 611
    A = rng.normal(size=(d, d))
    Q, _ = np.linalg.qr(A)
    scales = np.logspace(0, 2, d)
    X = (rng.normal(size=(N, d)) * scales) @ Q.T + 3.0
    w = np.exp(rng.normal(scale=3.0, size=N))
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    theta = np.concatenate([X[rng.integers(0, N, M - 100)]
                            + 0.1 * rng.normal(size=(M - 100, d)) * scales,
                            3.0 + 1.5 * (X[:100] - 3.0)])
    expect = ref.kde_transition_pd(theta, X, w, cov)
    pp = _packed(K, X, w, cov, "mfma")
    got = np.exp(host(pp.logpdf(dev(theta))))
    ok = expect > 0
    np.testing.assert_allclose(got[ok], expect[ok], rtol=1e-5)


@pytest.mark.parametrize("d", [1, 3, 8, 12])
def test_kde_mfma_out_of_grid_rows(K, d):
    """New rows beyond the population's grid range (f16 pieces: |y| > 2040 g)
    are flagged by the packer and evaluated by the exact fixup."""
    rng = np.random.default_rng(5)
    X = rng.normal(size=(2000, d))
    w = np.full(2000, 1 / 2000)
    cov = ref.mvn_fit_cov(X, w)
    theta = np.concatenate([X[:10] + 0.05, X[:5] * 40.0, X[:5] + 3.0])
    pp = _packed(K, X, w, cov, "mfma")
    lp = host(pp.logpdf(dev(theta)))
    U, rank, log_pdet = ref.psd_whitening(cov)
    ls = ref.kde_logsum(theta @ U, X @ U, np.log(w))
    expect = ls - 0.5 * (rank * ref.LOG_2PI + log_pdet)
    np.testing.assert_allclose(lp, expect, rtol=2e-6, atol=1e-5)


@pytest.mark.parametrize("d", [2, 8, 12])
@pytest.mark.parametrize("far,wfar", [(30.0, 1e-6), (3e3, 1e-12), (3e6, 1e-15)])
def test_kde_mfma_f16_grid_extremes(K, far, wfar, d):
    """f16 pieces (every d since round 4): a light particle far out makes the
    population's largest whitened norm 2^7 ... 2^24, i.e. the aH / bH pieces
    scaled by 2^-K (K = 2E - 13) and, past 2^13, the all-fixup packing;
    every row against the oracle."""
    rng = np.random.default_rng(int(far) + d)
    N, M = 3000, 300
    X = rng.normal(size=(N, d))
    X[0] = far
    w = rng.uniform(0.5, 1.5, N)
    w[0] = wfar
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    theta = np.concatenate([X[rng.integers(1, N, M - 2)]
                            + 0.3 * rng.normal(size=(M - 2, d)),
                            X[:1] + 0.1, X[1:2] * 3.0])
    pp = _packed(K, X, w, cov, "mfma")
    got = host(pp.logpdf(dev(theta)))
    U, rank, log_pdet = ref.psd_whitening(cov)
    ls = ref.kde_logsum(theta @ U, X @ U, np.log(w))
    expect = ls - 0.5 * (rank * ref.LOG_2PI + log_pdet)
    np.testing.assert_allclose(got, expect, rtol=1e-6, atol=1e-5)


def test_kde_mfma_rows_independent_of_launch(K):
    """A row's bits do not depend on M or on which rows share its tiles
    (the multi-GPU row split relies on it)."""
    rng = np.random.default_rng(9)
    N, M, d = 70000, 3000, 8
    X = rng.normal(size=(N, d))
    w = rng.uniform(0.5, 1.5, N)
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    theta = X[rng.integers(0, N, M)] + 0.1 * rng.normal(size=(M, d))
    pp = _packed(K, X, w, cov, "mfma")
    full = host(pp.logpdf(dev(theta)))
    for lo, hi in [(0, 1), (17, 1234), (1500, 3000), (2999, 3000)]:
        part = host(pp.logpdf(dev(theta[lo:hi])))
        np.testing.assert_array_equal(part, full[lo:hi])


KNOBS = {
    4: [("ABC_KDE_MFMA_PIPE", "0"), ("ABC_KDE_MFMA_IB", "1"),
        ("ABC_KDE_MFMA_IB", "2"), ("ABC_KDE_MFMA_SPLIT", "4"),
        ("ABC_KDE_MFMA_LDS2", "1"), ("ABC_KDE_MFMA_LDS2", "3"),
        ("ABC_KDE_MFMA_SMAJOR", "1")],
    8: [("ABC_KDE_MFMA_PIPE", "0"), ("ABC_KDE_MFMA_IB", "1"),
        ("ABC_KDE_MFMA_IB", "2"), ("ABC_KDE_MFMA_SPLIT", "1"),
        ("ABC_KDE_MFMA_SPLIT", "8"), ("ABC_KDE_MFMA_LDS2", "1"),
        ("ABC_KDE_MFMA_LDS2", "3"), ("ABC_KDE_MFMA_LDS2", "0"),
        ("ABC_KDE_MFMA_SMAJOR", "1")],
    20: [("ABC_KDE_MFMA_LDS2", "1"), ("ABC_KDE_MFMA_LDS2", "0"),
         ("ABC_KDE_MFMA_LDS2", "2"),
         ("ABC_KDE_MFMA_IB", "1"), ("ABC_KDE_MFMA_IB", "2"),
         ("ABC_KDE_MFMA_SPLIT", "2"), ("ABC_KDE_MFMA_PIPE", "1"),
         ("ABC_KDE_MFMA_SMAJOR", "1")],
}


@pytest.mark.parametrize("d", sorted(KNOBS))
def test_kde_mfma_launch_knobs_bit_identical(K, d, monkeypatch):
    """Every runtime knob of abc_kde_logpdf_mfma (kde_mfma.hip launch_mfma)
    is a launch-shape choice: the rows are bit-identical under each."""
    rng = np.random.default_rng(20 + d)
    N, M = 20000, 2500
    X = rng.normal(size=(N, d))
    w = rng.uniform(0.5, 1.5, N)
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    theta = np.concatenate([X[rng.integers(0, N, M - 500)]
                            + 0.2 * rng.normal(size=(M - 500, d)),
                            1.7 * X[:500]])          # low-density rows too
    pp = _packed(K, X, w, cov, "mfma")
    base = host(pp.logpdf(dev(theta)))
    want = ref.kde_transition_pd(theta[:64], X, w, cov)
    assert np.max(np.abs(np.exp(base[:64]) / want - 1)) < 1e-5
    for key, val in KNOBS[d]:
        monkeypatch.setenv(key, val)
        K.reload_tuning()
        got = host(pp.logpdf(dev(theta)))
        monkeypatch.delenv(key)
        K.reload_tuning()
        np.testing.assert_array_equal(got, base, err_msg=f"{key}={val}")


def test_kde_mfma_d8_ib_by_row_count(K):
    """d = 8 launches four i-tiles per wave from 375 000 new rows and three
    below (kde_mfma.hip kIb4MinRows; the padding unit follows): the rows
    common to a launch just below and one just above the switch are the
    same bits, on the LDS-DMA pass (N >= 2^16)."""
    rng = np.random.default_rng(8)
    N, d = 65536, 8
    X = rng.normal(size=(N, d))
    w = rng.uniform(0.5, 1.5, N)
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    M = 375_000
    theta = X[rng.integers(0, N, M)] + 0.2 * rng.normal(size=(M, d))
    pp = _packed(K, X, w, cov, "mfma")
    lo = host(pp.logpdf(dev(theta[:M - 1])))     # IB = 3, 768-row padding
    hi = host(pp.logpdf(dev(theta)))             # IB = 4, 512-row padding
    assert K.nat.lib().abc_kde_mfma_new_rows(M - 1, d) % 768 == 0
    assert K.nat.lib().abc_kde_mfma_new_rows(M, d) % 512 == 0
    np.testing.assert_array_equal(hi[:M - 1], lo)
    want = ref.kde_transition_pd(theta[:32], X, w, cov)
    assert np.max(np.abs(np.exp(hi[:32]) / want - 1)) < 1e-5


# ------------------------------------------------------------ (a1) fit
@pytest.mark.parametrize("name", golden_names("kde_"))
def test_weighted_moments_cov(K, name):
    g = load_golden(name)
    if g["X"].shape[0] < 2:
        pytest.skip("single particle: diag(|x|) handled on the host")
    w = ref.fit_normalize_weights(g["w"])
    mom = host(K.weighted_moments(dev(g["X"]), dev(w)))
    d = g["X"].shape[1]
    sw, sw2 = mom[0], mom[1]
    C = mom[2 + d:].reshape(d, d) / (sw - sw2 / sw)
    bw = ref.silverman_rule_of_thumb(1 / sw2, d)
    np.testing.assert_allclose(C * bw ** 2, g["cov"], rtol=1e-12, atol=1e-15)


# -------------------------------------------------------- (a2) proposals
@pytest.mark.parametrize("name", golden_names("resample_"))
def test_resample_perturb_bit_exact(K, name):
    g = load_golden(name)
    cdf_ref = ref.resample_cdf(g["w"])
    cdf = K.resample_cdf(dev(g["w"]))
    np.testing.assert_array_equal(host(cdf), cdf_ref)
    A = ref.svd_factor(g["cov"])
    theta, idx, sup = K.resample_perturb(dev(g["X"]), cdf, dev(g["u"]),
                                         dev(g["z"]), dev(A),
                                         dev(g["prior_lo"]),
                                         dev(g["prior_scale"]))
    np.testing.assert_array_equal(host(idx), g["idx"])
    np.testing.assert_allclose(host(theta), g["theta"], rtol=1e-13,
                               atol=1e-13)
    B = len(g["u"])
    np.testing.assert_array_equal(host(sup), g["in_support"][:B])


@pytest.mark.parametrize("name", golden_names("resample_"))
def test_support_boundary_probes(K, name):
    """theta exactly on / one ulp outside the box: scipy's inclusive test."""
    g = load_golden(name)
    P = g["probes"]
    n, d = P.shape
    cdf = K.resample_cdf(dev(np.ones(n)))
    u = (np.arange(n) + 0.5) / n
    theta, idx, sup = K.resample_perturb(dev(P), cdf, dev(u),
                                         dev(np.zeros((n, d))),
                                         dev(np.eye(d)), dev(g["prior_lo"]),
                                         dev(g["prior_scale"]))
    np.testing.assert_array_equal(host(idx), np.arange(n))
    np.testing.assert_array_equal(host(theta), P)
    B = len(g["u"])
    np.testing.assert_array_equal(host(sup), g["in_support"][B:])


def test_philox_streams_match_oracle(K):
    u = host(K.philox_uniform(1234, 7, 3, 100001))
    np.testing.assert_array_equal(u, ref.philox_uniform(1234, 7, 100004)[3:])
    z = host(K.philox_normal(99, 2, 0, 50001))
    np.testing.assert_allclose(z, ref.philox_normal(99, 2, 50001),
                               rtol=1e-13, atol=1e-13)


def test_propose_philox_consistent_with_injected(K):
    rng = np.random.default_rng(5)
    N, d, B = 5000, 6, 40000
    X = rng.normal(size=(N, d))
    w = rng.uniform(size=N)
    w /= w.sum()
    A = ref.svd_factor(ref.mvn_fit_cov(X, w))
    lo, sc = np.full(d, -2.0), np.full(d, 4.0)
    cdf = K.resample_cdf(dev(w))
    seed, sid, off = 42, 3, 1000
    th, idx, sup = K.propose_philox(dev(X), cdf, dev(A), dev(lo), dev(sc),
                                    seed, sid, off, B)
    u = ref.philox_uniform(seed, 2 * sid, off + B)[off:]
    z = ref.philox_normal(seed, 2 * sid + 1, (off + B) * d)[off * d:]
    idx_ref, th_ref = ref.resample_perturb(X, w, None if False else
                                           ref.mvn_fit_cov(X, w), u,
                                           z.reshape(B, d))
    np.testing.assert_array_equal(host(idx), idx_ref)
    np.testing.assert_allclose(host(th), th_ref, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(
        host(sup).astype(bool), ref.uniform_box_support(th_ref, lo, sc))
    # the bucket-table search gives the same indices and draws
    for log2k in (0, 4, 16, 20):
        tab = K.cdf_index(cdf, log2k)
        np.testing.assert_array_equal(
            host(tab), np.searchsorted(host(cdf), np.arange(2 ** log2k + 1)
                                       / 2 ** log2k, side="right"))
        th2, idx2, sup2 = K.propose_philox(dev(X), cdf, dev(A), dev(lo),
                                           dev(sc), seed, sid, off, B,
                                           tab=tab)
        np.testing.assert_array_equal(host(idx2), idx_ref)
        np.testing.assert_array_equal(host(th2), host(th))
        np.testing.assert_array_equal(host(sup2), host(sup))


@pytest.mark.parametrize("kind", ["one_heavy", "zeros", "tail"])
def test_cdf_index_search_skewed(K, kind):
    """Bucket-table search on skewed weights (one particle holding most of
    the mass, runs of zero weights, a heavy tail): indices equal numpy's
    searchsorted, including u on bucket edges."""
    rng = np.random.default_rng(8)
    N = 100_003
    w = rng.uniform(size=N)
    if kind == "one_heavy":
        w[777] = 1e7
    elif kind == "zeros":
        w[1000:90000] = 0.0
    else:
        w = rng.pareto(0.7, size=N)
    cdf = K.resample_cdf(dev(w / w.sum()))
    tab = K.cdf_index(cdf, 16)
    B = 300_000
    X = rng.normal(size=(N, 2))
    A = np.eye(2) * 0.1
    th, idx, _ = K.propose_philox(dev(X), cdf, dev(A), None, None, 9, 1, 0, B,
                                  tab=tab)
    u = ref.philox_uniform(9, 2, B)
    np.testing.assert_array_equal(host(idx), np.searchsorted(
        host(cdf), u, side="right"))


def test_compaction(K):
    rng = np.random.default_rng(3)
    for n in [1, 100, 4096, 4097, 1_000_003]:
        f = (rng.uniform(size=n) < 0.37).astype(np.uint8)
        idx, cnt = K.compact(dev(f, torch.uint8))
        c = int(host(cnt)[0])
        np.testing.assert_array_equal(host(idx)[:c], np.nonzero(f)[0])


# ------------------------------------------------------ (a5) distances
def test_pnorm_distances_and_accept(K):
    g = load_golden("pnorm_B1500_S100")
    stats_T = dev(g["stats"].T)
    for tag, p in [("1", 1), ("2", 2), ("3", 3), ("inf", math.inf)]:
        eps = float(g["eps_p2"]) if tag == "2" else math.inf
        d, acc, guard = K.pnorm_distance(stats_T, dev(g["x0"]), dev(g["fw"]),
                                         p, eps)
        np.testing.assert_allclose(host(d), g["d_p" + tag], rtol=1e-12)
        if tag == "2":
            np.testing.assert_array_equal(host(acc), g["accept_p2"])
            assert host(guard).sum() == 0


def _sqrt_pow_disagree(rng, n):
    """(t1, t2) with s = t1*t1 + t2*t2 and sqrt(s) != pow(s, .5) (libm: about
    1e-3 of generic s; a lone square t*t is almost never such an s), both
    ways."""
    up, down = [], []
    for _ in range(2_000_000):
        t1, t2 = (float(v) for v in rng.uniform(1, 100, 2))
        s = t1 * t1 + t2 * t2
        a, b = math.sqrt(s), math.pow(s, 0.5)
        if a > b and len(up) < n:
            up.append((t1, t2))
        elif a < b and len(down) < n:
            down.append((t1, t2))
        if len(up) == n and len(down) == n:
            return up, down
    raise AssertionError("no sqrt/pow disagreement found")


def test_stat_major_column_slices(K):
    """Column slices of a stat-major matrix (the recorded statistics of one
    round, first_m_sum_stats) go to the kernels as (pointer, row stride):
    median / MAD, std, p-norm and stochastic-kernel results equal those of
    the contiguous copy, bit for bit."""
    rng = np.random.default_rng(5)
    S, n, m = 7, 5000, 3111
    full = dev(rng.normal(size=(S, n)) * rng.uniform(0.1, 10, size=(S, 1)))
    view = full[:, :m]
    assert not view.is_contiguous()
    copy = view.contiguous()
    for f in (K.column_median_mad, K.column_std):
        for a, b in zip(f(view), f(copy)):
            np.testing.assert_array_equal(host(a), host(b))
    x0, fw = dev(rng.normal(size=S)), dev(rng.uniform(0.5, 2, size=S))
    for a, b in zip(K.pnorm_distance(view, x0, fw, 2, 3.0),
                    K.pnorm_distance(copy, x0, fw, 2, 3.0)):
        np.testing.assert_array_equal(host(a), host(b))
    prm = dev(rng.uniform(0.5, 2, size=S))
    a = K.stochastic_kernel(view, x0, prm, K.KERNEL_NORMAL, 0.0)[0]
    b = K.stochastic_kernel(copy, x0, prm, K.KERNEL_NORMAL, 0.0)[0]
    np.testing.assert_array_equal(host(a), host(b))
    one = full[:1, :m]                     # S = 1: any row stride
    np.testing.assert_array_equal(host(K.column_median_mad(one)[0]),
                                  np.median(host(copy)[:1], axis=1))


@pytest.mark.parametrize("p", [1, 2, 3, math.inf])
def test_sim_pnorm_fused(K, p):
    """The fused simulation + distance kernel (no statistics stored) gives
    the distances, accept and guard flags of abc_sim_linear_gaussian_f64
    followed by abc_pnorm_distance_f64, bit for bit, with and without the
    constant term c."""
    rng = np.random.default_rng(31)
    # d = 8 / 20 (the DMAX 8 / 24 forms with the model in LDS), S = 700 at
    # d = 20: A no longer fits the LDS stage (the global-A form)
    for B, d, S, c in ((20000, 8, 100, None), (20000, 8, 100, 1),
                       (9001, 20, 100, 1), (3001, 20, 700, 1)):
        _sim_pnorm_case(K, p, rng, B, d, S, c)


def _sim_pnorm_case(K, p, rng, B, d, S, c):
    theta = dev(rng.uniform(-2, 2, size=(B, d)))
    A = dev(rng.normal(size=(S, d)) / np.sqrt(d))
    x0, fw = dev(rng.normal(size=S)), dev(rng.uniform(0.5, 2, size=S))
    for c in ((None,) if c is None else (dev(rng.normal(size=S)),)):
        stats = K.sim_linear_gaussian(theta, A, c, 0.5, 7, 13, 12345)
        d1, a1, g1 = K.pnorm_distance(stats, x0, fw, p, 30.0)
        eps = float(np.median(host(d1)))
        d1, a1, g1 = K.pnorm_distance(stats, x0, fw, p, eps)
        d2, a2, g2 = K.sim_linear_gaussian_pnorm(theta, A, c, 0.5, 7, 13, 12345,
                                                 x0, fw, p, eps)
        np.testing.assert_array_equal(host(d1), host(d2))
        np.testing.assert_array_equal(host(a1), host(a2))
        np.testing.assert_array_equal(host(g1), host(g2))
        # the same pass writing the statistics too (round 6)
        d3, a3, g3, st3 = K.sim_linear_gaussian_pnorm(
            theta, A, c, 0.5, 7, 13, 12345, x0, fw, p, eps, keep_stats=True)
        np.testing.assert_array_equal(host(st3), host(stats))
        np.testing.assert_array_equal(host(d3), host(d1))
        np.testing.assert_array_equal(host(a3), host(a1))
        np.testing.assert_array_equal(host(g3), host(g1))


def test_engine_fused_round_equals_unfused(K):
    """A generation whose statistics are not kept (the bench's) runs the
    fused simulate_distance; population, distances, weights, log-densities
    and evaluation count equal the unfused engine's bit for bit."""
    from pyabc_amd.batch_models import LinearGaussianModel
    from pyabc_amd.engine import DeviceMVNFit, GenerationEngine
    model = LinearGaussianModel.benchmark(4, 30)
    x0 = dev(model._x0)
    fw = dev(np.ones(30))
    out = []
    for fuse, keep in ((False, False), (True, False), (False, True),
                       (True, True)):
        eng = GenerationEngine(model, np.full(4, -5.0), np.full(4, 10.0),
                               seed=99)
        eng.fuse_sim_distance = fuse
        r0 = eng.sample_prior(0, 8000)
        d0, _, _ = K.pnorm_distance(r0.stats_T, x0, fw, 2.0)
        w0 = torch.full((8000,), 1 / 8000, dtype=torch.float64, device="cuda")
        eps = float(np.quantile(host(d0), 0.3))
        # keep: the kept-statistics rounds (stored population, recorded
        # evaluations) through the stats-writing fused pass
        res = eng.sample_generation(1, 8000, DeviceMVNFit(r0.theta, w0), x0, fw,
                                    eps, keep_stats=keep, record=keep)
        out.append(res)
    a = out[0]
    for b in out[1:]:
        for f in ("theta", "d", "w", "logpd"):
            np.testing.assert_array_equal(host(getattr(a, f)),
                                          host(getattr(b, f)))
        assert a.n_eval == b.n_eval
    for f in ("stats_T", "rec_stats_T"):
        np.testing.assert_array_equal(host(getattr(out[2], f)),
                                      host(getattr(out[3], f)))


def test_pnorm_decide_one_read(K):
    """PNormAcceptance.decide (the engine's one-sync round) gives the
    distances, accept mask, compacted positions and counts of the plain
    call followed by a compaction, with the guard band re-decided."""
    from pyabc_amd.engine import PNormAcceptance
    rng = np.random.default_rng(8)
    S, B = 20, 40000
    stats = dev(rng.normal(size=(S, B)))
    x0, fw = dev(np.zeros(S)), dev(np.ones(S))
    eps = float(np.median(np.sqrt((host(stats) ** 2).sum(0))))
    a = PNormAcceptance(x0, fw, 2, eps)
    d1, acc1, g1, _ = a(stats, B, 0, 0, 0)
    pos1, c1 = K.compact(acc1)
    need = 5000
    d2, acc2, g2, _, pos2, n2, ng2, last = a.decide(stats, B, 0, 0, 0,
                                                    need=need)
    np.testing.assert_array_equal(host(d1), host(d2))
    np.testing.assert_array_equal(host(acc1), host(acc2))
    assert n2 == int(host(c1)[0]) and ng2 == int(host(g2).sum())
    np.testing.assert_array_equal(host(pos1)[:n2], host(pos2)[:n2])
    # the closing position read with the counts: the need-th acceptance
    # (None when the band moved positions or the round fell short)
    if ng2 == 0:
        assert last == int(host(pos1)[need - 1])
    *_, short = a.decide(stats, B, 0, 0, 0, need=n2 + 1)
    assert short is None


@pytest.mark.parametrize("p", [2, 3])
def test_guard_band_redecided_on_host(K, p):
    """A distance within 1 ulp of eps where the kernel's sqrt (or device
    pow) and the reference's libm pow disagree: the engine's host
    re-decision (engine.redecide_guard_band) makes the accept bit the
    reference's (distance.py:96-100, acceptor.py:241-242)."""
    from pyabc_amd.engine import PNormAcceptance, pnorm_host
    rng = np.random.default_rng(17)
    x0 = np.array([0.0, 0.0, -1.0])
    fw = np.array([1.0, 1.0, 1.0])
    if p == 2:
        up, down = _sqrt_pow_disagree(rng, 4)
        ts = up + down
    else:
        ts = [tuple(r) for r in rng.uniform(1, 100, (8, 2)).tolist()]
    cols = np.array([[t1, t2, -1.0] for t1, t2 in ts]).T     # [S, B]
    ref_d = np.array([pnorm_host(cols[:, i].tolist(), x0.tolist(),
                                 fw.tolist(), p) for i in range(len(ts))])
    stats = dev(cols)
    d_dev, _, _ = K.pnorm_distance(stats, dev(x0), dev(fw), p, math.inf)
    d_dev = host(d_dev)
    for i in range(len(ts)):
        # eps exactly at the reference's distance, and one ulp either side
        for eps in (ref_d[i], np.nextafter(ref_d[i], 0),
                    np.nextafter(ref_d[i], np.inf)):
            acc_obj = PNormAcceptance(dev(x0), dev(fw), p, float(eps))
            d, acc, guard, _ = acc_obj(stats, len(ts), 0, 0, 0)
            want = (ref_d <= eps).astype(np.uint8)
            np.testing.assert_array_equal(host(acc), want)
            assert host(d)[i] == ref_d[i]
            assert acc_obj.n_redecided >= 1
    if p == 2:
        # the kernel alone disagrees on these rows (what the guard is for)
        assert np.count_nonzero(d_dev != ref_d) == len(ts)


def test_guard_band_large_batch(K):
    """Many particles, eps at the reference median: accept mask equals the
    libm-pow decision for every particle; the band stays tiny."""
    from pyabc_amd.engine import PNormAcceptance, pnorm_host
    g = load_golden("pnorm_B1500_S100")
    stats = g["stats"].T
    x0, fw = g["x0"].tolist(), g["fw"].tolist()
    ref_d = np.array([pnorm_host(stats[:, i].tolist(), x0, fw, 2)
                      for i in range(stats.shape[1])])
    for eps in np.quantile(ref_d, [0.1, 0.5, 0.9], method="lower"):
        a = PNormAcceptance(dev(g["x0"]), dev(g["fw"]), 2, float(eps))
        d, acc, guard, _ = a(dev(stats), stats.shape[1], 0, 0, 0)
        np.testing.assert_array_equal(host(acc), (ref_d <= eps).astype(
            np.uint8))
        assert 1 <= a.n_redecided <= 8


# ---------------------------------------------- (a6) adaptive scales
@pytest.mark.parametrize("name", golden_names("adaptive_"))
def test_column_mad_and_std(K, name):
    g = load_golden(name)
    data = g["data"]
    med, mad = K.column_median_mad(dev(data.T))
    np.testing.assert_array_equal(host(med), np.median(data, axis=0))
    mad_ref = np.array([ref.median_absolute_deviation(data[:, k])
                        for k in range(data.shape[1])])
    np.testing.assert_array_equal(host(mad), mad_ref)
    _, std = K.column_std(dev(data.T))
    np.testing.assert_allclose(host(std), np.std(data, axis=0), rtol=1e-12)

    def weights(scale):
        w = np.array([0 if np.isclose(s, 0) else 1 / s for s in scale])
        return w / np.mean(w)
    np.testing.assert_array_equal(weights(host(mad)), g["w_mad"])
    np.testing.assert_allclose(weights(host(std)), g["w_std"], rtol=1e-12)


# ------------------------------------------------------ (a7) quantile
def test_weighted_quantile_golden(K):
    """The reference's own outputs (tests/golden/quantile.npz, written by
    weighted_quantile itself).  Random weights: within SURVEY 8(a7)'s local
    bound at the bracketing knots, and <= 1e-9 absolute.  Uniform weights
    (weights=None, np.ones(n) / n): bit for bit -- the device restates
    numpy's cumsum of equal weights (select.hip equal_weight_cumsum)."""
    from tests.wq_bound import local_bound, record
    g = load_golden("quantile")
    rows = []
    for N in [3, 4, 1000, 100000]:
        d, w = g[f"d_{N}"], g[f"w_{N}"]
        for j, a in enumerate(g["alphas"]):
            a = float(a)
            q = float(host(K.weighted_quantile(dev(d), dev(w), a))[0])
            want = float(g[f"q_{N}"][j])
            bound, exact = local_bound(d, w, a)
            tol = 0.0 if exact else 1e-12 * abs(want) + bound
            err = abs(q - want)
            rows.append(dict(N=N, alpha=a, weights="random", err=err,
                             tol=tol, rel=err / abs(want) if want else err))
            assert err <= tol, (N, a, q, want, tol)
            assert err <= 1e-9, (N, a, err)
            qu = float(host(K.weighted_quantile(dev(d), None, a))[0])
            wantu = float(g[f"qu_{N}"][j])
            rows.append(dict(N=N, alpha=a, weights="uniform (None)",
                             err=abs(qu - wantu), tol=0.0))
            assert qu == wantu, (N, a, qu, wantu)
            # the same equal weights passed as an array
            wu = np.ones(N) / N
            qa = float(host(K.weighted_quantile(dev(d), dev(wu), a))[0])
            assert qa == wantu, (N, a, qa, wantu)
    record("golden", rows)
    print(f"max |dq| random weights: "
          f"{max(r['err'] for r in rows if r['weights'] == 'random'):.3e}")


@pytest.mark.parametrize("N", [1, 2, 5, 64, 999, 4096, 100003, 1_000_000])
def test_weighted_quantile_equal_weights_bit_exact(K, N):
    """Equal weights -- none, np.ones(n) / n, and a constant that is not
    1/n (normalised weights of equal particles) -- with continuous and
    heavily tied points, alpha on a grid and at knots: equal to the
    reference's formula (np.argsort, np.cumsum, np.interp) bit for bit."""
    rng = np.random.default_rng(N)
    cont = rng.exponential(size=N) * 3.0
    tied = np.round(rng.normal(size=N) * 4.0) / 4.0
    alphas = [0.0, 1e-9, 0.1, 0.25, 0.5, 0.75, 0.9, 0.999, 1.0] + \
        list(rng.uniform(size=8)) + [(k + 0.5) / N for k in (0, N // 3, N - 1)]
    c = float(np.full(N, 0.37)[0] / np.sum(np.full(N, 0.37)))
    worst = 0.0
    for pts in (cont, tied):
        dd = dev(pts)
        for wname, w in (("none", None), ("ones/n", np.ones(N) / N),
                         ("const", np.full(N, c))):
            wd = None if w is None else dev(w)
            for a in alphas:
                a = float(a)
                q = float(host(K.weighted_quantile(dd, wd, a))[0])
                want = ref.weighted_quantile(pts, None if w is None else w, a)
                worst = max(worst, abs(q - want))
                assert q == want, (N, wname, a, q, want)
    assert worst == 0.0


def _wq_tie_blocks(d, w, alpha, first=np.min, last=np.min):
    """np.interp over knots where each run of equal points is one block
    whose first knot carries ``first`` and whose last knot carries
    ``last`` of the block's weights.  (np.min, np.min) is the device's
    convention for ties; the four (min / max) combinations bracket every
    result an order of the ties can give (the slope into a block edge grows
    with the last weight of the block before it and falls with the first
    weight of the block)."""
    order = np.argsort(d, kind="stable")
    p, ww = d[order], w[order]
    cs = np.cumsum(ww)
    xs, fs = [], []
    start = 0
    for i in range(1, len(p) + 1):
        if i == len(p) or p[i] != p[start]:
            if i - start > 1:
                xs += [(cs[start - 1] if start else 0.0)
                       + 0.5 * first(ww[start:i]),
                       cs[i - 1] - 0.5 * last(ww[start:i])]
                fs += [p[start]] * 2
            else:
                xs += [cs[i - 1] - 0.5 * ww[start]]
                fs += [p[start]]
            start = i
    return float(np.interp(alpha, xs, fs))


def _wq_tie_bracket(d, w, alpha):
    v = [_wq_tie_blocks(d, w, alpha, f, g) for f in (np.min, np.max)
         for g in (np.min, np.max)]
    return min(v), max(v)


def _wq_device_convention(d, w, alpha):
    """The device's general-weight path restated (select.hip
    wq_finalize_kernel: exact 2^62 fixed-point masses, the key whose mass
    interval holds alpha * W, tie blocks with their smallest weight at both
    end knots, the same double operations in the same order): the kernel's
    result bit for bit.  Not the reference -- the convention it follows
    where numpy's unstable argsort leaves the order of ties open."""
    d = np.asarray(d, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64)
    n = d.size
    E = math.frexp(float(n) * float(w.max()))[1]
    fw = np.rint(w * math.ldexp(1.0, 62 - E)).astype(np.uint64)
    order = np.argsort(d, kind="stable")
    ps, fs = d[order], fw[order]
    starts = np.flatnonzero(np.r_[True, ps[1:] != ps[:-1]])
    val = ps[starts]
    bmass = [int(x) for x in np.add.reduceat(fs, starts)]
    bmin = [int(x) for x in np.minimum.reduceat(fs, starts)]
    W = float(sum(bmass))
    t = alpha * W
    rem = 2 ** 64 - 1 if t >= 18446744073709551615.0 else int(t)
    excl = 0
    b = None
    for j, m in enumerate(bmass):
        if excl <= rem < excl + m:
            b = j
            break
        excl += m
    if b is None:
        return float(val[-1])
    pk, w_less, w_eq = float(val[b]), excl, bmass[b]
    wmk = min(bmin[b], w_eq)
    wk = float(wmk) / W
    csk = float(w_less + w_eq) / W
    xk = csk - 0.5 * wk
    xa = xk if wmk == w_eq else float(w_less) / W + 0.5 * wk
    if alpha >= xk:
        if b == len(val) - 1 or alpha == xk:
            return pk
        wn = float(min(bmin[b + 1], bmass[b + 1])) / W
        xn = csk + wn - 0.5 * wn
        slope = (float(val[b + 1]) - pk) / (xn - xk)
        return slope * (alpha - xk) + pk
    if alpha >= xa or b == 0:
        return pk
    pp = float(val[b - 1])
    wp = float(min(bmin[b - 1], bmass[b - 1])) / W
    xp = float(w_less) / W - 0.5 * wp
    if alpha == xp:
        return pp
    slope = (pk - pp) / (xa - xp)
    return slope * (alpha - xp) + pp


@pytest.mark.parametrize("case", ["ties70", "discrete", "zeros", "spike_edges"])
def test_weighted_quantile_ties_large(K, case):
    """N = 1.2e6 with heavy ties (the selected 22-bit bucket overflows the
    candidate buffer: the single-block finish reads the full arrays), few
    distinct values, a block of zero distances and a tie spike, alpha at
    0.1 / 0.5 / 0.9, in the middle of the tied block and at its edges.
    A run of equal points is a block of knots at one p: alpha between its
    first and last knot gives p exactly (weighted_statistics.py:26-43).
    * random weights, alpha away from block edges: the local bound
      (tests/wq_bound.py; 0, i.e. equality, inside a tie block);
    * uniform weights: bit for bit, edges included (equal weights: numpy's
      cumsum restated, the order of ties immaterial);
    * random weights at the block edges: numpy's unstable argsort leaves the
      order of ties open, so parity there is a convention (the block's
      smallest weight at both ends, include/abc_hip.h); the result equals
      that convention restated on the host bit for bit, and both it and the
      reference's result lie between the min- / max-weight placements of
      the edge knots, which bracket every order."""
    import time
    from tests.wq_bound import local_bound, record
    rng = np.random.default_rng({"ties70": 1, "discrete": 2, "zeros": 3,
                                 "spike_edges": 4}[case])
    N = 1_200_000
    if case == "ties70":
        d = np.where(rng.uniform(size=N) < 0.7, 3.0, rng.exponential(size=N) * 5)
    elif case == "discrete":
        d = rng.integers(0, 5, size=N).astype(float)
    elif case == "zeros":
        d = np.where(rng.uniform(size=N) < 0.4, 0.0, rng.uniform(1, 2, size=N))
    else:
        d = np.where(rng.uniform(size=N) < 0.5, 1.5, rng.normal(size=N))
    w = rng.uniform(0.5, 1.5, size=N)
    w /= w.sum()
    pt = {"ties70": 3.0, "discrete": 2.0, "zeros": 0.0, "spike_edges": 1.5}[case]
    below, inb = w[d < pt].sum(), w[d == pt].sum()
    dd, ww = dev(d), dev(w)
    rows = []
    for a in [0.1, 0.5, 0.9, below + 0.5 * inb]:
        a = float(a)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        q = float(host(K.weighted_quantile(dd, ww, a))[0])
        dt = time.perf_counter() - t0
        want = ref.weighted_quantile(d, w, a)
        bound, exact = local_bound(d, w, a)
        tol = 0.0 if exact else 1e-12 * abs(want) + bound
        rows.append(dict(alpha=a, weights="random", err=abs(q - want),
                         tol=tol))
        assert abs(q - want) <= tol, (case, a, q, want, tol)
        print(f"{case} alpha={a:.6f}: q={q!r} want={want!r} tol={tol:.2e} "
              f"({dt * 1e3:.2f} ms incl. host read)")
    assert float(host(K.weighted_quantile(dd, ww, below + 0.5 * inb))[0]) == pt
    # uniform weights: bit for bit, at and around the block edges too
    wu = np.full(N, 1.0 / N)
    cu = float((d < pt).sum()) / N
    cb = float((d == pt).sum()) / N
    for a in [cu, cu + 0.25 / N, cu + 0.5 / N, cu + cb - 0.25 / N,
              cu + cb - 0.5 / N, cu + cb, 0.5, 0.9]:
        a = float(a)
        want = ref.weighted_quantile(d, wu, a)
        q = float(host(K.weighted_quantile(dd, None, a))[0])
        rows.append(dict(alpha=a, weights="uniform", err=abs(q - want),
                         tol=0.0))
        assert q == want, (a, q, want)
    # random weights at the block edges: the convention (bit for bit), and
    # the reference's own result (numpy's order of the ties) inside the
    # bracket of the min- / max-weight placements of the edge knots
    for a in [below + 1e-9, below + inb - 1e-9, below + 0.1 / N,
              below + inb - 0.1 / N]:
        a = float(a)
        q = float(host(K.weighted_quantile(dd, ww, a))[0])
        conv = _wq_device_convention(d, w, a)
        assert q == conv, (a, q, conv)
        lo, hi = _wq_tie_bracket(d, w, a)
        want = ref.weighted_quantile(d, w, a)
        slack = 1e-12 * abs(want) + local_bound(d, w, a)[0]
        assert lo - slack <= want <= hi + slack, (a, want, lo, hi)
        assert lo - slack <= q <= hi + slack, (a, q, lo, hi)
        rows.append(dict(alpha=a, weights="random, tie edge (convention)",
                         err_vs_reference=abs(q - want), bracket=[lo, hi]))
    # the non-edge alphas: the same restatement, bit for bit
    for a in [0.1, 0.5, 0.9]:
        q = float(host(K.weighted_quantile(dd, ww, a))[0])
        assert q == _wq_device_convention(d, w, a), a
    record(f"ties_large_{case}", rows)


def test_weighted_quantile_kat(K):
    """test/test_weighted_statistics.py:6-20 on the device path."""
    pts = dev([1, 5, 2.5])
    w = dev([0.5, 0.2, 0.3])

    def q(a):
        return float(host(K.weighted_quantile(pts, w, a))[0])
    assert 1 < q(0.5) < 2.5
    assert q(0.2) == 1
    assert 2.5 < q(0.8) < 5
    assert q(0.9) == 5
    assert q(1.0) == 5


# ------------------------------------------------ (a8) LocalTransition
@pytest.mark.parametrize("name", [n for n in golden_names("local_")
                                  if not n.startswith("local_rvs")])
def test_local_transition(K, name):
    g = load_golden(name)
    X, w, k = g["X"], g["w"], int(g["k"])
    nbr, d2 = K.knn(dev(X), k)
    np.testing.assert_array_equal(np.sort(host(nbr), axis=1), g["nbr"])
    covs, invs, dets = K.local_cov(dev(X), dev(w), nbr)
    np.testing.assert_allclose(host(covs), g["covs"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(host(dets), g["dets"], rtol=1e-11)
    np.testing.assert_allclose(host(invs), g["inv_covs"], rtol=1e-9,
                               atol=1e-12)
    lp = K.local_logpdf(dev(g["pts"]), dev(X), dev(w), invs, dets)
    np.testing.assert_allclose(np.exp(host(lp)), g["pdf"], rtol=1e-11)


@pytest.mark.parametrize("d,k", [(1, 25), (4, 25), (5, 25), (7, 25), (9, 25),
                                 (3, 1), (1, 3), (6, 9), (6, 64)])
def test_local_cov_all_dims_vs_oracle(K, d, k):
    """local_cov_kernel's per-d register form (d <= 6) and its runtime-d
    form (d = 7..16) against the oracle's smart_cov / det / inv restatement
    (local_transition.py:77-101) on dimensions the goldens do not cover;
    k = 1 (smart_cov's diag(|delta|)), k below, near and above the 8 lanes
    that share a particle's neighbours."""
    rng = np.random.default_rng(40 + d + 100 * k)
    N = 700
    X = rng.normal(size=(N, d)) * rng.uniform(0.5, 2.0, d)
    w = rng.uniform(0.5, 1.5, N)
    w /= w.sum()
    # neighbour rows by numpy (the device kNN stops at d = 8); both sides
    # sum over the same rows in the same order
    d2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    nb = np.argsort(d2, axis=1, kind="stable")[:, :k].astype(np.int32)
    nbr = torch.as_tensor(nb, device="cuda")
    covs, invs, dets = K.local_cov(dev(X), dev(w), nbr)
    rc, ri, rd = ref.local_covs(X, w, nb)
    np.testing.assert_allclose(host(covs), rc, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(host(dets), rd, rtol=1e-11)
    np.testing.assert_allclose(host(invs), ri, rtol=1e-9, atol=1e-12)


# ------------------------------------------------------ simulators
def test_sim_linear_gaussian(K):
    rng = np.random.default_rng(1)
    B, d, S = 3000, 4, 100
    th = rng.normal(size=(B, d))
    A = rng.normal(size=(S, d))
    c = rng.normal(size=S)
    out = host(K.sim_linear_gaussian(dev(th), dev(A), dev(c), 0.5, 17, 4, 10))
    z = ref.philox_normal4_f32(17, 4, (10 + B) * S)[10 * S:].reshape(B, S)
    expect = (th @ A.T + c + 0.5 * z).T
    # the noise is fp32 Box-Muller on the hardware transcendentals: a few
    # fp32 ulps of |z| <= 5.8 (the rest of the model is fp64)
    np.testing.assert_allclose(out, expect, rtol=0, atol=0.5 * 6e-6)
    zz = (out - (th @ A.T + c).T) / 0.5
    assert abs(zz.mean()) < 0.01 and abs(zz.std() - 1) < 0.01


@pytest.mark.parametrize("kind", ["uniform", "lognormal", "zeros", "ties",
                                  "tiny", "steps", "equal", "descending"])
def test_cdf_scan_bit_exact(K, kind):
    """The parallel binade-grid scan equals numpy's sequential cumsum bit for
    bit (then /= cdf[-1]) on adversarial weight vectors."""
    rng = np.random.default_rng({"uniform": 1, "lognormal": 2, "zeros": 3,
                                 "ties": 4, "tiny": 5, "steps": 6, "equal": 7,
                                 "descending": 8}[kind])
    n = 1_000_003
    if kind == "uniform":
        w = rng.uniform(size=n)
    elif kind == "lognormal":
        w = np.exp(rng.normal(size=n) * 6)
    elif kind == "zeros":
        w = rng.uniform(size=n) * (rng.uniform(size=n) < 0.3)
        w[:1000] = 0
    elif kind == "ties":
        # dyadic weights: many increments land exactly half-way on the grid
        w = rng.integers(1, 1 << 12, size=n) * 2.0 ** -40
    elif kind == "equal":
        w = np.full(n, 1.0 / n)         # a prior population's weights
    elif kind == "descending":
        w = np.sort(rng.pareto(1.5, size=n))[::-1].copy()
    elif kind == "tiny":
        w = rng.uniform(size=n) * 1e-300
        w[n // 2:] *= 1e290
    else:
        w = np.repeat(rng.uniform(size=n // 1000 + 1) *
                      10.0 ** rng.integers(-12, 3, size=n // 1000 + 1),
                      1000)[:n]
    w = w / w.sum()
    ref_cdf = ref.resample_cdf(w)
    got = host(K.resample_cdf(dev(w)))
    np.testing.assert_array_equal(got, ref_cdf)


@pytest.mark.parametrize("n", [1, 2, 3, 1023, 1024, 1025, 4097, 2049 * 1024 + 5])
def test_cdf_scan_sizes(K, n):
    """Tile edges of the tiled exact scan (1024-element tiles, 2048 tile
    records per chain batch)."""
    rng = np.random.default_rng(n)
    w = rng.uniform(0.5, 1.5, size=n)
    w /= w.sum()
    np.testing.assert_array_equal(host(K.resample_cdf(dev(w))),
                                  ref.resample_cdf(w))


@pytest.mark.parametrize("k", [50, 64, 150])
@pytest.mark.parametrize("case", ["offset", "clustered", "d1", "d8"])
def test_knn_fp32_filter_exact(K, case, k):
    """The fp32 candidate filter never drops a true neighbour: sets, order
    and distances equal an fp64 brute force (the reference's sub/mul/add
    sequence) on data far from the origin (large fp32 rounding of the
    centred coordinates), near-duplicate clusters and d = 1 / 8; k <= 64
    takes the register-resident merged top-64 (k = 64: tau is its last
    element), k > 64 the 256-slot re-rank."""
    rng = np.random.default_rng({"offset": 1, "clustered": 2, "d1": 3,
                                 "d8": 4}[case])
    n, d = 3000, 6
    if case == "offset":
        X = rng.normal(size=(n, d)) * 1e-3 + 1e3
        X[0] -= 5e3                         # x0 far away: large bound A
    elif case == "clustered":
        X = np.repeat(rng.normal(size=(n // 30, d)), 30, axis=0)
        X += rng.normal(size=X.shape) * 1e-7
    elif case == "d1":
        d = 1
        X = rng.uniform(size=(n, d))
    else:
        d = 8
        X = rng.normal(size=(n, d))
    nbr, d2 = K.knn(dev(X), k)
    nbr, d2 = host(nbr), host(d2)
    diff = X[None, :, :] - X[:, None, :]
    D2 = np.zeros((n, n))
    for q in range(d):                        # sequential, no FMA
        D2 = D2 + diff[:, :, q] * diff[:, :, q]
    np.fill_diagonal(D2, np.inf)
    order = np.lexsort((np.broadcast_to(np.arange(n), (n, n)), D2), axis=1)
    want = order[:, :k]
    np.testing.assert_array_equal(nbr, want)
    np.testing.assert_array_equal(d2, np.take_along_axis(D2, want, axis=1))


def test_native_stream_follows_torch(K):
    """The launch stream the C-ABI calls receive is torch's current stream,
    inside and outside a side-stream context."""
    from pyabc_amd import _native as nat
    raw = lambda: nat.stream().value or 0  # NULL (the default stream) -> 0
    assert raw() == torch.cuda.current_stream().cuda_stream
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        assert raw() == side.cuda_stream != 0
    assert raw() == torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("n,k", [(2, 1), (11, 10), (65, 64), (65, 30),
                                 (130, 100)])
def test_knn_tiny_and_maximal_k(K, n, k):
    """Edge sizes of the kNN pass: one partial tile, k = N - 1 (every other
    particle is a neighbour), k at the 64-slot merge boundary and k > 64 on
    the re-rank path; sets, order and distances equal the fp64 brute force."""
    rng = np.random.default_rng(n * 1000 + k)
    d = 3
    X = rng.normal(size=(n, d))
    nbr, d2 = K.knn(dev(X), k)
    nbr, d2 = host(nbr), host(d2)
    diff = X[None, :, :] - X[:, None, :]
    D2 = np.zeros((n, n))
    for q in range(d):
        D2 = D2 + diff[:, :, q] * diff[:, :, q]
    np.fill_diagonal(D2, np.inf)
    order = np.lexsort((np.broadcast_to(np.arange(n), (n, n)), D2), axis=1)
    want = order[:, :k]
    np.testing.assert_array_equal(nbr, want)
    np.testing.assert_array_equal(d2, np.take_along_axis(D2, want, axis=1))


@pytest.mark.parametrize("prec,rtol", [("f64", 1e-11), ("f32", 1e-5), ("mfma", 1e-5)])
def test_local_logpdf_underflow_fixup(K, prec, rtol):
    """Points far from every particle: the fixed-offset sum underflows and
    the rows go through the exact max-then-sum fixup (log space), matching a
    numpy log-sum-exp of the same terms; near points take the main pass
    (fp64, fp32 pair loop or the z form on the matrix cores)."""
    rng = np.random.default_rng(11)
    n, d, k = 3000, 4, 20
    X = rng.normal(size=(n, d))
    w = rng.uniform(0.1, 1.0, size=n)
    nbr, _ = K.knn(dev(X), k)
    covs, invs, dets = K.local_cov(dev(X), dev(w), nbr)
    pts = np.concatenate([rng.normal(size=(5, d)),
                          np.full((3, d), 25.0) + rng.normal(size=(3, d))])
    got = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets, prec))
    inv, det = host(invs), host(dets)
    diff = pts[:, None, :] - X[None, :, :]
    q = np.einsum("mna,nab,mnb->mn", diff, inv, diff)
    e = np.log(w) - 0.5 * q - 0.5 * np.log((2 * np.pi) ** d * det)
    mx = e.max(axis=1, keepdims=True)
    want = (mx[:, 0] + np.log(np.exp(e - mx).sum(axis=1))) - np.log(w.sum())
    assert np.all(np.isfinite(got))
    # far rows: exact fixup at every precision
    np.testing.assert_allclose(got[5:], want[5:], rtol=1e-11)
    np.testing.assert_allclose(np.exp(got[:5] - want[:5]), 1.0, atol=rtol)


@pytest.mark.parametrize("n", [1, 2, 1023, 300_001])
def test_column_std_block_split(K, n):
    """abc_column_std_ws_f64: S * bps fixed-order partials; np.std to 1e-12
    and bit-identical run to run."""
    rng = np.random.default_rng(n)
    data = rng.normal(3.0, 2.0, size=(n, 7)) * np.array([1, 1e-3, 1e3, 1, 1,
                                                           1, 0])[None, :]
    data[:, 4] = 5.0                      # constant column: std exactly 0
    mean, std = K.column_std(dev(data.T))
    np.testing.assert_allclose(host(mean), data.mean(0), rtol=1e-12,
                               atol=1e-300)
    np.testing.assert_allclose(host(std), np.std(data, axis=0), rtol=1e-12,
                               atol=1e-300)
    assert host(std)[4] == 0.0
    _, std2 = K.column_std(dev(data.T))
    np.testing.assert_array_equal(host(std2), host(std))


@pytest.mark.parametrize("n", [200_000, 200_001])
def test_column_median_mad_skewed(K, n):
    """Wave-aggregated histogram counts: columns where most keys share one
    bin (ties, one dominant value, a tail of distinct values), and ragged
    tails (n not a multiple of 64) -- bit-exact np.median / MAD."""
    rng = np.random.default_rng(n)
    S = 5
    data = np.empty((n, S))
    data[:, 0] = 1.0
    data[:, 1] = np.where(rng.uniform(size=n) < 0.9, 2.5, rng.normal(size=n))
    data[:, 2] = rng.integers(0, 3, size=n).astype(float)
    data[:, 3] = rng.normal(size=n)
    data[:, 4] = np.where(rng.uniform(size=n) < 0.5, -0.0, 1e-300)
    med, mad = K.column_median_mad(dev(data.T))
    np.testing.assert_array_equal(host(med), np.median(data, axis=0))
    mad_ref = np.array([np.median(np.abs(data[:, k] - np.median(data[:, k])))
                        for k in range(S)])
    np.testing.assert_array_equal(host(mad), mad_ref)


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 16384, 16385, 300_001, 2_000_000])
def test_column_median_mad_sampled_splitters(K, n):
    """The sampled-splitter select (one read per order statistic) and its
    radix fallback on column orders and value sets that defeat a strided
    sample: sorted, reversed, sawtooth, constant, three values, a spike of
    ties at the median, and plain normal data -- bit-exact np.median / MAD
    for odd and even n."""
    rng = np.random.default_rng(n)
    cols = [np.sort(rng.normal(size=n)),
            np.sort(rng.normal(size=n))[::-1],
            np.tile(np.arange(97.0), n // 97 + 1)[:n] + 0.5 * (np.arange(n) % 2),
            np.full(n, 3.25),
            rng.integers(0, 3, size=n).astype(float),
            np.where(rng.uniform(size=n) < 0.3, 0.0, rng.normal(size=n)),
            rng.normal(size=n) * 1e-3 + 7.0]
    data = np.stack(cols, axis=1)
    med, mad = K.column_median_mad(dev(data.T))
    want = np.median(data, axis=0)
    np.testing.assert_array_equal(host(med), want)
    mad_ref = np.median(np.abs(data - want[None, :]), axis=0)
    np.testing.assert_array_equal(host(mad), mad_ref)


@pytest.mark.parametrize("prec", ["f32", "mfma"])
@pytest.mark.parametrize("d,offset", [(6, 0.0), (6, 40.0), (2, 0.0), (8, 3.0),
                                      (4, 0.0), (5, 1.0), (1, 0.0)])
def test_local_logpdf_f32_vs_exact(K, d, offset, prec):
    """precision="f32" LocalTransition density (pair loop in fp32, centred on
    X[0]) and precision="mfma" (z form on the f16 matrix cores): within 1e-5
    relative of the exact fp64 density (north_star's fp32 bar), including
    far points (exact fixup) and an offset population."""
    rng = np.random.default_rng(d * 7 + int(offset))
    n, k = 4000, 50
    X = rng.normal(size=(n, d)) @ (np.eye(d) + 0.4 * rng.normal(size=(d, d)))
    X += offset
    w = rng.uniform(0.1, 1.0, size=n)
    nbr, _ = K.knn(dev(X), k)
    covs, invs, dets = K.local_cov(dev(X), dev(w), nbr)
    pts = np.concatenate([X[rng.integers(0, n, 300)] +
                          0.3 * rng.normal(size=(300, d)),
                          rng.normal(size=(20, d)) * 3 + offset,
                          np.full((3, d), 30.0 + offset)])
    exact = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets))
    got = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets,
                              precision=prec))
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(np.exp(got - exact), 1.0, atol=1e-5)


@pytest.mark.parametrize("prec", ["f32", "mfma"])
@pytest.mark.parametrize("d", [3, 6])
def test_local_logpdf_f32_rows_independent(K, d, prec):
    """The fp32 pass cuts the particle range into chunks that depend on N
    only: a row's bits do not depend on which rows share its call (a subset
    in another order, a single row, duplicated rows), as the row-sharded
    generation needs."""
    rng = np.random.default_rng(90 + d)
    n, k = 20_000, 30
    X = rng.normal(size=(n, d))
    w = rng.uniform(0.1, 1.0, size=n)
    nbr, _ = K.knn(dev(X), k)
    covs, invs, dets = K.local_cov(dev(X), dev(w), nbr)
    pts = np.concatenate([X[rng.integers(0, n, 3000)] +
                          0.2 * rng.normal(size=(3000, d)),
                          rng.normal(size=(100, d)) * 4])
    full = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets, prec))
    sub = rng.permutation(len(pts))[:777]
    part = host(K.local_logpdf(dev(pts[sub]), dev(X), dev(w), invs, dets, prec))
    np.testing.assert_array_equal(part, full[sub])
    one = host(K.local_logpdf(dev(pts[sub[:1]]), dev(X), dev(w), invs, dets, prec))
    np.testing.assert_array_equal(one, full[sub[:1]])
    dup = np.repeat(pts[:50], 3, axis=0)
    got = host(K.local_logpdf(dev(dup), dev(X), dev(w), invs, dets, prec))
    np.testing.assert_array_equal(got, np.repeat(full[:50], 3))
    exact = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets))
    np.testing.assert_allclose(np.exp(full - exact), 1.0, atol=1e-5)


@pytest.mark.parametrize("d", [3, 6, 8])
def test_local_mfma_launch_knobs_bit_identical(K, d, monkeypatch):
    """The z-form pass's launch knobs (local_mfma.hip lz_run: ABC_LZ_IB point
    tiles per wave, ABC_LZ_TPB particle tiles per LDS buffer) only change the
    launch shape: every row is bit-identical under each."""
    rng = np.random.default_rng(130 + d)
    n, k = 12_000, 40
    X = rng.normal(size=(n, d))
    w = rng.uniform(0.1, 1.0, size=n)
    nbr, _ = K.knn(dev(X), k)
    covs, invs, dets = K.local_cov(dev(X), dev(w), nbr)
    pts = np.concatenate([X[rng.integers(0, n, 2000)] +
                          0.2 * rng.normal(size=(2000, d)),
                          rng.normal(size=(50, d)) * 4])
    base = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets, "mfma"))
    exact = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets))
    np.testing.assert_allclose(np.exp(base - exact), 1.0, atol=1e-5)
    for env in ({"ABC_LZ_IB": "2"}, {"ABC_LZ_IB": "1"}, {"ABC_LZ_TPB": "2"},
                {"ABC_LZ_TPB": "8"}, {"ABC_LZ_IB": "2", "ABC_LZ_TPB": "8"}):
        for key, val in env.items():
            monkeypatch.setenv(key, val)
        K.reload_tuning()
        got = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets, "mfma"))
        for key in env:
            monkeypatch.delenv(key)
        K.reload_tuning()
        np.testing.assert_array_equal(got, base, err_msg=str(env))


@pytest.mark.parametrize("d", [2, 6])
def test_knn_rows_tiled_equal_full(K, d):
    """Row ranges of the tiled kNN (the rank shares of the sharded fit) give
    the rows of the full call, and both equal an fp64 brute force on a
    sample of rows."""
    rng = np.random.default_rng(70 + d)
    n, k = 30_000, 50
    X = rng.normal(size=(n, d)) * np.linspace(0.5, 2.0, d)
    nbr, d2 = K.knn(dev(X), k)
    nbr, d2 = host(nbr), host(d2)
    for lo, m in [(0, 1), (12_345, 4321), (n - 77, 77)]:
        nb, dd = K.knn_rows(dev(X), k, lo, m)
        np.testing.assert_array_equal(host(nb), nbr[lo:lo + m])
        np.testing.assert_array_equal(host(dd), d2[lo:lo + m])
    # rows per wave (tuning knob ABC_KNN_ROWS): the same sets and distances
    for rpw in ("8",):
        os.environ["ABC_KNN_ROWS"] = rpw
        K.reload_tuning()
        try:
            nb, dd = K.knn(dev(X), k)
        finally:
            os.environ.pop("ABC_KNN_ROWS", None)
            K.reload_tuning()
        np.testing.assert_array_equal(host(nb), nbr, err_msg=rpw)
        np.testing.assert_array_equal(host(dd), d2, err_msg=rpw)
    rows = rng.choice(n, 200, replace=False)
    diff = X[None, :, :] - X[rows, None, :]
    D2 = np.zeros((len(rows), n))
    for q in range(d):
        D2 = D2 + diff[:, :, q] * diff[:, :, q]
    D2[np.arange(len(rows)), rows] = np.inf
    order = np.lexsort((np.broadcast_to(np.arange(n), D2.shape), D2), axis=1)
    np.testing.assert_array_equal(nbr[rows], order[:, :k])


@pytest.mark.parametrize("prec", ["f32", "mfma"])
@pytest.mark.parametrize("d,spread", [(6, 1e3), (3, 1e4), (8, 3e3)])
def test_local_logpdf_f32_wide_population(K, d, spread, prec):
    """A population whose extent is >= 1e3 local bandwidths (small k, far
    apart clusters, X[0] at one end): the fp32 pass's (hi, lo) centred
    coordinates keep it within 1e-5 of the exact fp64 density (a single
    fp32 rounding of x - X[0] would cost ~ sqrt(q) (R / sigma) 2^-23)."""
    rng = np.random.default_rng(int(spread) + d)
    # k >= 3d: with k = 10 at d = 8 the local covariances are near-singular
    # and the fp32 quadratic form's own conditioning (not the centring)
    # reaches 1.2e-5 on single rows -- kde_precision="f64" covers that case
    n_cl, per, k = 40, 100, max(10, 3 * d)
    centres = rng.uniform(-spread, spread, size=(n_cl, d))
    X = np.concatenate([c + rng.normal(size=(per, d)) for c in centres])
    X[0] = -spread                      # the centring anchor at the edge
    n = X.shape[0]
    w = rng.uniform(0.1, 1.0, size=n)
    nbr, _ = K.knn(dev(X), k)
    covs, invs, dets = K.local_cov(dev(X), dev(w), nbr)
    sig = np.sqrt(np.min(np.linalg.eigvalsh(host(covs)), axis=1))
    R = np.abs(X - X[0]).max()
    assert R / np.median(sig) > 1e3
    pts = X[rng.integers(1, n, 400)] + 0.5 * rng.normal(size=(400, d)) * \
        np.median(sig)
    exact = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets))
    got = host(K.local_logpdf(dev(pts), dev(X), dev(w), invs, dets,
                              precision=prec))
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(np.exp(got - exact), 1.0, atol=1e-5)


# ------------------------------------- SURVEY 8(b) minimum-set entry points
def _nat():
    from pyabc_amd import _native as nat
    return nat


def _ws(nbytes):
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device="cuda")


def test_philox_fill_reproduces_production_proposals(K):
    """abc_philox_fill hands out exactly the draws abc_propose_philox_f64
    makes in-kernel: injecting them into abc_resample_perturb_f64 gives the
    same indices, draws and support flags bit for bit."""
    nat = _nat()
    rng = np.random.default_rng(21)
    N, d, B = 3000, 5, 20000
    X = rng.normal(size=(N, d))
    w = rng.uniform(size=N)
    w /= w.sum()
    A = ref.svd_factor(ref.mvn_fit_cov(X, w))
    lo, sc = np.full(d, -2.0), np.full(d, 4.0)
    cdf = K.resample_cdf(dev(w))
    seed, sid, off = 99, 5, 777
    th, idx, sup = K.propose_philox(dev(X), cdf, dev(A), dev(lo), dev(sc),
                                    seed, sid, off, B)
    u = torch.empty(B, dtype=torch.float64, device="cuda")
    z = torch.empty(B * d, dtype=torch.float64, device="cuda")
    nat.call("abc_philox_fill", seed, sid, off, u.data_ptr(), B, z.data_ptr(),
             B * d, nat.stream())
    np.testing.assert_array_equal(host(u), ref.philox_uniform(
        seed, 2 * sid, off + B)[off:])
    th2, idx2, sup2 = K.resample_perturb(dev(X), cdf, u, z.view(B, d), dev(A),
                                         dev(lo), dev(sc))
    np.testing.assert_array_equal(host(idx2), host(idx))
    np.testing.assert_array_equal(host(th2), host(th))
    np.testing.assert_array_equal(host(sup2), host(sup))
    z32 = torch.empty(B * d, dtype=torch.float32, device="cuda")
    nat.call("abc_philox_fill_f32", seed, sid, off, u.data_ptr(), B,
             z32.data_ptr(), B * d, nat.stream())
    np.testing.assert_array_equal(host(z32), host(z).astype(np.float32))


def test_resample_perturb_f32(K):
    """fp32 storage: indices bit-exact with the fp64 oracle on the same u;
    theta within fp32 rounding of the oracle on the fp32 inputs; support
    flags equal wherever theta is not within fp32 rounding of a bound."""
    nat = _nat()
    rng = np.random.default_rng(22)
    N, d, B = 4096, 8, 30000
    X = rng.normal(size=(N, d)).astype(np.float32)
    w = rng.uniform(size=N)
    w /= w.sum()
    A = ref.svd_factor(ref.mvn_fit_cov(X.astype(np.float64), w)).astype(
        np.float32)
    u = rng.uniform(size=B)
    z = rng.normal(size=(B, d)).astype(np.float32)
    lo, sc = np.full(d, -2.5), np.full(d, 5.0)
    cdf = K.resample_cdf(dev(w))
    th = torch.empty((B, d), dtype=torch.float32, device="cuda")
    idx = torch.empty(B, dtype=torch.int64, device="cuda")
    sup = torch.empty(B, dtype=torch.uint8, device="cuda")
    Xd, zd, Ad = (dev(a, torch.float32) for a in (X, z, A))
    ud, lod, scd = dev(u), dev(lo), dev(sc)   # alive until the kernel ran
    nat.call("abc_resample_perturb_f32", Xd.data_ptr(), N, d, cdf.data_ptr(),
             ud.data_ptr(), zd.data_ptr(), Ad.data_ptr(), lod.data_ptr(),
             scd.data_ptr(), B, th.data_ptr(), idx.data_ptr(), sup.data_ptr(),
             nat.stream())
    torch.cuda.synchronize()
    idx_ref = ref.resample_indices(ref.resample_cdf(w), u)
    np.testing.assert_array_equal(host(idx), idx_ref)
    th_ref = X[idx_ref].astype(np.float64) + z.astype(np.float64) @ \
        A.astype(np.float64)
    scale = np.abs(X[idx_ref]).astype(np.float64) + np.abs(z).astype(
        np.float64) @ np.abs(A).astype(np.float64)
    err = np.abs(host(th) - th_ref)
    assert np.all(err <= (d + 2) * 2.0 ** -24 * scale)
    s_ref = ref.uniform_box_support(host(th).astype(np.float64), lo, sc)
    np.testing.assert_array_equal(host(sup).astype(bool), s_ref)


@pytest.mark.parametrize("d", [3, 8, 12])
def test_weighted_moments_f32(K, d):
    """fp32 X, w: the fp64 moments of the widened values (1e-12)."""
    nat = _nat()
    rng = np.random.default_rng(23 + d)
    n = 50001
    X = (rng.normal(size=(n, d)) * 2 + 1).astype(np.float32)
    w = rng.uniform(0.2, 1.0, n).astype(np.float32)
    out = torch.empty(2 + d + d * d, dtype=torch.float64, device="cuda")
    wsb = nat.lib().abc_moments_workspace_bytes(d)
    ws = _ws(wsb)
    Xd, wd = dev(X, torch.float32), dev(w, torch.float32)
    nat.call("abc_weighted_moments_f32", Xd.data_ptr(), wd.data_ptr(), n, d,
             out.data_ptr(), ws.data_ptr(), wsb, nat.stream())
    o = host(out)
    X64, w64 = X.astype(np.float64), w.astype(np.float64)
    np.testing.assert_allclose(o[0], w64.sum(), rtol=1e-12)
    np.testing.assert_allclose(o[1], (w64 ** 2).sum(), rtol=1e-12)
    mu = (w64[:, None] * X64).sum(0) / w64.sum()
    np.testing.assert_allclose(o[2:2 + d], mu, rtol=1e-12)
    C = ((X64 - mu) * w64[:, None]).T @ (X64 - mu)
    np.testing.assert_allclose(o[2 + d:].reshape(d, d), C, rtol=1e-11,
                               atol=1e-9)


@pytest.mark.parametrize("d", [1, 4, 8, 20])
def test_kde_logsum(K, d):
    """abc_kde_logsum_{f32,f64}: log_offset + log sum_j exp(logw_j -
    |y_i - y_j|^2 / 2) on pre-whitened rows: 1e-12 relative
    for fp64, 1e-5 relative (of the sum) for fp32."""
    nat = _nat()
    rng = np.random.default_rng(30 + d)
    N, M = 3001, 700
    Yp = rng.normal(size=(N, d)) * 1.5
    Yn = np.concatenate([Yp[:M - 50] + 0.1 * rng.normal(size=(M - 50, d)),
                         rng.normal(size=(50, d)) * 4])
    logw = np.log(rng.uniform(0.1, 1.0, N)) - 3.0
    off = 0.75
    d2 = ((Yn[:, None, :] - Yp[None, :, :]) ** 2).sum(-1)
    a = logw[None, :] - 0.5 * d2
    m = a.max(1)
    want = off + m + np.log(np.exp(a - m[:, None]).sum(1))
    for T, name, tol in ((np.float64, "f64", 1e-12), (np.float32, "f32", 1e-5)):
        tt = torch.float64 if T is np.float64 else torch.float32
        wsb = getattr(nat.lib(), f"abc_kde_logsum_workspace_bytes_{name}")(
            M, N, d)
        ws = _ws(wsb)
        out = torch.empty(M, dtype=tt, device="cuda")
        a1, a2, a3 = (dev(x.astype(T), tt) for x in (Yn, Yp, logw))
        nat.call(f"abc_kde_logsum_{name}", a1.data_ptr(), a2.data_ptr(),
                 a3.data_ptr(), M, N, d, float(off), out.data_ptr(),
                 ws.data_ptr(), wsb, nat.stream())
        got = host(out).astype(np.float64)
        if T is np.float32:
            # the reference value of the fp32-rounded inputs
            Yn32, Yp32, lw32 = (x.astype(np.float32).astype(np.float64)
                                for x in (Yn, Yp, logw))
            d2 = ((Yn32[:, None, :] - Yp32[None, :, :]) ** 2).sum(-1)
            a = lw32[None, :] - 0.5 * d2
            m = a.max(1)
            want32 = np.float32(off) + m + np.log(np.exp(a - m[:, None]).sum(1))
            err = np.abs(got - want32)
            bad = err > tol + 4e-7 * np.abs(want32)
            assert not bad.any(), (name, np.flatnonzero(bad)[:5],
                                   got[bad][:5], want32[bad][:5])
        else:
            np.testing.assert_allclose(got, want, rtol=tol, atol=tol)


def test_knn_topk_and_local_cov_f32(K):
    """fp32 storage kNN / local covariances: neighbour sets of the fp32
    points equal a brute force; covariances equal the fp64 kernel's on the
    widened points rounded to fp32."""
    nat = _nat()
    rng = np.random.default_rng(41)
    N, d, k = 1500, 6, 20
    X = rng.normal(size=(N, d)).astype(np.float32)
    w = rng.uniform(0.5, 1.5, N).astype(np.float32)
    nbr = torch.empty((N, k), dtype=torch.int32, device="cuda")
    d2 = torch.empty((N, k), dtype=torch.float32, device="cuda")
    wsb = nat.lib().abc_knn_topk_f32_workspace_bytes(N, d, k)
    ws = _ws(wsb)
    Xd, wd = dev(X, torch.float32), dev(w, torch.float32)
    nat.call("abc_knn_topk_f32", Xd.data_ptr(), N, d, k, nbr.data_ptr(),
             d2.data_ptr(), ws.data_ptr(), wsb, nat.stream())
    want = ref.knn_indices(X.astype(np.float64), k)
    got = host(nbr)
    for i in range(N):
        assert set(got[i]) == set(want[i])
    X64 = X.astype(np.float64)
    dd = ((X64[want] - X64[:, None, :]) ** 2).sum(-1)
    np.testing.assert_allclose(np.sort(host(d2), 1), np.sort(dd, 1),
                               rtol=1e-6)
    C = torch.empty((N, d, d), dtype=torch.float32, device="cuda")
    Ci = torch.empty_like(C)
    dt = torch.empty(N, dtype=torch.float32, device="cuda")
    wsb = nat.lib().abc_local_cov_f32_workspace_bytes(N, d)
    ws = _ws(wsb)
    nat.call("abc_local_cov_f32", Xd.data_ptr(), wd.data_ptr(), N, d,
             nbr.data_ptr(), k, 1.0, C.data_ptr(), Ci.data_ptr(),
             dt.data_ptr(), ws.data_ptr(), wsb, nat.stream())
    covs, invs, dets = ref.local_covs(X64, w.astype(np.float64), host(nbr))
    np.testing.assert_allclose(host(C), covs, rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(host(dt), dets, rtol=1e-5)
    np.testing.assert_allclose(host(Ci), invs, rtol=1e-4, atol=1e-4)
