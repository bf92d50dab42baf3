"""AdaptivePopulationSize (reference
pyabc/populationstrategy.py:140-358, cv/bootstrap.py, cv/powerlaw.py).

CPU: the CV formula and the power-law fit against the reference's outputs
(tests/golden/cv_bootstrap.npz, tools/gen_golden.py gen_cv), the oracle's
bootstrap KDE against the reference's fit_cov + pdf_static, and the strategy's
host path with a numpy transition.  GPU: the device bootstrap chain (Philox
draws -> moments kernel -> KDE pass) against the oracle on the same draws,
and an ABCSMC run that adapts its population size.
"""
import numpy as np
import pytest

from oracle import ref_cpu as ref
from pyabc_amd.populationstrategy import (AdaptivePopulationSize,
                                          calc_variation, fitpowerlaw,
                                          bootstrap_densities)
from tests.conftest import load_golden


def test_calc_variation_and_powerlaw_vs_reference():
    g = load_golden("cv_bootstrap")
    n = g["boots"].shape[1]
    cv = calc_variation([g["dens"]], np.array([n]), g["test_w"][None, :])
    np.testing.assert_allclose(cv, g["cv"], rtol=1e-13)
    cv2 = calc_variation([g["dens"], g["dens2"]], np.array([n, 3 * n]),
                         np.vstack([g["test_w"], g["test_w"][::-1]]))
    np.testing.assert_allclose(cv2, g["cv2"], rtol=1e-13)
    popt, f, finv = fitpowerlaw(g["xs"], g["ys"])
    np.testing.assert_allclose(popt, g["popt"], rtol=1e-6)
    np.testing.assert_allclose(finv(0.05), g["n_at_005"], rtol=1e-6)


def test_oracle_bootstrap_kde_vs_reference():
    g = load_golden("cv_bootstrap")
    n = g["boots"].shape[1]
    w0 = np.ones(n) / n
    for b in range(g["boots"].shape[0]):
        cov = ref.mvn_fit_cov(g["boots"][b], w0)
        np.testing.assert_allclose(cov, g["covs"][b], rtol=1e-12)
        dens = ref.kde_transition_pd(g["test_X"], g["boots"][b], w0, cov)
        np.testing.assert_allclose(dens, g["dens"][b], rtol=1e-10)


class _NumpyKDE:
    """Minimal host Transition (rvs / fit / pdf) for the generic path."""

    def __init__(self):
        self.rng = np.random.default_rng(3)

    def fit(self, X, w):
        self.X = np.asarray(X, dtype=float)
        self.w = np.asarray(w, dtype=float) / np.sum(w)
        self.cov = ref.mvn_fit_cov(self.X, self.w)

    def rvs(self, size=None):
        idx = self.rng.choice(len(self.X), size=size, p=self.w)
        L = np.linalg.cholesky(self.cov)
        return self.X[idx] + self.rng.normal(size=(size, self.X.shape[1])) @ L.T

    def pdf(self, x):
        return ref.kde_transition_pd(np.asarray(x), self.X, self.w, self.cov)


def test_adaptive_population_size_host_path():
    rng = np.random.default_rng(0)
    tr = _NumpyKDE()
    X = rng.normal(size=(300, 2))
    tr.fit(X, np.ones(300) / 300)
    np.random.seed(1)
    aps = AdaptivePopulationSize(300, mean_cv=0.05, n_bootstrap=4,
                                 max_population_size=5000,
                                 min_population_size=50)
    est = aps.predict_population_size(np.array([1.0]), [tr], n_steps=5)
    assert est.n_samples_list == list(range(100, 600, 60))
    cvs = np.asarray(est.cvs)
    assert np.all(cvs > 0) and cvs[0] > cvs[-1]   # CV falls with n
    aps.update([tr], np.array([1.0]), t=1)
    assert 50 <= aps() <= 5000
    assert aps(-1) == aps()
    cfg = aps.get_config()
    assert cfg["mean_cv"] == 0.05 and cfg["n_bootstrap"] == 4
    assert AdaptivePopulationSize(10, nr_calibration_particles=7)(-1) == 7


@pytest.mark.gpu
def test_device_bootstrap_chain_vs_oracle():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pyabc_amd import kernels as K
    from pyabc_amd.engine import DeviceMVNFit
    from pyabc_amd.transition import MultivariateNormalTransition
    g = load_golden("cv_bootstrap")
    dv = lambda a: torch.as_tensor(a, dtype=torch.float64, device="cuda")
    n = g["boots"].shape[1]
    # fit + KDE pass on the reference's own bootstrap samples
    for b in range(g["boots"].shape[0]):
        f = DeviceMVNFit(dv(g["boots"][b]), dv(np.ones(n) / n))
        np.testing.assert_allclose(f.cov, g["covs"][b], rtol=1e-12)
        dens = torch.exp(f.logpdf(dv(g["test_X"]))).cpu().numpy()
        np.testing.assert_allclose(dens, g["dens"][b], rtol=1e-5)
    # the device loop: re-draw the same Philox samples, check with the oracle
    tr = MultivariateNormalTransition()
    tr.fit(g["test_X"], g["test_w"])
    got = bootstrap_densities(tr, g["test_X"], 150, 3, seed=1234)
    fit = tr.device_fit
    for b in range(3):
        Xb, _, _ = K.propose_philox(fit.X, fit.cdf, fit.A, None, None, 1234,
                                    16 + b, 0, 150)
        Xb = Xb.cpu().numpy()
        w0 = np.ones(150) / 150
        want = ref.kde_transition_pd(g["test_X"], Xb, w0,
                                     ref.mvn_fit_cov(Xb, w0))
        np.testing.assert_allclose(got[b], want, rtol=1e-5)


@pytest.mark.gpu
def test_abcsmc_adaptive_population_size_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pyabc_amd as pa
    np.random.seed(2)
    prior = pa.Distribution(mean=pa.RV("uniform", 0, 5))
    aps = pa.AdaptivePopulationSize(500, mean_cv=0.1, n_bootstrap=5,
                                    min_population_size=300,
                                    max_population_size=4000)
    abc = pa.ABCSMC(pa.GaussianMeanModel(), prior, pa.PNormDistance(p=2),
                    population_size=aps, eps=pa.MedianEpsilon(),
                    sampler=pa.GPUBatchSampler(seed=4))
    abc.new("mem://aps", {"data": 2.5})
    h = abc.run(minimum_epsilon=0.2, max_nr_populations=4)
    sizes = h.get_nr_particles_per_population()
    assert len(sizes) >= 3
    assert all(300 <= int(s) <= 4000 for s in list(sizes)[1:])
    assert aps.last_estimate is not None and len(aps.last_estimate.cvs) > 0
    df, w = h.distribution_numpy(0, h.max_t)
    w = w / w.sum()
    m = float((df["mean"].values * w).sum())
    ess = 1.0 / float((w ** 2).sum())
    # posterior ~ N(2.5, 0.5^2): Monte Carlo bound from the weights' ESS
    assert abs(m - 2.5) < 4 * 0.5 / np.sqrt(ess) + 0.05, (m, ess)


@pytest.mark.gpu
def test_visualization_kde_grids_vs_reference():
    """kde_1d / kde_2d / kde_matrix grids (visualization/kde.py) through the
    device KDE pass vs the reference's own outputs (fp32-class KDE: 1e-5)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pandas as pd
    from pyabc_amd.visualization import kde_1d, kde_2d, kde_matrix
    g = load_golden("vis_kde")
    df = pd.DataFrame({"a": g["a"], "b": g["b"]})
    x1, pdf1 = kde_1d(df, g["w"], "a", numx=40)
    np.testing.assert_array_equal(x1, g["x1"])
    np.testing.assert_allclose(pdf1, g["pdf1"], rtol=1e-5)
    x1l, pdf1l = kde_1d(df, g["w"], "b", xmin=-1, xmax=9, numx=33)
    np.testing.assert_allclose(pdf1l, g["pdf1l"], rtol=1e-5, atol=1e-300)
    X, Y, PDF = kde_2d(df, g["w"], "a", "b", numx=20, numy=15)
    np.testing.assert_array_equal(X, g["X"])
    np.testing.assert_array_equal(Y, g["Y"])
    np.testing.assert_allclose(PDF, g["PDF"], rtol=1e-5)
    grids = kde_matrix(df, g["w"], numx=20, numy=15)
    np.testing.assert_allclose(grids[("a", "b")][2], g["PDF"], rtol=1e-5)
    assert set(grids) == {("a", "a"), ("b", "b"), ("a", "b"), ("b", "a")}
