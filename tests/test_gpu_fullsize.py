"""Full-size parity of the default KDE pass (exact-grid bf16 MFMA) at the
configurations the headline numbers are quoted on.

Reference: MultivariateNormalTransition.pdf (pyabc/transition/
multivariatenormal.py:102-125) via smc.py:722-733.  Tolerance (BASELINE
north star, fp32 kernel): 1e-5 relative on the transition density.

The population is the bench's own (LinearGaussianModel.benchmark, prior
population then ``GENS`` device generations), so bandwidth, grid g and the
spread of |y| are those of the timed run.  Two checks per configuration:

* every one of the M rows against the fp64 HIP pass (itself pinned at
  1e-12 against the reference's golden densities, test_gpu_kernels.py);
* sampled rows against the numpy oracle (oracle/ref_cpu.kde_logsum):
  random rows, the lowest-density tail rows, the rows with the largest
  max|y| (closest to the grid edge), and constructed rows displaced
  outward from the population's most extreme particle so that the largest
  exponent sits at -10 ... -70 (the rows where one fp32 rounding of e costs
  most), plus rows just inside and beyond the grid range (exact fixup).

Measured maxima are written to gpurun_out/kde_fullsize_parity.json when that
directory exists (DESIGN.md quotes them).
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu as ref

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RTOL = 1e-5


def _bench_population(d, N, gens, seed=2024):
    """Prior population + ``gens`` generations of the bench workload; returns
    the fit used by the last generation and that generation's result."""
    from pyabc_amd import kernels as K
    from pyabc_amd.batch_models import LinearGaussianModel
    from pyabc_amd.engine import GenerationEngine, DeviceMVNFit
    S = 100
    model = LinearGaussianModel.benchmark(d, S)
    x0 = torch.as_tensor(model._x0, device="cuda")
    fw = torch.ones(S, dtype=torch.float64, device="cuda")
    eng = GenerationEngine(model, np.full(d, -5.0), np.full(d, 10.0),
                           distance_p=2.0, seed=seed)
    r0 = eng.sample_prior(0, N)
    d0, _, _ = K.pnorm_distance(r0.stats_T, x0, fw, 2.0, math.inf,
                                with_accept=False)
    w = torch.full((N,), 1.0 / N, dtype=torch.float64, device="cuda")
    eps = float(K.weighted_quantile(d0, w, 0.5)[0].item())
    fit = DeviceMVNFit(r0.theta, w)
    res = None
    for t in range(1, gens + 1):
        prev = fit
        res = eng.sample_generation(t, N, fit, x0, fw, eps)
        th, dd, ww, _, _ = eng.gather_population(res)
        eps = float(K.weighted_quantile(dd, ww, 0.5)[0].item())
        fit = DeviceMVNFit(th, ww)
    return prev, res


def _rel_err(lp_a, lp_b):
    """|pd_a / pd_b - 1| from log densities."""
    return np.abs(np.expm1(np.asarray(lp_a) - np.asarray(lp_b)))


def _constructed_rows(fit, rng):
    """Rows displaced outward from the most extreme particle so that the
    largest exponent is about -E (log2 units), E = 10 ... 70, and rows just
    inside / beyond the grid range 256 g."""
    X = fit.X.cpu().numpy()
    mu = fit.packed.mu.cpu().numpy()
    Us = fit.packed.Us.cpu().numpy()          # y = (x - mu) Us  (log2 units)
    Uinv = np.linalg.pinv(Us)
    Y = (X - mu) @ Us
    r2 = np.sum(Y * Y, axis=1)
    rows = []
    for j in np.argsort(r2)[-4:]:
        u = Y[j] / math.sqrt(r2[j])
        for E in (10, 20, 30, 40, 50, 58, 62, 70):
            rows.append(Y[j] + math.sqrt(E) * u)
        # random directions around a central particle
        c = Y[rng.integers(0, len(Y))]
        for E in (15, 35, 55):
            v = rng.normal(size=Y.shape[1])
            rows.append(c + math.sqrt(E) * v / np.linalg.norm(v))
    g = float(fit.packed.gscale.item())
    k = int(np.argmax(np.abs(Y).max(0)))
    for f in (250.0, 255.9, 256.1, 300.0):
        y = Y[np.argmax(np.abs(Y[:, k]))].copy()
        y[k] = math.copysign(f * g, y[k])
        rows.append(y)
    Yc = np.array(rows)
    return mu + Yc @ Uinv, g


def _check(d, N, gens, n_random, n_tail, n_edge, tag):
    from pyabc_amd import kernels as K
    rng = np.random.default_rng(1000 + d)
    fit, res = _bench_population(d, N, gens)
    assert fit.packed.precision == "mfma"
    theta = res.theta
    M = theta.shape[0]
    lp_mfma = res.logpd.cpu().numpy()          # the production pass's output
    pp64 = K.PackedPopulation(fit.X, fit.w, fit.packed.mu, fit.packed.Us,
                              fit.rank, fit.log_pdet, "f64")
    lp64 = pp64.logpdf(theta).cpu().numpy()
    err_all = _rel_err(lp_mfma, lp64)
    worst = int(np.argmax(err_all))

    # sampled rows against the numpy oracle
    th = theta.cpu().numpy()
    Yn = (th - fit.packed.mu.cpu().numpy()) @ fit.packed.Us.cpu().numpy()
    pick = set(rng.choice(M, n_random, replace=False).tolist())
    pick |= set(np.argsort(lp64)[:n_tail].tolist())
    pick |= set(np.argsort(np.abs(Yn).max(1))[-n_edge:].tolist())
    pick.add(worst)
    pick = np.array(sorted(pick))
    extra, g = _constructed_rows(fit, rng)
    rows = np.concatenate([th[pick], extra])
    lp_rows_mfma = np.concatenate([
        lp_mfma[pick], fit.packed.logpdf(torch.as_tensor(
            extra, device="cuda")).cpu().numpy()])
    lp_rows_64 = np.concatenate([
        lp64[pick], pp64.logpdf(torch.as_tensor(extra, device="cuda"))
        .cpu().numpy()])
    U, rank, log_pdet = ref.psd_whitening(fit.cov)
    X = fit.X.cpu().numpy()
    w = fit.w.cpu().numpy()
    lp_ref = ref.kde_logsum(rows @ U, X @ U, np.log(w)) \
        - 0.5 * (rank * ref.LOG_2PI + log_pdet)
    err_ref = _rel_err(lp_rows_mfma, lp_ref)
    err_64_ref = _rel_err(lp_rows_64, lp_ref)
    # rows the MFMA pass hands to the exact fp64 fixup (sum below 2^-32 of
    # the largest weight's scale)
    off = math.log(2) * float(fit.packed.lw2max.item()) + fit.packed.log_const
    n_fix = int(np.sum(lp64 - off < -32 * math.log(2)))
    stats = dict(
        tag=tag, d=d, N=int(fit.n), M=int(M), gens=gens, grid_g=g,
        n_fixup_rows=n_fix,
        max_abs_y_new=float(np.abs(Yn).max()),
        max_rel_err_all_rows_vs_f64=float(err_all.max()),
        p99_rel_err_all_rows_vs_f64=float(np.quantile(err_all, 0.99)),
        worst_row=worst, worst_row_logpd=float(lp64[worst]),
        n_oracle_rows=int(len(rows)),
        max_rel_err_sampled_vs_oracle=float(err_ref.max()),
        max_rel_err_constructed_vs_oracle=float(
            err_ref[len(pick):].max()),
        max_rel_err_f64_kernel_vs_oracle=float(err_64_ref.max()),
        min_logpd_constructed=float(lp_ref[len(pick):].min()))
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        path = os.path.join(out, "kde_fullsize_parity.json")
        old = []
        if os.path.exists(path):
            with open(path) as f:
                old = [r for r in json.load(f) if r.get("tag") != tag]
        with open(path, "w") as f:
            json.dump(old + [stats], f, indent=1)
    print(json.dumps(stats))
    assert err_64_ref.max() < 1e-11, stats
    assert err_all.max() < RTOL, stats
    assert err_ref.max() < RTOL, stats


@pytest.mark.timeout(240)
def test_kde_mfma_headline_config_d8():
    """N = M = 1e6, d = 8: the bench's generation, every row."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _check(8, 1_000_000, 4, n_random=384, n_tail=96, n_edge=64, tag="d8_N1e6")


@pytest.mark.timeout(240)
def test_kde_mfma_c5_dim_d20():
    """N = M = 262144, d = 20 (config 5's dimension)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _check(20, 262_144, 4, n_random=384, n_tail=96, n_edge=64,
           tag="d20_N262144")
