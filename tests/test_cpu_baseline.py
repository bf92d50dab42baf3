"""The bench's CPU baseline leg (oracle/cpu_baseline.py) runs end to end on
a tiny generation: rate, physical-core count, the t(N) = aN + bN^2 fit and
the one-core KDE pairs/s are reported."""
import numpy as np

from oracle import cpu_baseline as cb
from oracle import ref_cpu as ref


def test_cpu_baseline_small_generation(tmp_path):
    rng = np.random.default_rng(0)
    N, d, S = 3000, 2, 5
    X = rng.normal(size=(N, d))
    w = rng.uniform(0.5, 1.5, N)
    w /= w.sum()
    cov = ref.mvn_fit_cov(X, w)
    A_model = rng.normal(size=(S, d))
    x0 = np.zeros(S)
    # two generations: every fit size runs the same schedule
    out = cb.run([(X, w, cov, 3.0), (X, w, cov, 2.5)], A_model, x0,
                 np.full(d, -5.0),
                 np.full(d, 10.0), 0.5, workers=2, seconds=0.6,
                 tmpdir=str(tmp_path), fit_sizes=(300, 1000, 2000),
                 fit_seconds=0.3, kde_dims=(2,), kde_n_prev=20000)
    assert out["workers"] == 2
    assert out["physical_cores"] >= 1
    assert out["rate"] > 0
    assert out["rate_all_physical_cores_ideal"] == \
        out["rate"] / 2 * out["physical_cores"]
    fit = out["tN_fit"]
    assert fit["sizes"] == [300, 1000, 2000] and fit["n"] == N
    assert fit["t_generation_extrapolated_s"] > 0
    assert len(out["per_generation"]) == 2
    assert fit["rate_measured"] == out["rate"]
    assert fit["fit_with_measured_n"]["rate_at_n"] > 0
    assert set(fit["us_per_accepted_per_prev_particle"]) == {
        "300", "1000", "2000", str(N)}
    assert out["kde_pairs_per_s_1core"]["d2"] > 0
    assert not list(tmp_path.iterdir())      # generation files removed


def test_physical_cores_and_share():
    assert cb.physical_cores() >= 1
    assert 1 <= cb.cpu_share()
