"""Exact-inference path on the CPU: the oracle against
the reference's golden vectors, and the host-side schemes / pdf norms against
the reference's values and its own known-answer tests
(``test/test_acceptor.py:117-147``, ``test/test_epsilon.py:56-163``).

Fixtures: ``tools/gen_golden.py`` (gen_stochastic, gen_temperature) ran the
reference pyabc 0.10.1 in the build container.
"""
import os
import tempfile

import numpy as np
import pandas as pd
import pytest

from oracle import ref_cpu as ref
from tests.conftest import load_golden

import pyabc_amd as pa


# ------------------------------------------------------------ oracle pins
@pytest.mark.parametrize("S", [5, 100, 300])
def test_oracle_independent_kernels_bit_exact(S):
    g = load_golden(f"stoch_kernel_S{S}")
    np.testing.assert_array_equal(
        ref.independent_normal_logpdf(g["X"], g["x0"], g["var"]), g["normal"])
    np.testing.assert_array_equal(
        ref.independent_laplace_logpdf(g["X"], g["x0"], g["scale"]),
        g["laplace"])
    # pdf_max = density at x_0
    np.testing.assert_array_equal(
        ref.independent_normal_logpdf(g["x0"][None], g["x0"], g["var"])[0],
        g["normal_pdf_max"])


def test_oracle_pairwise_sum_is_numpy():
    rng = np.random.default_rng(5)
    for n in [0, 1, 7, 8, 9, 100, 128, 129, 136, 300, 1000, 4096]:
        a = rng.random(n) * rng.random(n) * 1e3
        assert ref.np_pairwise_sum(a) == np.sum(a)


@pytest.mark.parametrize("scale", ["log", "lin"])
@pytest.mark.parametrize("temp", [1.0, 3.7])
@pytest.mark.parametrize("iw", [1, 0])
def test_oracle_stochastic_accept_bit_exact(scale, temp, iw):
    g = load_golden("stoch_accept")
    tag = f"{scale}_T{temp}_iw{iw}"
    _, acc, w = ref.stochastic_accept(g["pd_" + scale],
                                      float(g["pdf_max_" + scale]), temp,
                                      g["u_" + tag], scale == "log", bool(iw))
    np.testing.assert_array_equal(acc, g["accept_" + tag])
    np.testing.assert_array_equal(w, g["weight_" + tag])


@pytest.mark.parametrize("rate", [0.3, 0.05, 0.9])
def test_oracle_acceptance_rate_scheme(rate):
    g = load_golden("temperature")
    v = ref.acceptance_rate_temperature(g["pds"], g["tpp"], g["tp"],
                                        float(g["pds"].max()), True, rate)
    assert v == g[f"accrate_{rate}_log"]
    lin = np.exp(g["pds"] / 10)
    v = ref.acceptance_rate_temperature(lin, g["tpp"], g["tp"],
                                        float(lin.max()), False, rate)
    assert v == g[f"accrate_{rate}_lin"]


# ------------------------------------------------ host schemes vs reference
_SCHEMES = {"expiter": pa.ExpDecayFixedIterScheme,
            "expratio": pa.ExpDecayFixedRatioScheme,
            "poly": pa.PolynomialDecayFixedIterScheme,
            "daly": pa.DalyScheme, "friel": pa.FrielPettittScheme}


@pytest.mark.parametrize("name", sorted(_SCHEMES))
def test_scalar_schemes_match_reference(name):
    g = load_golden("temperature")
    for t, prev, rate in [(1, 50., 0.4), (3, 12.5, 1e-5), (2, 7.3, 0.7)]:
        s = _SCHEMES[name]()
        got = s(t=t, get_weighted_distances=None, get_all_records=None,
                max_nr_populations=6, pdf_norm=0.0,
                kernel_scale=pa.SCALE_LOG, prev_temperature=prev,
                acceptance_rate=rate)
        assert got == g[f"{name}_t{t}"], (name, t)


def test_schemes_without_previous_temperature():
    """test/test_epsilon.py:150-163: no base temperature -> inf."""
    for cls in _SCHEMES.values():
        assert cls()(t=0, get_weighted_distances=None, get_all_records=None,
                     max_nr_populations=3, pdf_norm=0.0,
                     kernel_scale=pa.SCALE_LOG, prev_temperature=None,
                     acceptance_rate=0.3) == np.inf
    s = pa.ExpDecayFixedIterScheme()
    assert s(t=2, get_weighted_distances=None, get_all_records=None,
             max_nr_populations=3, pdf_norm=0.0, kernel_scale=pa.SCALE_LOG,
             prev_temperature=7.53, acceptance_rate=0.4) == 1.0
    with pytest.raises(ValueError):
        s(t=2, get_weighted_distances=None, get_all_records=None,
          max_nr_populations=np.inf, pdf_norm=0.0, kernel_scale=pa.SCALE_LOG,
          prev_temperature=7.53, acceptance_rate=0.4)


def test_list_temperature():
    """test/test_epsilon.py:56-62."""
    eps = pa.ListTemperature(values=[10, 5, 1.5])
    assert eps(0) == 10
    assert eps(2) == 1.5


def test_temperature_initial_and_final_values():
    """Temperature bookkeeping without the data-driven schemes: initial value,
    monotone fallback, exact final temperature, log file
    (test/test_epsilon.py:65-91 with scalar schemes)."""
    log_file = tempfile.mkstemp(suffix=".json")[1]
    cfg = {"pdf_norm": 5, "kernel_scale": pa.SCALE_LOG}
    eps = pa.Temperature(schemes=[pa.ExpDecayFixedIterScheme(),
                                  pa.DalyScheme()],
                         initial_temperature=42, log_file=log_file)
    eps.initialize(0, None, None, 3, cfg)
    assert eps(0) == 42
    eps.update(1, None, None, 0.4, cfg)
    assert 1 < eps(1) < 42
    eps.update(2, None, None, 0.2, cfg)
    assert eps(2) == 1
    proposed = pa.storage.load_dict_from_json(log_file)
    assert proposed[0][0] == 42
    assert len(proposed[1]) == 2
    assert len(proposed[2]) == 1
    os.remove(log_file)


def test_pdf_norm_methods():
    """test/test_acceptor.py:117-147 (reference known answers)."""
    def wd():
        return pd.DataFrame({"distance": [1, 2, 3, 4], "w": [2, 1, 1, 0]})
    args = dict(kernel_val=42, prev_pdf_norm=3.5, get_weighted_distances=wd,
                prev_temp=10.3, acceptance_rate=0.3)
    assert pa.pdf_norm_max_found(**args) == 4
    assert pa.pdf_norm_from_kernel(**args) == 42
    assert pa.ScaledPDFNorm()(**args) == 4
    args["prev_pdf_norm"] = 4.5
    args["acceptance_rate"] = 0.05
    assert pa.pdf_norm_max_found(**args) == 4.5
    assert pa.ScaledPDFNorm()(**args) == 4.5 - np.log(10) * 0.5 * 10.3


def test_pdf_norms_match_reference_fixture():
    g = load_golden("temperature")
    df = pd.DataFrame({"distance": g["wd_d"], "w": g["wd_w"]})
    assert pa.pdf_norm_max_found(prev_pdf_norm=-3.0,
                                 get_weighted_distances=lambda: df) \
        == g["pdfnorm_maxfound"]
    s = pa.ScaledPDFNorm()
    assert s(prev_pdf_norm=-30.0, get_weighted_distances=lambda: df,
             prev_temp=5.0, acceptance_rate=0.5) == g["pdfnorm_scaled_hi"]
    assert s(prev_pdf_norm=-30.0, get_weighted_distances=lambda: df,
             prev_temp=5.0, acceptance_rate=0.01) == g["pdfnorm_scaled_lo"]


def test_kernel_api_errors():
    with pytest.raises(ValueError):
        pa.SimpleFunctionKernel(lambda **kw: 0.0, ret_scale="SCALE_X")
    with pytest.raises(ValueError):
        pa.BinomialKernel(p=1.5)


def test_discrete_kernels_host():
    """BinomialKernel / PoissonKernel semantics (kernel.py:360-470;
    closure-sampler path, scipy pmfs as the reference)."""
    import scipy.stats as st
    x0 = {"a": 3, "b": 7}
    x = {"a": 5, "b": 9}
    k = pa.BinomialKernel(p=0.6)
    k.initialize(0, None, x0)
    assert k(x, x0) == np.sum(st.binom.logpmf(k=[3, 7], n=[5, 9], p=0.6))
    k = pa.PoissonKernel(ret_scale=pa.SCALE_LIN)
    k.initialize(0, None, x0)
    assert k(x, x0) == np.prod(st.poisson.pmf(k=[3, 7], mu=[5, 9]))
