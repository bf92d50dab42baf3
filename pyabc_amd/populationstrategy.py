"""Population sizes (API of pyabc/populationstrategy.py:33-392).

AdaptivePopulationSize runs its bootstrap KDE
evaluations on the device: every bootstrap population is drawn by the Philox
proposal kernel, fitted by the weighted-moments kernel and evaluated at the
test points by the KDE pass (a3) -- the reference fans the same work out to
dask `pdf_static` blocks (populationstrategy.py:288-345, cv/bootstrap.py).
"""
import copy
import json
import logging
from typing import Callable, List, NamedTuple

import numpy as np

from .distributed import agree_int

logger = logging.getLogger("Adaptation")


class PopulationStrategy:
    def __init__(self, nr_particles, *, nr_samples_per_parameter=1):
        self.nr_particles = nr_particles
        self.nr_samples_per_parameter = nr_samples_per_parameter

    def update(self, transitions, model_weights, t=None):
        pass

    def __call__(self, t=None):
        return self.nr_particles

    def get_config(self):
        return {"name": self.__class__.__name__,
                "nr_particles": self.nr_particles}

    def to_json(self):
        return json.dumps(self.get_config())


class ConstantPopulationSize(PopulationStrategy):
    pass


class ListPopulationSize(PopulationStrategy):
    def __init__(self, values, *, nr_samples_per_parameter=1):
        super().__init__(nr_particles=list(values)[0],
                         nr_samples_per_parameter=nr_samples_per_parameter)
        self.values = list(values)

    def __call__(self, t=None):
        return self.values[t] if t is not None and t >= 0 else self.values[0]

    def get_config(self):
        return {"name": self.__class__.__name__,
                "population_values": self.values}


# --------------------------------------------------------------------------
# adaptive population size (populationstrategy.py:140-358, cv/*.py)
# --------------------------------------------------------------------------
class CVEstimate(NamedTuple):
    """populationstrategy.py CVEstimate: the suggested size, the probed
    sizes, their coefficients of variation and the fitted power law."""
    n_estimated: float
    n_samples_list: List[int]
    cvs: List[float]
    f: Callable = None
    popt: tuple = None


def power_law(x, a, b):
    """cv/powerlaw.py:5-6"""
    return a * x ** (-b)


def finverse(y, a, b):
    """cv/powerlaw.py:9-10"""
    return (a / y) ** (1 / b)


def fitpowerlaw(x, y):
    """cv/powerlaw.py:13-18 (scipy curve_fit, p0 = [.5, 1/5])."""
    from scipy.optimize import curve_fit
    popt, _ = curve_fit(power_law, np.array(x), np.array(y), p0=[.5, 1 / 5])
    return popt, lambda x: power_law(x, *popt), lambda y: finverse(y, *popt)


def calc_variation(per_model_w, n_per_model, test_w):
    """cv/bootstrap.py:12-32: scipy variation (std/mean, ddof 0) of the
    bootstrapped densities at each test point, weighted by the model's share
    of the samples and by the test point weights, summed."""
    from scipy import stats as st
    variations_at_X = np.stack([st.variation(ws, axis=0)
                                for ws in per_model_w])
    n_per_model = np.asarray(n_per_model)
    model_weighted = (variations_at_X * n_per_model[:, np.newaxis]
                      / np.sum(n_per_model))
    return (model_weighted * test_w).sum()


def _host(a):
    try:
        import torch
        if isinstance(a, torch.Tensor):
            return a.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(getattr(a, "values", a))


def bootstrap_densities(transition, test_X, n, n_bootstrap, seed=None):
    """[n_bootstrap, len(test_X)] densities of KDEs fitted (uniform weights)
    to n draws from `transition`, evaluated at test_X
    (populationstrategy.py:318-340 / cv/bootstrap.py:138-144).

    For the GPU MultivariateNormalTransition the whole loop stays on the
    device (Philox draws, moments kernel, KDE pass); any other Transition
    goes through its own rvs / fit / pdf."""
    if n == 0:  # model not drawn: zero variation, zero share
        return np.ones((n_bootstrap, len(test_X)))
    fit = getattr(transition, "device_fit", None)
    if fit is not None and hasattr(fit, "packed"):
        import torch
        from . import kernels as K
        from .engine import DeviceMVNFit
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 62))
        test = fit.X
        out = torch.empty((n_bootstrap, test.shape[0]), dtype=torch.float64,
                          device=test.device)
        for b in range(n_bootstrap):
            X_b, _, _ = K.propose_philox(fit.X, fit.cdf, fit.A, None, None,
                                         seed, 16 + b, 0, n)
            w_b = torch.full((n,), 1.0 / n, dtype=torch.float64,
                             device=test.device)
            f_b = DeviceMVNFit(X_b, w_b, transition.scaling,
                               transition.bandwidth_selector,
                               transition.kde_precision)
            out[b] = torch.exp(f_b.logpdf(test))
        return out.cpu().numpy()
    dens = []
    for _ in range(n_bootstrap):
        bootstr_X = transition.rvs(size=n)
        t_b = copy.deepcopy(transition)
        t_b.fit(bootstr_X, np.ones(len(bootstr_X)) / len(bootstr_X))
        dens.append(np.asarray(t_b.pdf(test_X), dtype=float))
    return np.stack(dens)


class AdaptivePopulationSize(PopulationStrategy):
    """Mean-CV population size adaptation (Klinger & Hasenauer 2017) with
    the reference's signature and semantics (populationstrategy.py:140-358).
    `client` is accepted for API compatibility and ignored: the bootstrap
    KDE evaluations run on the GPU instead of a dask cluster."""

    def __init__(self, start_nr_particles, mean_cv=0.05,
                 max_population_size=np.inf, min_population_size=10,
                 nr_samples_per_parameter=1, n_bootstrap=10,
                 nr_calibration_particles=None, client=None):
        super().__init__(start_nr_particles,
                         nr_samples_per_parameter=nr_samples_per_parameter)
        self.nr_calibration_particles = nr_calibration_particles
        self.start_nr_particles = start_nr_particles
        self.max_population_size = max_population_size
        self.min_population_size = min_population_size
        self.mean_cv = mean_cv
        self.n_bootstrap = n_bootstrap
        self.nr_particles = start_nr_particles
        self.last_estimate = None

    def get_config(self):
        return {"name": self.__class__.__name__,
                "nr_calibration_particles": self.nr_calibration_particles,
                "nr_samples_per_parameter": self.nr_samples_per_parameter,
                "start_nr_particles": self.start_nr_particles,
                "max_population_size": self.max_population_size,
                "min_population_size": self.min_population_size,
                "mean_cv": self.mean_cv,
                "n_bootstrap": self.n_bootstrap}

    def update(self, transitions, model_weights, t=None):
        """populationstrategy.py:218-229"""
        est = self.predict_population_size(np.asarray(model_weights),
                                           transitions)
        self.last_estimate = est
        ref = self.nr_particles
        if not np.isnan(est.n_estimated):
            self.nr_particles = max(min(int(est.n_estimated),
                                        self.max_population_size),
                                    self.min_population_size)
        # the estimate draws from numpy's global state (multinomial split,
        # bootstrap seeds); under torchrun every rank takes rank 0's size,
        # since the generation's collectives assume one n
        self.nr_particles = agree_int(self.nr_particles)
        logger.info(f"Change nr particles {ref} -> {self.nr_particles}")

    def __call__(self, t=None):
        if t == -1 and self.nr_calibration_particles is not None:
            return self.nr_calibration_particles
        return self.nr_particles

    def predict_population_size(self, model_weights, transitions, n_steps=10,
                                first_step_factor=3):
        """populationstrategy.py:237-358: probe sizes
        range(cur // first_step_factor, 2 cur, cur // n_steps), split each
        over the models by a multinomial draw, bootstrap n_bootstrap KDEs per
        model, CV at the models' own particles, fit cv(n) = a n^-b and
        invert at the target."""
        test_Xs = [tr.X for tr in transitions]
        test_w = np.vstack([_host(tr.w) for tr in transitions])
        cur = self.nr_particles
        if cur == 1:
            return CVEstimate(1, [], [], None, None)
        start = max(cur // first_step_factor, 1)
        stop = cur * 2
        step = max(cur // n_steps, 1)
        n_samples_list = list(range(start, stop, step))
        cvs = []
        for ns in n_samples_list:
            n_per_model = np.random.multinomial(ns, model_weights)
            per_model = [bootstrap_densities(tr, X, int(n), self.n_bootstrap)
                         for n, tr, X in zip(n_per_model, transitions,
                                             test_Xs)]
            cvs.append(calc_variation(per_model, n_per_model, test_w))
        try:
            popt, f, finv = fitpowerlaw(n_samples_list, cvs)
            return CVEstimate(finv(self.mean_cv), n_samples_list, cvs, f,
                              popt)
        except RuntimeError:
            logger.warning("Power law fit failed. Falling back to current "
                           f"nr particles {cur}")
            return CVEstimate(cur, n_samples_list, cvs, None, None)
