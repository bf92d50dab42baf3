"""Temperature schemes for exact-inference ABC with the StochasticAcceptor
(API of pyabc/epsilon/temperature.py:1-742).

The schemes that look at whole populations -- the AcceptanceRateScheme over
all recorded evaluations (smc.py:990-1017) and the EssScheme over the
weighted population -- evaluate their objectives with one device reduction
per objective call (``abc_tempered_sums_f64``); the records' transition
densities come from the device KDE pass (``DeviceRecords``).  The root /
minimum search around the objective is the reference's own scipy call, so
the search path is the reference's.
"""
import logging
import numbers

import numpy as np
import scipy.optimize
import torch

from . import kernels as K
from .acceptor import save_dict_to_json
from .distance import SCALE_LIN
from .epsilon import Epsilon

logger = logging.getLogger("Epsilon")


class DeviceRecords:
    """``get_all_records()`` of a device generation (smc.py:990-1017):
    every recorded evaluation's distance (the kernel density), the previous
    and the current transition log-densities of its parameter, and its
    acceptance flag, as device columns.  Iterates as the reference's list of
    dicts on demand."""

    def __init__(self, distance, log_transition_pd_prev, log_transition_pd,
                 accepted):
        self.distance = distance
        self.log_transition_pd_prev = log_transition_pd_prev
        self.log_transition_pd = log_transition_pd
        self.accepted = accepted

    def __len__(self):
        return self.distance.numel()

    def to_list(self):
        d = self.distance.cpu().numpy()
        a = torch.exp(self.log_transition_pd_prev).cpu().numpy()
        b = torch.exp(self.log_transition_pd).cpu().numpy()
        acc = self.accepted.cpu().numpy()
        return [{"distance": d[i], "transition_pd_prev": a[i],
                 "transition_pd": b[i], "accepted": bool(acc[i])}
                for i in range(d.size)]

    def __iter__(self):
        return iter(self.to_list())


def _dev():
    return torch.device("cuda", torch.cuda.current_device())


class _TemperedSums:
    """Device inputs of a tempered objective: densities and particle weights
    (linear, or the ratio of two log-densities)."""

    def __init__(self, pd, w=None, lnum=None, lden=None):
        self.pd, self.w, self.lnum, self.lden = pd, w, lnum, lden

    @staticmethod
    def from_records(records):
        if isinstance(records, DeviceRecords):
            return _TemperedSums(records.distance,
                                 lnum=records.log_transition_pd,
                                 lden=records.log_transition_pd_prev)
        pds = np.array([r["distance"] for r in records], dtype=float)
        tpp = np.array([r["transition_pd_prev"] for r in records], dtype=float)
        tp = np.array([r["transition_pd"] for r in records], dtype=float)
        return _TemperedSums(torch.as_tensor(pds, device=_dev()),
                             w=torch.as_tensor(tp / tpp, device=_dev()))

    @staticmethod
    def from_weighted_distances(df):
        d = getattr(df, "distance_tensor", None)
        if d is not None:
            return _TemperedSums(d, w=df.w_tensor)
        return _TemperedSums(
            torch.as_tensor(np.array(df["distance"], dtype=float),
                            device=_dev()),
            w=torch.as_tensor(np.array(df["w"], dtype=float), device=_dev()))

    def __len__(self):
        return self.pd.numel()

    def sums(self, c, beta, log_scale, clamp):
        """(sum w, sum w v^beta, sum (w v^beta)^2) as host floats."""
        out = K.tempered_sums(self.pd, c, [beta], w=self.w,
                              logw_num=self.lnum, logw_den=self.lden,
                              log_scale=log_scale, clamp=clamp).cpu().numpy()
        return out[0, 0], out[1, 0], out[1, 1]


class TemperatureBase(Epsilon):
    """Base of the temperature schemes (temperature.py:16-22)."""


class ListTemperature(TemperatureBase):
    """Temperatures given as a list (temperature.py:25-42)."""

    def __init__(self, values):
        super().__init__()
        self.values = values

    def __call__(self, t):
        return self.values[t]


class Temperature(TemperatureBase):
    """Adaptive temperature (temperature.py:45-192): each generation's
    temperature is the aggregate (default min) of the schemes' proposals,
    never above the previous one and never below 1; the last generation of a
    finite run is forced to 1."""

    def __init__(self, schemes=None, aggregate_fun=None,
                 initial_temperature=None,
                 enforce_exact_final_temperature=True, log_file=None):
        super().__init__()
        self.schemes = schemes
        self.aggregate_fun = aggregate_fun if aggregate_fun is not None \
            else min
        self.initial_temperature = initial_temperature \
            if initial_temperature is not None else AcceptanceRateScheme()
        self.enforce_exact_final_temperature = enforce_exact_final_temperature
        self.log_file = log_file
        self.max_nr_populations = None
        self.temperatures = {}
        self.temperature_proposals = {}

    def initialize(self, t, get_weighted_distances, get_all_records,
                   max_nr_populations, acceptor_config):
        self.max_nr_populations = max_nr_populations
        if self.schemes is None:
            acc_rate_scheme = AcceptanceRateScheme()
            decay_scheme = (ExpDecayFixedIterScheme()
                            if np.isfinite(max_nr_populations)
                            else ExpDecayFixedRatioScheme())
            self.schemes = [acc_rate_scheme, decay_scheme]
        self._update(t, get_weighted_distances, get_all_records, 1.0,
                     acceptor_config)

    def configure_sampler(self, sampler):
        if callable(self.initial_temperature):
            self.initial_temperature.configure_sampler(sampler)
        for scheme in self.schemes:
            scheme.configure_sampler(sampler)

    def update(self, t, get_weighted_distances, get_all_records,
               acceptance_rate, acceptor_config):
        self._update(t, get_weighted_distances, get_all_records,
                     acceptance_rate, acceptor_config)

    def _initial(self, **kwargs):
        init = self.initial_temperature
        if callable(init):
            return init(**kwargs)
        if isinstance(init, numbers.Number):
            return init
        raise ValueError("Initial temperature must be a float or a callable")

    def _update(self, t, get_weighted_distances, get_all_records,
                acceptance_rate, acceptor_config):
        kwargs = dict(t=t, get_weighted_distances=get_weighted_distances,
                      get_all_records=get_all_records,
                      max_nr_populations=self.max_nr_populations,
                      pdf_norm=acceptor_config["pdf_norm"],
                      kernel_scale=acceptor_config["kernel_scale"],
                      prev_temperature=self.temperatures.get(t - 1),
                      acceptance_rate=acceptance_rate)
        last = t >= self.max_nr_populations - 1
        if last and self.enforce_exact_final_temperature:
            proposals = [1.0]
        elif self.temperatures:
            proposals = [scheme(**kwargs) for scheme in self.schemes]
        else:
            proposals = [self._initial(**kwargs)]
        # never above the previous temperature, never below 1
        ceiling = self.temperatures.get(t - 1, np.inf)
        value = max(min(self.aggregate_fun(proposals), ceiling), 1.0)
        if not np.isfinite(value):
            raise ValueError("Temperature must be finite.")
        self.temperatures[t] = value
        self.temperature_proposals[t] = proposals
        logger.debug(f"Proposed temperatures for {t}: {proposals}.")
        if self.log_file:
            save_dict_to_json(self.temperature_proposals, self.log_file)

    def __call__(self, t):
        return self.temperatures[t]


class TemperatureScheme:
    """Proposes the next temperature (temperature.py:195-239)."""

    def __init__(self):
        pass

    def configure_sampler(self, sampler):
        pass

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        pass


class AcceptanceRateScheme(TemperatureScheme):
    """Temperature whose predicted acceptance rate over all recorded
    evaluations, importance-weighted by t_pd / t_pd_prev, is
    ``target_rate`` (temperature.py:242-303)."""

    def __init__(self, target_rate=0.3, min_rate=None):
        super().__init__()
        self.target_rate = target_rate
        self.min_rate = min_rate

    def configure_sampler(self, sampler):
        sampler.sample_factory.record_rejected = True

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if self.min_rate is not None and acceptance_rate < self.min_rate:
            return np.inf
        src = _TemperedSums.from_records(get_all_records())
        return match_acceptance_rate(src, pdf_norm, kernel_scale,
                                     self.target_rate)


def match_acceptance_rate(src, pdf_norm, kernel_scale, target_rate):
    """Root of sum(w/W min((pd/c)^beta, 1)) - target in b = log(beta) on
    [-100, 0] by scipy's bisect (temperature.py:306-345); every objective
    value is one device reduction."""
    log_scale = kernel_scale != SCALE_LIN

    def obj(b):
        W, A, _ = src.sums(pdf_norm, float(np.exp(b)), log_scale, True)
        return A / W - target_rate

    min_b = -100
    if obj(0) > 0:
        b_opt = 0
    elif obj(min_b) < 0:
        logger.info("AcceptanceRateScheme: Numerics limit temperature.")
        b_opt = min_b
    else:
        b_opt = scipy.optimize.bisect(obj, min_b, 0, maxiter=100000)
    return 1. / np.exp(b_opt)


class ExpDecayFixedIterScheme(TemperatureScheme):
    """T_j = T_{j-1}^((n-j)/(n-j+1)) (temperature.py:348-398)."""

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if max_nr_populations == np.inf:
            raise ValueError(
                "The ExpDecayFixedIterScheme requires a finite "
                "`max_nr_populations`.")
        if prev_temperature is None:
            return np.inf
        t_to_go = max_nr_populations - t
        return prev_temperature ** ((t_to_go - 1) / t_to_go)


class ExpDecayFixedRatioScheme(TemperatureScheme):
    """T_j = alpha T_{j-1}, alpha adapted to the acceptance rate
    (temperature.py:401-465)."""

    def __init__(self, alpha=0.5, min_rate=1e-4, max_rate=0.5):
        super().__init__()
        self.alpha = alpha
        self.min_rate = min_rate
        self.max_rate = max_rate
        self.alphas = {}

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if prev_temperature is None:
            return np.inf
        a = self.alphas.get(t - 1, self.alpha)
        if t > 1 and acceptance_rate > self.max_rate:
            # accepting easily: cool faster (halve alpha, or more)
            a = max(a / 2, a - 2 * (1 - a))
        if acceptance_rate < self.min_rate:
            # barely accepting: move alpha half-way towards 1
            a = a + (1 - a) / 2
        self.alphas[t] = a
        return a * prev_temperature


class PolynomialDecayFixedIterScheme(TemperatureScheme):
    """Pre-last entry of linspace(1, T^(1/e), t_to_go + 1)^e
    (temperature.py:468-531)."""

    def __init__(self, exponent=3):
        super().__init__()
        self.exponent = exponent

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if prev_temperature is None:
            return np.inf
        if max_nr_populations == np.inf:
            raise ValueError("Can only perform PolynomialDecayScheme step "
                             "with a finite max_nr_populations.")
        t_to_go = max_nr_populations - t
        temps = np.linspace(1, prev_temperature ** (1 / self.exponent),
                            t_to_go + 1) ** self.exponent
        return temps[-2]


class DalyScheme(TemperatureScheme):
    """Decrease sqrt(T) by k = min(k, alpha sqrt(T))
    (temperature.py:534-600)."""

    def __init__(self, alpha=0.5, min_rate=1e-4):
        super().__init__()
        self.alpha = alpha
        self.min_rate = min_rate
        self.k = {}

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if prev_temperature is None:
            return np.inf
        root = np.sqrt(prev_temperature)
        step = self.k[t - 1] if self.k else root
        if not self.k:
            self.k[t - 1] = root
        if acceptance_rate < self.min_rate:
            step = self.alpha * step
        self.k[t] = min(step, self.alpha * root)
        return (root - self.k[t]) ** 2


class FrielPettittScheme(TemperatureScheme):
    """beta = beta_{j-1} + ((1 - beta_{j-1}) / t_to_go)^2
    (temperature.py:603-639)."""

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        if prev_temperature is None:
            return np.inf
        if max_nr_populations == np.inf:
            raise ValueError("Can only perform FrielPettittScheme step with a "
                             "finite max_nr_populations.")
        beta = 1. / prev_temperature
        remaining = max_nr_populations - t
        beta = beta + ((1. - beta) / remaining) ** 2
        return 1. / beta


class EssScheme(TemperatureScheme):
    """Temperature keeping the relative effective sample size of the
    reweighted population at ``target_relative_ess``
    (temperature.py:642-742): scipy's bounded minimize of
    (ESS(beta) - target)^2, every ESS one device reduction."""

    def __init__(self, target_relative_ess=0.8):
        super().__init__()
        self.target_relative_ess = target_relative_ess

    def __call__(self, t, get_weighted_distances, get_all_records,
                 max_nr_populations, pdf_norm, kernel_scale,
                 prev_temperature, acceptance_rate):
        src = _TemperedSums.from_weighted_distances(get_weighted_distances())
        log_scale = kernel_scale != SCALE_LIN
        target_ess = len(src) * self.target_relative_ess
        beta_base = 0.0 if prev_temperature is None \
            else 1. / prev_temperature

        def obj(beta):
            _, A, Q = src.sums(pdf_norm, float(np.ravel(beta)[0]), log_scale,
                               False)
            return (A ** 2 / Q - target_ess) ** 2

        bounds = scipy.optimize.Bounds(lb=np.array([beta_base]),
                                       ub=np.array([1.]))
        ret = scipy.optimize.minimize(
            obj, x0=np.array([0.5 * (1 + beta_base)]), bounds=bounds)
        return float(1. / ret.x[0])
