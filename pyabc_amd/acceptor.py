"""Acceptors (API of pyabc/acceptor/acceptor.py:1-473, pdf_norm.py:1-110).
The batch sampler applies the uniform acceptance d <= eps(t) inside the
distance kernel and the stochastic acceptance inside the density kernel."""
import json
import logging

import numpy as np

logger = logging.getLogger("Acceptor")


class AcceptorResult(dict):
    def __init__(self, distance, accept, weight=1.0):
        super().__init__(distance=distance, accept=accept, weight=weight)

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError:
            raise AttributeError(key)

    __setattr__ = dict.__setitem__


class Acceptor:
    def __init__(self):
        pass

    def initialize(self, t, get_weighted_distances, distance_function, x_0):
        pass

    def update(self, t, get_weighted_distances, prev_temp, acceptance_rate):
        pass

    def __call__(self, distance_function, eps, x, x_0, t, par):
        raise NotImplementedError()

    def get_epsilon_config(self, t):
        return None

    @staticmethod
    def assert_acceptor(maybe_acceptor):
        return SimpleFunctionAcceptor.assert_acceptor(maybe_acceptor)


class SimpleFunctionAcceptor(Acceptor):
    def __init__(self, fun):
        super().__init__()
        self.fun = fun

    def __call__(self, distance_function, eps, x, x_0, t, par):
        return self.fun(distance_function, eps, x, x_0, t, par)

    @staticmethod
    def assert_acceptor(maybe_acceptor):
        if isinstance(maybe_acceptor, Acceptor):
            return maybe_acceptor
        return SimpleFunctionAcceptor(maybe_acceptor)


def accept_use_current_time(distance_function, eps, x, x_0, t, par):
    """d <= eps(t) (acceptor.py:235-244)."""
    d = distance_function(x, x_0, t, par)
    return AcceptorResult(distance=d, accept=d <= eps(t))


def accept_use_complete_history(distance_function, eps, x, x_0, t, par):
    d = distance_function(x, x_0, t, par)
    accept = d <= eps(t)
    if accept:
        for t_prev in range(0, t):
            try:
                accept = distance_function(x, x_0, t_prev, par) <= eps(t_prev)
                if not accept:
                    break
            except Exception:
                accept = True
    return AcceptorResult(distance=d, accept=accept)


class UniformAcceptor(Acceptor):
    def __init__(self, use_complete_history=False):
        super().__init__()
        self.use_complete_history = use_complete_history

    def __call__(self, distance_function, eps, x, x_0, t, par):
        if self.use_complete_history:
            return accept_use_complete_history(distance_function, eps, x,
                                               x_0, t, par)
        return accept_use_current_time(distance_function, eps, x, x_0, t, par)


# ---------------------------------------------------------------------------
# stochastic acceptance (acceptor/acceptor.py:309-473, pdf_norm.py:1-110)
# ---------------------------------------------------------------------------
def _distances(get_weighted_distances):
    df = get_weighted_distances()
    d = df["distance"]
    return np.asarray(d, dtype=np.float64)


def pdf_norm_from_kernel(kernel_val, **kwargs):
    """The kernel's pdf_max (pdf_norm.py:6-14)."""
    return kernel_val


def pdf_norm_max_found(prev_pdf_norm, get_weighted_distances, **kwargs):
    """max(prev, *distances of the current population) (pdf_norm.py:17-38)."""
    pdfs = _distances(get_weighted_distances)
    if prev_pdf_norm is None:
        prev_pdf_norm = -np.inf
    return max(prev_pdf_norm, float(np.max(pdfs))) if pdfs.size \
        else prev_pdf_norm


class ScaledPDFNorm:
    """pdf_norm_max_found, lowered by log(factor) x (the next temperature)
    from the first generation whose acceptance rate fell below
    ``min_acceptance_rate`` on (pdf_norm.py:41-110).  As in the reference,
    the factor is always 10 whatever is passed; the next temperature is
    alpha x the previous one (1 before any)."""

    def __init__(self, factor=10, alpha=0.5, min_acceptance_rate=0.1):
        self.factor = 10
        self.alpha = alpha
        self.min_acceptance_rate = min_acceptance_rate
        self._hit = False  # sticky once the rate has dropped

    def __call__(self, prev_pdf_norm, get_weighted_distances, prev_temp,
                 acceptance_rate, **kwargs):
        base = pdf_norm_max_found(prev_pdf_norm=prev_pdf_norm,
                                  get_weighted_distances=get_weighted_distances)
        self._hit = self._hit or not (
            acceptance_rate >= self.min_acceptance_rate)
        if not self._hit:
            return base
        t_next = 1 if prev_temp is None else self.alpha * prev_temp
        return base - np.log(self.factor) * t_next


class StochasticAcceptor(Acceptor):
    """Accept with probability (pdf(x_0|x)/c)^(1/T) (acceptor.py:309-473).

    The GPU batch sampler evaluates the kernel density, the uniform and the
    decision in one fused kernel (``abc_stochastic_kernel_f64``); the
    per-proposal ``__call__`` below is the closure-sampler path."""

    def __init__(self, pdf_norm_method=None, apply_importance_weighting=True,
                 log_file=None):
        super().__init__()
        self.pdf_norm_method = pdf_norm_method or pdf_norm_max_found
        self.apply_importance_weighting = apply_importance_weighting
        self.log_file = log_file
        self.pdf_norms = {}
        self.x_0 = None
        self.kernel_scale = None
        self.kernel_pdf_max = None

    def initialize(self, t, get_weighted_distances, distance_function, x_0):
        self.x_0 = x_0
        self.kernel_scale = distance_function.ret_scale
        self.kernel_pdf_max = distance_function.pdf_max
        self._update(t, get_weighted_distances)

    def update(self, t, get_weighted_distances, prev_temp, acceptance_rate):
        self._update(t, get_weighted_distances, prev_temp, acceptance_rate)

    def _update(self, t, get_weighted_distances, prev_temp=None,
                acceptance_rate=1.0):
        self.pdf_norms[t] = self.pdf_norm_method(
            kernel_val=self.kernel_pdf_max,
            get_weighted_distances=get_weighted_distances,
            prev_pdf_norm=None if not self.pdf_norms
            else max(self.pdf_norms.values()),
            acceptance_rate=acceptance_rate, prev_temp=prev_temp)
        logger.debug(f"pdf_norm={self.pdf_norms[t]:.4e} for t={t}.")
        if self.log_file:
            save_dict_to_json(self.pdf_norms, self.log_file)

    def get_epsilon_config(self, t):
        return dict(pdf_norm=self.pdf_norms[t], kernel_scale=self.kernel_scale)

    def __call__(self, distance_function, eps, x, x_0, t, par):
        """One proposal: the kernel value pd, acceptance probability
        (pd / c)^(1/T) (linear scale) or exp((pd - c) / T) (log scale), one
        U[0, 1) draw from numpy's global state, and the importance weight
        p / min(1, p) (1 without importance weighting, 0 when p = 0)."""
        from .distance import SCALE_LIN
        inv_temp = 1 / eps(t)
        pd = distance_function(x, x_0, t, par)
        c = self.pdf_norms[t]
        if distance_function.ret_scale == SCALE_LIN:
            p = (pd / c) ** inv_temp
        else:
            p = np.exp((pd - c) * inv_temp)
        u = np.random.uniform(low=0, high=1)
        if p == 0.0:
            weight = 0.0
        else:
            weight = p / min(1, p) if self.apply_importance_weighting else 1.0
        return AcceptorResult(pd, bool(p >= u), weight)


def save_dict_to_json(dct, file_):
    """storage/json.py: keys and values as JSON."""
    with open(file_, "w") as f:
        json.dump({str(k): v for k, v in dct.items()}, f, default=_to_py)


def load_dict_from_json(file_, key_type=int):
    with open(file_) as f:
        dct = json.load(f)
    return {key_type(k): v for k, v in dct.items()}


def _to_py(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    raise TypeError(type(v))
