"""Distances with the reference's plug-in API, computed by HIP kernels.

Reference: pyabc/distance/base.py:8-158 (Distance), distance.py:14-347
(PNormDistance, AdaptivePNormDistance), scale.py:1-156 (scale functions).

Every p-norm evaluation -- the batch one of the GPU sampler and the single
one of ``__call__`` -- runs through ``abc_pnorm_distance_f64``; the adaptive
scales median_absolute_deviation and standard_deviation run through the
column select / std kernels.  Other (user) scale functions are evaluated as
given, on host lists, exactly as the reference calls them.
"""
import json
import logging
from abc import ABC, abstractmethod

import numpy as np
import torch

from . import kernels as K

logger = logging.getLogger("Distance")


# ---------------------------------------------------------------------------
# scale functions (distance/scale.py) -- the reference semantics for user
# code; the two used on the hot path are recognised and run on the device.
# ---------------------------------------------------------------------------
def median_absolute_deviation(data, **kwargs):
    data = np.array(data)
    return np.median(np.abs(data - np.median(data)))


def mean_absolute_deviation(data, **kwargs):
    data = np.array(data)
    return np.mean(np.abs(data - np.mean(data)))


def standard_deviation(data, **kwargs):
    return np.std(data)


def bias(data, x_0, **kwargs):
    return np.abs(np.mean(data) - x_0)


def root_mean_square_deviation(data, x_0, **kwargs):
    return np.sqrt(bias(data, x_0) ** 2 + standard_deviation(data) ** 2)


def median_absolute_deviation_to_observation(data, x_0, **kwargs):
    return np.median(np.abs(np.array(data) - x_0))


def mean_absolute_deviation_to_observation(data, x_0, **kwargs):
    return np.mean(np.abs(np.array(data) - x_0))


def combined_median_absolute_deviation(data, x_0, **kwargs):
    return (median_absolute_deviation(data)
            + median_absolute_deviation_to_observation(data, x_0))


def combined_mean_absolute_deviation(data, x_0, **kwargs):
    return (mean_absolute_deviation(data)
            + mean_absolute_deviation_to_observation(data, x_0))


def standard_deviation_to_observation(data, x_0, **kwargs):
    return np.std(np.abs(np.array(data) - x_0))


def span(data, **kwargs):
    return max(data) - min(data)


def mean(data, **kwargs):
    return np.mean(data)


def median(data, **kwargs):
    return np.median(data)


DEVICE_SCALES = {median_absolute_deviation: "mad",
                 standard_deviation: "std"}


class DeviceStats:
    """Recorded summary statistics on the device, stat-major [S, n] in x_0
    key order (what the reference gathers per key from a list of dicts,
    distance.py:266-270).  ``stats_T`` is row-contiguous but its row stride
    may exceed n (a one-round generation hands out a column slice of the
    round's buffer): read it through (pointer, ``stats_T.stride(0)``), as
    ``kernels._stat_major`` does."""

    def __init__(self, stats_T, keys):
        self.stats_T = stats_T
        self.keys = list(keys)

    def __len__(self):
        return self.stats_T.shape[1]

    def to_dicts(self):
        a = self.stats_T.cpu().numpy()
        return [dict(zip(self.keys, a[:, j])) for j in range(a.shape[1])]

    def __iter__(self):
        return iter(self.to_dicts())

    def __getitem__(self, j):
        return dict(zip(self.keys, self.stats_T[:, j].cpu().numpy()))


def _rows_in_order(stats_T, have, want):
    """Rows of stat-major ``stats_T`` (statistics ``have``) reordered to the
    statistics ``want``; unchanged when the orders agree or ``have`` is
    unknown."""
    if have is None or list(have) == list(want):
        return stats_T
    idx = torch.as_tensor([list(have).index(k) for k in want],
                          device=stats_T.device)
    return stats_T.index_select(0, idx).contiguous()


def _stats_matrix(keys, all_sum_stats):
    """[S, n] device matrix from a DeviceStats or a list of dicts."""
    if isinstance(all_sum_stats, DeviceStats):
        if all_sum_stats.keys == list(keys):
            return all_sum_stats.stats_T, None
        idx = [all_sum_stats.keys.index(k) for k in keys]
        return all_sum_stats.stats_T[idx], None
    mask = np.array([[k in s for s in all_sum_stats] for k in keys])
    arr = np.array([[float(s[k]) if k in s else np.nan for s in all_sum_stats]
                    for k in keys], dtype=np.float64)
    return torch.as_tensor(arr.reshape(len(keys), -1), device="cuda"), mask


class Distance(ABC):
    def __init__(self):
        pass

    def initialize(self, t, get_all_sum_stats, x_0=None):
        """Calibrate before the first use (base.py:21-42)."""

    def configure_sampler(self, sampler):
        """Configure the sampler (base.py:44-65)."""

    def update(self, t, get_all_sum_stats):
        """Update for generation t; True if the distance changed."""
        return False

    @abstractmethod
    def __call__(self, x, x_0, t=None, par=None):
        """Distance of simulated to observed statistics."""

    def get_config(self):
        return {"name": self.__class__.__name__}

    def to_json(self):
        return json.dumps(self.get_config())


class NoDistance(Distance):
    def __call__(self, x, x_0, t=None, par=None):
        raise Exception(f"{self.__class__.__name__} is not intended to be called.")


class SimpleFunctionDistance(Distance):
    """Wraps a user function f(x, x_0) (user code, evaluated as given)."""

    def __init__(self, fun):
        super().__init__()
        self.fun = fun

    def __call__(self, x, x_0, t=None, par=None):
        return self.fun(x, x_0)

    def get_config(self):
        conf = super().get_config()
        conf["name"] = getattr(self.fun, "__name__", "function")
        return conf


def to_distance(maybe_distance):
    if maybe_distance is None:
        return NoDistance()
    if isinstance(maybe_distance, Distance):
        return maybe_distance
    return SimpleFunctionDistance(maybe_distance)


class PNormDistance(Distance):
    """Weighted p-norm (distance.py:14-133); evaluated by the device kernel."""

    def __init__(self, p=2, weights=None, factors=None):
        super().__init__()
        if p < 1:
            raise ValueError("It must be p >= 1")
        self.p = p
        self.weights = weights
        self.factors = factors
        self._dev_cache = {}

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t, get_all_sum_stats, x_0)
        self.format_weights_and_factors(t, x_0.keys())

    def format_weights_and_factors(self, t, sum_stat_keys):
        self.weights = PNormDistance.format_dict(self.weights, t, sum_stat_keys)
        self.factors = PNormDistance.format_dict(self.factors, t, sum_stat_keys)

    @staticmethod
    def format_dict(w, t, sum_stat_keys, default_val=1.):
        if w is None:
            return {t: {k: default_val for k in sum_stat_keys}}
        if not isinstance(next(iter(w.values())), dict):
            return {t: w}
        return w

    @staticmethod
    def get_for_t_or_latest(w, t):
        if t not in w:
            t = max(w)
        return w[t]

    # --- device parameters -------------------------------------------------
    def device_params(self, t, x_0):
        """(keys, x0[S], fw[S]) on the device in the key order of the weight
        dict (the reference sums over ``for key in w``, distance.py:96-100);
        keys missing from x_0 get fw = 0 (they contribute 0)."""
        self.format_weights_and_factors(t, x_0.keys())
        w = PNormDistance.get_for_t_or_latest(self.weights, t)
        f = PNormDistance.get_for_t_or_latest(self.factors, t)
        keys = list(w.keys())
        fw = np.array([(f[k] * w[k]) if k in x_0 and k in f else 0.0
                       for k in keys], dtype=np.float64)
        x0 = np.array([float(x_0[k]) if k in x_0 else 0.0 for k in keys],
                      dtype=np.float64)
        return (keys, torch.as_tensor(x0, device="cuda"),
                torch.as_tensor(fw, device="cuda"))

    def __call__(self, x, x_0, t=None, par=None):
        keys, x0d, fwd = self.device_params(t, x_0)
        present = [k in x for k in keys]
        if not all(present):
            fwd = fwd * torch.as_tensor(np.array(present, dtype=np.float64),
                                        device="cuda")
        xs = np.array([[float(x[k]) if k in x else 0.0] for k in keys],
                      dtype=np.float64).reshape(len(keys), 1)
        d, _, _ = K.pnorm_distance(torch.as_tensor(xs, device="cuda"), x0d,
                                   fwd, self.p, with_accept=False)
        return float(d.item())

    def batch(self, stats_T, t, x_0, eps=np.inf, n=None, keys=None):
        """Distances (and accept flags) of n stat-major columns whose rows
        are the statistics ``keys`` (default: the distance's key order)."""
        dkeys, x0d, fwd = self.device_params(t, x_0)
        stats_T = _rows_in_order(stats_T, keys, dkeys)
        return K.pnorm_distance(stats_T, x0d, fwd, self.p, eps, B=n)

    def get_config(self):
        return {"name": self.__class__.__name__, "p": self.p,
                "weights": self.weights, "factors": self.factors}

    def to_json(self):
        return json.dumps(self.get_config(), default=float)


class AdaptivePNormDistance(PNormDistance):
    """p-norm with per-generation scale-normalised weights
    (distance.py:136-347)."""

    def __init__(self, p=2, initial_weights=None, factors=None, adaptive=True,
                 scale_function=None, normalize_weights=True,
                 max_weight_ratio=None):
        super().__init__(p=p, weights=None, factors=factors)
        self.initial_weights = initial_weights
        self.factors = factors
        self.adaptive = adaptive
        self.scale_function = scale_function or standard_deviation
        self.normalize_weights = normalize_weights
        self.max_weight_ratio = max_weight_ratio
        self.x_0 = None

    def configure_sampler(self, sampler):
        if self.adaptive:
            sampler.sample_factory.record_rejected = True

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t, get_all_sum_stats, x_0)
        self.x_0 = x_0
        if self.initial_weights is not None:
            self.weights[t] = self.initial_weights
            return
        self._update(t, get_all_sum_stats())

    def update(self, t, get_all_sum_stats):
        if not self.adaptive:
            return False
        self._update(t, get_all_sum_stats())
        return True

    def _scales(self, keys, all_sum_stats):
        kind = DEVICE_SCALES.get(self.scale_function)
        if kind is not None:
            stats_T, mask = _stats_matrix(keys, all_sum_stats)
            if mask is None or mask.all():
                if kind == "mad":
                    _, s = K.column_median_mad(stats_T)
                else:
                    _, s = K.column_std(stats_T)
                return s.cpu().numpy()
        # ragged records or a user scale function: reference semantics
        recs = all_sum_stats.to_dicts() if isinstance(all_sum_stats,
                                                      DeviceStats) \
            else all_sum_stats
        out = []
        for key in keys:
            cur = [r[key] for r in recs if key in r]
            out.append(self.scale_function(data=cur, x_0=self.x_0[key]))
        return np.array(out, dtype=np.float64)

    def _update(self, t, all_sum_stats):
        keys = list(self.x_0.keys())
        scales = np.asarray(self._scales(keys, all_sum_stats),
                            dtype=np.float64)
        # 0 where np.isclose(s, 0), else 1 / s (elementwise: the same
        # values as the per-key loop, one numpy call instead of S)
        close = np.isclose(scales, 0)
        inv = np.where(close, 0.0, 1.0 / np.where(close, 1.0, scales))
        w = dict(zip(keys, inv.tolist()))
        w = self._normalize_weights(w)
        w = self._bound_weights(w)
        self.weights[t] = w
        logger.debug(f"updated weights[{t}] = {self.weights[t]}")

    def _normalize_weights(self, w):
        if not self.normalize_weights:
            return w
        vals = np.array(list(w.values()), dtype=np.float64)
        return dict(zip(w.keys(), (vals / np.mean(vals)).tolist()))

    def _bound_weights(self, w):
        if self.max_weight_ratio is None:
            return w
        arr = np.array(list(w.values()))
        min_abs = np.min(np.abs(arr[arr != 0]))
        for key, value in w.items():
            if abs(value) / min_abs > self.max_weight_ratio:
                w[key] = np.sign(value) * self.max_weight_ratio * min_abs
        return w

    def get_config(self):
        return {"name": self.__class__.__name__, "p": self.p,
                "factors": self.factors, "adaptive": self.adaptive,
                "scale_function": self.scale_function.__name__,
                "normalize_weights": self.normalize_weights,
                "max_weight_ratio": self.max_weight_ratio}


# ---------------------------------------------------------------------------
# stochastic kernels (distance/kernel.py:1-588): densities for the
# StochasticAcceptor.  Independent normal / Laplace kernels evaluate through
# abc_stochastic_kernel_f64 (single calls and the batch sampler alike).
# ---------------------------------------------------------------------------
SCALE_LIN = "SCALE_LIN"
SCALE_LOG = "SCALE_LOG"
SCALES = [SCALE_LIN, SCALE_LOG]


def _flat(x, keys):
    """Values of ``keys`` flattened into one float64 vector (kernel.py:563-588
    ``_diff_arr`` / ``_arr``: array-valued statistics are extended)."""
    out = []
    for key in keys:
        v = x[key]
        try:
            out.extend(v)
        except TypeError:
            out.append(v)
    return np.array(out, dtype=np.float64)


class StochasticKernel(Distance):
    """Base of the density kernels (kernel.py:12-80); ``ret_scale`` is
    SCALE_LIN or SCALE_LOG, ``keys`` default to sorted(x_0), ``pdf_max`` the
    density at x_0 unless given."""

    def __init__(self, ret_scale=SCALE_LIN, keys=None, pdf_max=None):
        super().__init__()
        StochasticKernel.check_ret_scale(ret_scale)
        self.ret_scale = ret_scale
        self.keys = keys
        self.pdf_max = pdf_max

    def initialize(self, t, get_all_sum_stats, x_0=None):
        if self.keys is None:
            self.initialize_keys(x_0)

    @staticmethod
    def check_ret_scale(ret_scale):
        if ret_scale not in SCALES:
            raise ValueError(
                f"The ret_scale {ret_scale} must be one of {SCALES}.")

    def initialize_keys(self, x):
        self.keys = sorted(x)

    def get_config(self):
        return {"name": self.__class__.__name__, "ret_scale": self.ret_scale,
                "keys": self.keys, "pdf_max": self.pdf_max}

    def to_json(self):
        return json.dumps(self.get_config(), default=str)


class SimpleFunctionKernel(StochasticKernel):
    """User density function fun(x, x_0, t, par) (kernel.py:82-107)."""

    def __init__(self, fun, ret_scale=SCALE_LIN, keys=None, pdf_max=None):
        super().__init__(ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)
        self.fun = fun

    def __call__(self, x, x_0, t=None, par=None):
        return self.fun(x=x, x_0=x_0, t=t, par=par)


class NormalKernel(StochasticKernel):
    """Multivariate normal density of x - x_0 (kernel.py:110-187), scipy's
    ``multivariate_normal`` semantics (host; d x d parameters)."""

    def __init__(self, cov=None, ret_scale=SCALE_LOG, keys=None,
                 pdf_max=None):
        super().__init__(ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)
        self.cov = cov

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t, get_all_sum_stats, x_0)
        if self.cov is None:
            self.cov = np.eye(sum(np.size(x_0[k]) for k in self.keys))
        self.cov = np.array(self.cov)
        import scipy.stats
        self.rv = scipy.stats.multivariate_normal(
            mean=np.zeros(self.cov.shape[0]), cov=self.cov)
        if self.pdf_max is None:
            self.pdf_max = self(x_0, x_0)

    def __call__(self, x, x_0, t=None, par=None):
        if self.keys is None:
            self.initialize_keys(x_0)
        diff = _flat(x, self.keys) - _flat(x_0, self.keys)
        if self.ret_scale == SCALE_LIN:
            return self.rv.pdf(diff)
        return self.rv.logpdf(diff)


class _IndependentKernel(StochasticKernel):
    """Shared device evaluation of the independent normal / Laplace kernels
    (kernel.py:190-357): prm is the variance (normal) or scale (Laplace)
    vector, a scalar broadcast over the statistics, or a callable of the
    parameters."""
    _kind = None

    def __init__(self, prm, keys=None, pdf_max=None):
        super().__init__(ret_scale=SCALE_LOG, keys=keys, pdf_max=pdf_max)
        self._prm = prm
        self._dev_cache = None

    def _const(self, prm):
        """The kernel's log-normalisation term c (numpy, as the reference)."""
        raise NotImplementedError

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t, get_all_sum_stats, x_0)
        dim = sum(np.size(x_0[k]) for k in self.keys)
        if self._prm is None:
            self._prm = np.ones(dim)
        if not callable(self._prm):
            self._prm = np.array(self._prm) * np.ones(dim)
        self._dev_cache = None
        if self.pdf_max is None and not callable(self._prm):
            self.pdf_max = self(x_0, x_0)

    def _evaluate(self, xs, x0s, prm):
        prm = np.asarray(prm, dtype=np.float64) * np.ones(xs.shape[0])
        dev = torch.device("cuda", torch.cuda.current_device())
        col = torch.as_tensor(xs.reshape(-1, 1), device=dev)
        pd, _, _, _ = K.stochastic_kernel(
            col, torch.as_tensor(x0s, device=dev),
            torch.as_tensor(prm, device=dev), self._kind, self._const(prm))
        return float(pd.item())

    def __call__(self, x, x_0, t=None, par=None):
        if self.keys is None:
            self.initialize_keys(x_0)
        prm = self._prm(par) if callable(self._prm) else self._prm
        return self._evaluate(_flat(x, self.keys), _flat(x_0, self.keys), prm)

    # --- batch (device) interface -----------------------------------------
    def batch_unsupported_reason(self, x_0):
        if callable(self._prm):
            return "kernel parameters depend on the particle parameters"
        if any(np.size(x_0[k]) != 1 for k in self.keys):
            return "array-valued summary statistics"
        return None

    def device_params(self, t, x_0):
        """(keys, x0[S], prm[S], kind, c) for the batch kernel, in the
        kernel's key order."""
        if self._dev_cache is None:
            dev = torch.device("cuda", torch.cuda.current_device())
            prm = np.asarray(self._prm, dtype=np.float64)
            self._dev_cache = (
                list(self.keys),
                torch.as_tensor(_flat(x_0, self.keys), device=dev),
                torch.as_tensor(prm, device=dev), self._kind,
                self._const(prm))
        return self._dev_cache

    def batch(self, stats_T, t, x_0, eps=np.inf, n=None, keys=None):
        """Log-densities of n stat-major columns whose rows are the
        statistics ``keys`` (default: the kernel's key order)."""
        dkeys, x0d, prmd, kind, c = self.device_params(t, x_0)
        stats_T = _rows_in_order(stats_T, keys, dkeys)
        pd, _, _, _ = K.stochastic_kernel(stats_T, x0d, prmd, kind, c, B=n)
        return pd, None, None


class IndependentNormalKernel(_IndependentKernel):
    """-0.5 (sum log(2 pi var) + sum diff^2 / var)  (kernel.py:190-282)."""
    _kind = K.KERNEL_NORMAL

    def __init__(self, var=None, keys=None, pdf_max=None):
        super().__init__(var, keys=keys, pdf_max=pdf_max)

    @property
    def var(self):
        return self._prm

    @var.setter
    def var(self, v):
        self._prm = v
        self._dev_cache = None

    def _const(self, prm):
        return float(np.sum(np.log(2) + np.log(np.pi) + np.log(prm)))


class IndependentLaplaceKernel(_IndependentKernel):
    """-(sum log(2 b) + sum |diff| / b)  (kernel.py:285-357)."""
    _kind = K.KERNEL_LAPLACE

    def __init__(self, scale=None, keys=None, pdf_max=None):
        super().__init__(scale, keys=keys, pdf_max=pdf_max)

    @property
    def scale(self):
        return self._prm

    @scale.setter
    def scale(self, v):
        self._prm = v
        self._dev_cache = None

    def _const(self, prm):
        return float(np.sum(np.log(2) + np.log(prm)))


class _DiscreteKernel(StochasticKernel):
    """Count-data likelihoods (kernel.py:360-560), scipy.stats pmfs of the
    observed counts given the simulated ones (host, closure sampler path)."""

    def __init__(self, p=None, ret_scale=SCALE_LOG, keys=None, pdf_max=None):
        super().__init__(ret_scale=ret_scale, keys=keys, pdf_max=pdf_max)
        if p is not None and not callable(p) and (p > 1 or p < 0):
            raise ValueError(
                f"The success probability p={p} must be in the interval"
                f"[0, 1].")
        self.p = p

    def _dist(self):
        raise NotImplementedError

    def _args(self, k, n, p):
        return dict(k=k, n=n, p=p)

    def __call__(self, x, x_0, t=None, par=None):
        n = _flat(x, self.keys).astype(int)
        k = _flat(x_0, self.keys).astype(int)
        p = self.p(par) if callable(self.p) else self.p
        dist, args = self._dist(), self._args(k, n, p)
        if self.ret_scale == SCALE_LIN:
            return np.prod(dist.pmf(**args))
        return np.sum(dist.logpmf(**args))


class BinomialKernel(_DiscreteKernel):
    """binom.pmf(k=x_0, n=x, p) (kernel.py:360-419)."""

    def __init__(self, p, ret_scale=SCALE_LOG, keys=None, pdf_max=None):
        super().__init__(p, ret_scale, keys, pdf_max)

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t, get_all_sum_stats, x_0)
        if self.pdf_max is None and not callable(self.p):
            self.pdf_max = binomial_pdf_max(x_0, self.keys, self.p,
                                            self.ret_scale)

    def _dist(self):
        import scipy.stats
        return scipy.stats.binom


class PoissonKernel(_DiscreteKernel):
    """poisson.pmf(k=x_0, mu=x) (kernel.py:422-470)."""

    def __init__(self, ret_scale=SCALE_LOG, keys=None, pdf_max=None):
        super().__init__(None, ret_scale, keys, pdf_max)

    def initialize(self, t, get_all_sum_stats, x_0=None):
        super().initialize(t, get_all_sum_stats, x_0)
        if self.pdf_max is None:
            self.pdf_max = self(x_0, x_0)

    def _dist(self):
        import scipy.stats
        return scipy.stats.poisson

    def _args(self, k, n, p):
        return dict(k=k, mu=n)


class NegativeBinomialKernel(_DiscreteKernel):
    """nbinom.pmf(k=x_0, n=x, p) (kernel.py:473-529)."""

    def __init__(self, p, ret_scale=SCALE_LOG, keys=None, pdf_max=None):
        super().__init__(p, ret_scale, keys, pdf_max)

    def _dist(self):
        import scipy.stats
        return scipy.stats.nbinom


def binomial_pdf_max(x_0, keys, p, ret_scale):
    """Max over n of binom.pmf(k=x_0, n, p): n = max(ceil((k-p)/p), 0)
    (kernel.py:532-551)."""
    import scipy.stats
    ks = _flat(x_0, keys).astype(int)
    ns = np.maximum(np.ceil((ks - p) / p), 0)
    lp = np.sum(scipy.stats.binom.logpmf(k=ks, n=ns, p=p))
    return np.exp(lp) if ret_scale == SCALE_LIN else lp
