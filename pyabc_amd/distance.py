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
    distance.py:266-270)."""

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

    def batch(self, stats_T, t, x_0, eps=np.inf, n=None):
        """Distances (and accept flags) of n stat-major columns."""
        _, x0d, fwd = self.device_params(t, x_0)
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
        scales = self._scales(keys, all_sum_stats)
        w = {}
        for key, s in zip(keys, scales):
            w[key] = 0 if np.isclose(s, 0) else 1 / s
        w = self._normalize_weights(w)
        w = self._bound_weights(w)
        self.weights[t] = w
        logger.debug(f"updated weights[{t}] = {self.weights[t]}")

    def _normalize_weights(self, w):
        if not self.normalize_weights:
            return w
        mean_weight = np.mean(list(w.values()))
        for key in w:
            w[key] /= mean_weight
        return w

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
