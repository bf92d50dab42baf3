"""Acceptance thresholds (API of pyabc/epsilon/base.py:10-167 and
epsilon.py:12-243).  QuantileEpsilon computes its weighted quantile with the
device radix select (abc_wquantile_f64)."""
import json
import logging
from abc import ABC, abstractmethod

import numpy as np
import torch

from . import kernels as K
from .distributed import Comm

logger = logging.getLogger("Epsilon")


class Epsilon(ABC):
    def __init__(self):
        pass

    def initialize(self, t, get_weighted_distances, get_all_records,
                   max_nr_populations, acceptor_config):
        pass

    def configure_sampler(self, sampler):
        pass

    def update(self, t, get_weighted_distances, get_all_records,
               acceptance_rate, acceptor_config):
        pass

    @abstractmethod
    def __call__(self, t):
        """Epsilon for generation t."""

    def get_config(self):
        return {"name": self.__class__.__name__}

    def to_json(self):
        return json.dumps(self.get_config())


class NoEpsilon(Epsilon):
    def __call__(self, t):
        return np.nan


class ConstantEpsilon(Epsilon):
    def __init__(self, constant_epsilon_value):
        super().__init__()
        self.constant_epsilon_value = constant_epsilon_value

    def get_config(self):
        c = super().get_config()
        c["constant_epsilon_value"] = self.constant_epsilon_value
        return c

    def __call__(self, t):
        return self.constant_epsilon_value


class ListEpsilon(Epsilon):
    def __init__(self, values):
        super().__init__()
        self.epsilon_values = list(values)

    def get_config(self):
        c = super().get_config()
        c["epsilon_values"] = self.epsilon_values
        return c

    def __call__(self, t):
        return self.epsilon_values[t]


def _columns(weighted_distances):
    """(distance, w) as device tensors from a DataFrame or the device
    WeightedDistances of a columnar population."""
    if hasattr(weighted_distances, "distance_tensor"):
        return (weighted_distances.distance_tensor,
                weighted_distances.w_tensor)
    d = torch.as_tensor(np.asarray(weighted_distances.distance.values,
                                   dtype=np.float64), device="cuda")
    w = torch.as_tensor(np.asarray(weighted_distances.w.values,
                                   dtype=np.float64), device="cuda")
    return d, w


class QuantileEpsilon(Epsilon):
    """alpha-quantile of the (weighted) distances of the last population
    (epsilon.py:68-228)."""

    def __init__(self, initial_epsilon='from_sample', alpha=0.5,
                 quantile_multiplier=1, weighted=True):
        super().__init__()
        self._initial_epsilon = initial_epsilon
        self.alpha = alpha
        self.quantile_multiplier = quantile_multiplier
        self.weighted = weighted
        self._look_up = {}
        if self.alpha > 1 or self.alpha <= 0:
            raise ValueError("It must be 0 < alpha <= 1")

    def get_config(self):
        c = super().get_config()
        c.update({"initial_epsilon": self._initial_epsilon,
                  "alpha": self.alpha,
                  "quantile_multiplier": self.quantile_multiplier,
                  "weighted": self.weighted})
        return c

    def initialize(self, t, get_weighted_distances, get_all_records,
                   max_nr_populations, acceptor_config):
        if self._initial_epsilon != 'from_sample':
            return
        self._update(t, get_weighted_distances())
        logger.info(f"initial epsilon is {self._look_up[t]}")

    def __call__(self, t):
        if not self._look_up:
            self._set_initial_value(t)
        try:
            return self._look_up[t]
        except KeyError as e:
            raise KeyError(f"The epsilon value for time {t} does not exist: "
                           f"{e!r} ")

    def _set_initial_value(self, t):
        self._look_up = {t: self._initial_epsilon}

    def update(self, t, get_weighted_distances, get_all_records,
               acceptance_rate, acceptor_config):
        self._update(t, get_weighted_distances())
        logger.debug(f"new eps, t={t}, eps={self._look_up[t]}")

    def _update(self, t, weighted_distances):
        d, w = _columns(weighted_distances)
        # weighted: w / sum(w) (epsilon.py:214-218); else uniform 1/n
        wq = w if self.weighted else None
        # a device population is the same global population on every rank:
        # each rank histograms its share, the histograms are all-reduced
        comm = Comm.current() if hasattr(weighted_distances,
                                         "distance_tensor") else None
        q = float(K.weighted_quantile(d, wq, self.alpha, comm=comm)[0].item())
        self._look_up[t] = q * self.quantile_multiplier


class MedianEpsilon(QuantileEpsilon):
    def __init__(self, initial_epsilon='from_sample', median_multiplier=1,
                 weighted=True):
        super().__init__(initial_epsilon=initial_epsilon, alpha=0.5,
                         quantile_multiplier=median_multiplier,
                         weighted=weighted)
