"""Particles and populations (API of pyabc/population.py:1-286), plus the
columnar device population the GPU sampler produces."""
import concurrent.futures
import logging
import threading

import numpy as np
import pandas as pd
import torch

from . import kernels as K
from .frames import DeviceFrame
from .distance import DeviceStats

logger = logging.getLogger("ABC.Population")


class Particle:
    def __init__(self, m, parameter, weight, accepted_sum_stats,
                 accepted_distances, rejected_sum_stats=None,
                 rejected_distances=None, accepted=True):
        self.m = m
        self.parameter = parameter
        self.weight = weight
        self.accepted_sum_stats = accepted_sum_stats
        self.accepted_distances = accepted_distances
        self.rejected_sum_stats = rejected_sum_stats or []
        self.rejected_distances = rejected_distances or []
        self.accepted = accepted


class Population:
    """List of particles; weights normalised per model on construction
    (population.py:120-142)."""

    def __init__(self, particles):
        self._list = list(particles)
        self._model_probabilities = None
        self._normalize_weights()

    def __len__(self):
        return len(self._list)

    def get_list(self):
        return self._list.copy()

    def to_dict(self):
        store = {}
        for p in self._list:
            store.setdefault(p.m, []).append(p)
        return store

    def _normalize_weights(self):
        store = self.to_dict()
        totals = {m: sum(p.weight for p in pl) for m, pl in store.items()}
        tot = sum(totals.values())
        self._model_probabilities = {m: w / tot for m, w in totals.items()}
        for m, pl in store.items():
            for p in pl:
                p.weight /= totals[m]

    def update_distances(self, distance_to_ground_truth):
        for p in self._list:
            for i in range(len(p.accepted_distances)):
                p.accepted_distances[i] = distance_to_ground_truth(
                    p.accepted_sum_stats[i], p.parameter)

    def get_model_probabilities(self):
        return self._model_probabilities

    def get_alive_models(self):
        return list(self._model_probabilities.keys())

    def nr_of_models_alive(self):
        return len(self.get_alive_models())

    def get_weighted_distances(self):
        rows = []
        for p in self._list:
            mp = self._model_probabilities[p.m]
            for d in p.accepted_distances:
                rows.append({"distance": d, "w": p.weight * mp})
        return pd.DataFrame(rows)

    def get_weighted_sum_stats(self):
        """(weights, sum_stats): one entry per accepted statistic, the
        particle's weight times its model probability (population.py:200-216)."""
        weights, sum_stats = [], []
        for p in self._list:
            w = p.weight * self._model_probabilities[p.m]
            for s in p.accepted_sum_stats:
                weights.append(w)
                sum_stats.append(s)
        return weights, sum_stats

    def get_accepted_sum_stats(self):
        out = []
        for p in self._list:
            out.extend(p.accepted_sum_stats)
        return out

    def get_for_keys(self, keys):
        """Same-ordered lists per key, one entry per accepted distance
        (population.py:228-262)."""
        _check_keys(keys)
        ret = {k: [] for k in keys}
        for p in self._list:
            n = len(p.accepted_distances)
            if "weight" in ret:
                ret["weight"].extend(
                    [p.weight * self._model_probabilities[p.m]] * n)
            if "parameter" in ret:
                ret["parameter"].extend([p.parameter] * n)
            if "distance" in ret:
                ret["distance"].extend(p.accepted_distances)
            if "sum_stat" in ret:
                ret["sum_stat"].extend(p.accepted_sum_stats)
        return ret

    def get_distribution(self, m=0):
        pl = [p for p in self._list if p.m == m]
        df = pd.DataFrame([dict(p.parameter) for p in pl])
        if len(df.columns):
            df = df[sorted(df.columns)]
        w = np.array([p.weight for p in pl], dtype=np.float64)
        return df, w


FOR_KEYS = ("weight", "distance", "parameter", "sum_stat")


def _check_keys(keys):
    for k in keys:
        if k not in FOR_KEYS:
            raise ValueError(f"Key {k} not in {list(FOR_KEYS)}.")


class DistanceToGroundTruth:
    """``lambda x, par: distance(x, x_0, t, par)`` (smc.py:978-984) that a
    device population can also evaluate with the distance's batch kernel."""

    def __init__(self, distance, x_0, t):
        self.distance, self.x_0, self.t = distance, x_0, t

    def __call__(self, x, par):
        return self.distance(x, self.x_0, self.t, par)


class WeightedDistances:
    """``get_weighted_distances`` of a device population: columns
    ``distance`` and ``w`` as device tensors (host copies on demand)."""

    def __init__(self, d, w):
        self.distance_tensor = d
        self.w_tensor = w

    @property
    def distance(self):
        return pd.Series(self.distance_tensor.cpu().numpy(), name="distance")

    @property
    def w(self):
        return pd.Series(self.w_tensor.cpu().numpy(), name="w")

    def __len__(self):
        return self.distance_tensor.numel()

    def __getitem__(self, col):
        if col == "distance":
            return self.distance
        if col == "w":
            return self.w
        raise KeyError(col)

    def to_pandas(self):
        return pd.DataFrame({"distance": self.distance.values,
                             "w": self.w.values})


class ColumnarPopulation:
    """Single-model population as device columns: theta [n, d], normalised
    weights [n], distances [n], accepted statistics [S, n] (optional).
    Same methods as :class:`Population`; ``get_list`` materialises particles
    on the host only when asked."""

    def __init__(self, theta, w, d, names, stats_T=None, stat_keys=None,
                 m=0, normalize=True):
        self._pending = None      # host offload in flight (to_host)
        self._offload_lock = threading.Lock()
        self.theta = theta
        self.d = d
        self.names = list(names)
        self.stats_T = stats_T
        self.stat_keys = list(stat_keys) if stat_keys is not None else None
        self.m = m
        if normalize:
            s = K.dsum(w)
            w = w.clone()
            K.scale_inplace(w, s)
        self.w = w
        self._model_probabilities = {m: 1.0}

    def __len__(self):
        return self.theta.shape[0]

    def to_host(self):
        """Move the columns to host memory (History keeps only the newest
        population on the device); readers work on either.

        The copy runs asynchronously: a worker thread copies the columns on
        a side stream (after an event recorded on the caller's stream), so
        the next generation's kernels are not held behind a D2H copy of the
        statistics matrix (80 MB at N = 1e5, S = 100).  The first access to
        a column waits for it."""
        if self._pending is not None:
            return self
        cols = {n: self.__dict__.get("_" + n) for n in _COLUMNS}
        if not any(t is not None and t.is_cuda for t in cols.values()):
            return self
        dev = next(t.device for t in cols.values()
                   if t is not None and t.is_cuda)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))

        def copy():
            with torch.cuda.device(dev):
                s = _side_stream(dev)
                with torch.cuda.stream(s):
                    s.wait_event(ev)
                    return {n: (t.to("cpu") if t is not None and t.is_cuda
                                else t) for n, t in cols.items()}

        self._pending = _offload_pool().submit(copy)
        return self

    def device_bytes(self):
        """Bytes of the columns held in device memory (0 once offloaded)."""
        if self._pending is not None:
            return 0
        return sum(t.numel() * t.element_size()
                   for t in (self.__dict__.get("_" + n) for n in _COLUMNS)
                   if t is not None and t.is_cuda)

    def _finish_offload(self):
        # readers may race (the History writer thread, the caller): the
        # first one installs the host columns, the others find _pending gone
        with self.__dict__.setdefault("_offload_lock", threading.Lock()):
            fut = self.__dict__.get("_pending")
            if fut is None:
                return
            for n, t in fut.result().items():
                self.__dict__["_" + n] = t
            self.__dict__["_pending"] = None

    def get_model_probabilities(self):
        return self._model_probabilities

    def get_alive_models(self):
        return [self.m]

    def nr_of_models_alive(self):
        return 1

    def get_weighted_distances(self):
        return WeightedDistances(self.d, self.w)

    def get_accepted_sum_stats(self):
        if self.stats_T is None:
            raise ValueError("statistics of this population were not kept")
        return DeviceStats(self.stats_T, self.stat_keys)

    def update_distances_device(self, distance, t, x_0):
        """Recompute distances under an updated distance (smc.py:978-984)
        with the batch kernel."""
        if self.stats_T is None:
            raise ValueError("statistics of this population were not kept")
        self.d, _, _ = distance.batch(self.stats_T, t, x_0, np.inf,
                                      keys=self.stat_keys)
        return self.d

    def update_distances(self, distance_to_ground_truth):
        """Population.update_distances (population.py:144-159): every
        accepted statistic's distance re-evaluated by the callable
        ``(sum_stat, parameter) -> float``.  A :class:`DistanceToGroundTruth`
        over a distance with a batch kernel runs on the device; any other
        callable is called once per particle on host copies."""
        f = distance_to_ground_truth
        if isinstance(f, DistanceToGroundTruth) and \
                hasattr(f.distance, "batch") and torch.cuda.is_available():
            if self.stats_T is None:
                raise ValueError("statistics of this population were not "
                                 "kept")
            if self.stats_T.is_cuda:
                return self.update_distances_device(f.distance, f.t, f.x_0)
            # offloaded by History (to_host): the statistics go back to the
            # device for the batch kernel (not O(N) host distance calls) and
            # the distances come home with the other columns
            d, _, _ = f.distance.batch(self.stats_T.cuda(), f.t, f.x_0,
                                       np.inf, keys=self.stat_keys)
            self.d = d.to(self.theta.device)
            return self.d
        if self.stats_T is None:
            raise ValueError("statistics of this population were not kept")
        if len(self) > 100000:
            logger.warning("update_distances: %d per-particle host distance "
                           "calls (no batch kernel for %r)", len(self), f)
        d = [float(f(s, p)) for s, p in
             zip(self._host_sum_stats(), self._host_parameters())]
        self.d = torch.as_tensor(np.asarray(d, dtype=np.float64),
                                 device=self.theta.device)
        return self.d

    def to_dict(self):
        """{model: [Particle, ...]} (population.py:264-286)."""
        return {self.m: self.get_list()} if len(self) else {}

    def _host_parameters(self):
        from .parameters import Parameter
        th = self.theta.cpu().numpy()
        return [Parameter(dict(zip(self.names, row))) for row in th]

    def _host_sum_stats(self):
        if self.stats_T is None:
            return [{} for _ in range(len(self))]
        st = self.stats_T.cpu().numpy()
        keys = self.stat_keys if self.stat_keys is not None \
            else list(range(st.shape[0]))
        return [dict(zip(keys, st[:, i])) for i in range(st.shape[1])]

    def get_weighted_sum_stats(self):
        """(weights, sum_stats) as host lists (population.py:200-216): one
        statistic per particle, weight x model probability."""
        mp = self._model_probabilities[self.m]
        w = (self.w.cpu().numpy() * mp).tolist() if mp != 1.0 \
            else self.w.cpu().numpy().tolist()
        return w, self._host_sum_stats()

    def get_for_keys(self, keys):
        """Population.get_for_keys (population.py:228-262) from the
        columns: weight (x model probability), distance, parameter,
        sum_stat, one entry per particle."""
        _check_keys(keys)
        ret = {}
        mp = self._model_probabilities[self.m]
        for k in keys:
            if k == "weight":
                w = self.w.cpu().numpy()
                ret[k] = (w * mp if mp != 1.0 else w).tolist()
            elif k == "distance":
                ret[k] = self.d.cpu().numpy().tolist()
            elif k == "parameter":
                ret[k] = self._host_parameters()
            else:
                if self.stats_T is None:
                    raise ValueError("statistics of this population were "
                                     "not kept")
                ret[k] = self._host_sum_stats()
        return ret

    def get_distribution(self, m=0):
        return DeviceFrame(self.theta, self.names), self.w

    def get_list(self):
        w = self.w.cpu().numpy()
        d = self.d.cpu().numpy()
        return [Particle(self.m, par, float(w[i]), [ss], [float(d[i])])
                for i, (par, ss) in enumerate(zip(self._host_parameters(),
                                                  self._host_sum_stats()))]


_COLUMNS = ("theta", "w", "d", "stats_T")
_pool = None
_side = {}
_pool_lock = threading.Lock()


def _offload_pool():
    global _pool
    with _pool_lock:
        if _pool is None:
            _pool = concurrent.futures.ThreadPoolExecutor(
                max_workers=1, thread_name_prefix="abc-offload")
        return _pool


def _side_stream(dev):
    with _pool_lock:
        if dev not in _side:
            _side[dev] = torch.cuda.Stream(device=dev)
        return _side[dev]


def _column(name):
    key = "_" + name

    def get(self):
        if self.__dict__.get("_pending") is not None:
            self._finish_offload()
        return self.__dict__.get(key)

    def set(self, value):
        if self.__dict__.get("_pending") is not None:
            self._finish_offload()
        self.__dict__[key] = value

    return property(get, set)


for _n in _COLUMNS:
    setattr(ColumnarPopulation, _n, _column(_n))
