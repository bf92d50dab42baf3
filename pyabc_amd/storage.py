"""In-memory History (the subset of pyabc/storage/history.py:104-1229 that
ABCSMC and the analysis helpers use).  Populations stay on the device as
columns; ``get_distribution`` hands the transition a DeviceFrame, so the fit
of the next generation never leaves HBM.  SQL persistence (the reference's
SQLAlchemy schema, db_model.py:35-127) is out of scope for this tier
(SURVEY 8(f) rank 1)."""
import datetime

import numpy as np
import pandas as pd

from .population import ColumnarPopulation
from .acceptor import save_dict_to_json, load_dict_from_json  # noqa: F401

_REGISTRY = {}


class History:
    PRE_TIME = -1

    def __init__(self, db="sqlite://", stores_sum_stats=True):
        self.db = db
        self.stores_sum_stats = stores_sum_stats
        self.id = 1
        self.start_time = None
        self._pops = {}        # t -> dict(population, eps, n_sim, names)
        self._pre_nr_samples = 0
        self._meta = {}
        _REGISTRY[db] = self

    @staticmethod
    def lookup(db):
        return _REGISTRY.get(db)

    # --- writing ----------------------------------------------------------
    def store_initial_data(self, ground_truth_model, options,
                           observed_summary_statistics, ground_truth_parameter,
                           model_names, distance_function_json_str,
                           eps_function_json_str, population_strategy_json_str):
        self._meta = dict(gt_model=ground_truth_model, options=options,
                          x_0=observed_summary_statistics,
                          gt_par=ground_truth_parameter,
                          model_names=model_names,
                          distance=distance_function_json_str,
                          eps=eps_function_json_str,
                          population_strategy=population_strategy_json_str)

    def update_nr_samples(self, t=PRE_TIME, nr_samples=0):
        if t == History.PRE_TIME:
            self._pre_nr_samples = nr_samples
        else:
            self._pops[t]["n_sim"] = nr_samples

    def append_population(self, t, current_epsilon, population, nr_simulations,
                          model_names):
        self._pops[t] = dict(population=population, eps=current_epsilon,
                             n_sim=nr_simulations, names=model_names,
                             end=datetime.datetime.now())

    def done(self):
        self._meta["end_time"] = datetime.datetime.now()

    # --- reading ----------------------------------------------------------
    @property
    def max_t(self):
        return max(self._pops) if self._pops else -1

    @property
    def n_populations(self):
        return len(self._pops)

    @property
    def total_nr_simulations(self):
        return self._pre_nr_samples + sum(p["n_sim"] for p in
                                          self._pops.values())

    def observed_sum_stat(self):
        return self._meta.get("x_0", {})

    def _t(self, t):
        return self.max_t if t is None else t

    def get_population(self, t=None):
        return self._pops[self._t(t)]["population"]

    def get_model_probabilities(self, t=None):
        if t is not None and t < 0:
            # before the first population: uniform over the model prior
            n = len(self._meta.get("model_names", [0]))
            return pd.DataFrame({"p": [1.0 / n] * n}, index=range(n))
        pop = self.get_population(t)
        mp = pop.get_model_probabilities()
        df = pd.DataFrame({"p": list(mp.values())}, index=list(mp.keys()))
        df.index.name = "m"
        return df

    def alive_models(self, t=None):
        mp = self.get_model_probabilities(t)
        return list(mp.index[mp.p > 0])

    def nr_of_models_alive(self, t=None):
        return len(self.alive_models(t))

    def get_distribution(self, m=0, t=None):
        return self.get_population(t).get_distribution(m)

    def get_weighted_distances(self, t=None):
        wd = self.get_population(t).get_weighted_distances()
        return wd.to_pandas() if hasattr(wd, "to_pandas") else wd

    def get_nr_particles_per_population(self):
        return pd.Series({t: len(p["population"])
                          for t, p in self._pops.items()})

    def get_all_populations(self):
        rows = [dict(t=t, population_end_time=p["end"], samples=p["n_sim"],
                     epsilon=p["eps"], particles=len(p["population"]))
                for t, p in sorted(self._pops.items())]
        return pd.DataFrame(rows)

    def get_ground_truth_parameter(self):
        return self._meta.get("gt_par", {})

    def distribution_numpy(self, m=0, t=None):
        """(DataFrame, ndarray) host copies of get_distribution."""
        df, w = self.get_distribution(m, t)
        if hasattr(df, "to_pandas"):
            df = df.to_pandas()
        if hasattr(w, "cpu"):
            w = w.cpu().numpy()
        return df, np.asarray(w)


def create_sqlite_db_id(dir_=None, file_="pyabc_test.db"):
    """A fresh in-memory history id (history.py:57-75 names a sqlite file;
    the in-memory History only needs a unique key)."""
    import uuid
    return f"sqlite:///{dir_ or '/tmp'}/{uuid.uuid4().hex}_{file_}"


def is_columnar(pop):
    return isinstance(pop, ColumnarPopulation)
