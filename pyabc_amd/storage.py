"""History: the run's populations, in memory and (for a file database) in the
reference's SQL schema.

Reference: ``pyabc/storage/history.py:104-1229`` (SQLAlchemy ORM), schema
``storage/db_model.py:35-127``, summary-statistic blobs
``storage/numpy_bytes_storage.py:5-28`` / ``dataframe_bytes_storage.py``.

* ``History("sqlite://")`` (the reference's in-memory database id) keeps the
  populations of this process only, as device columns.
* ``History("sqlite:///path.db")`` also writes every population to an SQLite
  file with exactly the reference's tables, columns, id order and value
  encodings, so the reference's ``History`` (and its analysis / plotting
  code) reads a file written here, and this History reads files the
  reference wrote (``tests/test_history.py`` against
  ``tests/golden/ref_history.db``).  Writes are bulk (``executemany`` over
  columns built with numpy; a float64 statistic's ``np.save`` blob is a
  fixed 128-byte header + the 8 value bytes) instead of one ORM object per
  particle, parameter, sample and statistic.

Readers prefer the device population when ``t`` was written by this process
(the ABCSMC loop never reads its own populations back from disk); other
generations, and files opened with ``create=False`` / ``ABCSMC.load``, are
read with set-based SQL queries that reproduce the reference's ordering.
"""
import datetime
import io
import json
import os
import sqlite3
import threading
import weakref
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pandas as pd
import torch

from .population import ColumnarPopulation, Particle, Population
from .parameters import Parameter
from .distributed import agree_int, env_rank, env_world
from .acceptor import save_dict_to_json, load_dict_from_json  # noqa: F401

# History objects by db id, held weakly (a finished run's device and host
# populations are freed with its last reference)
_REGISTRY = weakref.WeakValueDictionary()


def _device_budget():
    """Device bytes a History may keep in older populations
    (``ABC_HISTORY_DEVICE_BYTES``, default a tenth of the device memory)."""
    env = os.environ.get("ABC_HISTORY_DEVICE_BYTES")
    if env is not None:
        return int(float(env))
    if not torch.cuda.is_available():
        return 0
    return torch.cuda.get_device_properties(
        torch.cuda.current_device()).total_memory // 10

# CREATE TABLE statements as SQLAlchemy emits them for db_model.py:35-127
_DDL = [
    """CREATE TABLE abc_smc (
\tid INTEGER NOT NULL,
\tstart_time DATETIME,
\tend_time DATETIME,
\tjson_parameters VARCHAR(5000),
\tdistance_function VARCHAR(5000),
\tepsilon_function VARCHAR(5000),
\tpopulation_strategy VARCHAR(5000),
\tgit_hash VARCHAR(120),
\tPRIMARY KEY (id)
)""",
    """CREATE TABLE populations (
\tid INTEGER NOT NULL,
\tabc_smc_id INTEGER,
\tt INTEGER,
\tpopulation_end_time DATETIME,
\tnr_samples INTEGER,
\tepsilon FLOAT,
\tPRIMARY KEY (id),
\tFOREIGN KEY(abc_smc_id) REFERENCES abc_smc (id)
)""",
    """CREATE TABLE models (
\tid INTEGER NOT NULL,
\tpopulation_id INTEGER,
\tm INTEGER,
\tname VARCHAR(200),
\tp_model FLOAT,
\tPRIMARY KEY (id),
\tFOREIGN KEY(population_id) REFERENCES populations (id)
)""",
    """CREATE TABLE particles (
\tid INTEGER NOT NULL,
\tmodel_id INTEGER,
\tw FLOAT,
\tPRIMARY KEY (id),
\tFOREIGN KEY(model_id) REFERENCES models (id)
)""",
    """CREATE TABLE parameters (
\tid INTEGER NOT NULL,
\tparticle_id INTEGER,
\tname VARCHAR(200),
\tvalue FLOAT,
\tPRIMARY KEY (id),
\tFOREIGN KEY(particle_id) REFERENCES particles (id)
)""",
    """CREATE TABLE samples (
\tid INTEGER NOT NULL,
\tparticle_id INTEGER,
\tdistance FLOAT,
\tPRIMARY KEY (id),
\tFOREIGN KEY(particle_id) REFERENCES particles (id)
)""",
    """CREATE TABLE summary_statistics (
\tid INTEGER NOT NULL,
\tsample_id INTEGER,
\tname VARCHAR(200),
\tvalue BLOB,
\tPRIMARY KEY (id),
\tFOREIGN KEY(sample_id) REFERENCES samples (id)
)""",
]

# history.py:51-61 without the optional gitpython dependency
_NO_GIT = "Install pyABC's optional git dependency for git support"
_TIME_FMT = "%Y-%m-%d %H:%M:%S.%f"


def _now():
    return datetime.datetime.now().strftime(_TIME_FMT)


# --- value encodings (numpy_bytes_storage.py:5-54, bytes_storage.py) -------
def np_to_bytes(arr):
    f = io.BytesIO()
    np.save(f, arr, allow_pickle=False)
    return f.getvalue()


def np_from_bytes(arr_bytes):
    arr = np.load(io.BytesIO(arr_bytes), allow_pickle=False)
    if arr.size == 1:
        for type_ in (int, float, str):
            try:
                if type_(arr) == arr:
                    return type_(arr)
            except (TypeError, ValueError, OverflowError):
                # OverflowError (int(inf)) escapes the reference's loader;
                # here an infinite statistic loads as a float
                pass
    return arr


def to_bytes(obj):
    if isinstance(obj, pd.Series):
        obj = obj.to_frame()
    if isinstance(obj, pd.DataFrame):
        import pyarrow
        import pyarrow.parquet as parquet
        b = io.BytesIO()
        parquet.write_table(pyarrow.Table.from_pandas(obj), b)
        return b.getvalue()
    return np_to_bytes(obj)


def from_bytes(b):
    if b[:6] == b"\x93NUMPY":
        return np_from_bytes(b)
    import pyarrow.parquet as parquet
    return parquet.read_table(io.BytesIO(b)).to_pandas()


_F8_HEADER = np_to_bytes(np.float64(0.0))[:-8]


def _f8_blobs(values):
    """np.save blobs of float64 scalars, built column-wise."""
    v = np.ascontiguousarray(values, dtype="<f8").reshape(-1)
    rows = np.empty((v.size, len(_F8_HEADER) + 8), dtype=np.uint8)
    rows[:, :len(_F8_HEADER)] = np.frombuffer(_F8_HEADER, dtype=np.uint8)
    rows[:, len(_F8_HEADER):] = v.view(np.uint8).reshape(-1, 8)
    return [r.tobytes() for r in rows]


def _flat_parameter_items(parameter):
    """history.py:660-671: one nesting level flattened as key_subkey."""
    for key, value in parameter.items():
        if isinstance(value, dict):
            for k2, v2 in value.items():
                yield key + "_" + k2, v2
        else:
            yield key, value


def _db_path(db):
    """history.py:165-167: ``sqlite:///rel`` / ``sqlite:////abs`` files,
    ``sqlite://`` an in-memory SQLite database; any other id is a
    device-only History (no SQL at all)."""
    if db == "sqlite://":
        return ":memory:"
    if not db.startswith("sqlite:///"):
        return None
    return db[len("sqlite:///"):]


class _Run:
    """Row of the abc_smc table (the reference returns ORM objects)."""

    def __init__(self, row):
        (self.id, self.start_time, self.end_time, self.json_parameters,
         self.distance_function, self.epsilon_function,
         self.population_strategy, self.git_hash) = row

    def __repr__(self):
        return (f"<ABCSMC(id={self.id}, start_time={self.start_time}, "
                f"end_time={self.end_time})>")


class _SQLStore:
    """The reference schema in one SQLite file, written in bulk."""

    def __init__(self, path):
        self.path = path
        self.conn = sqlite3.connect(path, timeout=120,
                                    check_same_thread=False)
        self.lock = threading.RLock()
        # one writer thread: population writes overlap the next generation
        self._pool = ThreadPoolExecutor(max_workers=1,
                                        thread_name_prefix="history-writer")
        self._pending = []
        have = {r[0] for r in self.conn.execute(
            "SELECT name FROM sqlite_master WHERE type='table'")}
        for ddl in _DDL:
            name = ddl.split()[2]
            if name not in have:
                self.conn.execute(ddl)
        self.conn.commit()

    def submit(self, fn, *args):
        self._pending.append(self._pool.submit(fn, *args))

    def busy(self):
        return any(not f.done() for f in self._pending)

    def flush(self):
        """Wait for queued writes (re-raising their errors)."""
        pending, self._pending = self._pending, []
        for f in pending:
            f.result()

    def q(self, sql, args=()):
        self.flush()
        with self.lock:
            return self.conn.execute(sql, args).fetchall()

    def execute(self, sql, args=()):
        self.flush()
        with self.lock:
            self.conn.execute(sql, args)
            self.conn.commit()

    def _q(self, sql, args=()):
        return self.conn.execute(sql, args).fetchall()

    def next_id(self, table):
        return self._q(f"SELECT COALESCE(MAX(id), 0) + 1 FROM {table}")[0][0]

    def population_id(self, abc_id, t):
        r = self.q("SELECT id FROM populations WHERE abc_smc_id=? AND t=?",
                   (abc_id, t))
        if len(r) != 1:
            raise ValueError(f"population t={t} of run {abc_id}: {len(r)} "
                             "rows (history.py:516-520 expects one)")
        return r[0][0]

    def write_population(self, abc_id, t, eps, nr_samples, models,
                         stores_sum_stats, end_time=None):
        """One population: ``models`` = [(m, name, p_model, block)], each
        block = dict(w [n], theta [n, d] + names, or host parameter dicts,
        distances [n], stats (keys, [S, n] float64) or per-particle dicts).
        Ids follow the reference's insertion order (history.py:632-687)."""
        with self.lock:
            self.begin()
            try:
                self._write_population(abc_id, t, eps, nr_samples, models,
                                       stores_sum_stats, end_time)
            except BaseException:
                self.conn.rollback()
                raise
            self.conn.commit()

    def begin(self):
        """Take the write lock before reading the next ids, so Histories on
        other connections to the same file cannot race for them."""
        if not self.conn.in_transaction:
            self.conn.execute("BEGIN IMMEDIATE")

    def _write_population(self, abc_id, t, eps, nr_samples, models,
                          stores_sum_stats, end_time):
        c = self.conn
        pop_id = self.next_id("populations")
        c.execute("INSERT INTO populations VALUES (?,?,?,?,?,?)",
                  (pop_id, abc_id, t, end_time or _now(), nr_samples,
                   float(eps)))
        mid = self.next_id("models")
        pid = self.next_id("particles")
        parid = self.next_id("parameters")
        sid = self.next_id("samples")
        ssid = self.next_id("summary_statistics")
        for m, name, p_model, blk in models:
            c.execute("INSERT INTO models VALUES (?,?,?,?,?)",
                      (mid, pop_id, None if m is None else int(m),
                       None if name is None else str(name),
                       float(p_model)))
            w = np.asarray(blk["w"], dtype=np.float64)
            n = w.size
            pids = np.arange(pid, pid + n, dtype=np.int64)
            c.executemany("INSERT INTO particles VALUES (?,?,?)",
                          zip(pids.tolist(), [mid] * n, w.tolist()))
            # parameters: particle-major, columns in parameter order
            if "theta" in blk:
                th = np.asarray(blk["theta"], dtype=np.float64)
                names = list(blk["names"])
                d = len(names)
                ids = range(parid, parid + n * d)
                c.executemany(
                    "INSERT INTO parameters VALUES (?,?,?,?)",
                    zip(ids, np.repeat(pids, d).tolist(), names * n,
                        th.reshape(-1).tolist()))
                parid += n * d
            else:
                rows = []
                for k, par in zip(pids.tolist(), blk["parameters"]):
                    for key, value in _flat_parameter_items(par):
                        rows.append((parid, k, key, float(value)))
                        parid += 1
                c.executemany("INSERT INTO parameters VALUES (?,?,?,?)",
                              rows)
            # samples: one accepted sample per particle (or a list each)
            dists = blk["distances"]
            if isinstance(dists, np.ndarray):
                spid = pids
                dvals = dists.astype(np.float64).tolist()
            else:
                spid = np.repeat(pids, [len(x) for x in dists])
                dvals = [float(x) for xs in dists for x in xs]
            ns = len(dvals)
            samp_ids = np.arange(sid, sid + ns, dtype=np.int64)
            c.executemany("INSERT INTO samples VALUES (?,?,?)",
                          zip(samp_ids.tolist(), spid.tolist(), dvals))
            sid += ns
            if stores_sum_stats:
                st = blk.get("stats")
                if isinstance(st, tuple):
                    keys, vals = st        # [S, n] float64, sample-major out
                    S = len(keys)
                    blobs = _f8_blobs(np.asarray(vals, dtype=np.float64).T)
                    c.executemany(
                        "INSERT INTO summary_statistics VALUES (?,?,?,?)",
                        zip(range(ssid, ssid + ns * S),
                            np.repeat(samp_ids, S).tolist(), list(keys) * ns,
                            blobs))
                    ssid += ns * S
                elif st is not None:
                    rows = []
                    for k, ss in zip(samp_ids.tolist(), st):
                        for key, value in ss.items():
                            if key is None:
                                raise Exception(
                                    "Summary statistics need names.")
                            rows.append((ssid, k, key, to_bytes(value)))
                            ssid += 1
                    c.executemany(
                        "INSERT INTO summary_statistics VALUES (?,?,?,?)",
                        rows)
            pid += n
            mid += 1


class History:
    """pyabc.History (history.py:104-1229); ``db`` is an SQLAlchemy-style id:
    ``"sqlite://"`` in memory, ``"sqlite:///file.db"`` persistent."""
    DB_TIMEOUT = 120
    PRE_TIME = -1

    def __init__(self, db="sqlite://", stores_sum_stats=True, _id=None,
                 create=True):
        path = _db_path(db)
        if not create and (path in (None, ":memory:")
                           or not os.path.exists(path)):
            raise ValueError(f"Database file {db} does not exist.")
        self.db = db
        self.stores_sum_stats = stores_sum_stats
        self.start_time = None
        self._pops = {}        # t -> dict(population, eps, n_sim, names)
        self._pre_nr_samples = 0
        self._meta = {}
        self._path = path
        # under torchrun every rank holds the same (global) populations; only
        # rank 0 writes SQL.  Other ranks keep them on the device and open a
        # file only to read a run they continue (create=False).
        self._writer = env_rank() == 0
        self._sql = _SQLStore(path) if path and (
            self._writer or (not create and path != ":memory:")) else None
        self._readonly = self._sql is not None and not self._writer
        self._file_max_t = None
        self._max_t = None
        self._dup = set()      # t appended more than once: SQL readers only
        self._id = self._find_latest_id() if _id is None else _id
        if self._id is None and self._sql is None:
            self._id = 1
        _REGISTRY[db] = self

    def __getstate__(self):
        """history.py:595-600: connections do not pickle; a file History
        reconnects on unpickling (device populations are not carried)."""
        if self._sql is not None:
            self._sql.flush()
        dct = self.__dict__.copy()
        dct["_sql"] = None
        dct["_pops"] = {}
        return dct

    def __setstate__(self, dct):
        self.__dict__.update(dct)
        if self._path not in (None, ":memory:"):
            self._sql = _SQLStore(self._path)
            self._max_t = None

    @staticmethod
    def lookup(db):
        return _REGISTRY.get(db)

    # --- identity -----------------------------------------------------------
    def db_file(self):
        return self.db.split(":")[-1][3:]

    @property
    def in_memory(self):
        return self._path in (None, ":memory:")

    @property
    def db_size(self):
        try:
            return os.path.getsize(self.db_file()) / 10 ** 6
        except FileNotFoundError:
            return "Cannot calculate size"

    def all_runs(self):
        if self._sql is None:
            return []
        return [_Run(r) for r in self._sql.q("SELECT * FROM abc_smc")]

    def _find_latest_id(self):
        """history.py:202-215: the last run that has populations."""
        if self._sql is None:
            return None
        for (rid,) in reversed(self._sql.q("SELECT id FROM abc_smc")):
            if self._sql.q("SELECT 1 FROM populations WHERE abc_smc_id=? "
                           "LIMIT 1", (rid,)):
                return rid
        return None

    @property
    def id(self):
        return self._id

    @id.setter
    def id(self, val):
        if val is None:
            val = self._find_latest_id()
        elif self._sql is not None and val not in [
                r[0] for r in self._sql.q("SELECT id FROM abc_smc")]:
            raise ValueError(f"Specified id {val} does not exist in database.")
        self._id = val
        self._max_t = None

    # --- writing ----------------------------------------------------------
    def store_initial_data(self, ground_truth_model, options,
                           observed_summary_statistics, ground_truth_parameter,
                           model_names, distance_function_json_str,
                           eps_function_json_str, population_strategy_json_str):
        """history.py:372-496: run row + the PRE_TIME dummy population."""
        self._meta = dict(start_time=datetime.datetime.now(),
                          gt_model=ground_truth_model, options=options,
                          x_0=observed_summary_statistics,
                          gt_par=ground_truth_parameter,
                          model_names=model_names,
                          distance=distance_function_json_str,
                          eps=eps_function_json_str,
                          population_strategy=population_strategy_json_str)
        self._pops = {}
        if self._sql is None or self._readonly:
            if env_world() > 1 and self._path:
                self._id = agree_int(0)   # the run id rank 0 creates below
            return
        s = self._sql
        s.flush()
        with s.lock:
            s.begin()
            self._id = s.next_id("abc_smc")
            s.conn.execute("INSERT INTO abc_smc VALUES (?,?,?,?,?,?,?,?)",
                           (self._id, _now(), None, str(options),
                            distance_function_json_str,
                            eps_function_json_str,
                            population_strategy_json_str, _NO_GIT))
        gt = dict(w=np.ones(1), parameters=[dict(ground_truth_parameter)],
                  distances=[[0.0]],
                  stats=[dict(observed_summary_statistics)])
        models = [(ground_truth_model,
                   None if ground_truth_model is None
                   else model_names[ground_truth_model], 1.0, gt)]
        models += [(m, name, 0.0, dict(w=np.zeros(0), parameters=[],
                                       distances=[], stats=[]))
                   for m, name in enumerate(model_names)
                   if m != ground_truth_model]
        s.write_population(self._id, History.PRE_TIME, np.inf, 0, models,
                           True)
        self._max_t = History.PRE_TIME
        if env_world() > 1:
            agree_int(self._id)

    def _offload_over_budget(self, t_new):
        held = []
        for t_old in sorted(self._pops):
            pop = self._pops[t_old]["population"]
            if t_old != t_new and hasattr(pop, "device_bytes"):
                held.append((t_old, pop))
        total = sum(p.device_bytes() for _, p in held)
        budget = _device_budget()
        for _, pop in held:          # oldest first
            if total <= budget:
                break
            total -= pop.device_bytes()
            pop.to_host()

    def update_nr_samples(self, t=PRE_TIME, nr_samples=0):
        if t == History.PRE_TIME:
            self._pre_nr_samples = nr_samples
        elif t in self._pops:
            self._pops[t]["n_sim"] = nr_samples
        if self._sql is not None and not self._readonly:
            pid = self._sql.population_id(self._id, t)
            self._sql.execute(
                "UPDATE populations SET nr_samples=? WHERE id=?",
                (int(nr_samples), pid))

    def append_population(self, t, current_epsilon, population, nr_simulations,
                          model_names):
        """history.py:696-729 (+ _save_to_population_db :616-693)."""
        if t in self._pops:
            self._dup.add(t)
        self._pops[t] = dict(population=population, eps=current_epsilon,
                             n_sim=nr_simulations, names=model_names,
                             end=datetime.datetime.now())
        # populations stay on the device up to a byte budget (default a tenth
        # of the device's memory: ~29 GB on an MI355X, ten generations of
        # N = 1e6, S = 100 statistics); beyond it the oldest move to host
        # memory (asynchronously, ColumnarPopulation.to_host), where every
        # reader still finds them.  The newest always stays (the next fit
        # and the loop read it).
        self._offload_over_budget(t)
        if self._sql is None or self._readonly:
            return
        mp = population.get_model_probabilities()
        if isinstance(population, ColumnarPopulation):
            blk = dict(w=population.w.cpu().numpy(),
                       theta=population.theta.cpu().numpy(),
                       names=population.names,
                       distances=population.d.cpu().numpy())
            if self.stores_sum_stats and population.stats_T is not None:
                blk["stats"] = (population.stat_keys,
                                population.stats_T.cpu().numpy())
            models = [(population.m, model_names[population.m],
                       mp[population.m], blk)]
        else:
            models = []
            for m, plist in population.to_dict().items():
                blk = dict(
                    w=np.array([p.weight for p in plist], dtype=np.float64),
                    parameters=[p.parameter for p in plist],
                    distances=[list(p.accepted_distances) for p in plist],
                    stats=[s for p in plist for s in p.accepted_sum_stats])
                models.append((int(m), model_names[m], mp[m], blk))
        self._max_t = max(int(t), self.max_t if self.max_t is not None
                          else int(t))
        # host copies are taken above; the SQL write runs on the writer
        # thread (readers and done() wait for it)
        self._sql.submit(
            self._sql.write_population, self._id, int(t), current_epsilon,
            int(nr_simulations), models, self.stores_sum_stats,
            self._pops[t]["end"].strftime(_TIME_FMT))

    def done(self):
        self._meta["end_time"] = datetime.datetime.now()
        if self._sql is not None and not self._readonly:
            self._sql.execute("UPDATE abc_smc SET end_time=? WHERE id=?",
                              (_now(), self._id))

    # --- reading ----------------------------------------------------------
    def _mem(self, t):
        """This process's population at t, when readers may use it: every
        population of a device-only History; with SQL, device populations
        appended once (host particle lists are read back through SQL, as
        the reference does, e.g. without their statistics when
        stores_sum_stats is off)."""
        e = self._pops.get(t)
        if self._sql is None or e is None:
            return e
        if t in self._dup or not isinstance(e["population"],
                                            ColumnarPopulation):
            return None
        return e

    def _q(self, sql, args=()):
        return self._sql.q(sql, args)

    _JOIN = ("FROM models mo JOIN populations po ON mo.population_id = po.id "
             "WHERE po.abc_smc_id = ? AND po.t = ?")

    @property
    def max_t(self):
        if self._sql is None:
            return max(self._pops) if self._pops else -1
        if self._readonly:
            # the file as opened (rank 0 appends to it asynchronously)
            # plus this process's own populations
            if self._file_max_t is None:
                self._file_max_t = self._q(
                    "SELECT MAX(t) FROM populations WHERE abc_smc_id=?",
                    (self._id,))[0][0]
                if self._file_max_t is None:
                    self._file_max_t = History.PRE_TIME
            return max([self._file_max_t] + list(self._pops))
        if self._max_t is not None and self._sql.busy():
            # while this History's writes are queued, the generation loop
            # reads the value append_population keeps current instead of
            # waiting for the writer thread
            return self._max_t
        # otherwise the file's value (another History may have appended)
        self._max_t = self._q("SELECT MAX(t) FROM populations WHERE "
                              "abc_smc_id=?", (self._id,))[0][0]
        return self._max_t

    @property
    def n_populations(self):
        return self.max_t + 1

    @property
    def total_nr_simulations(self):
        if self._sql is None:
            return self._pre_nr_samples + sum(p["n_sim"] for p in
                                              self._pops.values())
        return self._q("SELECT SUM(nr_samples) FROM populations "
                       "WHERE abc_smc_id=?", (self._id,))[0][0]

    def _t(self, t):
        return self.max_t if t is None else int(t)

    def observed_sum_stat(self):
        if self._sql is None:
            return self._meta.get("x_0", {})
        rows = self._q(
            "SELECT ss.name, ss.value FROM summary_statistics ss "
            "JOIN samples s ON ss.sample_id = s.id "
            "JOIN particles p ON s.particle_id = p.id "
            "JOIN models mo ON p.model_id = mo.id "
            "JOIN populations po ON mo.population_id = po.id "
            "WHERE po.abc_smc_id = ? AND po.t = ? AND mo.p_model = 1 "
            "ORDER BY ss.id", (self._id, History.PRE_TIME))
        return {name: from_bytes(v) for name, v in rows}

    def get_ground_truth_parameter(self):
        if self._sql is None:
            return Parameter(self._meta.get("gt_par", {}))
        rows = self._q(
            "SELECT pa.name, pa.value FROM parameters pa "
            "JOIN particles p ON pa.particle_id = p.id "
            "JOIN models mo ON p.model_id = mo.id "
            "JOIN populations po ON mo.population_id = po.id "
            "WHERE po.abc_smc_id = ? AND po.t = ? AND mo.p_model = 1 "
            "ORDER BY pa.id", (self._id, History.PRE_TIME))
        return Parameter({n: v for n, v in rows})

    def get_population_strategy(self):
        if self._sql is None:
            return json.loads(self._meta["population_strategy"])
        return json.loads(self._q(
            "SELECT population_strategy FROM abc_smc WHERE id=?",
            (self._id,))[0][0])

    def get_abc(self):
        return _Run(self._q("SELECT * FROM abc_smc WHERE id=?",
                            (self._id,))[0])

    def model_names(self, t=PRE_TIME):
        if self._sql is None:
            return list(self._meta.get("model_names", []))
        rows = self._q("SELECT DISTINCT mo.name, mo.m " + self._JOIN +
                       " AND mo.name IS NOT NULL ORDER BY mo.m",
                       (self._id, int(t)))
        return [r[0] for r in rows]

    def get_population(self, t=None):
        t = self._t(t)
        mem = self._mem(t)
        if mem is not None or self._sql is None:
            return mem["population"]
        return self._sql_population(t)

    def get_model_probabilities(self, t=None):
        """history.py:731-773."""
        if self._sql is None or (t is not None and t >= 0
                                 and self._mem(int(t)) is not None):
            if t is not None and t < 0:
                # before the first population: uniform over the model prior
                n = len(self._meta.get("model_names", [0]))
                return pd.DataFrame({"p": [1.0 / n] * n}, index=range(n))
            if t is None:
                return pd.DataFrame(
                    {t_: self._pops[t_]["population"]
                     .get_model_probabilities() for t_ in sorted(self._pops)}
                ).T.fillna(0)
            mp = self._pops[int(t)]["population"].get_model_probabilities()
            df = pd.DataFrame({"p": list(mp.values())}, index=list(mp.keys()))
            df.index.name = "m"
            return df
        if t is not None:
            rows = self._q("SELECT mo.p_model, mo.m " + self._JOIN +
                           " ORDER BY mo.m", (self._id, int(t)))
            df = pd.DataFrame(rows, columns=["p", "m"]).set_index("m")
            return df[df.p >= 0]
        rows = self._q(
            "SELECT mo.p_model, mo.m, po.t FROM models mo JOIN populations po "
            "ON mo.population_id = po.id WHERE po.abc_smc_id = ? AND po.t >= 0"
            " ORDER BY mo.m", (self._id,))
        return (pd.DataFrame(rows, columns=["p", "m", "t"])
                .pivot(index="t", columns="m", values="p").fillna(0))

    def model_probabilities_dict(self, t):
        """{m: p} of generation t, as get_model_probabilities(t)'s rows
        (the generation loop's fast path: no DataFrame for a population
        held in memory)."""
        if self._sql is None or (t >= 0 and self._mem(int(t)) is not None):
            if t < 0:
                n = len(self._meta.get("model_names", [0]))
                return {i: 1.0 / n for i in range(n)}
            return dict(self._pops[int(t)]["population"]
                        .get_model_probabilities())
        df = self.get_model_probabilities(t)
        return dict(zip(df.index, df.p))

    def alive_models(self, t=None):
        t = self._t(t)
        if self._sql is None or self._mem(t) is not None:
            return [m for m, p in self.model_probabilities_dict(t).items()
                    if p > 0]
        return sorted(r[0] for r in self._q("SELECT mo.m " + self._JOIN,
                                            (self._id, t)))

    def nr_of_models_alive(self, t=None):
        mp = self.model_probabilities_dict(self._t(t))
        return int(sum(1 for p in mp.values() if p > 0))

    def get_distribution(self, m=0, t=None):
        """history.py:268-313 (device frame for a population of this
        process; otherwise the reference's pivot of the parameters table)."""
        m, t = int(m), self._t(t)
        if self._sql is None or self._mem(t) is not None:
            return self.get_population(t).get_distribution(m)
        # the particles of (m, t) are one contiguous id range in files
        # written by either History: then two range scans replace the
        # four-table join (same rows)
        mids = [r[0] for r in self._q("SELECT mo.id " + self._JOIN +
                                      " AND mo.m = ?", (self._id, t, m))]
        rng = self._q("SELECT MIN(id), MAX(id), COUNT(*) FROM particles "
                      "WHERE model_id = ?", (mids[0],)) \
            if len(mids) == 1 else [(None, None, -1)]
        lo, hi, cnt = rng[0]
        if cnt > 0 and hi - lo + 1 == cnt:
            pw = self._q("SELECT id, w FROM particles WHERE id BETWEEN ? "
                         "AND ? ORDER BY id", (lo, hi))
            rows = self._q("SELECT particle_id, name, value FROM parameters"
                           " WHERE particle_id BETWEEN ? AND ?", (lo, hi))
            return self._pivot(rows, pw)
        else:
            rows = self._q(
                "SELECT p.id, pa.name, pa.value, p.w FROM parameters pa "
                "JOIN particles p ON pa.particle_id = p.id "
                "JOIN models mo ON p.model_id = mo.id "
                "JOIN populations po ON mo.population_id = po.id "
                "WHERE mo.m = ? AND po.t = ? AND po.abc_smc_id = ?",
                (m, t, self._id))
        pw = {}
        for r in rows:
            pw[r[0]] = r[3]
        return self._pivot([r[:3] for r in rows], sorted(pw.items()))

    @staticmethod
    def _pivot(rows, pw):
        """The reference's ``pivot(id, name, value).sort_index()`` and
        sorted weights (history.py:306-313), assembled with numpy (a pandas
        pivot of n*d rows takes tens of seconds at n = 1e6)."""
        n = len(rows)
        uid = np.fromiter((r[0] for r in pw), np.int64, len(pw))
        w_arr = np.fromiter((r[1] for r in pw), np.float64, len(pw))
        ids = np.fromiter((r[0] for r in rows), np.int64, n)
        vals = np.fromiter((r[2] for r in rows), np.float64, n)
        ucol = sorted({r[1] for r in rows})
        code = {c: i for i, c in enumerate(ucol)}
        col = np.fromiter((code[r[1]] for r in rows), np.int64, n)
        X = np.full((uid.size, len(ucol)), np.nan)
        X[np.searchsorted(uid, ids), col] = vals
        pars = pd.DataFrame(X, index=pd.Index(uid, name="id"),
                            columns=pd.Index(ucol, name="name"))
        if w_arr.size > 0 and not np.isclose(w_arr.sum(), 1):
            raise AssertionError(
                "Weight not close to 1, w.sum()={}".format(w_arr.sum()))
        return pars, w_arr

    def _samples(self, t, extra=""):
        return self._q(
            "SELECT p.w * mo.p_model, s.distance, s.id, p.id, mo.m, p.w "
            "FROM samples s JOIN particles p ON s.particle_id = p.id "
            "JOIN models mo ON p.model_id = mo.id "
            "JOIN populations po ON mo.population_id = po.id "
            "WHERE po.abc_smc_id = ? AND po.t = ?" + extra +
            " ORDER BY mo.id, p.id, s.id", (self._id, t))

    def _stats_of(self, sample_ids):
        out = {k: {} for k in sample_ids}
        if not sample_ids:
            return out
        lo, hi = min(sample_ids), max(sample_ids)
        for sid, name, v in self._q(
                "SELECT sample_id, name, value FROM summary_statistics "
                "WHERE sample_id BETWEEN ? AND ? ORDER BY id", (lo, hi)):
            if sid in out:
                out[sid][name] = from_bytes(v)
        return out

    def get_weighted_distances(self, t=None):
        """history.py:801-857."""
        t = self._t(t)
        if self._sql is None or self._mem(t) is not None:
            wd = self.get_population(t).get_weighted_distances()
            return wd.to_pandas() if hasattr(wd, "to_pandas") else wd
        rows = self._samples(t)
        return pd.DataFrame({"distance": [r[1] for r in rows],
                             "w": [r[0] for r in rows]})

    def get_weighted_sum_stats(self, t=None):
        """history.py:947-1001."""
        t = self._t(t)
        if self._sql is None or self._mem(t) is not None:
            pop = self.get_population(t)
            if isinstance(pop, ColumnarPopulation):
                pop = Population(pop.get_list())
            ws, ss = [], []
            mp = pop.get_model_probabilities()
            for p in pop.get_list():
                for s in p.accepted_sum_stats:
                    ws.append(p.weight * mp[p.m])
                    ss.append(s)
            return ws, ss
        rows = self._samples(t)
        st = self._stats_of([r[2] for r in rows])
        return [r[0] for r in rows], [st[r[2]] for r in rows]

    def get_weighted_sum_stats_for_model(self, m=0, t=None):
        """history.py:900-945 (weights without the model probability)."""
        m, t = int(m), self._t(t)
        if self._sql is None or self._mem(t) is not None:
            pop = self.get_population(t)
            plist = [p for p in pop.get_list() if p.m == m]
            ws = [p.weight for p in plist for _ in p.accepted_sum_stats]
            return np.array(ws), [s for p in plist
                                  for s in p.accepted_sum_stats]
        rows = self._samples(t, " AND mo.m = %d" % m)
        st = self._stats_of([r[2] for r in rows])
        return np.array([r[5] for r in rows]), [st[r[2]] for r in rows]

    def _sql_population(self, t):
        """history.py:1003-1078: host Population of stored particles."""
        rows = self._samples(t)
        st = self._stats_of([r[2] for r in rows])
        pars = {}
        for pid, name, v in self._q(
                "SELECT pa.particle_id, pa.name, pa.value FROM parameters pa "
                "JOIN particles p ON pa.particle_id = p.id "
                "JOIN models mo ON p.model_id = mo.id "
                "JOIN populations po ON mo.population_id = po.id "
                "WHERE po.abc_smc_id = ? AND po.t = ? ORDER BY pa.id",
                (self._id, t)):
            pars.setdefault(pid, {})[name] = v
        parts, by_pid = [], {}
        for wpm, dist, sid, pid, m, _ in rows:
            p = by_pid.get(pid)
            if p is None:
                p = Particle(m=m, parameter=Parameter(pars.get(pid, {})),
                             weight=wpm, accepted_sum_stats=[],
                             accepted_distances=[], accepted=True)
                by_pid[pid] = p
                parts.append(p)
            p.accepted_sum_stats.append(st[sid])
            p.accepted_distances.append(dist)
        return Population(parts)

    def get_nr_particles_per_population(self):
        """history.py:859-879."""
        if self._sql is None:
            return pd.Series({t: len(p["population"])
                              for t, p in self._pops.items()})
        rows = self._q(
            "SELECT po.t, COUNT(p.id) FROM populations po "
            "JOIN models mo ON mo.population_id = po.id "
            "JOIN particles p ON p.model_id = mo.id "
            "WHERE po.abc_smc_id = ? GROUP BY po.t ORDER BY po.t",
            (self._id,))
        return pd.Series([r[1] for r in rows],
                         index=pd.Index([r[0] for r in rows], name="t"),
                         name="count")

    def get_all_populations(self):
        """history.py:344-370."""
        if self._sql is None:
            # the PRE_TIME row first, as the reference's table holds it
            rows = [dict(t=History.PRE_TIME,
                         population_end_time=self._meta.get("start_time"),
                         samples=self._pre_nr_samples, epsilon=np.inf,
                         particles=1)]
            rows += [dict(t=t, population_end_time=p["end"],
                          samples=p["n_sim"], epsilon=p["eps"],
                          particles=len(p["population"]))
                     for t, p in sorted(self._pops.items())]
            return pd.DataFrame(rows)
        rows = self._q("SELECT t, population_end_time, nr_samples, epsilon "
                       "FROM populations WHERE abc_smc_id=? ORDER BY id",
                       (self._id,))
        df = pd.DataFrame(rows, columns=["t", "population_end_time",
                                         "nr_samples", "epsilon"])
        df["population_end_time"] = pd.to_datetime(df["population_end_time"])
        particles = self.get_nr_particles_per_population()
        particles.index += 1
        df["particles"] = particles
        return df.rename(columns={"nr_samples": "samples"})

    def get_population_extended(self, *, m=None, t="last", tidy=True):
        """history.py:1092-1204 (file databases)."""
        if self._sql is None:
            raise NotImplementedError(
                "get_population_extended reads the SQL store: use a "
                "'sqlite:///file.db' History")
        if t == "last":
            t = self.max_t
        sql = ("SELECT po.t, po.epsilon, po.nr_samples, mo.m, mo.name, "
               "mo.p_model, p.w, p.id, s.distance, pa.name, pa.value, "
               "ss.name, ss.value FROM populations po "
               "JOIN models mo ON mo.population_id = po.id "
               "JOIN particles p ON p.model_id = mo.id "
               "JOIN samples s ON s.particle_id = p.id "
               "JOIN summary_statistics ss ON ss.sample_id = s.id "
               "JOIN parameters pa ON pa.particle_id = p.id "
               "WHERE po.abc_smc_id = ?")
        args = [self._id]
        if m is not None:
            sql += " AND mo.m = ?"
            args.append(int(m))
        if t != "all":
            sql += " AND po.t = ?"
            args.append(int(t))
        cols = ["t", "epsilon", "samples", "m", "model_name", "p_model", "w",
                "particle_id", "distance", "par_name", "par_val",
                "sumstat_name", "sumstat_val"]
        rows = self._q(sql + " ORDER BY p.id, ss.id, pa.id", args)
        df = pd.DataFrame(rows, columns=cols)
        df["sumstat_val"] = [from_bytes(v) for v in df["sumstat_val"]]
        if len(df.m.unique()) == 1:
            del df["m"], df["model_name"], df["p_model"]
        if isinstance(t, int):
            del df["t"]
        if tidy and isinstance(t, int) and "m" not in df:
            df = df.set_index("particle_id")
            df_unique = df[["distance", "w"]].drop_duplicates()
            df_par = (df[["par_name", "par_val"]].reset_index()
                      .drop_duplicates(subset=["particle_id", "par_name"])
                      .pivot(index="particle_id", columns="par_name",
                             values="par_val"))
            df_par.columns = ["par_" + c for c in df_par.columns]
            df_ss = (df[["sumstat_name", "sumstat_val"]].reset_index()
                     .drop_duplicates(subset=["particle_id", "sumstat_name"])
                     .pivot(index="particle_id", columns="sumstat_name",
                            values="sumstat_val"))
            df_ss.columns = ["sumstat_" + c for c in df_ss.columns]
            df = df_unique.merge(df_par, left_index=True, right_index=True) \
                .merge(df_ss, left_index=True, right_index=True)
        return df

    def distribution_numpy(self, m=0, t=None):
        """(DataFrame, ndarray) host copies of get_distribution."""
        df, w = self.get_distribution(m, t)
        if hasattr(df, "to_pandas"):
            df = df.to_pandas()
        if hasattr(w, "cpu"):
            w = w.cpu().numpy()
        return df, np.asarray(w)


def create_sqlite_db_id(dir_=None, file_="pyabc_test.db"):
    """history.py:64-83: ``sqlite:///`` + a file in ``dir_`` (default: the
    temp dir)."""
    import tempfile
    if dir_ is None:
        dir_ = tempfile.gettempdir()
    return "sqlite:///" + os.path.join(dir_, file_)


def is_columnar(pop):
    return isinstance(pop, ColumnarPopulation)
