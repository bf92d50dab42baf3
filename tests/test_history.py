"""Persistent History in the reference's SQL schema, on
the CPU.  Pinned by ``tests/golden/ref_history.db`` (written by the
reference's own History, ``tools/gen_golden_history.py``) and
``ref_history_read.npz`` (its readers' outputs on that file).  The same
script's ``--check-ours`` mode has the reference History read a file written
here (run in the build container, where the reference is importable)."""
import os
import shutil
import sqlite3
import sys

import numpy as np
import pandas as pd
import pytest
import torch

import pyabc_amd as pa
from pyabc_amd.population import ColumnarPopulation

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
import gen_golden_history as G  # noqa: E402  (run_data / readers / compare)

REF_DB = os.path.join(HERE, "golden", "ref_history.db")
TIME_COLS = {"abc_smc": (1, 2), "populations": (3,)}
TABLES = ["abc_smc", "populations", "models", "particles", "parameters",
          "samples", "summary_statistics"]


def write_ours(path, columnar=False):
    init, gens = G.run_data()
    h = pa.History("sqlite:///" + path)
    h.store_initial_data(init["gt_model"], init["options"], init["x_0"],
                         init["gt_par"], init["names"], init["dist"],
                         init["eps"], init["pop"])
    h.update_nr_samples(-1, 13)
    for t, eps, nsim, parts in gens:
        single = len({p[0] for p in parts}) == 1
        if columnar and single:
            names = list(parts[0][2])
            w = np.array([p[1] for p in parts])
            keys = ["y1", "y0"]
            pop = ColumnarPopulation(
                torch.tensor([[p[2][k] for k in names] for p in parts],
                             dtype=torch.float64),
                torch.tensor(w / w.sum()),
                torch.tensor([p[3] for p in parts], dtype=torch.float64),
                names,
                torch.tensor([[p[4][k] for p in parts] for k in keys],
                             dtype=torch.float64), keys, m=parts[0][0],
                normalize=False)
        else:
            pop = pa.Population([
                pa.Particle(m, pa.Parameter(par), w, [st], [dd])
                for m, w, par, dd, st in parts])
        h.append_population(t, eps, pop, nsim, init["names"])
    h.done()
    return h


def table_rows(path, table):
    c = sqlite3.connect(path)
    rows = c.execute(f"SELECT * FROM {table} ORDER BY id").fetchall()
    c.close()
    drop = TIME_COLS.get(table, ())
    return [tuple(v for i, v in enumerate(r) if i not in drop) for r in rows]


def test_schema_equals_reference(tmp_path):
    p = str(tmp_path / "h.db")
    pa.History("sqlite:///" + p)
    norm = lambda db: sorted(  # noqa: E731
        " ".join(s.split()) for (s,) in sqlite3.connect(db).execute(
            "SELECT sql FROM sqlite_master WHERE type='table'"))
    assert norm(p) == norm(REF_DB)


def test_rows_equal_reference_file(tmp_path):
    """Every table, row by row (ids, foreign keys, values, np.save blobs),
    equals the file the reference wrote for the same run; only the
    wall-clock columns differ."""
    p = str(tmp_path / "h.db")
    write_ours(p)
    for tb in TABLES:
        assert table_rows(p, tb) == table_rows(REF_DB, tb), tb


def test_reads_reference_file():
    """The reference's file, read here: every reader equals the reference's
    readers on it (history.py:236-1229)."""
    h = pa.History("sqlite:///" + REF_DB, create=False)
    want = dict(np.load(os.path.join(HERE, "golden",
                                     "ref_history_read.npz")))
    want.pop("_ref")
    G.compare(G.readers(h), want)


def test_reads_own_file_like_reference(tmp_path):
    p = str(tmp_path / "h.db")
    write_ours(p)
    want = dict(np.load(os.path.join(HERE, "golden",
                                     "ref_history_read.npz")))
    want.pop("_ref")
    G.compare(G.readers(pa.History("sqlite:///" + p, create=False)), want)


def test_columnar_bulk_write_equals_particle_write(tmp_path):
    """The bulk writer of a device population (columns -> executemany,
    vectorised np.save blobs) produces the same rows as the per-particle
    path, except the statistics it does not hold (here 'arr')."""
    a, b = str(tmp_path / "a.db"), str(tmp_path / "b.db")
    write_ours(a)
    write_ours(b, columnar=True)
    for tb in TABLES[:-1]:
        assert table_rows(a, tb) == table_rows(b, tb), tb
    ca = [r for r in table_rows(a, "summary_statistics") if r[2] != "arr"]
    cb = [r for r in table_rows(b, "summary_statistics") if r[2] != "arr"]
    # the columnar statistics are y1, y0 per sample (no array statistic), so
    # ids differ; sample ids, names and blobs agree in order
    assert len(ca) == len(cb) > 0
    assert [r[1:] for r in ca] == [r[1:] for r in cb]


def test_blob_codec_matches_np_save():
    vals = np.array([0.0, -0.25, np.inf, np.nan, 1e-300, 3.5])
    from pyabc_amd import storage as S
    for v, blob in zip(vals, S._f8_blobs(vals)):
        assert blob == S.np_to_bytes(np.float64(v))
        got = S.from_bytes(blob)
        assert (got == v) or (np.isnan(got) and np.isnan(v))
    arr = np.arange(6.0).reshape(2, 3)
    np.testing.assert_array_equal(S.from_bytes(S.to_bytes(arr)), arr)


def test_open_errors_and_ids(tmp_path):
    with pytest.raises(ValueError):
        pa.History("sqlite:///" + str(tmp_path / "missing.db"), create=False)
    p = str(tmp_path / "h.db")
    shutil.copy(REF_DB, p)
    h = pa.History("sqlite:///" + p)
    assert h.id == 1 and len(h.all_runs()) == 1
    with pytest.raises(ValueError):
        h.id = 7
    # a second run in the same file gets the next id; readers follow it
    h2 = write_ours(p)
    assert h2.id == 2
    assert pa.History("sqlite:///" + p).id == 2
    assert h2.max_t == 1 and h2.total_nr_simulations == 13 + 21 + 28
    assert pa.History("sqlite:///" + p, _id=1).max_t == 1


def test_in_memory_id_keeps_device_populations():
    h = pa.History("sqlite://")
    assert h.in_memory and h.all_runs() == []


# --- the reference's storage contract (test/test_storage.py), file and
# in-memory SQL databases; R data frames (rpy2) are not available here ----
def _example_df():
    return pd.DataFrame({"col_a": [1, 2], "col_b": [1.1, 2.2],
                         "col_c": ["foo", "bar"]},
                        index=["ind_first", "ind_second"])


def _one(w=.2):
    return [pa.Particle(0, pa.Parameter({"a": 23, "b": 12}), w,
                        [{"ss": .1}], [.1])]


def _rand_pop_list(m, rng):
    return [pa.Particle(m, pa.Parameter({"a": int(rng.integers(10)),
                                         "b": float(rng.normal())}),
                        float(rng.uniform()) * 42,
                        [{"ss_float": 0.1, "ss_int": 42,
                          "ss_str": "foo bar string",
                          "ss_np": rng.uniform(size=(13, 42)),
                          "ss_df": _example_df()}],
                        [float(rng.uniform())])
            for _ in range(int(rng.integers(10)) + 3)]


@pytest.fixture(params=["file", "memory"])
def history(request, tmp_path):
    db = ("sqlite:///" + str(tmp_path / "history_test.db")
          if request.param == "file" else "sqlite://")
    h = pa.History(db)
    h.store_initial_data(0, {}, {}, {},
                         [f"fake_name_{k}" for k in range(50)], "", "",
                         '{"name": "pop_strategy_str_test"}')
    return h


def test_ref_single_particle_np_int64_indexing(history):
    history.append_population(0, 42, pa.Population(_one()), 2, [""])
    for m in (0, np.int64(0)):
        for t in (0, np.int64(0)):
            df, w = history.get_distribution(m, t)
            assert w[0] == 1 and df.a.iloc[0] == 23 and df.b.iloc[0] == 12


def test_ref_save_no_sum_stats(history):
    rng = np.random.default_rng(0)
    plist = [pa.Particle(0, pa.Parameter({"th0": float(rng.uniform())}), .2,
                         [{"ss0": float(rng.uniform()),
                           "ss1": float(rng.uniform())}],
                         [float(rng.uniform())]) for _ in range(6)]
    pop = pa.Population(plist)
    history.stores_sum_stats = False
    history.append_population(t=0, current_epsilon=42.97, population=pop,
                              nr_simulations=10, model_names=[""])
    history.get_distribution(0, 0)
    wd_h = history.get_weighted_distances()
    wd = pop.get_weighted_distances()
    assert (wd_h[["distance", "w"]] == wd[["distance", "w"]]).all().all()
    weights, sum_stats = history.get_weighted_sum_stats(t=0)
    assert len(weights) == len(plist)
    assert all(not s for s in sum_stats)
    history.get_population_extended()


def test_ref_get_population(history):
    rng = np.random.default_rng(1)
    pop = pa.Population(_rand_pop_list(0, rng))
    history.append_population(t=0, current_epsilon=7.0, population=pop,
                              nr_simulations=200, model_names=["m0"])
    pop_h = history.get_population(t=0)
    assert len(pop) == len(pop_h)
    np.testing.assert_allclose(
        sum((p.accepted_distances for p in pop.get_list()), []),
        sum((p.accepted_distances for p in pop_h.get_list()), []))
    np.testing.assert_allclose([p.weight for p in pop.get_list()],
                               [p.weight for p in pop_h.get_list()])


def test_ref_sum_stats_save_load(history):
    rng = np.random.default_rng(2)
    arr, arr2 = rng.uniform(size=10), rng.uniform(size=(10, 2))
    plist = [pa.Particle(0, pa.Parameter({"a": 23, "b": 12}), .2,
                         [{"ss1": .1, "ss2": arr2, "ss3": _example_df()}],
                         [.1]),
             pa.Particle(0, pa.Parameter({"a": 23, "b": 12}), .2,
                         [{"ss12": .11, "ss22": arr, "ss33": _example_df()}],
                         [.1])]
    history.append_population(0, 42, pa.Population(plist), 2, ["m1", "m2"])
    weights, ss = history.get_weighted_sum_stats_for_model(0, 0)
    assert (weights == 0.5).all()
    assert ss[0]["ss1"] == .1 and (ss[0]["ss2"] == arr2).all()
    assert (ss[0]["ss3"] == _example_df()).all().all()
    assert ss[1]["ss12"] == .11 and (ss[1]["ss22"] == arr).all()
    assert (ss[1]["ss33"] == _example_df()).all().all()


def test_ref_total_nr_samples_and_t_count(history):
    pop = pa.Population(_one())
    history.append_population(0, 42, pop, 4234, ["m1"])
    history.append_population(0, 42, pop, 3, ["m1"])
    assert history.total_nr_simulations == 4237
    for t in range(1, 10):
        history.append_population(t, 42, pa.Population(_one()), 2, ["m1"])
        assert history.max_t == t


def test_ref_population_retrieval_and_models(history):
    rng = np.random.default_rng(3)
    history.append_population(1, .23, pa.Population(_rand_pop_list(0, rng)),
                              234, ["m1"])
    history.append_population(2, .123, pa.Population(_rand_pop_list(0, rng)),
                              345, ["m1"])
    history.append_population(2, .1235,
                              pa.Population(_rand_pop_list(5, rng)), 20345,
                              ["m1"] * 6)
    history.append_population(3, .12330,
                              pa.Population(_rand_pop_list(30, rng)), 30345,
                              ["m1"] * 31)
    df = history.get_all_populations()
    assert list(df[df.t == 2].epsilon) == [.123, .1235]
    assert list(df[df.t == 2].samples) == [345, 20345]
    assert df[df.t == 3].samples.iloc[0] == 30345
    assert history.alive_models(1) == [0]
    assert history.alive_models(2) == [0, 5]
    assert history.alive_models(3) == [30]
    assert history.get_population_strategy()["name"] == \
        "pop_strategy_str_test"


def test_ref_model_probabilities(history):
    rng = np.random.default_rng(4)
    history.append_population(1, .23, pa.Population(_rand_pop_list(3, rng)),
                              234, ["m0", "m1", "m2", "m3"])
    probs = history.get_model_probabilities(1)
    assert probs.p[3] == 1 and probs.index.tolist() == [3]
    assert (history.get_model_probabilities()[3].values == [1]).all()


def test_ref_population_extended_and_update_nr_samples(history):
    rng = np.random.default_rng(5)
    for t in range(3):
        for m in range(4):
            history.append_population(t, .23,
                                      pa.Population(_rand_pop_list(m, rng)),
                                      234, ["m0", "m1", "m2", "m3"])
    df = history.get_population_extended(m=0)
    assert len(df) > 0 and "sumstat_ss_np" in df.columns
    history.store_initial_data(None, {}, {}, {}, ["m0"], "", "", "")
    pops = history.get_all_populations()
    assert pops[pops.t == pa.History.PRE_TIME].samples.values == 0
    history.update_nr_samples(pa.History.PRE_TIME, 43)
    pops = history.get_all_populations()
    assert pops[pops.t == pa.History.PRE_TIME].samples.values == 43


def test_ref_pickle(history):
    import pickle
    history.append_population(0, 42, pa.Population(_one()), 2, [""])
    h2 = pickle.loads(pickle.dumps(history))
    if not history.in_memory:
        assert h2.get_distribution(0, 0)[0].a.iloc[0] == 23


@pytest.mark.parametrize("gt_model", [0, None])
def test_ref_observed_sum_stats_and_names(tmp_path, gt_model):
    db = "sqlite:///" + str(tmp_path / "h.db")
    obs = {"s1": 1, "s2": 1.1, "s3": np.array(.1),
           "s4": np.random.default_rng(6).uniform(size=10)}
    pa.History(db).store_initial_data(gt_model, {}, obs, {},
                                      ["m1", "m2", "m3"], "", "", "")
    h2 = pa.History(db)
    got = h2.observed_sum_stat()
    for k in ["s1", "s2", "s3"]:
        assert got[k] == obs[k]
    assert type(got["s1"]) is int and type(got["s2"]) is float
    assert (got["s4"] == obs["s4"]).all() and got["s4"] is not obs["s4"]
    assert h2.model_names() == ["m1", "m2", "m3"]


def test_ref_dataframe_storage_readout(tmp_path):
    """Four Histories (four connections) on one file, five models each."""
    db = "sqlite:///" + str(tmp_path / "h.db")
    rng = np.random.default_rng(7)
    names = ["fake_name"] * 5
    hs = []
    for _ in range(4):
        h = pa.History(db)
        h.store_initial_data(0, {}, {}, {}, names, "", "", "")
        hs.append(h)
    pops = {}
    for k, h in enumerate(hs):
        for t in range(4):
            plist = []
            for m in range(5):
                pops[(k, m, t)] = _rand_pop_list(m, rng)
                plist += pops[(k, m, t)]
            h.append_population(t, .1, pa.Population(plist), 2, names)
    for k, h in enumerate(hs):
        for t in range(4):
            for m in range(5):
                df, w = h.get_distribution(m, t)
                assert np.isclose(w.sum(), 1)
                exp = pops[(k, m, t)]
                np.testing.assert_array_equal(df.a.values,
                                              [p.parameter["a"] for p in exp])
                np.testing.assert_array_equal(df.b.values,
                                              [p.parameter["b"] for p in exp])


def test_ref_create_db(tmp_path):
    import tempfile
    f = tempfile.mkstemp(suffix=".db", dir=str(tmp_path))[1]
    pa.History("sqlite:///" + f, create=False)
    os.remove(f)
    with pytest.raises(ValueError):
        pa.History("sqlite:///" + f, create=False)
