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
