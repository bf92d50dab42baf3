"""Multi-rank host logic under torchrun semantics, on the CPU (gloo,
world size 2): decisions every rank must share come from rank 0, and only
rank 0 writes the SQL History (a run is one abc_smc row however many ranks
drive it)."""
import os
import socket
import sqlite3
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo")


def _history_rank(rank, world, port, path, out):
    _init(rank, world, port)
    import torch.distributed as dist
    from tests.test_history import write_ours
    from pyabc_amd.distributed import agree_int
    # rank-local numpy states differ: the agreed value is rank 0's
    np.random.seed(100 + rank)
    out[f"seed{rank}"] = agree_int(int(np.random.randint(0, 2 ** 62)))
    h = write_ours(path)
    out[f"id{rank}"] = h.id
    out[f"max_t{rank}"] = h.max_t
    df, w = h.get_distribution(0, h.max_t)
    out[f"dist{rank}"] = (df.values.tolist(), list(w))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_ranks_one_sql_run(tmp_path):
    """Two ranks drive the same run into one sqlite file: one abc_smc row,
    one row per population, the same run id and the same readers' answers
    on both ranks (rank 1 serves them from memory)."""
    path = str(tmp_path / "run.db")
    # a previous run in the file: the new run's id is 2 on both ranks
    sys.path.insert(0, ROOT)
    from tests.test_history import write_ours
    write_ours(path)
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_history_rank, args=(2, port, path, out), nprocs=2,
                 join=True)
        res = dict(out)
    assert res["seed0"] == res["seed1"]
    assert res["id0"] == res["id1"] == 2
    assert res["max_t0"] == res["max_t1"]
    assert res["dist0"] == res["dist1"]
    c = sqlite3.connect(path)
    runs = c.execute("SELECT id FROM abc_smc").fetchall()
    n_pops = c.execute("SELECT COUNT(*) FROM populations WHERE abc_smc_id=2"
                       ).fetchone()[0]
    n_pops1 = c.execute("SELECT COUNT(*) FROM populations WHERE abc_smc_id=1"
                        ).fetchone()[0]
    c.close()
    assert [r[0] for r in runs] == [1, 2]
    assert n_pops == n_pops1 > 1


def _forced_rank(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      ABC_COMM_FORCE="1")
    sys.path.insert(0, ROOT)
    import torch
    from pyabc_amd.distributed import Comm
    comm = Comm.from_env("gloo")
    assert comm.active and comm.world == 1
    assert Comm.current().active
    x = torch.arange(12, dtype=torch.float64).reshape(6, 2)
    out["rows"] = comm.all_gather_rows(x).numpy().tolist()
    out["ints"] = comm.all_gather_ints(5)
    out["lists"] = comm.all_gather_int_lists([1, 2, 3])
    out["sum"] = comm.all_reduce_ints([4, 7])
    comm.barrier()
    torch.distributed.destroy_process_group()


def test_forced_one_rank_group_runs_collectives():
    """ABC_COMM_FORCE=1 under a one-rank process group: the communicator is
    active and every collective runs (the RCCL self-test's host path) with
    the identity result."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_forced_rank, args=(port, out), nprocs=1, join=True)
        res = dict(out)
    assert res["rows"] == np.arange(12.0).reshape(6, 2).tolist()
    assert res["ints"] == [5]
    assert res["lists"] == [[1, 2, 3]]
    assert res["sum"] == [4, 7]


def test_rank_slice_comm_matches_identical_ranks():
    """bench.py --rank-slice R: RankSliceComm answers every collective as R
    ranks holding this rank's data would (sums x R, maxima / minima as is,
    gathers replicate this rank's rows), and counts calls and bytes."""
    import torch
    from pyabc_amd.distributed import RankSliceComm
    from pyabc_amd.engine import gather_segments, selection_plan
    c = RankSliceComm(4)
    assert c.active and c.world == 4 and c.rank == 0
    assert c.all_gather_ints(torch.tensor(7)) == [7] * 4
    assert c.all_reduce_ints([3, 5]) == [12, 20]
    assert c.all_gather_int_lists([1, 2]) == [[1, 2]] * 4
    words = torch.tensor([5, 9], dtype=torch.int64)
    c.all_reduce_words(words, 1)
    assert words.tolist() == [20, 36]
    c.all_reduce_words(words, 4)
    assert words.tolist() == [20, 36]
    assert c.all_reduce_max_float(1.5) == 1.5
    rows = torch.arange(12, dtype=torch.float64).reshape(6, 2)
    g = c.all_gather_rows(rows, [6, 6, 4, 0])
    assert g.shape == (16, 2)
    assert torch.equal(g[6:12], rows) and torch.equal(g[12:], rows[:4])
    # a rank holding no rows still returns sum(sizes) rows (advisor r04)
    g0 = RankSliceComm(4).all_gather_rows(rows[:0], [0, 3, 2, 0])
    assert g0.shape == (5, 2)
    # the engine's selection and segment gather run on it unchanged
    takes, closing = selection_plan([[5] * 4, [5] * 4], [[2] * 4, [3] * 4], 13)
    counts = [[t[s] for t in takes] for s in range(4)]
    got = gather_segments(c, [rows[:2], rows[2:5]], (2,), counts, "cpu")
    assert got.shape[0] == 13
    s = c.summary()
    assert s["all_gather_rows"][0] == 2
    # 6 + 5 rows sent, (16 - 6) + (13 - 5) received, 16 B per row
    assert s["all_gather_rows"][1:] == [(6 + 5) * 16, (10 + 8) * 16]
