"""Multi-rank generation path on ONE GPU (rehearsal of SURVEY 8(e)).

Two ranks share cuda:0 and exchange through gloo (host-staged all-gather),
so the exact engine / bench code that runs one rank per GPU over RCCL is
exercised with real HIP kernels: global-id Philox streams, the per-round
count exchange, the all-gather of the accepted rows, the row-parallel KDE
pass with its all-gathered log-densities, and the redundant deterministic
fit / epsilon on every rank -- checked bit for bit against one rank.
"""
import json
import math
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _generation(comm, n, min_batch, record):
    """Prior population, one SMC generation, the next epsilon: the bench's
    and the sampler's sequence of engine calls."""
    from pyabc_amd import kernels as K
    from pyabc_amd.batch_models import LinearGaussianModel
    from pyabc_amd.engine import GenerationEngine, DeviceMVNFit
    d, S = 4, 20
    model = LinearGaussianModel.benchmark(d, S)
    x0 = torch.as_tensor(model._x0, device="cuda")
    fw = torch.ones(S, dtype=torch.float64, device="cuda")
    eng = GenerationEngine(model, np.full(d, -5.0), np.full(d, 10.0),
                           distance_p=2.0, comm=comm, seed=7,
                           min_batch=min_batch)
    eng.max_batch = min_batch     # several sampling rounds per generation
    r0 = eng.sample_prior(0, n)
    d0, _, _ = K.pnorm_distance(r0.stats_T, x0, fw, 2.0, math.inf,
                                with_accept=False)
    theta = comm.all_gather_rows(r0.theta)
    dist = comm.all_gather_rows(d0)
    w = torch.full((theta.shape[0],), 1.0 / theta.shape[0],
                   dtype=torch.float64, device="cuda")
    eps = float(K.weighted_quantile(dist, w, 0.5, comm=comm)[0].item())
    fit = DeviceMVNFit(theta, w)
    res = eng.sample_generation(1, n, fit, x0, fw, eps, keep_stats=True,
                                record=record)
    th, dd, ww, n_eval, _ = eng.gather_population(res)
    eps1 = float(K.weighted_quantile(dd, ww, 0.5, comm=comm)[0].item())
    # the sharded protocol (histograms all-reduced between passes) gives
    # the same bits as each rank's own select
    assert float(K.weighted_quantile(dd, ww, 0.5, comm=comm, shard=True)[0]
                 .item()) == eps1
    # heavily tied distances (the sharded tie-block words, exchange step 33)
    dt = torch.round(dd * 2.0) / 2.0
    eps_ties = [float(K.weighted_quantile(dt, wq, a, comm=comm,
                                          shard=True)[0].item())
                for wq in (ww, None) for a in (0.3, 0.5, 0.7, 0.9)]
    fit1 = DeviceMVNFit(th, ww)
    # exact-inference generation: stochastic acceptance with u keyed by the
    # global evaluation id, acceptance weights, particle records
    from pyabc_amd.engine import StochasticAcceptance
    var = torch.full((S,), 0.25, dtype=torch.float64, device="cuda")
    c = float(np.sum(np.log(2) + np.log(np.pi) + np.log(np.full(S, 0.25))))
    acc = StochasticAcceptance(x0, var, K.KERNEL_NORMAL, c, -0.5 * c, 20.0)
    rs = eng.sample_generation(2, n, fit1, None, None, None, keep_stats=False,
                               record=False, acceptance=acc,
                               record_particles=True)
    return dict(theta0=theta.cpu().numpy(), eps0=eps, d0=dist.cpu().numpy(),
                theta=th.cpu().numpy(),
                d=dd.cpu().numpy(), w=ww.cpu().numpy(),
                logpd=res.logpd.cpu().numpy(), n_eval=int(n_eval),
                stats=res.stats_T.cpu().numpy(),
                rec=None if res.rec_stats_T is None
                else res.rec_stats_T.cpu().numpy(),
                eps1=eps1, eps_ties=np.array(eps_ties), cov1=fit1.cov,
                s_theta=rs.theta.cpu().numpy(), s_d=rs.d.cpu().numpy(),
                s_w=rs.w.cpu().numpy(), s_accw=rs.accw.cpu().numpy(),
                s_rec_theta=rs.rec_theta.cpu().numpy(),
                s_rec_d=rs.rec_d.cpu().numpy(),
                s_rec_acc=rs.rec_acc.cpu().numpy(), s_n_eval=int(rs.n_eval))


def _rank_main(rank, world, port, n, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from pyabc_amd.distributed import Comm
    comm = Comm.from_env("gloo", device=0)
    multi = _generation(comm, n, 1 << 11, record=True)
    if rank == 0:
        # the same generation on one rank, with a different round size
        single = _generation(Comm.single(), n, 1 << 12, record=True)
        out["single"] = single
    out[rank] = multi
    torch.distributed.destroy_process_group()


def _generations_parents(comm, n, min_batch):
    """d = 12 (KL >= 4: the MFMA pass evaluates each row relative to its
    parent's term): two generations, the second on the fit of
    engine.next_generation_inputs (CDF and KDE pack on the side stream)."""
    from pyabc_amd import kernels as K
    from pyabc_amd.batch_models import LinearGaussianModel
    from pyabc_amd.engine import (GenerationEngine, DeviceMVNFit,
                                  next_generation_inputs)
    d, S = 12, 24
    model = LinearGaussianModel.benchmark(d, S)
    x0 = torch.as_tensor(model._x0, device="cuda")
    fw = torch.ones(S, dtype=torch.float64, device="cuda")
    eng = GenerationEngine(model, np.full(d, -5.0), np.full(d, 10.0),
                           distance_p=2.0, comm=comm, seed=11,
                           min_batch=min_batch)
    eng.max_batch = min_batch
    r0 = eng.sample_prior(0, n)
    d0, _, _ = K.pnorm_distance(r0.stats_T, x0, fw, 2.0, math.inf,
                                with_accept=False)
    theta = comm.all_gather_rows(r0.theta)
    dist = comm.all_gather_rows(d0)
    w = torch.full((theta.shape[0],), 1.0 / theta.shape[0],
                   dtype=torch.float64, device="cuda")
    eps = float(K.weighted_quantile(dist, w, 0.5, comm=comm)[0].item())
    fit = DeviceMVNFit(theta, w)
    out = {}
    for t in (1, 2):
        res = eng.sample_generation(t, n, fit, x0, fw, eps)
        th, dd, ww, _, _ = eng.gather_population(res)
        out[f"theta{t}"] = th.cpu().numpy()
        out[f"parent{t}"] = res.parent.cpu().numpy()
        out[f"logpd{t}"] = res.logpd.cpu().numpy()
        out[f"w{t}"] = ww.cpu().numpy()
        eps, fit = next_generation_inputs(th, dd, ww, 0.5, comm=comm)
        out[f"eps{t}"] = eps
    return out


def _rank_main_parents(rank, world, port, n, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from pyabc_amd.distributed import Comm
    comm = Comm.from_env("gloo", device=0)
    multi = _generations_parents(comm, n, 1 << 11)
    if rank == 0:
        out["single"] = _generations_parents(Comm.single(), n, 1 << 12)
    out[rank] = multi
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 4])
def test_two_ranks_equal_one_rank_parents_d12(world):
    """At d > 8 the accepted rows' parents travel with theta through the
    all-gather to the row-parallel KDE pass (per-row offsets), and the next
    fit comes from next_generation_inputs: two (four) ranks reproduce one
    rank's parents, log-densities, weights and epsilons bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 3001
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rank_main_parents, args=(world, port, n, out),
                 nprocs=world, join=True)
        res = dict(out)
    one = res["single"]
    for r in range(world):
        for k, v in one.items():
            if isinstance(v, float):
                assert res[r][k] == v, k
            else:
                np.testing.assert_array_equal(res[r][k], v, err_msg=k)
    # the parents index the previous population and are real draws
    for t in (1, 2):
        p = one[f"parent{t}"]
        assert p.min() >= 0 and p.max() < n and len(np.unique(p)) > n // 4


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 4])
def test_two_ranks_equal_one_rank_bit_for_bit(world):
    """Global-id sampling (engine.sample_generation): two (and four) ranks
    sharing cuda:0 over gloo produce exactly the population, distances, weights,
    evaluation count, recorded statistics, next epsilon and next fit that
    one rank produces -- with different sampling-round sizes too; and the
    same for a stochastic-acceptance generation (acceptance weights and
    particle records)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 6001          # odd: uneven row slices for the weight pass
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rank_main, args=(world, port, n, out), nprocs=world,
                 join=True)
        res = dict(out)
    one = res["single"]
    for r in range(world):
        got = res[r]
        for k in ("theta0", "d0", "theta", "d", "w", "logpd", "stats", "rec",
                  "cov1", "eps_ties", "s_theta", "s_d", "s_w", "s_accw", "s_rec_theta",
                  "s_rec_d", "s_rec_acc"):
            np.testing.assert_array_equal(got[k], one[k], err_msg=k)
        for k in ("eps0", "eps1", "n_eval", "s_n_eval"):
            assert got[k] == one[k], k
    # stochastic generation: records are every evaluation up to the n-th
    # acceptance, the accepted ones in order are the population
    assert one["s_rec_d"].shape[0] == one["s_n_eval"] > n
    acc = one["s_rec_acc"] > 0
    assert acc.sum() == n
    np.testing.assert_array_equal(one["s_rec_theta"][acc], one["s_theta"])
    np.testing.assert_array_equal(one["s_rec_d"][acc], one["s_d"])
    assert np.all(one["s_accw"] >= 1.0)
    assert one["theta"].shape == (n, 4)
    assert one["rec"].shape[1] == one["n_eval"] >= n
    assert np.all(one["d"] <= one["eps0"])
    assert abs(one["w"].sum() - 1.0) < 1e-12
    assert one["eps1"] <= one["eps0"]
    # the (one- and two-rank) epsilons against the reference's formula:
    # random weights within SURVEY 8(a7)'s local bound, equal weights bit
    # for bit (tests/wq_bound.py)
    from oracle import ref_cpu as ref
    from tests.wq_bound import local_bound
    want = ref.weighted_quantile(one["d"], one["w"], 0.5)
    bound, exact = local_bound(one["d"], one["w"], 0.5)
    assert abs(one["eps1"] - want) <= (0.0 if exact else
                                       1e-12 * abs(want) + bound)
    assert one["eps0"] == ref.weighted_quantile(
        one["d0"], np.full(len(one["d0"]), 1.0 / len(one["d0"])), 0.5)
    dt = np.round(one["d"] * 2.0) / 2.0
    for i, a in enumerate((0.3, 0.5, 0.7, 0.9)):
        assert one["eps_ties"][4 + i] == ref.weighted_quantile(dt, None, a)


def _rccl_main(rank, port, n, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      ABC_COMM_FORCE="1")
    sys.path.insert(0, ROOT)
    from pyabc_amd.distributed import Comm
    comm = Comm.from_env("nccl")
    assert comm.active and torch.distributed.get_backend() == "nccl"
    out["rccl"] = _generation(comm, n, 1 << 11, record=True)
    out["single"] = _generation(Comm.single(), n, 1 << 11, record=True)
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(240)
def test_rccl_collectives_one_rank_equal_no_comm():
    """The "nccl" (RCCL) branches of pyabc_amd.distributed on the GPU: a
    one-rank process group whose collectives still run (ABC_COMM_FORCE=1)
    drives the whole generation -- count all-gathers, row all-gathers of the
    population and statistics, the log-density all-gather, the sharded
    quantile's histogram all-reduces -- through RCCL, and gives exactly the
    no-communicator result."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rccl_main, args=(_free_port(), 5001, out), nprocs=1,
                 join=True)
        res = dict(out)
    one, got = res["single"], res["rccl"]
    for k in ("theta0", "theta", "d", "w", "logpd", "stats", "rec", "cov1",
              "s_theta", "s_d", "s_w", "s_accw", "s_rec_theta", "s_rec_d",
              "s_rec_acc"):
        np.testing.assert_array_equal(got[k], one[k], err_msg=k)
    for k in ("eps0", "eps1", "n_eval", "s_n_eval"):
        assert got[k] == one[k], k


@pytest.mark.timeout(300)
def test_bench_rccl_one_rank():
    """bench.py under torchrun over RCCL ("nccl" backend), one rank with its
    collectives forced on: barrier, all-gathers and the max-over-ranks
    timing run through RCCL and rank 0 prints one line."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "1", "--warmup", "1", "--particles",
           "40000", "--no-cpu-baseline"]
    env = dict(os.environ, ABC_COMM_FORCE="1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280,
                       cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines()
             if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    assert lines[0]["n_gpus"] == 1 and lines[0]["value"] > 0


@pytest.mark.timeout(300)
def test_bench_two_rank_rehearsal():
    """bench.py's own N>1 path (barrier, max-over-ranks timing, rank-0 JSON)
    under torchrun with two ranks on cuda:0."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--particles", "40000",
           "--rehearse-gloo", "--no-cpu-baseline"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines()
             if ln.startswith("{")]
    assert len(lines) == 1, p.stdout          # rank 0 prints one line
    r = lines[0]
    assert r["n_gpus"] == 2 and r["value"] > 0 and r["steps"] == 1
    rl = r["roofline"]
    # frac = issue-ceiling time / launch time of the KDE pass: a fraction of
    # the ceiling the kernel is bound by, <= 1 at any size
    assert 0 < rl["frac"] <= 1
    assert rl["peak"] >= rl["achieved"] > 0
    assert rl["ceiling_ms"] <= rl["avg_launch_ms"]


def _abcsmc_rank(rank, world, port, path, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from pyabc_amd.distributed import Comm
    Comm.from_env("gloo", device=0)
    import pyabc_amd as pa
    from pyabc_amd.batch_models import LinearGaussianModel
    np.random.seed(1000 + rank)        # rank-local numpy states differ
    d, S = 3, 20
    model = LinearGaussianModel.benchmark(d, S)
    names = [f"p{k}" for k in range(d)]
    prior = pa.Distribution(**{n: pa.RV("uniform", -5, 10) for n in names})
    abc = pa.ABCSMC(model, prior, pa.PNormDistance(p=2), population_size=1500,
                    eps=pa.QuantileEpsilon(alpha=0.5),
                    sampler=pa.GPUBatchSampler(min_batch=1 << 11))
    abc.new("sqlite:///" + path, model.observed())
    h = abc.run(max_nr_populations=3)
    df, w = h.distribution_numpy(0, h.max_t)
    out[rank] = dict(id=h.id, max_t=h.max_t, theta=np.asarray(df.values),
                     w=np.asarray(w), eps=list(h.get_all_populations()
                                               .epsilon.values))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_rank_abcsmc_one_sql_run(tmp_path):
    """ABCSMC + GPUBatchSampler under two ranks (one GPU, gloo) with a file
    History and no explicit seed: the ranks agree on rank 0's Philox seed,
    hold identical populations, and the file holds ONE run written by
    rank 0 (rank-0-only SQL)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import sqlite3
    path = str(tmp_path / "run.db")
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_abcsmc_rank, args=(2, port, path, out), nprocs=2, join=True)
        res = dict(out)
    a, b = res[0], res[1]
    assert a["id"] == b["id"] == 1 and a["max_t"] == b["max_t"] == 2
    np.testing.assert_array_equal(a["theta"], b["theta"])
    np.testing.assert_array_equal(a["w"], b["w"])
    assert a["eps"] == b["eps"]
    c = sqlite3.connect(path)
    assert c.execute("SELECT COUNT(*) FROM abc_smc").fetchone()[0] == 1
    assert c.execute("SELECT COUNT(*) FROM populations").fetchone()[0] == 4
    n_par = c.execute("SELECT COUNT(*) FROM particles").fetchone()[0]
    c.close()
    assert n_par == 3 * 1500 + 1


def _local_fit_data():
    rng = np.random.default_rng(31)
    X = rng.normal(size=(5001, 4)) * [1.0, 2.0, 0.5, 1.5]
    w = rng.uniform(0.2, 1.0, size=5001)
    return X, w / w.sum()


def _local_generation(comm):
    """LocalTransition fit (sharded over ranks when comm is active) and one
    engine generation with it: the C4 path."""
    import pandas as pd
    import pyabc_amd as pa
    from pyabc_amd.batch_models import LinearGaussianModel
    from pyabc_amd.engine import GenerationEngine
    X, w = _local_fit_data()
    tr = pa.LocalTransition(k=20, k_fraction=None)
    tr.fit(pd.DataFrame(X, columns=[f"p{k}" for k in range(4)]), w)
    d, S = 4, 20
    model = LinearGaussianModel.benchmark(d, S)
    x0 = torch.as_tensor(model._x0, device="cuda")
    fw = torch.ones(S, dtype=torch.float64, device="cuda")
    eng = GenerationEngine(model, np.full(d, -5.0), np.full(d, 10.0),
                           distance_p=2.0, comm=comm, seed=3,
                           min_batch=1 << 11)
    eng.max_batch = 1 << 11
    res = eng.sample_generation(1, 3001, tr.device_fit, x0, fw, 40.0)
    return dict(covs=tr.covs, invs=tr.inv_covs, dets=tr.determinants,
                nbr=tr.nbr.cpu().numpy(), theta=res.theta.cpu().numpy(),
                logpd=res.logpd.cpu().numpy(), n_eval=int(res.n_eval))


def _local_rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from pyabc_amd.distributed import Comm
    comm = Comm.from_env("gloo", device=0)
    out[rank] = _local_generation(comm)
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_ranks_local_transition_fit_sharded_bit_for_bit():
    """each rank fits kNN + covariances for its row share and
    the shares are all-gathered; the fit (neighbour sets, covariances,
    inverses, determinants) and a LocalTransition generation (population,
    log-densities, evaluation count) equal the one-rank result bit for bit
    (local_transition.py:77-96)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_local_rank, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    from pyabc_amd.distributed import Comm
    one = _local_generation(Comm.single())
    for r in (0, 1):
        for k in ("covs", "invs", "dets", "nbr", "theta", "logpd"):
            np.testing.assert_array_equal(res[r][k], one[k], err_msg=k)
        assert res[r]["n_eval"] == one["n_eval"]


@pytest.mark.timeout(300)
def test_bench_rank_slice():
    """bench.py --rank-slice 4: one process runs rank 0's share of a 4-GPU
    generation (a quarter of the KDE rows, every full-population stage) and
    prints the stage breakdown, the collectives' calls and bytes and the
    xGMI-model prediction."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--rank-slice",
           "4", "--steps", "2", "--warmup", "1", "--particles", "40000",
           "--no-cpu-baseline"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines()
             if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = lines[0]
    assert r["R"] == 4 and r["steps"] == 2
    assert r["kde_rows_per_launch"] == pytest.approx(10000, rel=1e-9)
    ag = r["collectives_per_step"]["all_gather_rows"]
    assert ag["calls"] >= 3 and ag["bytes_received"] > ag["bytes_sent"] > 0
    assert r["predicted_ms_per_step"] >= r["rank0_ms_per_step"] > 0
    assert r["largest_non_scaling_term"] in r["stage_ms"]
