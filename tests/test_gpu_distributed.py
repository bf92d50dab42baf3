"""Multi-rank generation path on ONE GPU (rehearsal of SURVEY 8(e)).

Two ranks share cuda:0 and exchange through gloo (host-staged all-gather),
so the exact engine / bench code that runs one rank per GPU over RCCL is
exercised with real HIP kernels: per-rank Philox streams and quotas, the
all-gather of the accepted rows, the all-reduced evaluation count, and the
redundant deterministic fit / epsilon on every rank.
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


def _rank_main(rank, world, port, n, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from pyabc_amd import kernels as K
    from pyabc_amd.batch_models import LinearGaussianModel
    from pyabc_amd.distributed import Comm
    from pyabc_amd.engine import GenerationEngine, DeviceMVNFit
    comm = Comm.from_env("gloo", device=0)
    d, S = 4, 20
    model = LinearGaussianModel.benchmark(d, S)
    x0 = torch.as_tensor(model._x0, device="cuda")
    fw = torch.ones(S, dtype=torch.float64, device="cuda")
    eng = GenerationEngine(model, np.full(d, -5.0), np.full(d, 10.0),
                           distance_p=2.0, comm=comm, seed=7,
                           min_batch=1 << 12)
    r0 = eng.sample_prior(0, n)
    d0, _, _ = K.pnorm_distance(r0.stats_T, x0, fw, 2.0, math.inf,
                                with_accept=False)
    theta = comm.all_gather_rows(r0.theta)
    dist = comm.all_gather_rows(d0)
    w = torch.full((theta.shape[0],), 1.0 / theta.shape[0],
                   dtype=torch.float64, device="cuda")
    eps = float(K.weighted_quantile(dist, w, 0.5)[0].item())
    fit = DeviceMVNFit(theta, w)
    res = eng.sample_generation(1, n, fit, x0, fw, eps)
    th, dd, ww, n_eval, _ = eng.gather_population(res)
    eps1 = float(K.weighted_quantile(dd, ww, 0.5)[0].item())
    # the rank-local KDE weights must equal a recomputation of the same rows
    # against the same (gathered) previous population
    logpd = fit.logpdf(res.theta)
    out[rank] = dict(
        n_local=int(res.theta.shape[0]), quota=eng.quota(n),
        n_total=int(th.shape[0]), n_eval=int(n_eval),
        local_eval=int(res.n_eval),
        wsum=float(ww.sum().item()),
        theta_sum=float(th.sum().item()), eps0=eps, eps1=eps1,
        all_accepted=bool((dd <= eps).all().item()),
        logpd_err=float((logpd - res.logpd).abs().max().item()),
        mean=th.mul(ww[:, None]).sum(0).cpu().numpy().tolist())
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_ranks_share_one_gpu_generation():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 6001          # odd: uneven per-rank quotas
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rank_main, args=(2, port, n, out), nprocs=2, join=True)
        res = dict(out)
    r0, r1 = res[0], res[1]
    assert r0["quota"] + r1["quota"] == n and abs(r0["quota"] - r1["quota"]) == 1
    assert r0["n_local"] == r0["quota"] and r1["n_local"] == r1["quota"]
    for k in ("n_total", "n_eval", "wsum", "theta_sum", "eps0", "eps1", "mean"):
        assert r0[k] == r1[k], k           # identical replicated state
    assert r0["n_total"] == n
    assert r0["n_eval"] == r0["local_eval"] + r1["local_eval"]
    assert abs(r0["wsum"] - 1.0) < 1e-12
    assert r0["all_accepted"] and r0["eps1"] <= r0["eps0"]
    assert r0["logpd_err"] == 0.0 and r1["logpd_err"] == 0.0
    assert np.all(np.abs(r0["mean"]) < 5.0)     # inside the prior box


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
    assert 0 < r["roofline"]["frac"] < 1
