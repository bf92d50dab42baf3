"""Host-side logic of the drop-in API (no GPU): configuration objects,
contracts and the multi-process plumbing (gloo, world_size 2)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import pyabc_amd as pa
from pyabc_amd.distributed import Comm
from pyabc_amd.sampler.gpu import BatchSpec


def test_uniform_box_and_rv_bounds():
    prior = pa.Distribution(b=pa.RV("uniform", -1, 2),
                            a=pa.RV("uniform", loc=0.5, scale=3))
    names, lo, sc = prior.uniform_box()
    assert names == ["a", "b"]
    np.testing.assert_array_equal(lo, [0.5, -1])
    np.testing.assert_array_equal(sc, [3, 2])
    assert pa.Distribution(x=pa.RV("norm", 0, 1)).uniform_box() is None
    # scipy support semantics at the boundary
    assert prior.pdf(pa.Parameter(a=3.5, b=1.0)) > 0
    assert prior.pdf(pa.Parameter(a=np.nextafter(3.5, 4), b=0.0)) == 0


def test_population_normalisation_matches_reference_fixture(golden):
    g = golden("kde_N4096_M1024_d8")
    parts = [pa.Particle(0, pa.Parameter(x=float(i)), float(w), [{}], [0.0])
             for i, w in enumerate(g["weight"])]
    pop = pa.Population(parts)
    w = np.array([p.weight for p in pop.get_list()])
    np.testing.assert_array_equal(w, g["weight_norm"])
    assert pop.get_model_probabilities() == {0: 1.0}


class _WrongOutputSampler(pa.SingleCoreSampler):
    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False):
        return super().sample_until_n_accepted(n + 1, simulate_one, max_eval,
                                               all_accepted)


def test_sampler_meta_contract():
    """test/test_samplers.py:66-70, 206-214: wrong n raises."""
    def sim():
        return pa.Particle(0, {}, 1.0, [{}], [0.0], accepted=True)
    s = _WrongOutputSampler()
    with pytest.raises(AssertionError):
        s.sample_until_n_accepted(10, sim)
    ok = pa.SingleCoreSampler().sample_until_n_accepted(10, sim)
    assert ok.n_accepted == 10


def test_singlecore_counts_evaluations():
    rng = np.random.default_rng(0)

    def sim():
        acc = bool(rng.uniform() < 0.3)
        return pa.Particle(0, {}, 1.0, [{"a": 1}], [0.0], [{"a": 2}], [1.0],
                           accepted=acc)
    smp = pa.SingleCoreSampler()
    smp.sample_factory.record_rejected = True
    sample = smp.sample_until_n_accepted(50, sim)
    assert sample.n_accepted == 50
    assert len(sample.first_m_particles(10 ** 9)) == smp.nr_evaluations_


def test_pnorm_weight_formatting():
    w = pa.PNormDistance.format_dict(None, 3, ["a", "b"])
    assert w == {3: {"a": 1., "b": 1.}}
    assert pa.PNormDistance.format_dict({"a": 2}, 1, ["a"]) == {1: {"a": 2}}
    assert pa.PNormDistance.get_for_t_or_latest({0: 1, 5: 2}, 7) == 2
    with pytest.raises(ValueError):
        pa.PNormDistance(p=0.5)


def test_epsilon_api():
    with pytest.raises(ValueError):
        pa.QuantileEpsilon(alpha=0)
    assert np.isclose(pa.ConstantEpsilon(42)(100), 42)
    with pytest.raises(Exception):
        pa.ListEpsilon([3.5, 2.3, 1, 0.3])(4)
    assert not np.isfinite(pa.NoEpsilon()(42))
    assert np.isclose(pa.MedianEpsilon().alpha, 0.5)


def test_batch_spec_support_rules():
    prior = pa.Distribution(a=pa.RV("uniform", 0, 1))
    model = pa.GaussianMeanModel()
    ident = pa.smc.identity
    base = dict(priors=[prior], transitions=[pa.MultivariateNormalTransition()],
                distance=pa.PNormDistance(), eps=pa.MedianEpsilon(),
                acceptor=pa.UniformAcceptor(), x_0={"data": 1.0},
                nr_samples_per_parameter=1, summary_statistics=ident)
    assert BatchSpec(1, "smc", [model], **base).unsupported_reason() is None
    assert "BatchModel" in BatchSpec(1, "smc", [lambda p: p],
                                     **base).unsupported_reason()
    assert "several" in BatchSpec(1, "smc", [model, model],
                                  **base).unsupported_reason()
    b2 = dict(base, priors=[pa.Distribution(a=pa.RV("norm", 0, 1))])
    assert "uniform" in BatchSpec(1, "smc", [model], **b2).unsupported_reason()
    b3 = dict(base, transitions=[pa.LocalTransition()])
    assert BatchSpec(1, "smc", [model], **b3).unsupported_reason() is None

    class UserTransition(pa.Transition):
        def fit(self, X, w):
            pass

        def rvs_single(self):
            return None

        def pdf(self, x):
            return 1.0
    b4 = dict(base, transitions=[UserTransition()])
    assert "Multivariate" in BatchSpec(1, "smc", [model],
                                       **b4).unsupported_reason()


def test_fast_random_choice():
    np.random.seed(0)
    c = [pa.smc.fast_random_choice([0.2, 0.5, 0.3]) for _ in range(20000)]
    f = np.bincount(c, minlength=3) / len(c)
    np.testing.assert_allclose(f, [0.2, 0.5, 0.3], atol=0.02)


def test_quota_split():
    from pyabc_amd.engine import GenerationEngine
    for R in [1, 2, 3, 8]:
        for n in [1, 7, 1000, 10 ** 6 + 3]:
            q = []
            for r in range(R):
                e = GenerationEngine.__new__(GenerationEngine)
                e.comm = Comm(r, R)
                q.append(e.quota(n))
            assert sum(q) == n and max(q) - min(q) <= 1


def test_transition_weight_normalisation_and_empty():
    tr = pa.MultivariateNormalTransition()
    import pandas as pd
    with pytest.raises(pa.NotEnoughParticles):
        tr.fit(pd.DataFrame({"a": []}), np.array([]))
    tr.fit(pd.DataFrame(index=[0, 1]), np.array([0.5, 0.5]))
    assert tr.no_parameters and tr.pdf(pd.Series(dtype=float)) == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    comm = Comm.from_env("gloo")
    # uneven per-rank row counts, as the per-rank quotas give
    rows = torch.arange((rank + 2) * 3, dtype=torch.float64).view(-1, 3) \
        + 100 * rank
    g = comm.all_gather_rows(rows)
    n = comm.all_reduce_int(rank + 1)
    mx = comm.all_reduce_max_float(float(rank) * 1.5)
    out[rank] = (g.numpy().tolist(), n, mx)
    torch.distributed.destroy_process_group()


def test_comm_gloo_world2():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_gloo_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    exp = np.concatenate([np.arange(6).reshape(-1, 3),
                          np.arange(9).reshape(-1, 3) + 100])
    for r in range(2):
        np.testing.assert_array_equal(np.array(res[r][0]), exp)
        assert res[r][1] == 3
        assert res[r][2] == 1.5


def _emulate_rounds(sup, acc, n, R, B):
    """The engine's round loop on host flags: raw ids split into rounds of
    R adjacent slices of B; returns the selected eval ids and n_eval."""
    from pyabc_amd.engine import selection_plan
    nvs, nas, apos, evals = [], [], [], []
    raw = 0
    ev = 0
    tot = 0
    while tot < n:
        nv_k, na_k, ap_k, ev_k = [], [], [], []
        for s in range(R):
            sl = slice(raw + s * B, raw + (s + 1) * B)
            ids_ev = ev + np.arange(int(sup[sl].sum()))
            ev += len(ids_ev)
            a = acc[ids_ev]
            nv_k.append(len(ids_ev))
            na_k.append(int(a.sum()))
            ap_k.append(np.flatnonzero(a))
            ev_k.append(ids_ev)
        raw += R * B
        tot += sum(na_k)
        nvs.append(nv_k)
        nas.append(na_k)
        apos.append(ap_k)
        evals.append(ev_k)
    takes, closing = selection_plan(nvs, nas, n)
    sel, n_eval = [], 0
    for k in range(len(nvs)):
        for s in range(R):
            t = takes[k][s]
            sel.extend(evals[k][s][apos[k][s][:t]])
            if closing[k][s] == 1:
                n_eval += apos[k][s][t - 1] + 1
            elif closing[k][s] == 0:
                n_eval += nvs[k][s]
    return np.array(sel, dtype=np.int64), n_eval


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_selection_plan_global_id_order(seed):
    """The population is the first n accepted evaluation ids and n_eval
    counts evaluations through the n-th acceptance, for any rank count and
    round size (SingleCoreSampler semantics, singlecore.py:19-38)."""
    rng = np.random.default_rng(seed)
    sup = rng.uniform(size=200000) < 0.8
    acc = rng.uniform(size=200000) < 0.3
    for n in [1, 17, 1000, 5003]:
        ev_acc = np.flatnonzero(acc)
        want = ev_acc[:n]
        want_eval = want[-1] + 1
        for R, B in [(1, 64), (1, 4096), (2, 50), (3, 1000), (8, 257)]:
            got, n_eval = _emulate_rounds(sup, acc, n, R, B)
            np.testing.assert_array_equal(got, want)
            assert n_eval == want_eval


def _gather_worker(rank, world, port, out):
    from pyabc_amd.engine import gather_segments
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    comm = Comm.from_env("gloo")
    # counts[s][k]: rows rank s holds from round k; row value = global id
    counts = [[2, 0, 1], [0, 3, 2], [1, 1, 0]][:world]
    ids, gid = {}, 0
    for k in range(3):
        for s in range(world):
            ids[(s, k)] = list(range(gid, gid + counts[s][k]))
            gid += counts[s][k]
    pieces = [torch.tensor(ids[(rank, k)], dtype=torch.float64).view(-1, 1)
              .repeat(1, 2) for k in range(3) if counts[rank][k]]
    g = gather_segments(comm, pieces, (2,), counts, torch.device("cpu"))
    ints = comm.all_gather_ints(rank * 10 + 1)
    lists = comm.all_gather_int_lists([rank, rank + 5])
    red = comm.all_reduce_ints([rank, 2])
    out[rank] = (g[:, 0].tolist(), ints, lists, red, gid)
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_segments_gloo(world):
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_gather_worker, args=(world, port, out), nprocs=world,
                 join=True)
        res = dict(out)
    for r in range(world):
        g, ints, lists, red, gid = res[r]
        assert g == list(range(gid))            # global id order
        assert ints == [s * 10 + 1 for s in range(world)]
        assert lists == [[s, s + 5] for s in range(world)]
        assert red == [sum(range(world)), 2 * world]


def test_columnar_offload_finish_is_thread_safe():
    """Two readers of an offloaded population racing on the first column
    access: both get the host columns, nothing raises."""
    import concurrent.futures as cf
    import threading
    import time
    from pyabc_amd.population import ColumnarPopulation
    th = torch.arange(12, dtype=torch.float64).reshape(6, 2)
    w = torch.full((6,), 1 / 6, dtype=torch.float64)
    d = torch.arange(6, dtype=torch.float64)
    pop = ColumnarPopulation(th, w, d, ["a", "b"], normalize=False)
    gate = threading.Event()

    def slow_copy():
        gate.wait(5)
        time.sleep(0.05)
        return {"theta": th.clone(), "w": w.clone(), "d": d.clone(),
                "stats_T": None}
    with cf.ThreadPoolExecutor(4) as ex:
        pop._pending = ex.submit(slow_copy)
        readers = [ex.submit(lambda: pop.theta.sum().item()) for _ in range(2)]
        readers.append(ex.submit(lambda: pop.w.sum().item()))
        gate.set()
        got = [r.result(timeout=10) for r in readers]
    assert got[0] == got[1] == float(th.sum())
    assert pop._pending is None


def test_fused_path_only_for_the_mirrored_simulate():
    """engine.mirrors_simulate: the fused simulate + distance kernel is used
    only when simulate_distance comes from the class whose simulate it
    mirrors -- a subclass overriding simulate() is never fused."""
    from pyabc_amd.batch_models import LinearGaussianModel
    from pyabc_amd.engine import mirrors_simulate

    class Noisier(LinearGaussianModel):
        def simulate(self, theta, seed, sid, offset):  # pragma: no cover
            return super().simulate(theta, seed, sid, offset) * 2.0

    class Both(Noisier):
        def simulate(self, theta, seed, sid, offset):  # pragma: no cover
            return super().simulate(theta, seed, sid, offset)

        def simulate_distance(self, *a):  # pragma: no cover
            return None

    class Stale(Both):   # simulate overridden again, the fused one inherited
        def simulate(self, theta, seed, sid, offset):  # pragma: no cover
            return super().simulate(theta, seed, sid, offset) + 1.0

    m = LinearGaussianModel.benchmark(2, 3)
    assert mirrors_simulate(m)
    assert not mirrors_simulate(Noisier(m.A_host, m.sigma))
    assert mirrors_simulate(Both(m.A_host, m.sigma))
    assert not mirrors_simulate(Stale(m.A_host, m.sigma))
    assert not mirrors_simulate(object())
    # simulate replaced on the instance: its distances must come from it
    inst = LinearGaussianModel.benchmark(2, 3)
    inst.simulate = lambda theta, seed, sid, offset: None
    assert not mirrors_simulate(inst)
    inst.simulate_distance = lambda *a: None   # both from the instance
    assert mirrors_simulate(inst)
