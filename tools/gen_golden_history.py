"""Golden History database written and read by the reference (THIS container
only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_history.py

1. The reference's own ``pyabc.History`` (``storage/history.py:372-729``,
   schema ``storage/db_model.py:35-127``, blobs
   ``storage/numpy_bytes_storage.py:5-28``) writes a small run to
   ``tests/golden/ref_history.db``: a calibration pre-population, t = 0 with
   two models, t = 1 with one model, scalar and array summary statistics,
   parameter columns out of name order.
2. The reference's readers are called on it; their outputs go to
   ``tests/golden/ref_history_read.npz`` (arrays + a JSON string).
3. With ``--check-ours DB``: the reference History reads a database written by
   ``pyabc_amd.storage.History`` and the same readers must agree with (2).

Only data is written: the .db file is the reference's output for fixed
inputs.  No reference source travels; the GPU box never runs this.
"""
import argparse
import datetime
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import ref_stub  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden")


def run_data():
    """The fixed run: list of (t, eps, nr_sim, [(m, weight, par, dist,
    stats)]) plus the initial data."""
    rng = np.random.default_rng(11)
    gens = []
    for t, models, n in ((0, (0, 1), 7), (1, (0,), 9)):
        parts = []
        for i in range(n):
            m = models[i % len(models)]
            par = {"b": float(rng.normal()), "a": float(rng.normal())}
            if m == 1:
                par["c"] = float(rng.uniform())
            stats = {"y1": float(rng.normal()), "y0": float(rng.normal()),
                     "arr": rng.normal(size=3)}
            parts.append((m, float(rng.uniform(0.5, 1.5)), par,
                          float(rng.uniform()), stats))
        gens.append((t, float(2.0 / (t + 1)), int(3 * n + t), parts))
    init = dict(gt_model=0, options={"seed": 11},
                x_0={"y1": 0.5, "y0": -0.25, "arr": np.array([1., 2., 3.])},
                gt_par={"a": 0.1, "b": -0.2},
                names=["m0", "m1"], dist='{"name": "PNorm"}',
                eps='{"name": "Quantile"}', pop='{"name": "Constant"}')
    return init, gens


def readers(h):
    """Outputs of the reference History's readers (history.py:236-1229)."""
    out = {}
    meta = {}
    meta["max_t"] = int(h.max_t)
    meta["n_populations"] = int(h.n_populations)
    meta["total_nr_simulations"] = int(h.total_nr_simulations)
    meta["alive_0"] = [int(x) for x in h.alive_models(0)]
    meta["alive_1"] = [int(x) for x in h.alive_models(1)]
    meta["model_names"] = h.model_names()
    meta["nr_particles"] = {str(k): int(v) for k, v in
                            h.get_nr_particles_per_population().items()}
    meta["gt_par"] = dict(h.get_ground_truth_parameter())
    oss = h.observed_sum_stat()
    meta["x0_keys"] = sorted(oss)
    for k, v in oss.items():
        out[f"x0_{k}"] = np.asarray(v)
    ap = h.get_all_populations()
    meta["all_pops_columns"] = list(ap.columns)
    out["all_pops_t"] = ap.t.values
    out["all_pops_samples"] = ap.samples.values
    out["all_pops_eps"] = ap.epsilon.values
    out["all_pops_particles"] = ap.particles.values.astype(float)
    for t in (0, 1):
        mp = h.get_model_probabilities(t)
        out[f"mp{t}_m"] = mp.index.values
        out[f"mp{t}_p"] = mp.p.values
        wd = h.get_weighted_distances(t)
        out[f"wd{t}_distance"] = wd.distance.values
        out[f"wd{t}_w"] = wd.w.values
        ws, ss = h.get_weighted_sum_stats(t)
        out[f"wss{t}_w"] = np.asarray(ws)
        out[f"wss{t}_y0"] = np.array([s["y0"] for s in ss])
        out[f"wss{t}_arr"] = np.array([s["arr"] for s in ss])
        for m in h.alive_models(t):
            df, w = h.get_distribution(m, t)
            meta[f"dist{t}_{m}_columns"] = list(df.columns)
            out[f"dist{t}_{m}_X"] = df.values
            out[f"dist{t}_{m}_index"] = df.index.values
            out[f"dist{t}_{m}_w"] = w
            wm, ssm = h.get_weighted_sum_stats_for_model(m, t)
            out[f"wssm{t}_{m}_w"] = wm
            out[f"wssm{t}_{m}_y1"] = np.array([s["y1"] for s in ssm])
        pop = h.get_population(t)
        out[f"pop{t}_m"] = np.array([p.m for p in pop.get_list()])
        out[f"pop{t}_w"] = np.array([p.weight for p in pop.get_list()])
    mpa = h.get_model_probabilities()
    out["mp_all"] = mpa.values
    ext = h.get_population_extended(t=1)
    meta["ext1_columns"] = list(ext.columns)
    out["ext1_index"] = ext.index.values
    out["ext1_par_a"] = ext.par_a.values
    out["ext1_sumstat_y0"] = ext.sumstat_y0.values.astype(float)
    out["_meta"] = np.array(json.dumps(meta, sort_keys=True))
    return out


def write_ref(path, pyabc):
    from pyabc.population import Particle, Population
    from pyabc.parameters import Parameter
    init, gens = run_data()
    h = pyabc.History("sqlite:///" + path)
    h.store_initial_data(init["gt_model"], init["options"], init["x_0"],
                         init["gt_par"], init["names"], init["dist"],
                         init["eps"], init["pop"])
    h.update_nr_samples(-1, 13)
    for t, eps, nsim, parts in gens:
        plist = [Particle(m=m, parameter=Parameter(par), weight=w,
                          accepted_sum_stats=[st], accepted_distances=[dd],
                          accepted=True)
                 for m, w, par, dd, st in parts]
        h.append_population(t, eps, Population(plist), nsim, init["names"])
    h.done()
    return h


def compare(a, b):
    assert set(a) == set(b), (set(a) ^ set(b))
    for k in a:
        if k == "_meta":
            ma, mb = json.loads(str(a[k])), json.loads(str(b[k]))
            assert ma == mb, (ma, mb)
        else:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check-ours", default=None)
    args = ap.parse_args()
    pyabc = ref_stub.import_pyabc()
    if args.check_ours:
        got = readers(pyabc.History("sqlite:///" + args.check_ours))
        want = dict(np.load(os.path.join(OUT, "ref_history_read.npz")))
        want.pop("_ref")
        compare(got, want)
        print(f"reference History reads {args.check_ours}: all readers equal")
        return
    path = os.path.join(OUT, "ref_history.db")
    if os.path.exists(path):
        os.remove(path)
    write_ref(path, pyabc)
    h = pyabc.History("sqlite:///" + path)
    out = readers(h)
    out["_ref"] = np.array("pyabc/storage/history.py:236-1229, "
                           "db_model.py:35-127, numpy_bytes_storage.py:5-28")
    np.savez_compressed(os.path.join(OUT, "ref_history_read.npz"), **out)
    print("wrote", path, os.path.getsize(path), "bytes;",
          datetime.datetime.now())


if __name__ == "__main__":
    main()
