"""GPUBatchSampler: the drop-in sampler that runs a whole generation on the
MI355X (reference boundary: ``Sampler.sample_until_n_accepted``,
pyabc/sampler/base.py:196-234, called at pyabc/smc.py:888 and 524).

The reference hands the sampler an opaque per-proposal closure
(``_create_simulate_function``, smc.py:536-600).  :class:`pyabc_amd.ABCSMC`
attaches a :class:`BatchSpec` to that closure; when the spec describes a
configuration the device engine covers (one :class:`BatchModel`, uniform-box
prior, :class:`MultivariateNormalTransition` / :class:`LocalTransition`,
p-norm distance with uniform acceptance or an independent normal / Laplace
kernel with the :class:`StochasticAcceptor`, one simulation per parameter),
the generation runs through
:mod:`pyabc_amd.engine`.  Otherwise the closure is called proposal by
proposal with SingleCoreSampler semantics (user Python models), its
transition / distance / epsilon calls still computing on the device.
"""
import numpy as np
import torch

from .base import Sampler, Sample
from ..distance import DeviceStats, PNormDistance, _IndependentKernel
from ..distributed import Comm
from ..engine import GenerationEngine, StochasticAcceptance
from ..population import ColumnarPopulation
from ..batch_models import BatchModel
from .. import kernels as K


class BatchSpec:
    """Everything ``simulate_one`` closes over, for batch evaluation."""

    def __init__(self, t, kind, models, priors, transitions, distance, eps,
                 acceptor, x_0, nr_samples_per_parameter, summary_statistics,
                 model_probabilities=None):
        self.t = t
        self.kind = kind           # "calibration" (all accepted) or "smc"
        self.models = models
        self.priors = priors
        self.transitions = transitions
        self.distance = distance
        self.eps = eps
        self.acceptor = acceptor
        self.x_0 = x_0
        self.nr_samples_per_parameter = nr_samples_per_parameter
        self.summary_statistics = summary_statistics
        self.model_probabilities = model_probabilities

    def stochastic(self):
        from ..acceptor import StochasticAcceptor
        return isinstance(self.acceptor, StochasticAcceptor)

    def unsupported_reason(self):
        from ..acceptor import UniformAcceptor
        from ..transition import MultivariateNormalTransition, LocalTransition
        if len(self.models) != 1:
            return "model selection (several models)"
        if not isinstance(self.models[0], BatchModel):
            return "model is not a BatchModel"
        if self.priors[0].uniform_box() is None:
            return "prior is not a product of uniform marginals"
        if self.nr_samples_per_parameter != 1:
            return "nr_samples_per_parameter != 1"
        if getattr(self.summary_statistics, "__name__", "") != "identity":
            return "custom summary_statistics"
        if self.kind == "smc" and self.stochastic():
            if not isinstance(self.distance, _IndependentKernel):
                return ("StochasticAcceptor kernel is not an Independent"
                        "Normal/LaplaceKernel")
            why = self.distance.batch_unsupported_reason(self.x_0)
            if why is not None:
                return why
        elif self.kind == "smc":
            if not isinstance(self.distance, PNormDistance):
                return "distance is not a (Adaptive)PNormDistance"
            if not isinstance(self.acceptor, UniformAcceptor) or \
                    self.acceptor.use_complete_history:
                return "acceptor is not UniformAcceptor(current time)"
        if self.kind == "smc":
            if self.t > 0 and not isinstance(
                    self.transitions[0],
                    (MultivariateNormalTransition, LocalTransition)):
                return "transition is not MultivariateNormal/LocalTransition"
        return None


class BatchSample(Sample):
    """Columnar sample: the accepted population on the device plus the
    recorded statistics (accepted and rejected, evaluation order)."""

    def __init__(self, population, recorded, record_rejected, ok=True,
                 rec_particles=None):
        super().__init__(record_rejected=record_rejected, ok=ok)
        self.population = population
        self.recorded = recorded
        # (theta [n_rec, d], distance [n_rec], accepted [n_rec]) of every
        # recorded evaluation, for the temperature schemes' records
        self.rec_particles = rec_particles

    @property
    def n_accepted(self):
        return 0 if self.population is None else len(self.population)

    def get_accepted_population(self):
        return self.population

    @property
    def all_sum_stats(self):
        return self.recorded

    def first_m_sum_stats(self, m):
        if self.recorded is None:
            return self.population.get_accepted_sum_stats()
        n = len(self.recorded)
        if m >= n:
            return self.recorded
        return DeviceStats(self.recorded.stats_T[:, :int(m)],
                           self.recorded.keys)

    def first_m_particles(self, m):
        return self.population.get_list()[:int(min(m, len(self.population)))]


class GPUBatchSampler(Sampler):
    """Runs each generation as batched HIP kernels on the current device.

    Parameters: ``seed`` (Philox seed; default drawn from numpy's global
    state, rank 0's under torchrun), ``min_batch`` / ``max_batch``
    proposals per round, ``kde_precision`` ("mfma" default, "f32" or "f64"
    KDE kernel), ``comm`` (multi-GPU sharding, default from the torchrun
    environment), ``check_max_eval`` (as SingleCoreSampler's,
    singlecore.py:15-17: stop a generation at ``max_eval`` evaluations,
    off by default).
    """

    def __init__(self, seed=None, min_batch=1 << 14, max_batch=1 << 22,
                 kde_precision="mfma", comm=None, check_max_eval=False):
        super().__init__()
        self.check_max_eval = check_max_eval
        self.seed = seed
        self.min_batch = min_batch
        self.max_batch = max_batch
        self.kde_precision = kde_precision
        self.comm = comm
        self._engines = {}
        self.last_timers = {}
        self.timer_log = []     # per-call engine timers (tools/bench_configs.py)
        self.fallback_reason = None

    def _engine(self, spec):
        model = spec.models[0]
        names, lo, sc = spec.priors[0].uniform_box()
        key = (id(model), tuple(lo), tuple(sc))
        eng = self._engines.get(key)
        if eng is None:
            comm = self.comm or Comm.from_env()
            seed = self.seed if self.seed is not None else int(
                np.random.randint(0, 2 ** 62, dtype=np.int64))
            # every rank must draw from the same Philox streams (global-id
            # sampling): rank 0's seed, whatever each rank's numpy state
            seed = comm.broadcast_int(seed)
            eng = GenerationEngine(
                model, lo, sc, comm=comm,
                seed=seed, min_batch=self.min_batch,
                max_batch=self.max_batch, kde_precision=self.kde_precision)
            eng.max_rounds = 100000
            self._engines[key] = eng
        return eng, names

    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False):
        spec = getattr(simulate_one, "batch_spec", None)
        reason = "no batch spec" if spec is None else spec.unsupported_reason()
        self.fallback_reason = reason
        if reason is not None:
            return self._closure_path(n, simulate_one, max_eval)
        eng, names = self._engine(spec)
        cap = max_eval if self.check_max_eval else np.inf
        model = spec.models[0]
        keys = list(model.keys)
        record = self.sample_factory.record_rejected
        if spec.kind == "calibration":
            res = eng.sample_generation(spec.t, n, None, None, None, np.inf,
                                        keep_stats=True, record=False,
                                        stream_base=2, max_eval=cap)
            if not res.ok:
                return self._not_ok(res, record)
            # calibration distances are computed later (smc.py:516-534)
            res.d = K.full(res.w.numel(), np.inf)
        else:
            fit = spec.transitions[0].device_fit if spec.t > 0 and \
                spec.transitions[0].device_fit is not None else None
            if spec.stochastic():
                keys_d, x0d, prmd, kind, c = spec.distance.device_params(
                    spec.t, spec.x_0)
                acceptance = StochasticAcceptance(
                    x0d, prmd, kind, c, spec.acceptor.pdf_norms[spec.t],
                    spec.eps(spec.t),
                    spec.acceptor.apply_importance_weighting)
                x0d = fwd = eps = None
            else:
                keys_d, x0d, fwd = spec.distance.device_params(spec.t,
                                                               spec.x_0)
                eps = spec.eps(spec.t)
                acceptance = None
            if keys_d != keys:
                perm = [keys.index(k) for k in keys_d]
                model = _PermutedModel(model, perm)
                eng.model = model
            res = eng.sample_generation(spec.t, n, fit, x0d, fwd, eps,
                                        keep_stats=True, record=record,
                                        acceptance=acceptance,
                                        record_particles=record and
                                        acceptance is not None,
                                        max_eval=cap)
            eng.model = spec.models[0]
            if not res.ok:
                return self._not_ok(res, record)
            keys = keys_d
        # the engine returns the global population, identical on every rank
        rec = None
        if res.rec_stats_T is not None:
            rec = DeviceStats(res.rec_stats_T, keys)
        self.nr_evaluations_ = int(res.n_eval)
        self.last_timers = dict(eng.timers)
        self.timer_log.append(self.last_timers)
        pop = ColumnarPopulation(res.theta, res.w, res.d, names,
                                 res.stats_T, keys)
        recp = None
        if getattr(res, "rec_theta", None) is not None:
            recp = (res.rec_theta, res.rec_d, res.rec_acc,
                    getattr(res, "rec_parent", None))
        return BatchSample(pop, rec, record, rec_particles=recp)

    def _not_ok(self, res, record):
        """max_eval reached before n acceptances (singlecore.py:35-38):
        ABCSMC.run stops on ``ok = False`` without reading a population."""
        self.nr_evaluations_ = int(res.n_eval)
        return BatchSample(None, None, record, ok=False)

    def _closure_path(self, n, simulate_one, max_eval):
        """SingleCoreSampler.sample_until_n_accepted (singlecore.py:19-38)."""
        nr = 0
        sample = self._create_empty_sample()
        for _ in range(n):
            while True:
                if self.check_max_eval and nr >= max_eval:
                    break
                p = simulate_one()
                sample.append(p)
                nr += 1
                if p.accepted:
                    break
        self.nr_evaluations_ = nr
        if sample.n_accepted < n:
            sample.ok = False
        return sample


class _PermutedModel(BatchModel):
    """Presents a model's statistics in the distance's key order."""

    def __init__(self, model, perm):
        self.model = model
        self.perm = torch.as_tensor(perm, device="cuda")
        self.keys = tuple(model.keys[i] for i in perm)
        self.name = model.name

    def simulate(self, theta, seed, sid, offset):
        return self.model.simulate(theta, seed, sid, offset).index_select(
            0, self.perm).contiguous()
