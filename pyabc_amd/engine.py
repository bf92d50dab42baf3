"""Device-resident ABC-SMC generation engine (the batch hot path).

One call of :meth:`GenerationEngine.sample_generation` performs, on the GPU,
everything the reference does per proposal inside ``simulate_one`` for a
whole generation t >= 1 (reference pyabc/smc.py:580-792, driven by
``sample_until_n_accepted`` pyabc/sampler/singlecore.py:19-38):

  rounds of B proposals until n are accepted:
    resample + perturb + prior-support test          (propose_philox)
    in-support compaction -> proposal ids            (compact, gather)
    batch simulation -> stat-major statistics        (model.simulate)
    p-norm distance + acceptance d <= eps            (pnorm_distance)
  the first n accepted in proposal-id order (SingleCoreSampler semantics)
  KDE importance weights prior / transition        (PackedPopulation.logpdf)
  weight normalisation                             (dsum / scale)

and between generations (``_prepare_next_iteration`` smc.py:942-1022):
  transition fit (weighted moments + host d x d finish), adaptive distance
  weights (column MAD / std), distance recompute, quantile epsilon.

Multi-GPU: ranks shard proposals and new particles (their own Philox streams
and quotas of the population); the previous population is replicated by an
all-gather of the accepted rows once per generation, weight normalisers are
all-reduced, and every rank then runs the same deterministic fit / epsilon on
identical inputs.  ``comm`` is a :class:`pyabc_amd.distributed.Comm`.
"""
import math
import time

import numpy as np
import torch

from . import kernels as K
from .distributed import Comm

F64 = torch.float64


def silverman_rule_of_thumb(n_samples, dimension):
    """(4 / (n (d+2)))^(1/(d+4))  (transition/multivariatenormal.py:27-37)."""
    return (4 / n_samples / (dimension + 2)) ** (1 / (dimension + 4))


def scott_rule_of_thumb(n_samples, dimension):
    """n^(-1/(d+4))  (transition/multivariatenormal.py:14-24)."""
    return n_samples ** (-1. / (dimension + 4))


class DeviceMVNFit:
    """MultivariateNormalTransition state on the device: covariance (host
    d x d), perturbation factor A (numpy svd semantics), and the packed
    previous population for the KDE pass (scipy _PSD whitening)."""

    def __init__(self, X, w, scaling=1.0, bandwidth_selector=None,
                 precision="f32", moments=None):
        self.X = X
        self.w = w
        n, d = X.shape
        self.n, self.d = n, d
        bw_sel = bandwidth_selector or silverman_rule_of_thumb
        if n == 1:
            # smart_cov: a single row gives diag(|x_0|) (transition/util.py:8-11)
            x0 = X[0].double().cpu().numpy()
            sample_cov = np.diag(np.abs(x0))
            sw2 = float((w.double() ** 2).sum().item())
            mu = x0
        else:
            mom = (moments if moments is not None
                   else K.weighted_moments(X, w)).cpu().numpy()
            sw, sw2 = mom[0], mom[1]
            mu = mom[2:2 + d]
            fact = sw - sw2 / sw
            with np.errstate(divide="ignore", invalid="ignore"):
                sample_cov = mom[2 + d:].reshape(d, d) * (
                    1.0 / fact if fact > 0 else np.inf)
        ess = 1.0 / sw2
        self.ess = ess
        self.cov = sample_cov * bw_sel(ess, d) ** 2 * scaling
        # numpy legacy multivariate_normal factor: A = sqrt(s)[:,None] * V
        _, s, v = np.linalg.svd(self.cov)
        self.A_host = np.sqrt(s)[:, None] * v
        self.A = torch.as_tensor(self.A_host, dtype=F64, device=X.device)
        U, rank, log_pdet = K.psd_whitening(self.cov)
        self.rank, self.log_pdet = rank, log_pdet
        Us = torch.as_tensor(U * math.sqrt(0.5 * K.LOG2E), dtype=F64,
                             device=X.device)
        mu_t = torch.as_tensor(mu, dtype=F64, device=X.device)
        self.packed = K.PackedPopulation(X, w, mu_t, Us, rank, log_pdet,
                                         precision)
        self._cdf = None

    @property
    def cdf(self):
        if self._cdf is None:
            self._cdf = K.resample_cdf(self.w)
        return self._cdf

    def logpdf(self, theta):
        return self.packed.logpdf(theta)

    def propose(self, lo, scale, seed, sid, offset, B):
        """B draws of resample + perturb + support flag (Philox)."""
        return K.propose_philox(self.X, self.cdf, self.A, lo, scale, seed,
                                sid, offset, B)


class GenerationResult:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class GenerationEngine:
    """Runs generations of a batch model on the current device."""

    def __init__(self, model, prior_lo, prior_scale, distance_p=2.0,
                 comm=None, seed=0, min_batch=1 << 16, max_batch=1 << 22,
                 kde_precision="f32", record_stats=False):
        self.model = model
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.lo = torch.as_tensor(np.asarray(prior_lo, dtype=np.float64),
                                  device=self.dev)
        self.scale = torch.as_tensor(np.asarray(prior_scale, dtype=np.float64),
                                     device=self.dev)
        self.d = self.lo.numel()
        self.prior_pd = float(np.prod(1.0 / np.asarray(prior_scale)))
        self.p = distance_p
        self.comm = comm or Comm.single()
        self.seed = int(seed)
        self.min_batch = min_batch
        self.max_batch = max_batch
        self.kde_precision = kde_precision
        self.record_stats = record_stats
        self.acc_rate_est = 0.5
        self.valid_rate_est = 1.0
        self.timers = {}
        self.kde_events = None   # list -> (start, end, M, N) per KDE launch
        self.max_rounds = None

    # ------------------------------------------------------------------
    def _sid(self, t, kind):
        # disjoint Philox stream ids per (generation, rank, purpose)
        return ((int(t) * 4096 + self.comm.rank) * 8 + kind)

    def quota(self, n):
        """Accepted particles this rank contributes to a population of n."""
        R, r = self.comm.world, self.comm.rank
        return n // R + (1 if r < n % R else 0)

    # ------------------------------------------------------------------
    def sample_prior(self, t, n):
        """t = 0 / calibration: theta ~ prior, all accepted
        (smc.py:486-534 with all_accepted=True)."""
        nq = self.quota(n)
        theta = K.prior_uniform(self.lo, self.scale, self.seed,
                                self._sid(t, 0), 0, nq)
        stats = self.model.simulate(theta, self.seed, self._sid(t, 1), 0)
        return GenerationResult(theta=theta, stats_T=stats, n_eval=nq,
                                rec_stats_T=stats, n_rec=nq)

    def sample_generation(self, t, n, fit, x0, fw, eps, keep_stats=None,
                          record=None, stream_base=0):
        """Proposals until this rank's quota of n is accepted, then KDE
        weights.  ``fit=None`` proposes from the prior (generation 0,
        weight 1).  Returns the rank-local accepted rows; with ``record``
        also the statistics of every evaluated proposal up to the last
        acceptance (record_rejected, sampler/base.py:119-141)."""
        keep_stats = self.record_stats if keep_stats is None else keep_stats
        record = self.record_stats if record is None else record
        nq = self.quota(n)
        tm = {}
        t0 = time.perf_counter()
        rounds = []
        n_acc = 0
        prop_off = 0
        sim_off = 0
        while n_acc < nq:
            need = nq - n_acc
            B = int(min(self.max_batch, max(
                self.min_batch,
                math.ceil(1.2 * need / max(self.acc_rate_est, 1e-3)
                          / max(self.valid_rate_est, 1e-3)))))
            if fit is None:
                theta = K.prior_uniform(self.lo, self.scale, self.seed,
                                        self._sid(t, stream_base), prop_off, B)
                nv = B
            else:
                theta_all, idx, sup = fit.propose(
                    self.lo, self.scale, self.seed,
                    self._sid(t, stream_base), prop_off, B)
                vpos, vcount = K.compact(sup)
                nv = int(vcount.item())                             # sync 1
                self.valid_rate_est = max(nv / B, 1e-3)
                theta = K.gather_rows(theta_all, vpos, nv) if nv else None
            prop_off += B
            if nv == 0:
                continue
            stats = self.model.simulate(theta, self.seed,
                                        self._sid(t, stream_base + 1), sim_off)
            sim_off += nv
            if x0 is None:
                # calibration sample: everything accepted, distances later
                # (smc.py:486-514: accepted_distances = [inf])
                d = torch.full((nv,), math.inf, dtype=F64, device=self.dev)
                guard = torch.zeros(nv, dtype=torch.uint8, device=self.dev)
                apos = torch.arange(nv, dtype=torch.int64, device=self.dev)
                na = nv
            else:
                d, acc, guard = K.pnorm_distance(stats, x0, fw, self.p, eps,
                                                 B=nv)
                apos, acount = K.compact(acc)
                na = int(acount.item())                             # sync 2
            self.acc_rate_est = max(na / nv, 1e-4)
            rounds.append((theta, stats, d, apos, na, nv, guard))
            n_acc += na
            if self.max_rounds is not None and len(rounds) >= self.max_rounds \
                    and n_acc < nq:
                raise RuntimeError("acceptance rate too low: "
                                   f"{n_acc}/{sim_off} after {len(rounds)} "
                                   "rounds")
        tm["propose_sim_dist"] = time.perf_counter() - t0
        # first nq accepted in proposal order; evaluations up to the nq-th
        thetas, ds, stats_acc, recs = [], [], [], []
        n_eval = 0
        left = nq
        n_guard = 0
        for (theta, stats, d, apos, na, nv, guard) in rounds:
            take = min(left, na)
            sel = apos[:take]
            # the round holding the nq-th acceptance counts evaluations up
            # to and including it (singlecore.py:24-35)
            last = int(apos[take - 1].item()) + 1 if take == left else nv
            n_eval += last
            thetas.append(theta.index_select(0, sel))
            ds.append(d.index_select(0, sel))
            if keep_stats:
                stats_acc.append(stats.index_select(1, sel))
            if record:
                recs.append(stats[:, :last])
            n_guard += int(guard[:last].sum().item())
            left -= take
            if left == 0:
                break
        theta_acc = torch.cat(thetas) if thetas else torch.empty(
            (0, self.d), dtype=F64, device=self.dev)
        d_acc = torch.cat(ds) if ds else torch.empty(0, dtype=F64,
                                                     device=self.dev)
        torch.cuda.synchronize()
        tm["select"] = time.perf_counter() - t0 - tm["propose_sim_dist"]
        t1 = time.perf_counter()
        if fit is None:
            logpd = None
            w = torch.ones(theta_acc.shape[0], dtype=F64, device=self.dev)
        else:
            if self.kde_events is not None and hasattr(fit, "packed"):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                Y = fit.packed.whiten(theta_acc)
                e0.record()
                logpd = fit.packed.logpdf_whitened(Y)
                e1.record()
                self.kde_events.append((e0, e1, theta_acc.shape[0], fit.n))
            else:
                logpd = fit.logpdf(theta_acc)
            w = K.importance_weights(logpd, None, self.prior_pd)
        torch.cuda.synchronize()
        tm["kde"] = time.perf_counter() - t1
        self.timers = tm
        return GenerationResult(
            theta=theta_acc, d=d_acc, w=w, logpd=logpd, n_eval=n_eval,
            n_guard=n_guard,
            stats_T=torch.cat(stats_acc, 1) if stats_acc else None,
            rec_stats_T=torch.cat(recs, 1) if recs else None)

    # ------------------------------------------------------------------
    def gather_population(self, res):
        """All-gather the rank-local accepted rows (rank-major order) and
        normalise the weights by the global sum (population.py:120-142)."""
        comm = self.comm
        theta = comm.all_gather_rows(res.theta)
        d = comm.all_gather_rows(res.d)
        w = comm.all_gather_rows(res.w)
        s = K.dsum(w)
        K.scale_inplace(w, s)
        n_eval = comm.all_reduce_int(res.n_eval)
        return theta, d, w, n_eval, s
