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
import os
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
                 precision="mfma", moments=None, pack_stream=None):
        self.X = X
        self.w = w
        self.precision = precision
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
            if moments is None:
                moments = K.weighted_moments(X, w)
            mom = moments.cpu().numpy() if torch.is_tensor(moments) \
                else np.asarray(moments, dtype=np.float64)
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
        U, rank, log_pdet = K.psd_whitening(self.cov)
        self.rank, self.log_pdet = rank, log_pdet
        # A, the whitening Us and mu in ONE host-to-device copy
        host = np.concatenate([self.A_host.ravel(),
                               (U * math.sqrt(0.5 * K.LOG2E)).ravel(),
                               np.asarray(mu, dtype=np.float64).ravel()])
        if pack_stream is not None:
            # page-locked staging: an asynchronous copy (the buffer is
            # reused a generation later, after the stream has passed it)
            pin = _pinned("h2d", host.size)
            pin[:host.size].numpy()[:] = host
            dev = torch.empty(host.size, dtype=F64, device=X.device)
            dev.copy_(pin[:host.size], non_blocking=True)
            _pinned_used("h2d")
        else:
            dev = torch.as_tensor(host, dtype=F64, device=X.device)
        self.A = dev[:d * d].view(d, d)
        Us = dev[d * d:2 * d * d].view(d, d)
        mu_t = dev[2 * d * d:]
        self._pack_ev = None
        self._pack_args = None
        if pack_stream is None:
            self._packed = K.PackedPopulation(X, w, mu_t, Us, rank, log_pdet,
                                              precision)
        else:
            # the KDE pack on another stream, launched by start_pack() --
            # the engine calls it right after the next generation's first
            # proposal launch, so the pack's host work no longer sits
            # between this fit and those proposals (round 6: ~0.15 ms of
            # host time per generation, 1 % of a rank's step at R = 8); its
            # first user (the density pass, through .packed) waits for it
            self._packed = None
            self._pack_args = (X, w, mu_t, Us, rank, log_pdet, precision,
                               pack_stream)
        self._cdf = None
        self._tab = None
        self._cdf_ev = None

    def start_pack(self):
        """Launch the deferred KDE pack on its stream (no-op once launched,
        or when the pack ran at construction)."""
        if self._pack_args is None:
            return
        X, w, mu_t, Us, rank, log_pdet, precision, pack_stream = \
            self._pack_args
        self._pack_args = None
        main = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(main)
        with torch.cuda.stream(pack_stream):
            pack_stream.wait_event(ev)
            pp = K.PackedPopulation(X, w, mu_t, Us, rank, log_pdet,
                                    precision, ws_tag="pack_side")
            self._pack_ev = torch.cuda.Event()
            self._pack_ev.record(pack_stream)
        for t in (pp.P, pp.lw2max, getattr(pp, "A", None),
                  getattr(pp, "gscale", None)):
            if t is not None:
                t.record_stream(main)
        self._packed = pp

    @property
    def packed(self):
        """The packed previous population (launches a deferred pack, and
        waits for its stream's pack at first use)."""
        self.start_pack()
        if self._pack_ev is not None:
            torch.cuda.current_stream().wait_event(self._pack_ev)
            self._pack_ev = None
        return self._packed

    @property
    def cdf(self):
        if self._cdf is None:
            self._cdf = K.resample_cdf(self.w)
            self._tab = K.cdf_index(self._cdf)
        if self._cdf_ev is not None:   # computed on a side stream
            torch.cuda.current_stream().wait_event(self._cdf_ev)
            self._cdf_ev = None
        return self._cdf

    def adopt_cdf(self, cdf, tab, event):
        """The resampling CDF and its bucket table, computed on another
        stream; ``event`` marks their completion (waited at first use)."""
        self._cdf, self._tab, self._cdf_ev = cdf, tab, event

    def logpdf(self, theta, parent=None):
        """log transition density; ``parent``: per row the population index
        its proposal was resampled from (optional; same density, the MFMA
        pass then evaluates the row relative to its parent's term)."""
        return self.packed.logpdf(theta, parent)

    def propose(self, lo, scale, seed, sid, offset, B):
        """B draws of resample + perturb + support flag (Philox); the CDF
        search is bracketed by the bucket table (same indices)."""
        cdf = self.cdf
        return K.propose_philox(self.X, cdf, self.A, lo, scale, seed, sid,
                                offset, B, tab=self._tab)


_SIDE = {}
_PINNED = {}


def _side_stream():
    dev = torch.cuda.current_device()
    if dev not in _SIDE:
        _SIDE[dev] = torch.cuda.Stream(device=dev)
    return _SIDE[dev]


def _pinned(key, n):
    """A cached page-locked host buffer of >= n float64 for asynchronous
    copies.  Waits for the copy that last used the buffer (its event, see
    _pinned_used) before handing it out again."""
    b, ev = _PINNED.get(key, (None, None))
    if ev is not None:
        ev.synchronize()
    if b is None or b.numel() < n:
        b = torch.empty(max(n, 256), dtype=F64, pin_memory=True)
    _PINNED[key] = (b, None)
    return b


def _pinned_used(key):
    """Mark the buffer's pending copy (an event on the current stream)."""
    b, _ = _PINNED[key]
    ev = torch.cuda.Event()
    ev.record()
    _PINNED[key] = (b, ev)


def start_cdf(w):
    """The resampling CDF of w and its bucket table, launched on the side
    stream after the launching stream's work so far; returns (cdf, tab,
    event) for DeviceMVNFit.adopt_cdf (waited at first use)."""
    main = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(main)
    side = _side_stream()
    with torch.cuda.stream(side):
        side.wait_event(ev)
        # its own scratch: a main-stream CDF (LocalTransition.fit) may run
        # at the same time
        cdf = K.resample_cdf(w, ws_tag="cdf_side")
        tab = K.cdf_index(cdf)
        cdf_ev = torch.cuda.Event()
        cdf_ev.record(side)
    # allocated on the side stream, read on the main one
    cdf.record_stream(main)
    tab.record_stream(main)
    return cdf, tab, cdf_ev


def next_generation_inputs(theta, d, w, alpha, comm=None, scaling=1.0,
                           bandwidth_selector=None, precision="mfma"):
    """QuantileEpsilon(alpha)'s next epsilon and the MultivariateNormal fit
    of the new population (``smc.py:942-1061``: epsilon update, then
    ``_fit_transitions``), with the stages that do not depend on each other
    overlapped: the resampling CDF (latency-bound binade walks) runs on a
    side stream while the main stream computes the weighted moments and then
    the quantile; the host's d x d finish starts as soon as the moments are
    back (the quantile's kernels still running), and the KDE pack goes to
    the side stream after the CDF (the next generation's density pass waits
    for it, its proposals do not).  Every rank holds the whole population and computes
    the same bits (no collective).  Returns (eps, fit)."""
    main = torch.cuda.current_stream()
    side = _side_stream()
    cdf, tab, cdf_ev = start_cdf(w)
    mom = K.weighted_moments(theta, w)
    nm = mom.numel()
    pin = _pinned("d2h", nm + 1)
    pin[:nm].copy_(mom, non_blocking=True)
    mom_ev = torch.cuda.Event()
    mom_ev.record(main)
    q = K.weighted_quantile(d, w, alpha, comm=comm)
    pin[nm:nm + 1].copy_(q[:1], non_blocking=True)
    q_ev = torch.cuda.Event()
    q_ev.record(main)
    # the host's d x d finish runs while the quantile's kernels do; the
    # KDE pack follows the CDF on the side stream (needed only by the next
    # generation's density pass)
    mom_ev.synchronize()
    fit = DeviceMVNFit(theta, w, scaling, bandwidth_selector, precision,
                       moments=pin[:nm].numpy().copy(), pack_stream=side)
    fit.adopt_cdf(cdf, tab, cdf_ev)
    q_ev.synchronize()
    eps = float(pin[nm].item())
    _PINNED["d2h"] = (pin, None)
    return eps, fit


def selection_plan(nvs, nas, n):
    """Which rows of each (round k, rank s) segment form the population.

    ``nvs[k][s]`` / ``nas[k][s]``: in-support evaluations / acceptances of
    rank s in round k; within a round rank s's evaluation ids precede rank
    s+1's, and rounds follow each other.  Returns ``takes[k][s]`` (the first
    takes accepted rows of the segment belong to the first n accepted) and
    ``closing[k][s]`` = 0 before the segment holding the n-th acceptance
    (all its evaluations count), 1 for that segment, 2 after it.
    """
    takes, closing = [], []
    acc = 0
    state = 0
    for nv_k, na_k in zip(nvs, nas):
        tk, cl = [], []
        for s in range(len(na_k)):
            t = int(min(max(n - acc, 0), na_k[s]))
            if state == 0 and t > 0 and acc + t == n:
                cl.append(1)
                state = 2
            else:
                cl.append(state)
            tk.append(t)
            acc += int(na_k[s])
        takes.append(tk)
        closing.append(cl)
    return takes, closing


def copy_rows(dst, src):
    """dst[:] = src (same shape, rows of 8-byte words): the library's strided
    word copy on the device (no torch kernel), a plain copy for the host
    tensors of the gloo rehearsals."""
    if src.shape[0] == 0:
        return dst
    if dst.is_cuda:
        if src.dim() == 1:
            return K.gather_words(src, None, src.shape[0], dst)
        return K.gather_words(src.reshape(src.shape[0], -1), None,
                              src.shape[0], dst.view(dst.shape[0], -1))
    dst.copy_(src)
    return dst


def cat_rows(pieces, row_shape, device, dtype=F64):
    """torch.cat of row pieces through :func:`copy_rows` (a single piece is
    returned as is)."""
    if len(pieces) == 1:
        return pieces[0]
    n = sum(int(p.shape[0]) for p in pieces)
    out = torch.empty((n,) + tuple(row_shape), dtype=dtype, device=device)
    r = 0
    for p in pieces:
        copy_rows(out[r:r + p.shape[0]], p)
        r += p.shape[0]
    return out


def gather_segments(comm, pieces, row_shape, counts, device, dtype=F64):
    """Global row order from per-rank pieces: ``pieces`` are this rank's
    non-empty segments in round order (a list, or one tensor holding them
    back to back), ``counts[s][k]`` the rows rank s holds from round k.
    Returns the rows ordered round-major, then by rank -- the global id
    order -- on every rank (one all-gather; the reorder is a block copy, and
    none at all when one round produced every row)."""
    if torch.is_tensor(pieces):
        local = pieces
    elif pieces:
        local = cat_rows(pieces, row_shape, device, pieces[0].dtype)
    else:
        local = torch.empty((0,) + tuple(row_shape), dtype=dtype, device=device)
    R = comm.world
    if not comm.active:
        return local
    allr = comm.all_gather_rows(local, [sum(c) for c in counts])
    starts = [0]
    for s in range(R):
        starts.append(starts[-1] + sum(counts[s]))
    blocks = []
    for k in range(len(counts[0])):
        for s in range(R):
            c = counts[s][k]
            if c:
                blocks.append((starts[s] + sum(counts[s][:k]), c))
    pos = 0
    for off, c in blocks:     # already in global order (one round): no copy
        if off != pos:
            break
        pos += c
    else:
        return allr
    out = torch.empty_like(allr)
    pos = 0
    for off, c in blocks:
        copy_rows(out[pos:pos + c], allr[off:off + c])
        pos += c
    return out


def mirrors_simulate(model):
    """True when ``model.simulate_distance`` is defined by the same class as
    the ``simulate`` it mirrors: a subclass that overrides ``simulate``
    (other noise, other statistics) without its own fused method is not
    fused, so its distances always come from its own simulate()."""
    inst = vars(model) if hasattr(model, "__dict__") else {}
    if "simulate" in inst or "simulate_distance" in inst:
        # replaced on the instance: fused only if both come from it
        return "simulate" in inst and "simulate_distance" in inst

    def owner(name):
        return next((c for c in type(model).__mro__ if name in c.__dict__),
                    None)
    o = owner("simulate_distance")
    return o is not None and o is owner("simulate")


def fused_keeps_stats(model):
    """True when the model's ``simulate_distance`` can also return the
    statistics it simulates (a ``keep_stats`` parameter): rounds that keep
    them then run one pass instead of simulate() + the distance kernel."""
    import inspect
    try:
        return "keep_stats" in inspect.signature(
            model.simulate_distance).parameters
    except (TypeError, ValueError):
        return False


def pnorm_host(x, x0, fw, p):
    """One particle's distance exactly as the reference evaluates it
    (distance/distance.py:88-100): Python floats, libm ``pow`` for every
    term and for the root, ``sum`` sequential from int 0 in key order."""
    if p == math.inf:
        return max(abs(f * (a - b)) for a, b, f in zip(x, x0, fw))
    return math.pow(sum(math.pow(abs(f * (a - b)), p)
                        for a, b, f in zip(x, x0, fw)), 1 / p)


def redecide_guard_band(stats, B, d, acc, guard, x0_host, fw_host, p, eps,
                        band=None):
    """Host re-decision of the guard band (acceptor.py:241-242).

    The kernel squares with ``t*t`` and roots with ``sqrt``; the reference
    calls libm ``pow`` for both.  ``t*t == pow(t, 2.)`` bit for bit, but
    ``pow(s, .5)`` differs from ``sqrt(s)`` by one ulp for about 1e-3 of all
    s (general p: a few ulp), so a particle whose device distance lies within
    the flagged band around eps could be decided differently.  Those
    columns -- normally none -- are copied to the host, re-evaluated with
    :func:`pnorm_host`, and their distance and accept bit overwritten, so
    the accept mask equals the reference's.  ``band`` = (positions, count)
    of the flagged columns when the caller has compacted them already.
    Returns the band's size."""
    if guard is None or B == 0:
        return 0
    if band is None:
        gpos, gcount = K.compact(guard[:B])
        n = int(gcount.item())
    else:
        gpos, n = band
    if n == 0:
        return 0
    sel = gpos[:n]
    cols = stats.index_select(1, sel).cpu().numpy()
    dh = np.array([pnorm_host(cols[:, i].tolist(), x0_host, fw_host, p)
                   for i in range(n)], dtype=np.float64)
    d.index_copy_(0, sel, torch.as_tensor(dh, device=d.device))
    acc.index_copy_(0, sel, torch.as_tensor((dh <= eps).astype(np.uint8),
                                            device=acc.device))
    return n


def _count_slots(dev):
    """int64[3] device slots: accepted count, guard-band count, closing
    position (filled by the compactions / a word copy, read in one go)."""
    return torch.empty(3, dtype=torch.int64, device=dev)


def _read_counts(cbuf, apos, nv, need):
    """[accepted, guard band, apos[need - 1]] in one host read of ``cbuf``
    (the first two slots written by the compactions); the last is the
    position of the round's need-th acceptance (valid only when accepted >=
    need) -- the selection's closing position without a read of its own."""
    k = 2
    if need is not None and nv:
        p = min(need, nv) - 1
        K.gather_words(apos[p:p + 1], None, 1, cbuf[2:3])
        k = 3
    vals = cbuf[:k].cpu().tolist()
    last = vals[2] if k == 3 and vals[0] >= need else None
    return int(vals[0]), int(vals[1]), last


def decide(acceptance, stats, nv, seed, stream, eval_off, need=None):
    """One round's acceptance with ONE host read: distances / flags, the
    order-preserving positions of the accepted columns, the accepted and
    guard-band counts as host ints and, given ``need``, the position of
    the need-th acceptance if the round reached it -> (d, acc, guard, accw,
    apos, n_acc, n_guard, apos_need)."""
    if hasattr(acceptance, "decide"):
        return acceptance.decide(stats, nv, seed, stream, eval_off,
                                 need=need)
    d, acc, guard, accw = acceptance(stats, nv, seed, stream, eval_off)
    cbuf = _count_slots(acc.device)
    apos, _ = K.compact(acc, count=cbuf[0:1])
    if guard is not None:
        K.compact(guard[:nv], count=cbuf[1:2])
    else:
        K.compact(acc[:0], count=cbuf[1:2])    # writes a zero count
    n_acc, n_guard, last = _read_counts(cbuf, apos, nv, need)
    return d, acc, guard, accw, apos, n_acc, n_guard, last


class PNormAcceptance:
    """Uniform acceptance d <= eps of a p-norm distance
    (distance/distance.py:76-102, acceptor/acceptor.py:235-244), with the
    guard band re-decided on the host (:func:`redecide_guard_band`)."""

    def __init__(self, x0, fw, p, eps):
        self.x0, self.fw, self.p, self.eps = x0, fw, p, eps
        self._host = None
        self.n_redecided = 0

    def _host_params(self):
        if self._host is None:
            self._host = (self.x0.cpu().tolist(), self.fw.cpu().tolist())
        return self._host

    def __call__(self, stats, nv, seed, stream, eval_off):
        d, acc, guard = K.pnorm_distance(stats, self.x0, self.fw, self.p,
                                         self.eps, B=nv)
        x0h, fwh = self._host_params()
        self.n_redecided += redecide_guard_band(
            stats, nv, d, acc, guard, x0h, fwh, self.p, self.eps)
        return d, acc, guard, None

    def decide(self, stats, nv, seed, stream, eval_off, fused=None,
               need=None):
        """:func:`decide` for the p-norm: the accepted and the guard-band
        columns are compacted together and their counts read in one host
        sync; the (rare) band is then re-decided and the accepted columns
        compacted again.  ``fused`` = (d, acc, guard, simulate) when the
        round ran the fused simulation + distance: ``stats`` is None and
        the band's statistics come from ``simulate()`` (same Philox noise,
        so the same columns)."""
        x0h, fwh = self._host_params()
        if fused is None:
            d, acc, guard = K.pnorm_distance(stats, self.x0, self.fw, self.p,
                                             self.eps, B=nv)
        else:
            d, acc, guard, simulate = fused
        cbuf = _count_slots(acc.device)
        gpos, _ = K.compact(guard[:nv], count=cbuf[1:2])
        apos, _ = K.compact(acc, count=cbuf[0:1])
        n_acc, n_guard, last = _read_counts(cbuf, apos, nv, need)
        if n_guard:
            if stats is None:
                stats = simulate()
            self.n_redecided += redecide_guard_band(
                stats, nv, d, acc, guard, x0h, fwh, self.p, self.eps,
                band=(gpos, int(n_guard)))
            apos, acount = K.compact(acc)
            n_acc = acount.item()
            last = None  # the band's flags moved the positions
        return d, acc, guard, None, apos, int(n_acc), int(n_guard), last


class StochasticAcceptance:
    """StochasticAcceptor over an independent normal / Laplace kernel
    (acceptor/acceptor.py:440-473, distance/kernel.py:256-357): the log
    density, u ~ U[0,1) from Philox keyed by the GLOBAL evaluation id, the
    decision acc >= u and the acceptance weight, in one fused kernel."""

    def __init__(self, x0, prm, kind, c, pdf_norm, temperature,
                 apply_importance_weighting=True):
        self.x0, self.prm, self.kind, self.c = x0, prm, kind, c
        self.pdf_norm = float(pdf_norm)
        self.inv_temp = 1 / temperature
        self.apply_iw = apply_importance_weighting

    def __call__(self, stats, nv, seed, stream, eval_off):
        pd, acc, accw, guard = K.stochastic_kernel(
            stats, self.x0, self.prm, self.kind, self.c, B=nv,
            pdf_norm=self.pdf_norm, inv_temp=self.inv_temp,
            apply_iw=self.apply_iw, seed=seed, stream=stream, offset=eval_off)
        return pd, acc, guard, accw


class GenerationResult:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class GenerationEngine:
    """Runs generations of a batch model on the current device."""

    def __init__(self, model, prior_lo, prior_scale, distance_p=2.0,
                 comm=None, seed=0, min_batch=1 << 16, max_batch=1 << 22,
                 kde_precision="mfma", record_stats=False):
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
        # rounds whose statistics are not kept run the model's fused
        # simulate_distance when it has one (bit-identical distances)
        self.fuse_sim_distance = True
        self.acc_rate_est = 0.5
        self.valid_rate_est = 1.0
        self.timers = {}
        self.kde_events = None   # list -> (start, end, M, N) per KDE launch
        # wait for the generation's device work before returning (so the
        # "kde" stage timer holds the density pass): diagnostics only.  By
        # default the host returns at once and enqueues the normalisation
        # and the next generation's inputs behind the density pass (round
        # 6: the host's ~0.25 ms between the pass and those kernels no
        # longer leaves the GPU idle); every host read of the results
        # synchronises on its own (.item(), .cpu(), events)
        self.stage_sync = os.environ.get("ABC_STAGE_SYNC") == "1"
        self.max_rounds = None
        # load the library's code objects now, not inside the first
        # generation that launches a unit's kernels (abc_preload)
        K.preload()

    # ------------------------------------------------------------------
    def _sid(self, t, kind):
        # disjoint Philox stream ids per (generation, purpose); shared by all
        # ranks -- a proposal's random numbers are keyed by its GLOBAL id, so
        # the draws do not depend on the number of ranks.  Proposal kernels
        # use the raw streams 2*sid and 2*sid+1; single-stream consumers get
        # _stream() = 2*sid, so no two purposes ever share a raw stream.
        return int(t) * 8 + kind

    def _stream(self, t, kind):
        return 2 * self._sid(t, kind)

    def quota(self, n):
        """Rows of a population of n this rank owns for row-parallel work."""
        lo, hi = self.row_range(n)
        return hi - lo

    def row_ranges(self, n):
        """[lo, hi) of every rank in the balanced contiguous split of n."""
        R = self.comm.world
        q, m = divmod(n, R)
        return [(r * q + min(r, m), r * q + min(r, m) + q + (1 if r < m else 0))
                for r in range(R)]

    def row_range(self, n):
        """[lo, hi) of this rank's rows."""
        return self.row_ranges(n)[self.comm.rank]

    # ------------------------------------------------------------------
    def sample_prior(self, t, n):
        """t = 0 / calibration: theta ~ prior, all accepted
        (smc.py:486-534 with all_accepted=True).  Rank r draws the global
        rows row_range(n); all-gathering in rank order gives the population
        a single GPU would draw."""
        lo, hi = self.row_range(n)
        theta = K.prior_uniform(self.lo, self.scale, self.seed,
                                self._stream(t, 0), lo, hi - lo)
        stats = self.model.simulate(theta, self.seed, self._stream(t, 1), lo)
        return GenerationResult(theta=theta, stats_T=stats, n_eval=hi - lo,
                                rec_stats_T=stats, n_rec=hi - lo)

    def sample_generation(self, t, n, fit, x0, fw, eps, keep_stats=None,
                          record=None, stream_base=0, acceptance=None,
                          record_particles=False, max_eval=math.inf):
        """Proposals until n are accepted (over all ranks), then KDE weights.

        Global-id semantics (SingleCoreSampler, singlecore.py:19-38): raw
        proposal p draws its resample/perturbation numbers from Philox
        counter p; the in-support proposals get consecutive evaluation ids
        (their simulation noise is keyed by that id); the population is the
        first n accepted evaluation ids.  Each round the ranks take adjacent
        slices of the raw-id range and exchange their in-support and accepted
        counts, so the result -- rows, order, evaluation count, recorded
        statistics -- is the same bit for bit for any number of ranks.

        ``fit=None`` proposes from the prior (generation 0, weight 1).
        Returns the GLOBAL population (identical on every rank): theta, d,
        unnormalised w, logpd, n_eval, and with ``keep_stats`` / ``record``
        the accepted statistics / the statistics of every evaluation up to
        the n-th acceptance (record_rejected, sampler/base.py:119-141),
        stat-major.  ``acceptance`` (default: p-norm with ``x0, fw, eps``)
        decides acceptance per evaluation; a stochastic acceptance also
        returns acceptance weights that enter the importance weights.
        ``record_particles`` keeps parameters, distances and accept flags of
        the recorded evaluations (the temperature schemes' records,
        smc.py:990-1017).  ``max_eval`` (SingleCoreSampler's
        check_max_eval, singlecore.py:24-35): no round starts once that
        many evaluations are done; if fewer than n were accepted by then the
        result has ``ok = False`` and no population."""
        keep_stats = self.record_stats if keep_stats is None else keep_stats
        record = self.record_stats if record is None else record
        if acceptance is None and x0 is not None:
            acceptance = PNormAcceptance(x0, fw, self.p, eps)
        comm = self.comm
        R, r = comm.world, comm.rank
        tm = {}
        t0 = time.perf_counter()
        rounds = []
        n_acc = 0
        raw_off = 0
        eval_off = 0
        # the accepted rows' parents (resample indices) travel with theta to
        # the MFMA KDE pass, which evaluates each row relative to its
        # parent's term (kde_mfma.hip, per-row offsets)
        # (the pass uses parents where KL >= 4 lo MFMAs fold: d > 8)
        use_parent = fit is not None and self.d > 8 and getattr(
            fit, "precision", None) == "mfma"
        # SingleCoreSampler starts evaluation k (1-based) iff k - 1 <
        # max_eval: at most ceil(max_eval) evaluations (singlecore.py:24-30)
        cap = math.ceil(max_eval) if math.isfinite(max_eval) else math.inf
        while n_acc < n:
            if eval_off >= cap:
                tm["propose_sim_dist"] = time.perf_counter() - t0
                self.timers = tm
                return GenerationResult(ok=False, n_eval=int(cap))
            need = n - n_acc
            B_glob = int(min(self.max_batch * R, max(
                self.min_batch,
                math.ceil(1.2 * need / max(self.acc_rate_est, 1e-3)
                          / max(self.valid_rate_est, 1e-3)))))
            B = -(-B_glob // R)
            my_raw = raw_off + r * B
            if fit is None:
                theta = K.prior_uniform(self.lo, self.scale, self.seed,
                                        self._stream(t, stream_base), my_raw,
                                        B)
                nvs = [B] * R
            else:
                theta_all, idx, sup = fit.propose(
                    self.lo, self.scale, self.seed,
                    self._sid(t, stream_base), my_raw, B)
                if hasattr(fit, "start_pack"):
                    fit.start_pack()   # a deferred pack: after the proposals
                vpos, vcount = K.compact(sup)
                nvs = comm.all_gather_ints(vcount)                  # sync 1
                nv = nvs[r]
                theta = K.gather_rows(theta_all, vpos, nv) if nv else None
                # the in-support proposals' resample indices (int64)
                pid = K.gather_words(idx, vpos, nv, torch.empty(
                    nv, dtype=torch.int64, device=self.dev)) \
                    if nv and use_parent else None
            nv = nvs[r]
            my_eval = eval_off + sum(nvs[:r])
            sim_sid = self._stream(t, stream_base + 1)
            # statistics nobody keeps: simulation and distance in one pass
            # (kept statistics: the same pass writes them, when the model's
            # fused method can -- round 6)
            keep_any = bool(keep_stats or record)
            fuse = (nv and self.fuse_sim_distance
                    and isinstance(acceptance, PNormAcceptance)
                    and mirrors_simulate(self.model)
                    and (not keep_any or fused_keeps_stats(self.model)))
            if nv and not fuse:
                stats = self.model.simulate(theta, self.seed, sim_sid,
                                            my_eval)
            else:
                stats = None
            accw = acc = None
            alast = None
            # one rank: this round's take is `need` if it closes the
            # generation, so decide's read also brings the closing position
            need1 = need if R == 1 else None
            if acceptance is None:
                # calibration sample: everything accepted, distances later
                # (smc.py:486-514: accepted_distances = [inf])
                d = K.full(nv, math.inf)
                guard = K.full(nv, 0, torch.uint8)
                apos = K.arange(nv)
                nas = list(nvs)
            elif fuse and keep_any:
                a = acceptance
                fd = self.model.simulate_distance(
                    theta, self.seed, sim_sid, my_eval, a.x0, a.fw, a.p, a.eps,
                    keep_stats=True)
                stats = fd[3]
                d, acc, guard, accw, apos, acount, gcount, alast = a.decide(
                    stats, nv, self.seed, self._stream(t, stream_base + 4),
                    my_eval, fused=fd[:3] + (None,), need=need1)    # sync 2
                nas = comm.all_gather_ints(acount)
            elif fuse:
                a = acceptance
                fd = self.model.simulate_distance(
                    theta, self.seed, sim_sid, my_eval, a.x0, a.fw, a.p, a.eps)
                th_, me_ = theta, my_eval
                d, acc, guard, accw, apos, acount, gcount, alast = a.decide(
                    None, nv, self.seed, self._stream(t, stream_base + 4),
                    my_eval, fused=fd + (lambda: self.model.simulate(
                        th_, self.seed, sim_sid, me_),), need=need1)  # sync 2
                nas = comm.all_gather_ints(acount)
            elif nv:
                d, acc, guard, accw, apos, acount, gcount, alast = decide(
                    acceptance, stats, nv, self.seed,
                    self._stream(t, stream_base + 4), my_eval,
                    need=need1)                                     # sync 2
                nas = comm.all_gather_ints(acount)
            else:
                d = guard = apos = None
                nas = comm.all_gather_ints(0)
            if acceptance is None or not nv:
                gcount = 0
            rounds.append(dict(theta=theta, pid=pid if use_parent else None,
                               stats=stats, d=d, apos=apos,
                               guard=guard, accw=accw, acc=acc, nvs=nvs,
                               nas=nas, acc0=n_acc, gcount=gcount,
                               need=need1, alast=alast))
            raw_off += R * B
            eval_off += sum(nvs)
            n_acc += sum(nas)
            self.valid_rate_est = max(sum(nvs) / (R * B), 1e-3)
            if sum(nvs):
                self.acc_rate_est = max(sum(nas) / sum(nvs), 1e-4)
            if self.max_rounds is not None and len(rounds) >= self.max_rounds \
                    and n_acc < n:
                raise RuntimeError("acceptance rate too low: "
                                   f"{n_acc}/{eval_off} after {len(rounds)} "
                                   "rounds")
        tm["propose_sim_dist"] = time.perf_counter() - t0

        # the first n accepted in global id order; evaluations up to the
        # n-th.  Segment (round k, rank s) holds takes[k][s] accepted rows
        # and last[k][s] recorded evaluations; the local pieces are ours.
        takes, closing = selection_plan([rd["nvs"] for rd in rounds],
                                        [rd["nas"] for rd in rounds], n)
        lasts = []
        rec_loc = []
        rth_loc, rd_loc, ra_loc, rp_loc = [], [], [], []
        stochastic = isinstance(acceptance, StochasticAcceptance)
        n_guard = 0
        n_eval_loc = 0
        # this rank's accepted rows of every round land in one buffer per
        # quantity (the library's word gathers; parents as an int64 column
        # beside theta, so one all-gather carries both)
        k_loc = sum(tk[r] for tk in takes)
        wth = self.d + int(use_parent)
        th_buf = torch.empty((k_loc, wth), dtype=F64, device=self.dev)
        d_buf = torch.empty(k_loc, dtype=F64, device=self.dev)
        aw_buf = torch.empty(k_loc, dtype=F64, device=self.dev) \
            if stochastic else None
        st_buf = torch.empty((self.model.n_stats, k_loc), dtype=F64,
                             device=self.dev) if keep_stats else None
        row = 0
        for rd, take, cl in zip(rounds, takes, closing):
            k = take[r]
            if cl[r] == 1:          # this rank holds the n-th acceptance
                if rd["alast"] is not None and k == rd["need"]:
                    last = int(rd["alast"]) + 1     # read with the counts
                else:
                    last = int(rd["apos"][k - 1].item()) + 1
            elif cl[r] == 0:        # before it: every evaluation counts
                last = rd["nvs"][r]
            else:                   # after it
                last = 0
            lasts.append(last)
            n_eval_loc += last
            if k:
                sel = rd["apos"]
                rows_ = slice(row, row + k)
                K.gather_words(rd["theta"], sel, k, th_buf[rows_, :self.d])
                if use_parent:
                    K.gather_words(rd["pid"], sel, k, th_buf[rows_, self.d:])
                K.gather_words(rd["d"], sel, k, d_buf[rows_])
                if stochastic:
                    K.gather_words(rd["accw"], sel, k, aw_buf[rows_])
                if keep_stats:
                    K.gather_cols(rd["stats"], sel, k, st_buf[:, rows_])
                row += k
            if last:
                if record:
                    rec_loc.append(rd["stats"][:, :last])
                if record_particles:
                    rth_loc.append(rd["theta"][:last])
                    if use_parent:
                        rp_loc.append(rd["pid"][:last])
                    rd_loc.append(rd["d"][:last])
                    ra_loc.append(rd["acc"][:last].to(F64) if rd["acc"]
                                  is not None else K.full(last, 1.0))
                if rd["gcount"]:     # no flag in the round: no host read
                    n_guard += int(rd["guard"][:last].sum().item())
        n_eval, n_guard = comm.all_reduce_ints([n_eval_loc, n_guard])
        if n_eval > cap:
            # the n-th acceptance lies past the evaluation cap: the reference
            # stops at cap evaluations without it (sample.ok = False)
            tm["select"] = time.perf_counter() - t0 - tm["propose_sim_dist"]
            self.timers = tm
            return GenerationResult(ok=False, n_eval=int(cap))
        take_counts = [[tk[s] for tk in takes] for s in range(R)]
        theta_acc = self._gather(th_buf, (wth,), take_counts)
        parent_acc = None
        if use_parent:
            T = theta_acc.shape[0]
            parent_acc = K.gather_words(
                theta_acc[:, self.d:], None, T,
                torch.empty((T, 1), dtype=torch.int64, device=self.dev)).view(-1)
            theta_acc = K.gather_words(
                theta_acc[:, :self.d], None, T,
                torch.empty((T, self.d), dtype=F64, device=self.dev))
        d_acc = self._gather(d_buf, (), take_counts)
        stats_acc = None
        if keep_stats:
            stats_acc = self._gather_cols([st_buf], take_counts)
        accw_acc = self._gather(aw_buf, (), take_counts) if stochastic \
            else None
        rec = None
        last_counts = None
        if record or record_particles:
            last_counts = comm.all_gather_int_lists(lasts)
        if record:
            rec = self._gather_cols(rec_loc, last_counts)
        rec_theta = rec_d = rec_acc = rec_parent = None
        if record_particles:
            rec_theta = self._gather(rth_loc, (self.d,), last_counts)
            if use_parent:
                rec_parent = self._gather(rp_loc, (), last_counts,
                                          dtype=torch.int64)
            rec_d = self._gather(rd_loc, (), last_counts)
            rec_acc = self._gather(ra_loc, (), last_counts)
        # host time (the device work of the selection overlaps the KDE pass)
        tm["select"] = time.perf_counter() - t0 - tm["propose_sim_dist"]
        t1 = time.perf_counter()
        if fit is None:
            logpd = None
            # t = 0: weight = 1 * prod(acceptance weights) (smc.py:762-770)
            w = accw_acc.clone() if stochastic else K.full(
                theta_acc.shape[0], 1.0)
        else:
            # row-parallel weight pass: rank r weights rows row_range(n)
            lo, hi = self.row_range(theta_acc.shape[0])
            mine = theta_acc[lo:hi]
            pm = parent_acc[lo:hi] if parent_acc is not None else None
            if self.kde_events is not None and hasattr(fit, "packed"):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                Y = fit.packed.whiten(mine, pm)
                e0.record()
                lp = fit.packed.logpdf_whitened(Y)
                e1.record()
                self.kde_events.append((e0, e1, hi - lo, fit.n))
            elif pm is not None:
                lp = fit.logpdf(mine, pm)
            else:
                lp = fit.logpdf(mine)
            logpd = comm.all_gather_rows(
                lp, [b - a for a, b in self.row_ranges(theta_acc.shape[0])])
            if stochastic:
                w = K.importance_weights_scaled(logpd, accw_acc, self.prior_pd)
            else:
                w = K.importance_weights(logpd, None, self.prior_pd)
        if self.stage_sync:
            torch.cuda.synchronize()
        tm["kde"] = time.perf_counter() - t1
        self.timers = tm
        return GenerationResult(
            ok=True, theta=theta_acc, parent=parent_acc, d=d_acc, w=w,
            logpd=logpd, n_eval=n_eval,
            n_guard=n_guard, stats_T=stats_acc, rec_stats_T=rec,
            accw=accw_acc, rec_theta=rec_theta, rec_d=rec_d, rec_acc=rec_acc,
            rec_parent=rec_parent)

    def _gather(self, pieces, row_shape, counts, dtype=F64):
        return gather_segments(self.comm, pieces, row_shape, counts, self.dev,
                               dtype)

    def _gather_cols(self, pieces, counts):
        """Stat-major [S, cols] version of :meth:`_gather`.  Row-contiguous
        with any row stride: a single round's piece is returned as the
        column slice of that round's [S, B] buffer itself (no copy), so
        consumers take (pointer, ``stride(0)``) -- the kernels do, through
        ``kernels._stat_major`` -- and never assume ``stride(0) == cols``."""
        S = self.model.n_stats
        if not self.comm.active:
            if len(pieces) == 1:
                # one round: the column slice itself (row stride = the
                # round's batch; the kernels take (pointer, ld), no copy)
                return pieces[0]
            n = sum(int(x.shape[1]) for x in pieces)
            out = torch.empty((S, n), dtype=F64, device=self.dev)
            c = 0
            for x in pieces:   # column blocks through the library's copy
                K.gather_cols(x, None, x.shape[1], out[:, c:c + x.shape[1]])
                c += x.shape[1]
            return out
        # several ranks: the row all-gather takes [cols, S] rows (a
        # transpose; the recorded statistics of multi-rank runs only)
        local = torch.cat([x.t() for x in pieces]) if pieces else torch.empty(
            (0, S), dtype=F64, device=self.dev)
        rows = self._gather(local, (S,), counts)
        return rows.t().contiguous()

    # ------------------------------------------------------------------
    def gather_population(self, res):
        """Normalise the (already global) population's weights by their sum
        (population.py:120-142).  Kept for callers of the per-rank API."""
        w = res.w.clone()
        s = K.dsum(w)
        K.scale_inplace(w, s)
        return res.theta, res.d, w, res.n_eval, s
