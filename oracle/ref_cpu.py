"""CPU oracle: a numpy restatement of the reference's per-generation numerics.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline.  The product path (``pyabc_amd``) never
imports it and fails loudly when its HIP library is missing.

Each function restates (it does not copy) the reference semantics of
chrhck/pyABC 0.10.1 at the cited ``file:line`` (paths relative to the
reference checkout).  Where the arithmetic lives in numpy/scipy/glibc the
restatement follows the published algorithm of numpy 2.2 / scipy 1.15 (the
versions the golden fixtures were generated with; ``tools/gen_golden.py``).

Parity status: pinned.  ``tests/test_oracle_golden.py`` checks every function
here against the fixtures under ``tests/golden/`` generated from the reference
itself, and against the reference's own known-answer tests
(``test/test_weighted_statistics.py:6-39``, ``test/test_epsilon.py:25-47``,
``test/test_distance_function.py:75-91,132-150``).
"""
import math

import numpy as np

LOG2E = 1.4426950408889634
LN2 = 0.6931471805599453
LOG_2PI = 1.8378770664093453


# ---------------------------------------------------------------------------
# (a1) Transition.fit wrapper + MultivariateNormalTransition.fit
# ---------------------------------------------------------------------------
def fit_normalize_weights(w):
    """``w /= w.sum()`` unless already close to 1 (transition/transitionmeta.py:16-18)."""
    w = np.array(w, dtype=np.float64)
    if w.size > 0 and not np.isclose(w.sum(), 1):
        w = w / w.sum()
    return w


def silverman_rule_of_thumb(n_samples, dimension):
    """(4 / (n (d+2)))^(1/(d+4))  (transition/multivariatenormal.py:27-37)."""
    return (4 / n_samples / (dimension + 2)) ** (1 / (dimension + 4))


def scott_rule_of_thumb(n_samples, dimension):
    """n^(-1/(d+4))  (transition/multivariatenormal.py:14-24)."""
    return n_samples ** (-1. / (dimension + 4))


def weighted_cov(X, w):
    """``smart_cov`` (transition/util.py:4-15) = np.cov(X, aweights=w, rowvar=False).

    mu = sum w x / sum w ; C = sum w (x-mu)(x-mu)^T / (sum w - sum w^2 / sum w).
    A single row gives diag(|x_0|).
    """
    X = np.asarray(X, dtype=np.float64)
    if X.shape[0] == 1:
        return np.diag(np.abs(X[0]))
    w = np.asarray(w, dtype=np.float64)
    v1 = w.sum()
    mu = (X * w[:, None]).sum(0) / v1
    fact = v1 - (w * w).sum() / v1
    if fact <= 0:
        fact = 0.0
    Xc = X - mu
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.atleast_2d((Xc.T @ (Xc * w[:, None])) * (1.0 / fact))


def mvn_fit_cov(X, w, scaling=1.0, bandwidth_selector=silverman_rule_of_thumb):
    """MultivariateNormalTransition.fit_cov (transition/multivariatenormal.py:67-73)."""
    cov = weighted_cov(X, w)
    d = cov.shape[0]
    ess = 1 / (np.asarray(w) ** 2).sum()
    bw = bandwidth_selector(ess, d)
    return cov * bw ** 2 * scaling


# ---------------------------------------------------------------------------
# (a2) rvs: weighted ancestor resampling + Gaussian perturbation + support
# ---------------------------------------------------------------------------
def resample_cdf(w):
    """numpy legacy ``choice(p=w)`` CDF: sequential cumsum, divided by its last
    entry (multivariatenormal.py:89 -> numpy RandomState.choice)."""
    cdf = np.cumsum(np.asarray(w, dtype=np.float64))
    cdf /= cdf[-1]
    return cdf


def resample_indices(cdf, u):
    """``cdf.searchsorted(u, side='right')`` (numpy RandomState.choice)."""
    return np.searchsorted(cdf, u, side="right")


def svd_factor(cov):
    """numpy legacy ``multivariate_normal`` factor A = sqrt(s)[:,None] * V from
    ``U, s, V = svd(cov)`` so that theta = mean + z @ A  (multivariatenormal.py:91-94)."""
    _, s, v = np.linalg.svd(np.asarray(cov, dtype=np.float64))
    return np.sqrt(s)[:, None] * v


def resample_perturb(X, w, cov, u, z):
    """Batch ``MultivariateNormalTransition.rvs(size=B)`` given its uniforms
    ``u[B]`` and normals ``z[B,d]`` (multivariatenormal.py:87-95)."""
    idx = resample_indices(resample_cdf(w), u)
    A = svd_factor(cov)
    theta = np.asarray(X, dtype=np.float64)[idx] + (np.asarray(z) @ A)
    return idx, theta


def uniform_box_support(theta, lo, scale):
    """``Distribution.pdf(theta) > 0`` for a product of ``RV('uniform', lo, scale)``
    priors (random_variables.py:425-452 -> scipy uniform.pdf): x=(theta-lo)/scale
    in fp64, support is 0 <= x <= 1 inclusive."""
    x = (np.asarray(theta, dtype=np.float64) - lo) / scale
    return np.all((x >= 0) & (x <= 1), axis=-1)


def uniform_box_pdf(theta, lo, scale):
    """Product of the uniform marginal densities (random_variables.py:445-451)."""
    ins = uniform_box_support(theta, lo, scale)
    return np.where(ins, np.prod(1.0 / np.asarray(scale)), 0.0)


# ---------------------------------------------------------------------------
# (a3) KDE transition density and importance weight
# ---------------------------------------------------------------------------
def psd_whitening(cov):
    """scipy ``_PSD`` (scipy/stats/_multivariate.py) as used by
    ``multivariate_normal(cov, allow_singular=True)`` (multivariatenormal.py:85,119):
    s,u = eigh(cov); cut = 1e6 * eps64 * max|s|; U = u / sqrt(s) on s > cut
    (pseudo-inverse); rank; log_pdet = sum log s over s > cut."""
    cov = np.asarray(cov, dtype=np.float64)
    s, u = np.linalg.eigh(cov)
    eps = 1e6 * np.finfo(np.float64).eps * np.max(np.abs(s))
    keep = s > eps
    s_pinv = np.array([0.0 if not k else 1.0 / x for x, k in zip(s, keep)])
    U = u * np.sqrt(s_pinv)
    rank = int(keep.sum())
    log_pdet = float(np.sum(np.log(s[keep])))
    return U, rank, log_pdet


def kde_transition_pd(theta, X, w, cov):
    """MVN.pdf / pdf_static (multivariatenormal.py:102-125):
    sum_j w_j N(theta_i; X_j, cov), evaluated as scipy does it (exp of the
    log-density, then a plain weighted sum)."""
    theta = np.atleast_2d(np.asarray(theta, dtype=np.float64))
    X = np.asarray(X, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64)
    U, rank, log_pdet = psd_whitening(cov)
    Yp = X @ U
    out = np.empty(theta.shape[0])
    for i in range(theta.shape[0]):
        diff = theta[i] @ U - Yp
        maha = np.sum(diff * diff, axis=1)
        out[i] = np.sum(np.exp(-0.5 * (rank * LOG_2PI + log_pdet + maha)) * w)
    return out


def kde_logsum(Ynew, Yprev, logw):
    """Contract of the device KDE pass: log sum_j exp(logw_j - 1/2 |y_i - y_j|^2)
    for pre-whitened coordinates (the host adds -1/2(rank log 2pi + log_pdet))."""
    Ynew = np.atleast_2d(np.asarray(Ynew, dtype=np.float64))
    Yprev = np.atleast_2d(np.asarray(Yprev, dtype=np.float64))
    out = np.empty(Ynew.shape[0])
    for i in range(Ynew.shape[0]):
        diff = Ynew[i] - Yprev
        e = logw - 0.5 * np.sum(diff * diff, axis=1)
        m = e.max()
        out[i] = m + np.log(np.sum(np.exp(e - m)))
    return out


def importance_weight(prior_pd, transition_pd, n_accepted=1,
                      nr_samples_per_parameter=1, acceptance_weight=1.0):
    """weight = prior * acceptance_weight * (n_acc / nr_samples) / transition
    (smc.py:776-792)."""
    with np.errstate(divide="ignore"):
        return (np.asarray(prior_pd) * acceptance_weight
                * (n_accepted / nr_samples_per_parameter)
                / np.asarray(transition_pd))


# ---------------------------------------------------------------------------
# (a4) population weight normalisation, ESS
# ---------------------------------------------------------------------------
def normalize_population_weights(w):
    """Single-model ``Population._normalize_weights`` (population.py:120-142):
    sequential Python sum, then divide."""
    w = np.asarray(w, dtype=np.float64)
    total = 0.0
    for x in w.tolist():
        total += x
    return w / total, total


def effective_sample_size(w):
    """(sum w)^2 / sum w^2  (weighted_statistics.py:73-83)."""
    w = np.asarray(w, dtype=np.float64)
    return np.sum(w) ** 2 / np.sum(w ** 2)


# ---------------------------------------------------------------------------
# (a5) p-norm distance + uniform acceptance
# ---------------------------------------------------------------------------
def pnorm_distance(stats, x0, fw, p):
    """PNormDistance.__call__ (distance/distance.py:76-102), vectorised over rows.

    ``stats[B,S]`` columns in x_0 key order; ``fw = f*w`` per key (multiplied
    first, as the reference does).  The key sum is sequential from 0 in key
    order; powers use C ``pow`` (Python float semantics), evaluated by
    ``math.pow`` element-wise so numpy's x*x / sqrt fast paths are avoided.
    """
    stats = np.atleast_2d(np.asarray(stats, dtype=np.float64))
    B, S = stats.shape
    fw = np.asarray(fw, dtype=np.float64)
    x0 = np.asarray(x0, dtype=np.float64)
    out = np.empty(B)
    if p == np.inf:
        return np.max(np.abs(fw[None, :] * (stats - x0[None, :])), axis=1) \
            if S else np.zeros(B)
    pw = float(p)
    inv = 1 / p
    for b in range(B):
        acc = 0
        row = stats[b]
        for k in range(S):
            acc = acc + math.pow(abs(fw[k] * (row[k] - x0[k])), pw)
        out[b] = math.pow(acc, inv)
    return out


def accept(d, eps):
    """``d <= eps(t)`` (acceptor/acceptor.py:241-242)."""
    return np.asarray(d) <= eps


# ---------------------------------------------------------------------------
# (a6) adaptive distance scale functions and weights
# ---------------------------------------------------------------------------
def median_absolute_deviation(x):
    """median(|x - median(x)|) with np.median even-n = mean of the two middle
    values (distance/scale.py:38-47)."""
    x = np.asarray(x, dtype=np.float64)
    return np.median(np.abs(x - np.median(x)))


def standard_deviation(x):
    """np.std, ddof 0 (distance/scale.py:59-65)."""
    return np.std(np.asarray(x, dtype=np.float64))


def adaptive_pnorm_weights(data, scale="std", normalize=True,
                           max_weight_ratio=None):
    """AdaptivePNormDistance._update/_normalize_weights/_bound_weights
    (distance/distance.py:253-338).  ``data[n,S]`` in x_0 key order."""
    data = np.asarray(data, dtype=np.float64)
    fn = median_absolute_deviation if scale == "mad" else standard_deviation
    w = []
    for k in range(data.shape[1]):
        s = fn(data[:, k])
        w.append(0 if np.isclose(s, 0) else 1 / s)
    w = np.array(w, dtype=np.float64)
    if normalize:
        w = w / np.mean(w)
    if max_weight_ratio is not None:
        nz = np.abs(w[w != 0])
        mn = np.min(nz)
        big = np.abs(w) / mn > max_weight_ratio
        w[big] = np.sign(w[big]) * max_weight_ratio * mn
    return w


# ---------------------------------------------------------------------------
# (a7) weighted quantile epsilon
# ---------------------------------------------------------------------------
def weighted_quantile(points, weights=None, alpha=0.5):
    """argsort, sequential cumsum, interp(alpha, cs - w/2, sorted points)
    (weighted_statistics.py:26-43)."""
    points = np.asarray(points, dtype=np.float64)
    order = np.argsort(points)
    p = points[order]
    if weights is None:
        w = np.ones(len(p)) / len(p)
    else:
        w = np.asarray(weights, dtype=np.float64)[order]
    cs = np.cumsum(w)
    return float(np.interp(alpha, cs - 0.5 * w, p))


def quantile_epsilon(distances, w, alpha=0.5, multiplier=1.0, weighted=True):
    """QuantileEpsilon._update (epsilon/epsilon.py:202-228)."""
    distances = np.asarray(distances, dtype=np.float64)
    if weighted:
        w = np.asarray(w, dtype=np.float64)
        w = w / w.sum()
    else:
        w = np.ones(len(distances)) / len(distances)
    return weighted_quantile(distances, w, alpha) * multiplier


# ---------------------------------------------------------------------------
# (a8) LocalTransition
# ---------------------------------------------------------------------------
def knn_indices(X, k):
    """Brute-force k nearest neighbours excluding self (the reference queries
    cKDTree with k+1 and drops column 0; local_transition.py:82-83).  Rows are
    returned sorted by distance (tie-free inputs assumed)."""
    X = np.asarray(X, dtype=np.float64)
    n = X.shape[0]
    kk = min(k + 1, n)
    out = np.empty((n, kk - 1), dtype=np.int64)
    for i in range(n):
        d2 = np.sum((X - X[i]) ** 2, axis=1)
        order = np.argsort(d2, kind="stable")[:kk]
        out[i] = order[1:]
    return out


def local_k(k, k_fraction, n, d, min_k=10):
    """LocalTransition.k (local_transition.py:60-75)."""
    k_ = int(k_fraction * n) if k_fraction is not None else k
    return max([k_, min_k, d])


def knn_rows(X, k, rows):
    """knn_indices for the particles ``rows`` only (sorted by distance)."""
    X = np.asarray(X, dtype=np.float64)
    kk = min(k + 1, X.shape[0])
    out = np.empty((len(rows), kk - 1), dtype=np.int64)
    for r, i in enumerate(rows):
        d2 = np.sum((X - X[i]) ** 2, axis=1)
        out[r] = np.argsort(d2, kind="stable")[:kk][1:]
    return out


def local_covs(X, w, nbr, scaling=1.0, eps=1e-3, rows=None):
    """LocalTransition._cov / _cov_and_inv (local_transition.py:112-139).
    ``rows``: evaluate only these particles (``nbr`` then holds their
    neighbour rows, in the same order)."""
    X = np.asarray(X, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64)
    n, d = X.shape
    rows = np.arange(n) if rows is None else np.asarray(rows)
    covs = np.empty((len(rows), d, d))
    invs = np.empty((len(rows), d, d))
    dets = np.empty(len(rows))
    for r, i in enumerate(rows):
        if nbr.shape[1] >= 1:
            deltas = X[nbr[r]] - X[i]
            lw = w[nbr[r]]
            c = weighted_cov(deltas, lw / lw.sum())
        else:
            c = weighted_cov(np.abs(X), np.array([1.0]))
        if np.abs(c.sum()) == 0:
            for j in range(d):
                c[j, j] = np.abs(X[0, j])
        c = c * scaling
        det = np.linalg.det(c)
        while det <= 0:
            c = c + np.identity(d) * eps
            det = np.linalg.det(c)
        covs[r] = c
        invs[r] = np.linalg.inv(c)
        dets[r] = det
    return covs, invs, dets


def local_rvs(X, w, covs, u, z):
    """``LocalTransition.rvs_single`` per draw (local_transition.py:141-145):
    ``choice(N, p=w)`` = searchsorted(cumsum(w)/sum, u, 'right'), then legacy
    ``multivariate_normal(X[idx], C[idx])`` = X[idx] + z @ (sqrt(s)[:, None]
    * V) with (U, s, V) = svd(C[idx])."""
    idx = resample_indices(resample_cdf(w), np.asarray(u))
    theta = np.empty((len(idx), X.shape[1]))
    for b, i in enumerate(idx):
        _, s, v = np.linalg.svd(covs[i])
        theta[b] = np.asarray(z[b]) @ (np.sqrt(s)[:, None] * v) + X[i]
    return idx, theta


def local_pdf(pts, X, w, invs, dets):
    """LocalTransition._pdf_single (local_transition.py:103-110):
    sum_n w_n exp(-1/2 q_n) / sqrt((2 pi)^d det_n) / sum w."""
    pts = np.atleast_2d(np.asarray(pts, dtype=np.float64))
    X = np.asarray(X, dtype=np.float64)
    d = X.shape[1]
    norm = np.sqrt((2 * np.pi) ** d * dets)
    out = np.empty(pts.shape[0])
    for i in range(pts.shape[0]):
        dist = X - pts[i]
        q = np.einsum("ij,ijk,ik->i", dist, invs, dist)
        out[i] = np.average(np.exp(-.5 * q) / norm, weights=w)
    return out


# ---------------------------------------------------------------------------
# Philox4x32-10 (Salmon et al., SC'11 "Parallel random numbers: as easy as
# 1, 2, 3").  The device RNG of the production path; no reference
# counterpart (the reference draws from numpy's legacy MT19937).
# ---------------------------------------------------------------------------
PHILOX_M0 = 0xD2511F53
PHILOX_M1 = 0xCD9E8D57
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85


def philox4x32_10(ctr, key):
    """Vectorised Philox4x32 with 10 rounds.  ``ctr`` is uint32[...,4], ``key``
    uint32[...,2]; returns uint32[...,4]."""
    c = np.array(ctr, dtype=np.uint64) & 0xFFFFFFFF
    k = np.array(key, dtype=np.uint64) & 0xFFFFFFFF
    c0, c1, c2, c3 = (c[..., i].copy() for i in range(4))
    k0, k1 = k[..., 0].copy(), k[..., 1].copy()
    for r in range(10):
        p0 = c0 * PHILOX_M0
        p1 = c2 * PHILOX_M1
        hi0, lo0 = p0 >> 32, p0 & 0xFFFFFFFF
        hi1, lo1 = p1 >> 32, p1 & 0xFFFFFFFF
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        if r < 9:
            k0 = (k0 + PHILOX_W0) & 0xFFFFFFFF
            k1 = (k1 + PHILOX_W1) & 0xFFFFFFFF
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def philox_block(seed, stream, idx):
    """Block ``idx`` of the library's stream layout: counter = (idx_lo,
    idx_hi, stream_lo, stream_hi), key = (seed_lo, seed_hi)."""
    idx = np.asarray(idx, dtype=np.uint64)
    ctr = np.stack([idx & 0xFFFFFFFF, idx >> 32,
                    np.full_like(idx, stream & 0xFFFFFFFF),
                    np.full_like(idx, (stream >> 32) & 0xFFFFFFFF)], axis=-1)
    key = np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF],
                   dtype=np.uint64)
    return philox4x32_10(ctr, np.broadcast_to(key, ctr.shape[:-1] + (2,)))


def u01_from_words(hi, lo):
    """53-bit uniform in [0,1): ((hi << 21) ^ (lo >> 11)) ... as
    (hi*2^21 + (lo >> 11)) * 2^-53 with hi the top 32 bits."""
    hi = np.asarray(hi, dtype=np.uint64)
    lo = np.asarray(lo, dtype=np.uint64)
    return ((hi << np.uint64(21)) | (lo >> np.uint64(11))).astype(np.float64) \
        * (1.0 / 9007199254740992.0)


def philox_uniform(seed, stream, n):
    """u[i], i < n: block i//2, words (0,1) for even i and (2,3) for odd i."""
    i = np.arange(n, dtype=np.uint64)
    blk = philox_block(seed, stream, i // np.uint64(2))
    odd = (i & np.uint64(1)).astype(bool)
    hi = np.where(odd, blk[:, 2], blk[:, 0])
    lo = np.where(odd, blk[:, 3], blk[:, 1])
    return u01_from_words(hi, lo)


def philox_normal(seed, stream, n):
    """z[i]: Box-Muller on a pair of 53-bit uniforms from block i//2 (even i
    -> cos branch, odd i -> sin branch); u1 in (0,1]."""
    i = np.arange(n, dtype=np.uint64)
    blk = philox_block(seed, stream, i // np.uint64(2))
    u1 = 1.0 - u01_from_words(blk[:, 0], blk[:, 1])
    u2 = u01_from_words(blk[:, 2], blk[:, 3])
    r = np.sqrt(-2.0 * np.log(u1))
    ang = 2.0 * np.pi * u2
    odd = (i & np.uint64(1)).astype(bool)
    return np.where(odd, r * np.sin(ang), r * np.cos(ang))


def philox_normal4_f32(seed, stream, n):
    """The synthetic simulators' noise z[i] (library: philox.hpp
    box_muller4_f32): block i//4, 24-bit uniforms (w >> 8) * 2^-24 of each
    word, fp32 Box-Muller -- words (0,1) give members 0 (cos) and 1 (sin),
    words (2,3) members 2 and 3; u1 = 1 - U.  Restated in float32 with
    numpy's log2 / sin / cos: the device's hardware transcendentals agree to
    a few fp32 ulps, not bit for bit."""
    i = np.arange(n, dtype=np.uint64)
    blk = philox_block(seed, stream, i // np.uint64(4))
    k24 = np.float32(2.0 ** -24)
    m = (i & np.uint64(3)).astype(np.int64)
    w1 = np.where(m < 2, blk[:, 0], blk[:, 2])
    w2 = np.where(m < 2, blk[:, 1], blk[:, 3])
    u1 = np.float32(1) - (w1 >> np.uint64(8)).astype(np.float32) * k24
    u2 = (w2 >> np.uint64(8)).astype(np.float32) * k24
    r = np.sqrt(np.float32(-2 * LN2) * np.log2(u1).astype(np.float32))
    ang = (np.float32(2 * np.pi) * u2).astype(np.float32)
    z = np.where(m % 2 == 0, r * np.cos(ang), r * np.sin(ang))
    return z.astype(np.float32).astype(np.float64)


# ---------------------------------------------------------------------------
# (f3) exact inference: stochastic kernels, stochastic acceptance,
#      temperature schemes
# ---------------------------------------------------------------------------
def np_pairwise_sum(a):
    """numpy's float64 ``np.sum`` of a contiguous vector: 0 + pairwise(a).

    pairwise(n < 8): sequential; n <= 128: eight strided accumulators seeded
    with a[0..7], combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the
    n % 8 tail sequentially; n > 128: split at n2 = n//2 rounded down to a
    multiple of 8 (numpy/_core/src/umath/loops_utils.h.src pairwise_sum)."""
    a = [float(x) for x in a]

    def pw(lo, n):
        if n < 8:
            r = 0.0
            for i in range(lo, lo + n):
                r += a[i]
            return r
        if n <= 128:
            r = a[lo:lo + 8]
            i = 8
            while i < n - (n % 8):
                for j in range(8):
                    r[j] += a[lo + i + j]
                i += 8
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
            while i < n:
                res += a[lo + i]
                i += 1
            return res
        n2 = n // 2
        n2 -= n2 % 8
        return pw(lo, n2) + pw(lo + n2, n - n2)
    return 0.0 + pw(0, len(a))


def independent_normal_logpdf(stats, x0, var):
    """IndependentNormalKernel.__call__ (distance/kernel.py:256-282), rows of
    ``stats[B,S]`` in the kernel's key order:
    -0.5 * (sum(log 2 + log pi + log var) + sum(diff**2 / var)), both sums
    numpy pairwise, diff = x - x_0."""
    stats = np.atleast_2d(np.asarray(stats, dtype=np.float64))
    var = np.asarray(var, dtype=np.float64)
    c = np.sum(np.log(2) + np.log(np.pi) + np.log(var))
    diff = stats - np.asarray(x0, dtype=np.float64)[None, :]
    sq = np.array([np_pairwise_sum((r ** 2) / var) for r in diff])
    return -0.5 * (c + sq)


def independent_laplace_logpdf(stats, x0, scale):
    """IndependentLaplaceKernel.__call__ (distance/kernel.py:332-357):
    -(sum(log 2 + log b) + sum(|diff| / b))."""
    stats = np.atleast_2d(np.asarray(stats, dtype=np.float64))
    scale = np.asarray(scale, dtype=np.float64)
    c = np.sum(np.log(2) + np.log(scale))
    diff = stats - np.asarray(x0, dtype=np.float64)[None, :]
    ab = np.array([np_pairwise_sum(np.abs(r) / scale) for r in diff])
    return -(c + ab)


def stochastic_accept(pd, pdf_norm, temp, u, log_scale=True,
                      apply_importance_weighting=True):
    """StochasticAcceptor.__call__ (acceptor/acceptor.py:440-473):
    acc_prob = exp((pd - c) * (1/T)) [log] or (pd / c) ** (1/T) [lin];
    accept iff acc_prob >= u; weight 0 if acc_prob == 0, else
    acc_prob / min(1, acc_prob) (or 1 without importance weighting)."""
    pd = np.asarray(pd, dtype=np.float64)
    inv_t = 1 / temp
    if log_scale:
        with np.errstate(over="ignore"):
            acc = np.exp((pd - pdf_norm) * inv_t)   # numpy's exp, as the ref
    else:
        acc = np.array([(p / pdf_norm) ** inv_t for p in pd])
    accept = acc >= np.asarray(u)
    w = np.where(acc == 0.0, 0.0,
                 acc / np.minimum(1.0, acc) if apply_importance_weighting
                 else 1.0)
    return acc, accept, w


def pdf_norm_max_found(prev_pdf_norm, pds):
    """max(prev, *pds) (acceptor/pdf_norm.py:17-38)."""
    prev = -np.inf if prev_pdf_norm is None else prev_pdf_norm
    return max(prev, *pds)


def match_acceptance_rate(weights, pds, pdf_norm, log_scale, target_rate):
    """epsilon/temperature.py:306-345: bisection in b = log(beta) on
    sum(w * min(acc_prob(beta), 1)) - target over [-100, 0]; T = 1/exp(b)."""
    import scipy.optimize
    weights = np.asarray(weights, dtype=np.float64)
    pds = np.asarray(pds, dtype=np.float64)

    def obj(b):
        beta = np.exp(b)
        if log_scale:
            acc = np.exp((pds - pdf_norm) * beta)
        else:
            acc = (pds / pdf_norm) ** beta
        return np.sum(weights * np.minimum(acc, 1.0)) - target_rate
    min_b = -100
    if obj(0) > 0:
        b = 0
    elif obj(min_b) < 0:
        b = min_b
    else:
        b = scipy.optimize.bisect(obj, min_b, 0, maxiter=100000)
    return 1. / np.exp(b)


def acceptance_rate_temperature(pds, t_pd_prev, t_pd, pdf_norm, log_scale,
                                target_rate=0.3):
    """AcceptanceRateScheme.__call__ (epsilon/temperature.py:280-303):
    importance weights t_pd / t_pd_prev normalised by a sequential sum."""
    w = np.asarray(t_pd, dtype=np.float64) / np.asarray(t_pd_prev,
                                                         dtype=np.float64)
    w = w / sum(w)
    return match_acceptance_rate(w, pds, pdf_norm, log_scale, target_rate)
