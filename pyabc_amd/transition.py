"""GPU-backed transitions with the reference's plug-in API.

Reference: pyabc/transition/base.py:13-123 (Transition), transitionmeta.py:
7-51 (no-parameter handling and fit-weight normalisation),
multivariatenormal.py:42-125 (MultivariateNormalTransition) and
local_transition.py:13-145 (LocalTransition).  fit / rvs / pdf compute through
the HIP kernels (weighted moments, Philox proposals, KDE pass; kNN, local
covariances, local density); only d x d factorisations run on the host, where
the reference also calls numpy/scipy on d x d matrices.
"""
import functools
import math
from abc import ABCMeta, abstractmethod

import numpy as np
import pandas as pd
import torch

from . import kernels as K
from .distributed import Comm
from .engine import (DeviceMVNFit, _side_stream, start_cdf,
                     silverman_rule_of_thumb,
                     scott_rule_of_thumb)
from .frames import DeviceFrame, as_device_matrix, as_device_vector

__all__ = ["Transition", "DiscreteTransition", "MultivariateNormalTransition",
           "LocalTransition", "NotEnoughParticles", "silverman_rule_of_thumb",
           "scott_rule_of_thumb"]


class NotEnoughParticles(Exception):
    pass


def _ncols(X):
    return len(X.columns) if hasattr(X, "columns") else np.shape(X)[1]


def _wrap_fit(f):
    @functools.wraps(f)
    def fit(self, X, w):
        self.X = X
        self.w = w
        if _ncols(X) == 0:
            self.no_parameters = True
            return
        self.no_parameters = False
        if isinstance(w, torch.Tensor):
            if w.numel() > 0:
                s = float(K.dsum(as_device_vector(w)).item())
                if not np.isclose(s, 1):
                    w = w / s
                    self.w = w
        elif np.size(w) > 0:
            if not np.isclose(w.sum(), 1):
                w /= w.sum()
        f(self, X, w)
    return fit


def _wrap_pdf(f):
    @functools.wraps(f)
    def pdf(self, x):
        if self.no_parameters:
            return 1
        return f(self, x)
    return pdf


def _wrap_rvs_single(f):
    @functools.wraps(f)
    def rvs_single(self):
        if self.no_parameters:
            return pd.Series(dtype=float)
        return f(self)
    return rvs_single


class TransitionMeta(ABCMeta):
    """Wraps fit/pdf/rvs_single for the zero-parameter case and normalises
    the fit weights (transitionmeta.py:7-51)."""

    def __init__(cls, name, bases, attrs):
        ABCMeta.__init__(cls, name, bases, attrs)
        if "fit" in attrs:
            cls.fit = _wrap_fit(attrs["fit"])
        if "pdf" in attrs:
            cls.pdf = _wrap_pdf(attrs["pdf"])
        if "rvs_single" in attrs:
            cls.rvs_single = _wrap_rvs_single(attrs["rvs_single"])


class Transition(metaclass=TransitionMeta):
    NR_BOOTSTRAP = 5
    X = None
    w = None
    no_parameters = False

    @abstractmethod
    def fit(self, X, w):
        """Fit to the weighted population ``X`` (DataFrame / DeviceFrame)."""

    @abstractmethod
    def rvs_single(self):
        """One sample as a pd.Series indexed by the parameter names."""

    def rvs(self, size=None):
        if size is None:
            return self.rvs_single()
        return pd.DataFrame([self.rvs_single() for _ in range(size)])

    @abstractmethod
    def pdf(self, x):
        """Density at a Series (-> float) or DataFrame (-> ndarray)."""

    def score(self, X, w):
        return (np.log(self.pdf(X)) * w).sum()

    def no_meaningful_particles(self):
        return len(self.X) == 0 or self.no_parameters

    def get_params(self, deep=True):
        return {}

    def set_params(self, **params):
        for k, v in params.items():
            setattr(self, k, v)
        return self


class DiscreteTransition(Transition):
    """Base class of discrete transition kernels."""


def _columns(X):
    return list(X.columns)


def _draw_seed():
    # the reference draws from numpy's global RandomState; seeding it with
    # np.random.seed therefore also fixes the device Philox streams here
    return int(np.random.randint(0, 2 ** 62, dtype=np.int64))


def _as_output(arr, single, columns):
    if single:
        return pd.Series(arr[0], index=columns)
    return pd.DataFrame(arr, columns=columns)


class MultivariateNormalTransition(Transition):
    """Gaussian KDE perturbation kernel on the GPU.

    fit: weighted moments kernel + host d x d finish (smart_cov * bw^2 *
    scaling, multivariatenormal.py:67-85).  rvs: device resampling +
    perturbation (Philox).  pdf: device KDE pass (exact-grid f16 MFMA by
    default; ``kde_precision="f32"`` for the direct fp32 kernel,
    ``kde_precision="f64"`` for the fp64 kernel).
    """

    def __init__(self, scaling=1, bandwidth_selector=silverman_rule_of_thumb,
                 kde_precision="mfma"):
        self.scaling = scaling
        self.bandwidth_selector = bandwidth_selector
        self.kde_precision = kde_precision
        self._fit = None

    def fit(self, X, w):
        if len(X) == 0:
            raise NotEnoughParticles("Fitting not possible.")
        Xd, _ = as_device_matrix(X)
        wd = as_device_vector(w)
        if Xd.is_cuda:
            # the resampling CDF and the KDE pack on the side stream,
            # overlapping the host's d x d finish (engine.start_cdf)
            c = start_cdf(wd)
            self._fit = DeviceMVNFit(Xd, wd, self.scaling,
                                     self.bandwidth_selector,
                                     self.kde_precision,
                                     pack_stream=_side_stream())
            self._fit.adopt_cdf(*c)
        else:
            self._fit = DeviceMVNFit(Xd, wd, self.scaling,
                                     self.bandwidth_selector,
                                     self.kde_precision)
        self.cov = self._fit.cov

    # device-level API used by the batch sampler
    @property
    def device_fit(self):
        return self._fit

    def rvs(self, size=None):
        if size is None:
            return self.rvs_single()
        return self._draw(size, single=False)

    def rvs_single(self):
        return self._draw(1, single=True)

    def _draw(self, size, single):
        f = self._fit
        theta, _, _ = K.propose_philox(f.X, f.cdf, f.A, None, None,
                                       _draw_seed(), 0, 0, size)
        return _as_output(theta.cpu().numpy(), single, _columns(self.X))

    def pdf(self, x):
        single = isinstance(x, pd.Series) or (
            not isinstance(x, (pd.DataFrame, DeviceFrame, torch.Tensor))
            and np.ndim(x) == 1)
        theta, _ = as_device_matrix(x, columns=_columns(self.X)
                                    if isinstance(x, (pd.Series, pd.DataFrame,
                                                      DeviceFrame)) else None)
        dens = torch.exp(self._fit.logpdf(theta)).cpu().numpy()
        if single or dens.size == 1:
            return float(dens[0])
        return dens

    def logpdf_device(self, theta, parent=None):
        """log density at device rows; ``parent`` (optional): per row an
        index into the fitted population (kde_mfma.hip per-row offsets;
        the density does not depend on it)."""
        return self._fit.logpdf(theta, parent)


class LocalTransition(Transition):
    """Local (k-nearest-neighbour covariance) Gaussian kernel on the GPU
    (local_transition.py:13-145): kNN by the one-pass device top-k, per
    particle weighted covariance + LU det/inverse, density by the device
    quadratic-form pass."""
    EPS = 1e-3
    MIN_K = 10

    def __init__(self, k=None, k_fraction=1 / 4, scaling=1,
                 kde_precision="mfma"):
        # kde_precision: the density pass as the z form on the f16 matrix
        # cores "mfma" (the default: 1e-5 relative, measured 1.4e-6 at C4;
        # 21.5 vs 35.1 ms for "f32" at N = M = 2e5, d = 6), the fp32 pair
        # loop "f32" (1e-5) or "f64" (1e-12)
        if kde_precision not in ("f32", "f64", "mfma"):
            raise ValueError(f"unknown kde_precision {kde_precision!r}")
        self.kde_precision = kde_precision
        if k_fraction is not None:
            self.k_fraction = k_fraction
            self._k = None
        else:
            self.k_fraction = None
            self._k = k
        self.scaling = scaling

    @property
    def k(self):
        if self.k_fraction is not None:
            k_ = 0 if self.w is None else int(self.k_fraction * len(self.w))
        else:
            k_ = self._k
        try:
            dim = self._Xd.shape[1]
        except AttributeError:
            dim = 0
        return max([k_, self.MIN_K, dim])

    def fit(self, X, w):
        if len(X) == 0:
            raise NotEnoughParticles("Fitting not possible.")
        self._Xd, _ = as_device_matrix(X)
        self._wd = as_device_vector(w)
        n, d = self._Xd.shape
        kk = min(self.k + 1, n) - 1          # query(k+1) minus self
        if kk == 0:
            # single particle: deltas = |X|, one unit weight (:126-128)
            x0 = self._Xd[0].cpu().numpy()
            c = np.diag(np.abs(x0))
            if np.abs(c.sum()) == 0:
                c = np.diag(np.abs(x0))
            c = c * self.scaling
            det = np.linalg.det(c)
            while det <= 0:
                c += np.identity(d) * self.EPS
                det = np.linalg.det(c)
            covs = torch.as_tensor(c[None], device=self._Xd.device)
            invs = torch.as_tensor(np.linalg.inv(c)[None],
                                   device=self._Xd.device)
            dets = torch.as_tensor([det], device=self._Xd.device)
        else:
            comm = Comm.current()
            if comm.active:
                # each rank fits its row share, one all-gather
                # of (covs, inverses, dets); every row equals the 1-rank fit
                q, m = divmod(n, comm.world)
                r = comm.rank
                lo = r * q + min(r, m)
                hi = lo + q + (1 if r < m else 0)
                sizes = [q + (1 if s < m else 0) for s in range(comm.world)]
                nbr, _ = K.knn_rows(self._Xd, kk, lo, hi - lo)
                c, i, dt = K.local_cov_rows(self._Xd, self._wd, nbr, lo,
                                            self.scaling)
                packed = torch.cat([c.reshape(hi - lo, -1),
                                    i.reshape(hi - lo, -1),
                                    dt.view(-1, 1)], 1)
                allp = comm.all_gather_rows(packed, sizes)
                covs = allp[:, :d * d].reshape(n, d, d).contiguous()
                invs = allp[:, d * d:2 * d * d].reshape(n, d, d).contiguous()
                dets = allp[:, 2 * d * d].contiguous()
                nbr = comm.all_gather_rows(nbr.to(torch.int64), sizes).to(
                    torch.int32)
            else:
                nbr, _ = K.knn(self._Xd, kk)
                covs, invs, dets = K.local_cov(self._Xd, self._wd, nbr,
                                               self.scaling)
            self.nbr = nbr
        self._covs, self._invs, self._dets = covs, invs, dets
        self._cdf = K.resample_cdf(self._wd)

    # device-level API used by the batch sampler (engine.GenerationEngine)
    @property
    def device_fit(self):
        if getattr(self, "_covs", None) is None:
            return None
        return _LocalDeviceFit(self)

    @property
    def covs(self):
        return self._covs.cpu().numpy()

    @property
    def inv_covs(self):
        return self._invs.cpu().numpy()

    @property
    def determinants(self):
        return self._dets.cpu().numpy()

    @property
    def normalization(self):
        d = self._Xd.shape[1]
        return np.sqrt((2 * np.pi) ** d * self.determinants)

    @property
    def X_arr(self):
        return self._Xd.cpu().numpy()

    def pdf(self, x):
        single = isinstance(x, pd.Series)
        theta, _ = as_device_matrix(x, columns=_columns(self.X)
                                    if isinstance(x, (pd.Series, pd.DataFrame,
                                                      DeviceFrame)) else None)
        dens = torch.exp(self.logpdf_device(theta)).cpu().numpy()
        if single:
            return float(dens[0])
        return dens

    def logpdf_device(self, theta, parent=None):
        return K.local_logpdf(theta, self._Xd, self._wd, self._invs,
                              self._dets, self.kde_precision)

    def rvs_single(self):
        return self._draw(1, True)

    def rvs(self, size=None):
        if size is None:
            return self.rvs_single()
        return self._draw(size, False)

    def _draw(self, size, single):
        theta, _, _ = K.propose_local(self._Xd, self._cdf, self._covs,
                                      _draw_seed(), 0, 0, size)
        return _as_output(theta.cpu().numpy(), single, _columns(self.X))

    def svd_factors(self):
        """numpy's legacy ``multivariate_normal`` factor of every local
        covariance, A_n = sqrt(s)[:, None] * V with (U, s, V) = svd(C_n),
        as a device tensor [N, d, d] (the reference's draw,
        local_transition.py:141-145).  The production proposal kernel uses
        the Cholesky factor instead (the same distribution); this factor
        makes draws from given (u, z) equal the reference's."""
        _, s, v = np.linalg.svd(self.covs)
        return torch.as_tensor(np.sqrt(s)[..., :, None] * v,
                               device=self._Xd.device)

    def rvs_from(self, u, z):
        """Draws from the reference's random numbers: u[B] uniforms (the
        ``choice``) and z[B, d] normals (the ``multivariate_normal``), in
        the order rvs_single consumes them.  Returns (theta [B, d], idx)."""
        dev = self._Xd.device
        theta, idx, _ = K.resample_perturb_local(
            self._Xd, self._cdf, torch.as_tensor(np.asarray(u), device=dev),
            torch.as_tensor(np.asarray(z), device=dev), self.svd_factors())
        return theta, idx


class _LocalDeviceFit:
    """LocalTransition state as the generation engine consumes it:
    ``propose`` = rvs_single for a whole batch (choice by the weight CDF,
    then N(X_idx, C_idx), local_transition.py:141-145) with the prior-support
    flag, ``logpdf`` = the density pass (local_transition.py:103-110)."""

    def __init__(self, tr):
        self.X = tr._Xd
        self.w = tr._wd
        self.n = self.X.shape[0]
        self.cdf = tr._cdf
        self._covs, self._invs, self._dets = tr._covs, tr._invs, tr._dets
        self.kde_precision = tr.kde_precision

    def propose(self, lo, scale, seed, sid, offset, B):
        return K.propose_local(self.X, self.cdf, self._covs, seed, sid,
                               offset, B, lo, scale)

    def logpdf(self, theta):
        return K.local_logpdf(theta, self.X, self.w, self._invs, self._dets,
                              self.kde_precision)
