"""Batch simulators for the GPU sampler.

The reference evaluates one Python model call per proposal
(pyabc/model.py:92-123, 176-239).  The batch sampler instead asks a
:class:`BatchModel` for the statistics of B proposals at once, stat-major
``[S, B]`` on the device.  The two synthetic models below are the benchmark
models of BASELINE.json; each is one HIP kernel with
Philox4x32-10 noise.
"""
import numpy as np
import torch

from . import kernels as K


class BatchModel:
    """Interface: ``simulate(theta[B, d], seed, sid, offset) -> stats_T[S, B]``.

    ``keys`` are the summary-statistic names in x_0 order; ``name`` as in
    pyabc.Model.  ``offset`` is the global index of the first row, so that
    the noise of proposal i is the same however the batch is cut.
    """
    name = "batch_model"
    keys = ()

    @property
    def n_stats(self):
        return len(self.keys)

    def simulate(self, theta, seed, sid, offset):  # pragma: no cover
        raise NotImplementedError

    def observed(self):
        """x_0 as a dict in key order (optional)."""
        raise NotImplementedError


class LinearGaussianModel(BatchModel):
    """y = A theta + c + sigma * eps, eps ~ N(0, I_S)  (SURVEY C2/C5)."""

    def __init__(self, A, c=None, sigma=0.5, keys=None, name="linear_gaussian",
                 x0=None):
        A = np.asarray(A, dtype=np.float64)
        self.S, self.d = A.shape
        self.A_host = A
        self.c_host = None if c is None else np.asarray(c, dtype=np.float64)
        self.sigma = float(sigma)
        self.keys = tuple(keys) if keys is not None else tuple(
            f"y{k:03d}" for k in range(self.S))
        self.name = name
        self._x0 = x0
        self._dev = {}

    def _tensors(self):
        dev = torch.cuda.current_device()
        if dev not in self._dev:
            A = torch.as_tensor(self.A_host, device="cuda")
            c = None if self.c_host is None else torch.as_tensor(
                self.c_host, device="cuda")
            self._dev[dev] = (A, c)
        return self._dev[dev]

    def simulate(self, theta, seed, sid, offset):
        A, c = self._tensors()
        return K.sim_linear_gaussian(theta, A, c, self.sigma, seed, sid,
                                     offset)

    def simulate_distance(self, theta, seed, sid, offset, x0, fw, p, eps,
                          keep_stats=False):
        """simulate + p-norm distance + d <= eps in one pass (x0 / fw rows
        in the model's key order): (d, accept, guard), bit-identical to
        simulate() followed by the distance kernel; ``keep_stats``: the
        statistics simulate() returns as a fourth item, written by the same
        pass."""
        A, c = self._tensors()
        return K.sim_linear_gaussian_pnorm(theta, A, c, self.sigma, seed, sid,
                                           offset, x0, fw, p, eps,
                                           keep_stats=keep_stats)

    def simulate_host(self, theta, rng):
        """numpy reference of the same model (for CPU baselines)."""
        theta = np.atleast_2d(theta)
        y = theta @ self.A_host.T + self.sigma * rng.normal(
            size=(theta.shape[0], self.S))
        if self.c_host is not None:
            y = y + self.c_host
        return y

    def observed(self):
        return dict(zip(self.keys, self._x0))

    @staticmethod
    def benchmark(d, S=100, seed_A=42, seed_x0=7, sigma=0.5):
        """The synthetic inference problem of SURVEY 8(d): A =
        RandomState(42).randn(S,d)/sqrt(d), theta_true = linspace(-1,1,d),
        x_0 = A theta_true + sigma * RandomState(7).randn(S)."""
        A = np.random.RandomState(seed_A).randn(S, d) / np.sqrt(d)
        theta_true = np.linspace(-1, 1, d)
        x0 = A @ theta_true + sigma * np.random.RandomState(seed_x0).randn(S)
        m = LinearGaussianModel(A, None, sigma, x0=x0)
        m.theta_true = theta_true
        return m


class GaussianMeanModel(BatchModel):
    """Quickstart model: y = mean + 0.5 N(0,1)  (doc/examples/
    parameter_inference.ipynb, model cell)."""

    def __init__(self, sigma=0.5, key="data", name="model"):
        self.sigma = float(sigma)
        self.keys = (key,)
        self.name = name

    def simulate(self, theta, seed, sid, offset):
        out = K.sim_gaussian_mean(theta, self.sigma, seed, sid, offset)
        return out.view(1, -1)


def _per_particle_accept(model, t, pars, sum_stats_calculator,
                         distance_calculator, eps_calculator, acceptor, x_0):
    """One proposal through a batch model (closure sampling path): B = 1 on
    the device, then the acceptor, as Model.accept does (model.py:176-239)."""
    from .model import ModelResult
    res = model.summary_statistics(t, pars, sum_stats_calculator)
    acc = acceptor(distance_function=distance_calculator, eps=eps_calculator,
                   x=res.sum_stats, x_0=x_0, t=t, par=pars)
    res.distance = acc.distance
    res.accepted = acc.accept
    res.weight = acc.weight
    return res


def _per_particle_stats(model, t, pars, sum_stats_calculator):
    from .model import ModelResult
    names = sorted(pars.keys())
    theta = torch.as_tensor(np.array([[float(pars[k]) for k in names]]),
                            device="cuda")
    seed = int(np.random.randint(0, 2 ** 62, dtype=np.int64))
    stats = model.simulate(theta, seed, 0, 0)[:, 0].cpu().numpy()
    return ModelResult(sum_stats=sum_stats_calculator(
        dict(zip(model.keys, stats))))


BatchModel.summary_statistics = _per_particle_stats
BatchModel.accept = _per_particle_accept
