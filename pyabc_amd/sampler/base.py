"""Sampler base classes (API of pyabc/sampler/base.py:1-234)."""
from abc import ABC, ABCMeta, abstractmethod

import numpy as np

from ..population import Population


class Sample:
    """Particles gathered while sampling a generation (base.py:8-116)."""

    def __init__(self, record_rejected=False, ok=True):
        self._particles = []
        self.record_rejected = record_rejected
        self.ok = ok

    @property
    def all_sum_stats(self):
        out = []
        for p in self._particles:
            out.extend(p.accepted_sum_stats)
            out.extend(p.rejected_sum_stats)
        return out

    def first_m_sum_stats(self, m):
        # linear-time concatenation (the reference's sum(lists, []) is O(n^2))
        m = min(len(self._particles), m)
        out = []
        for p in self._particles[:m]:
            out.extend(p.accepted_sum_stats)
            out.extend(p.rejected_sum_stats)
        return out

    def first_m_particles(self, m):
        m = min(len(self._particles), m)
        return self._particles[:m]

    @property
    def _accepted_particles(self):
        return [p for p in self._particles if p.accepted]

    def append(self, particle):
        if particle.accepted or self.record_rejected:
            self._particles.append(particle)

    def __add__(self, other):
        s = Sample(self.record_rejected)
        s._particles = self._particles + other._particles
        return s

    @property
    def n_accepted(self):
        return len(self._accepted_particles)

    def get_accepted_population(self):
        return Population(self._accepted_particles)


class SampleFactory:
    def __init__(self, record_rejected=False):
        self.record_rejected = record_rejected

    def __call__(self):
        return Sample(self.record_rejected)


def wrap_sample(f):
    """Checks the sampler output (base.py:144-157)."""
    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False):
        sample = f(self, n, simulate_one, max_eval, all_accepted)
        if sample.n_accepted != n and sample.ok:
            raise AssertionError(
                f"Expected {n} but got {sample.n_accepted} acceptances.")
        return sample
    return sample_until_n_accepted


class SamplerMeta(ABCMeta):
    def __init__(cls, name, bases, attrs):
        ABCMeta.__init__(cls, name, bases, attrs)
        cls.sample_until_n_accepted = wrap_sample(cls.sample_until_n_accepted)


class Sampler(ABC, metaclass=SamplerMeta):
    def __init__(self):
        self.nr_evaluations_ = 0
        self.sample_factory = SampleFactory(record_rejected=False)

    def _create_empty_sample(self):
        return self.sample_factory()

    @abstractmethod
    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False):
        """Run simulate_one until n particles are accepted."""
