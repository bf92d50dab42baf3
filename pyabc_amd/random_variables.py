"""Priors (API of pyabc/random_variables.py:1-538).

Marginals wrap scipy.stats exactly as the reference's ``RV`` does; this is
host-side configuration, evaluated per particle only on the per-particle
(closure) sampling path.  The batch GPU path needs the prior's support test
and density on the device: :meth:`Distribution.uniform_box` exposes a
product of ``RV('uniform', loc, scale)`` marginals as (names, lo, scale)
for the device kernels (prior support, random_variables.py:425-452).
"""
from functools import reduce

import numpy as np

from .parameters import Parameter, ParameterStructure


class RVBase:
    def copy(self):  # pragma: no cover
        raise NotImplementedError

    def rvs(self, *args, **kwargs):  # pragma: no cover
        raise NotImplementedError

    def pmf(self, x, *args, **kwargs):  # pragma: no cover
        raise NotImplementedError

    def pdf(self, x, *args, **kwargs):  # pragma: no cover
        raise NotImplementedError

    def cdf(self, x, *args, **kwargs):  # pragma: no cover
        raise NotImplementedError


class RV(RVBase):
    """A scipy.stats distribution by name, e.g. ``RV("uniform", 0, 5)``."""

    @classmethod
    def from_dictionary(cls, dictionary):
        return cls(dictionary["type"], *dictionary.get("args", []),
                   **dictionary.get("kwargs", {}))

    def __init__(self, name, *args, **kwargs):
        self.name = name
        self.args = args
        self.kwargs = kwargs
        self.distribution = None
        self.__setstate__(self.__getstate__())

    def __getattr__(self, item):
        if item in ("distribution", "name", "args", "kwargs"):
            raise AttributeError(item)
        return getattr(self.distribution, item)

    def __getstate__(self):
        return self.name, self.args, self.kwargs

    def __setstate__(self, state):
        import scipy.stats as st
        self.name, self.args, self.kwargs = state
        self.distribution = getattr(st, self.name)(*self.args, **self.kwargs)

    def copy(self):
        return self.__class__(self.name, *self.args, **self.kwargs)

    def rvs(self, *args, **kwargs):
        return self.distribution.rvs(*args, **kwargs)

    def pmf(self, x, *args, **kwargs):
        return self.distribution.pmf(x, *args, **kwargs)

    def pdf(self, x, *args, **kwargs):
        return self.distribution.pdf(x, *args, **kwargs)

    def cdf(self, x, *args, **kwargs):
        return self.distribution.cdf(x, *args, **kwargs)

    def uniform_bounds(self):
        """(loc, scale) when this is scipy's uniform, else None."""
        if self.name != "uniform":
            return None
        names = ("loc", "scale")
        vals = list(self.args) + [None] * (2 - len(self.args))
        loc = self.kwargs.get("loc", vals[0] if vals[0] is not None else 0.0)
        scale = self.kwargs.get("scale",
                                vals[1] if vals[1] is not None else 1.0)
        del names
        return float(loc), float(scale)

    def __repr__(self):
        return f"<RV(name={self.name}, args={self.args} kwargs={self.kwargs})>"


class RVDecorator(RVBase):
    def __init__(self, component):
        self.component = component

    def rvs(self, *args, **kwargs):
        return self.component.rvs(*args, **kwargs)

    def pmf(self, x, *args, **kwargs):
        return self.component.pmf(x, *args, **kwargs)

    def pdf(self, x, *args, **kwargs):
        return self.component.pdf(x, *args, **kwargs)

    def cdf(self, x, *args, **kwargs):
        return self.component.cdf(x, *args, **kwargs)

    def copy(self):
        return self.__class__(self.component.copy())

    def decorator_repr(self):
        return "Decorator"

    def uniform_bounds(self):
        return None

    def __repr__(self):
        return f"[{self.decorator_repr()}]" + repr(self.component)


class LowerBoundDecorator(RVDecorator):
    """Condition X > lower_bound by rejection (random_variables.py:232-305)."""
    MAX_TRIES = 10000

    def __init__(self, component, lower_bound):
        if component.cdf(lower_bound) == 1:
            raise Exception(
                "LowerBoundDecorator: Conditioning on a set of measure zero.")
        self.lower_bound = lower_bound
        super().__init__(component)

    def copy(self):
        return self.__class__(self.component.copy(), self.lower_bound)

    def decorator_repr(self):
        return "Lower: X > {:2f}".format(self.lower_bound)

    def rvs(self, *args, **kwargs):
        for _ in range(self.MAX_TRIES):
            s = self.component.rvs()
            if not s <= self.lower_bound:
                return s
        return None

    def pdf(self, x, *args, **kwargs):
        if x <= self.lower_bound:
            return 0.
        return self.component.pdf(x) / (1 - self.component.cdf(self.lower_bound))

    def pmf(self, x, *args, **kwargs):
        if x <= self.lower_bound:
            return 0.
        return self.component.pmf(x) / (1 - self.component.cdf(self.lower_bound))

    def cdf(self, x, *args, **kwargs):
        if x <= self.lower_bound:
            return 0.
        lm = self.component.cdf(self.lower_bound)
        return (self.component.cdf(x) - lm) / (1 - lm)


class Distribution(ParameterStructure):
    """Independent product of RVs keyed by parameter name."""

    def __repr__(self):
        return "<Distribution {}>".format(
            str(list(self.get_parameter_names()))[1:-1])

    @classmethod
    def from_dictionary_of_dictionaries(cls, dict_of_dicts):
        return cls({k: RV.from_dictionary(v) for k, v in dict_of_dicts.items()})

    def copy(self):
        return self.__class__(**{k: v.copy() for k, v in self.items()})

    def update_random_variables(self, **random_variables):
        self.update(random_variables)

    def get_parameter_names(self):
        return sorted(self.keys())

    def rvs(self):
        return Parameter(**{k: v.rvs() for k, v in self.items()})

    def pdf(self, x):
        if sorted(x.keys()) != sorted(self.keys()):
            raise Exception("Random variable parameter mismatch. Expected: "
                            + str(sorted(self.keys())) + " got "
                            + str(sorted(x.keys())))
        if len(self) == 0:
            return 1
        res = []
        for key, val in x.items():
            try:
                res.append(self[key].pdf(val))
            except AttributeError:
                res.append(self[key].pmf(val))
        return reduce(lambda s, t: s * t, res)

    def uniform_box(self):
        """(sorted names, lo[d], scale[d]) if every marginal is uniform."""
        names = self.get_parameter_names()
        lo, sc = [], []
        for n in names:
            rv = self[n]
            b = rv.uniform_bounds() if hasattr(rv, "uniform_bounds") else None
            if b is None:
                return None
            lo.append(b[0])
            sc.append(b[1])
        return names, np.array(lo), np.array(sc)


class ModelPerturbationKernel:
    """Model jump kernel (random_variables.py:455-538)."""

    def __init__(self, nr_of_models, probability_to_stay=None):
        self.nr_of_models = nr_of_models
        if nr_of_models == 1:
            self.probability_to_stay = 1
        elif probability_to_stay is None:
            self.probability_to_stay = 1 / nr_of_models
        else:
            self.probability_to_stay = min(max(probability_to_stay, 0), 1)

    def _get_discrete_rv(self, m):
        p_stay = self.probability_to_stay
        p_move = (1 - p_stay) / (self.nr_of_models - 1)
        probs = [p_stay if n == m else p_move for n in range(self.nr_of_models)]
        return RV("rv_discrete", values=(range(len(probs)), probs))

    def rvs(self, m):
        if not 0 <= m <= self.nr_of_models - 1:
            raise Exception("m has to be between 0 and nr_of_models - 1")
        if self.nr_of_models == 1:
            return 0
        return self._get_discrete_rv(m).rvs()

    def pmf(self, n, m):
        if not (0 <= n <= self.nr_of_models
                and 0 <= m <= self.nr_of_models - 1):
            raise Exception("n and m have to be between 0 and nr_of_models - 1")
        if self.nr_of_models == 1:
            return 1 if n == m else 0
        return self._get_discrete_rv(m).pmf(n)
