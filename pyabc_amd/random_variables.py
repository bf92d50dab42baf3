"""Priors (API of pyabc/random_variables.py:1-538).

Marginals wrap scipy.stats exactly as the reference's ``RV`` does; this is
host-side configuration, evaluated per particle only on the per-particle
(closure) sampling path.  The batch GPU path needs the prior's support test
and density on the device: :meth:`Distribution.uniform_box` exposes a
product of ``RV('uniform', loc, scale)`` marginals as (names, lo, scale)
for the device kernels (prior support, random_variables.py:425-452).
"""
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


def _forward(method):
    """A decorator method that hands the call to the wrapped component."""
    def call(self, *args, **kwargs):
        return getattr(self.component, method)(*args, **kwargs)
    call.__name__ = method
    return call


class RVDecorator(RVBase):
    """Wraps another RV; every method not overridden is the component's
    (random_variables.py:185-229)."""

    def __init__(self, component):
        self.component = component

    rvs = _forward("rvs")
    pmf = _forward("pmf")
    pdf = _forward("pdf")
    cdf = _forward("cdf")

    def copy(self):
        return type(self)(self.component.copy())

    def decorator_repr(self):
        return "Decorator"

    def uniform_bounds(self):
        return None  # a decorated RV is never the plain uniform box

    def __repr__(self):
        return "[" + self.decorator_repr() + "]" + repr(self.component)


class LowerBoundDecorator(RVDecorator):
    """The component conditioned on X > lower_bound
    (random_variables.py:232-305): draws by rejection (None after
    MAX_TRIES), densities renormalised by the mass above the bound."""
    MAX_TRIES = 10000

    def __init__(self, component, lower_bound):
        below = component.cdf(lower_bound)
        if below == 1:
            raise Exception(
                "LowerBoundDecorator: Conditioning on a set of measure zero.")
        self.lower_bound = lower_bound
        super().__init__(component)

    def _mass_below(self):
        return self.component.cdf(self.lower_bound)

    def copy(self):
        return type(self)(self.component.copy(), self.lower_bound)

    def decorator_repr(self):
        return f"Lower: X > {self.lower_bound:2f}"

    def rvs(self, *args, **kwargs):
        tries = 0
        while tries < self.MAX_TRIES:
            draw = self.component.rvs()
            if draw > self.lower_bound or draw != draw:  # NaN is not <= lb
                return draw
            tries += 1
        return None

    def _renormalised(self, density, x):
        if x <= self.lower_bound:
            return 0.
        return density(x) / (1 - self._mass_below())

    def pdf(self, x, *args, **kwargs):
        return self._renormalised(self.component.pdf, x)

    def pmf(self, x, *args, **kwargs):
        return self._renormalised(self.component.pmf, x)

    def cdf(self, x, *args, **kwargs):
        if x <= self.lower_bound:
            return 0.
        below = self._mass_below()
        return (self.component.cdf(x) - below) / (1 - below)


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
        """Product of the marginal densities (pmf for discrete marginals)."""
        expected, got = sorted(self.keys()), sorted(x.keys())
        if got != expected:
            raise Exception("Random variable parameter mismatch. Expected: "
                            + str(expected) + " got " + str(got))
        if not self:
            return 1
        value = None
        for key, v in x.items():
            rv = self[key]
            try:
                f = rv.pdf(v)
            except AttributeError:  # discrete scipy marginals have no pdf
                f = rv.pmf(v)
            value = f if value is None else value * f
        return value

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
    """Model jump kernel (random_variables.py:455-538): stay in model m with
    probability p_stay, else move to one of the other models uniformly."""

    def __init__(self, nr_of_models, probability_to_stay=None):
        self.nr_of_models = nr_of_models
        if nr_of_models == 1:
            p = 1
        elif probability_to_stay is None:
            p = 1 / nr_of_models
        else:
            p = float(np.clip(probability_to_stay, 0, 1))
        self.probability_to_stay = p

    def _probabilities(self, m):
        k = self.nr_of_models
        probs = [(1 - self.probability_to_stay) / (k - 1)] * k
        probs[m] = self.probability_to_stay
        return probs

    def _get_discrete_rv(self, m):
        probs = self._probabilities(m)
        return RV("rv_discrete", values=(range(len(probs)), probs))

    def rvs(self, m):
        if m < 0 or m >= self.nr_of_models:
            raise Exception("m has to be between 0 and nr_of_models - 1")
        if self.nr_of_models == 1:
            return 0
        return self._get_discrete_rv(m).rvs()

    def pmf(self, n, m):
        if not (0 <= m < self.nr_of_models and 0 <= n <= self.nr_of_models):
            raise Exception("n and m have to be between 0 and nr_of_models - 1")
        if self.nr_of_models == 1:
            return int(n == m)
        return self._get_discrete_rv(m).pmf(n)
