"""Models (API of pyabc/model.py:1-356) and the batch-model interface.

``Model.accept`` / ``summary_statistics`` are the per-particle path of the
reference; batch models (:mod:`pyabc_amd.batch_models`) are what the GPU
sampler evaluates B proposals at a time on the device.
"""
from .batch_models import BatchModel, LinearGaussianModel, GaussianMeanModel

__all__ = ["ModelResult", "Model", "SimpleModel", "IntegratedModel",
           "BatchModel", "LinearGaussianModel", "GaussianMeanModel"]


class ModelResult:
    def __init__(self, sum_stats=None, distance=None, accepted=None,
                 weight=1.0):
        self.sum_stats = sum_stats if sum_stats is not None else {}
        self.distance = distance
        self.accepted = accepted
        self.weight = weight


class Model:
    def __init__(self, name="model"):
        self.name = name

    def __repr__(self):
        return f"<{self.__class__.__name__} {self.name}>"

    def sample(self, pars):
        raise NotImplementedError()

    def summary_statistics(self, t, pars, sum_stats_calculator):
        raw = self.sample(pars)
        return ModelResult(sum_stats=sum_stats_calculator(raw))

    def distance(self, t, pars, sum_stats_calculator, distance_calculator,
                 x_0):
        res = self.summary_statistics(t, pars, sum_stats_calculator)
        res.distance = distance_calculator(res.sum_stats, x_0, t, pars)
        return res

    def accept(self, t, pars, sum_stats_calculator, distance_calculator,
               eps_calculator, acceptor, x_0):
        """Simulate, summarise, distance, accept (model.py:176-239)."""
        res = self.summary_statistics(t, pars, sum_stats_calculator)
        acc = acceptor(distance_function=distance_calculator,
                       eps=eps_calculator, x=res.sum_stats, x_0=x_0, t=t,
                       par=pars)
        res.distance = acc.distance
        res.accepted = acc.accept
        res.weight = acc.weight
        return res


class SimpleModel(Model):
    def __init__(self, sample_function, name=None):
        if name is None:
            name = sample_function.__name__
        super().__init__(name)
        self.sample_function = sample_function

    def sample(self, pars):
        return self.sample_function(pars)

    @staticmethod
    def assert_model(model_or_function):
        if isinstance(model_or_function, (Model, BatchModel)):
            return model_or_function
        return SimpleModel(model_or_function)


class IntegratedModel(Model):
    def integrated_simulate(self, pars, eps):
        raise NotImplementedError()

    def accept(self, t, pars, sum_stats_calculator, distance_calculator,
               eps_calculator, acceptor, x_0):
        return self.integrated_simulate(pars, eps_calculator(t))
