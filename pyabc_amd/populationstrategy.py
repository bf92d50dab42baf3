"""Population sizes (API of pyabc/populationstrategy.py:33-136, 361-392).
AdaptivePopulationSize is out of scope for this tier."""
import json
import logging

logger = logging.getLogger("Adaptation")


class PopulationStrategy:
    def __init__(self, nr_particles, *, nr_samples_per_parameter=1):
        self.nr_particles = nr_particles
        self.nr_samples_per_parameter = nr_samples_per_parameter

    def update(self, transitions, model_weights, t=None):
        pass

    def __call__(self, t=None):
        return self.nr_particles

    def get_config(self):
        return {"name": self.__class__.__name__,
                "nr_particles": self.nr_particles}

    def to_json(self):
        return json.dumps(self.get_config())


class ConstantPopulationSize(PopulationStrategy):
    pass


class ListPopulationSize(PopulationStrategy):
    def __init__(self, values, *, nr_samples_per_parameter=1):
        super().__init__(nr_particles=list(values)[0],
                         nr_samples_per_parameter=nr_samples_per_parameter)
        self.values = list(values)

    def __call__(self, t=None):
        return self.values[t] if t is not None and t >= 0 else self.values[0]

    def get_config(self):
        return {"name": self.__class__.__name__,
                "population_values": self.values}
