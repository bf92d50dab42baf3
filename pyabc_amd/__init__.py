"""pyabc_amd: MI355X-native per-generation ABC-SMC particle update.

Drop-in for the hot path of pyABC (reference chrhck/pyABC 0.10.1): the GPU
batch sampler, GPU-backed MultivariateNormalTransition / LocalTransition,
PNorm / AdaptivePNorm distances and the quantile epsilon, computing through
hand-written HIP kernels (``libabc_hip.so``, C-ABI in ``include/abc_hip.h``).
The public names mirror ``pyabc/__init__.py`` for the covered components.
"""
import logging
import os

__version__ = "0.1.0"

from .parameters import Parameter  # noqa: E402
from .random_variables import (RV, RVBase, RVDecorator,  # noqa: E402
                               LowerBoundDecorator, Distribution,
                               ModelPerturbationKernel)
from .distance import (Distance, NoDistance, SimpleFunctionDistance,  # noqa: E402
                       PNormDistance, AdaptivePNormDistance, to_distance,
                       median_absolute_deviation, mean_absolute_deviation,
                       standard_deviation, bias, root_mean_square_deviation,
                       median_absolute_deviation_to_observation,
                       mean_absolute_deviation_to_observation,
                       combined_median_absolute_deviation,
                       combined_mean_absolute_deviation,
                       standard_deviation_to_observation, span, mean, median,
                       SCALE_LIN, SCALE_LOG, StochasticKernel,
                       SimpleFunctionKernel, NormalKernel,
                       IndependentNormalKernel, IndependentLaplaceKernel,
                       BinomialKernel, PoissonKernel, NegativeBinomialKernel)
from .epsilon import (Epsilon, NoEpsilon, ConstantEpsilon,  # noqa: E402
                      ListEpsilon, QuantileEpsilon, MedianEpsilon)
from .acceptor import (Acceptor, SimpleFunctionAcceptor,  # noqa: E402
                       UniformAcceptor, AcceptorResult,
                       accept_use_current_time, accept_use_complete_history,
                       StochasticAcceptor, pdf_norm_from_kernel,
                       pdf_norm_max_found, ScaledPDFNorm)
from .temperature import (TemperatureBase, ListTemperature,  # noqa: E402
                          Temperature, TemperatureScheme,
                          AcceptanceRateScheme, ExpDecayFixedIterScheme,
                          ExpDecayFixedRatioScheme,
                          PolynomialDecayFixedIterScheme, DalyScheme,
                          FrielPettittScheme, EssScheme)
from .model import (Model, SimpleModel, ModelResult,  # noqa: E402
                    IntegratedModel, BatchModel, LinearGaussianModel,
                    GaussianMeanModel)
from .population import Particle, Population, ColumnarPopulation  # noqa: E402
from .populationstrategy import (PopulationStrategy,  # noqa: E402
                                 ConstantPopulationSize, ListPopulationSize,
                                 AdaptivePopulationSize)
from .sampler import (Sample, SampleFactory, Sampler,  # noqa: E402
                      SingleCoreSampler, GPUBatchSampler)
from .storage import History, create_sqlite_db_id  # noqa: E402
from .transition import (Transition, MultivariateNormalTransition,  # noqa: E402
                         LocalTransition, NotEnoughParticles,
                         silverman_rule_of_thumb, scott_rule_of_thumb)
from .smc import ABCSMC  # noqa: E402
from . import weighted_statistics  # noqa: E402
from . import storage  # noqa: E402

DefaultSampler = GPUBatchSampler

try:
    _lvl = os.environ["ABC_LOG_LEVEL"]
    logging.getLogger().setLevel(_lvl)
except KeyError:
    pass
