"""Samplers: the reference's sampler API plus the GPU batch sampler."""
from .base import Sample, SampleFactory, Sampler
from .singlecore import SingleCoreSampler
from .gpu import GPUBatchSampler, BatchSample, BatchSpec

__all__ = ["Sample", "SampleFactory", "Sampler", "SingleCoreSampler",
           "GPUBatchSampler", "BatchSample", "BatchSpec"]
