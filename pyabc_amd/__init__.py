"""pyabc_amd: MI355X-native per-generation ABC-SMC particle update.

Drop-in for pyABC's hot path (reference chrhck/pyABC 0.10.1): the GPU batch
sampler, GPU-backed MultivariateNormalTransition / LocalTransition,
PNorm / AdaptivePNorm distances and the quantile epsilon, all computing
through hand-written HIP kernels (``libabc_hip.so``, C-ABI in
``include/abc_hip.h``).
"""
__version__ = "0.1.0"
