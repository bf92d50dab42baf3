"""Weighted statistics (API of pyabc/weighted_statistics.py:1-160).

``weighted_quantile`` (the epsilon hot path, :26-43) runs on the device radix
select; ``effective_sample_size`` (:73-83) on the device sums when given a
device tensor.  The remaining helpers are the reference's analysis utilities
(not on the per-generation path) and keep their numpy definitions.
"""
from functools import wraps

import numpy as np
import torch

from . import kernels as K


def _is_dev(x):
    return isinstance(x, torch.Tensor)


def weight_checked(function):
    @wraps(function)
    def function_with_checking(points, weights=None, **kwargs):
        if weights is not None:
            s = float(K.dsum(weights.double()).item()) if _is_dev(weights) \
                else np.asarray(weights).sum()
            if not np.isclose(s, 1):
                raise AssertionError(f"Weights not normalized: {s}.")
        return function(points, weights, **kwargs)
    return function_with_checking


def _to_dev(x):
    if _is_dev(x):
        return x.to("cuda", torch.float64).contiguous().view(-1)
    return torch.as_tensor(np.ascontiguousarray(np.asarray(x, dtype=np.float64)
                                                ).reshape(-1), device="cuda")


@weight_checked
def weighted_quantile(points, weights=None, alpha=0.5):
    """interp(alpha, cumsum(w) - w/2, sorted points) by the device select."""
    d = _to_dev(points)
    w = None if weights is None else _to_dev(weights)
    return float(K.weighted_quantile(d, w, alpha)[0].item())


@weight_checked
def weighted_median(points, weights):
    return weighted_quantile(points, weights, alpha=0.5)


@weight_checked
def weighted_mean(points, weights):
    return (np.asarray(points) * np.asarray(weights)).sum()


@weight_checked
def weighted_std(points, weights):
    points = np.asarray(points)
    weights = np.asarray(weights)
    m = weighted_mean(points, weights)
    return np.sqrt(((points - m) ** 2 * weights).sum())


def effective_sample_size(weights):
    if _is_dev(weights):
        w = weights.double().contiguous()
        s = float(K.dsum(w).item())
        s2 = float(K.dsum(w, squares=True).item())
        return s * s / s2
    weights = np.asarray(weights)
    return np.sum(weights) ** 2 / np.sum(weights ** 2)


def resample(points, weights, n):
    weights = np.array(weights)
    weights /= np.sum(weights)
    return np.random.choice(points, size=n, p=weights)


def resample_deterministic(points, weights, n, enforce_n=False):
    weights = np.array(weights)
    numbers_f = weights * (n / np.sum(weights))
    numbers = np.round(numbers_f)
    if enforce_n and np.sum(numbers) != n:
        order = np.argsort(numbers_f - numbers)
        while np.sum(numbers) < n:
            numbers[order[-1]] += 1
            order = order[:-1]
        while np.sum(numbers) > n:
            numbers[order[0]] -= 1
            order = order[1:]
    out = []
    for i, ni in enumerate(numbers):
        out.extend([points[i]] * int(ni))
    return out
