import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")
    config.addinivalue_line(
        "markers", "slow: long-running CPU test")


def load_golden(name):
    path = os.path.join(GOLDEN, name + ".npz")
    with np.load(path, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def golden_names(prefix):
    return sorted(f[:-4] for f in os.listdir(GOLDEN)
                  if f.startswith(prefix) and f.endswith(".npz"))


@pytest.fixture
def golden():
    return load_golden
