"""How many rows of the exact-inference run's KDE passes take the refine
(rows outside the folded pass's routing range) or the fp64 fixup: wraps
MultivariateNormalTransition.logpdf_device and prints M, refined and fixup
rows per call while tools/bench_configs.py's x1 config runs.

    python tools/x1_refine_count.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tools.bench_configs as bc  # noqa: E402
from pyabc_amd import transition as tr  # noqa: E402

_orig = tr.MultivariateNormalTransition.logpdf_device


def logpdf_device(self, theta, parent=None):
    out = _orig(self, theta, parent)
    pp = getattr(self._fit, "packed", None)
    if pp is not None and hasattr(pp, "refined_rows"):
        print(f"logpdf M={theta.shape[0]} refined={pp.refined_rows()} "
              f"fixup={pp.fixup_rows()}", flush=True)
    return out


tr.MultivariateNormalTransition.logpdf_device = logpdf_device
torch.cuda.set_device(0)
bc.x1()
