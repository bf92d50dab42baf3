"""Import shim for the read-only reference checkout (THIS container only).

The reference (pyabc 0.10.1 under /root/reference) imports optional
dependencies that are absent here (redis, dask, ...).  They are unused on the
hot path, so they are replaced by inert module objects.  pandas>=2 rejects the
positional ``DataFrame.pivot`` call in ``pyabc/storage/history.py:307``; a
keyword-forwarding shim restores it.  Nothing here ships to the GPU box.
"""
import sys
import types

REF_ROOT = "/root/reference"


class _Any(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return type(name, (), {"__init__": lambda self, *a, **k: None})


def install():
    for name in ["redis", "distributed", "dask", "dask.array",
                 "dask.distributed", "dask.delayed", "memory_profiler",
                 "tlz", "feather", "bkcharts", "bokeh", "flask_bootstrap"]:
        if name not in sys.modules:
            try:
                __import__(name)
            except Exception:
                sys.modules[name] = _Any(name)
    sys.modules["memory_profiler"].profile = lambda f: f
    sys.modules["dask"].array = sys.modules["dask.array"]
    sys.modules["dask"].distributed = sys.modules["dask.distributed"]
    import pandas as _pd
    if not getattr(_pd.DataFrame.pivot, "_graft_shim", False):
        _p = _pd.DataFrame.pivot

        def _pivot(self, *a, **k):
            return _p(self, **{**dict(zip(["index", "columns", "values"], a)),
                               **k})
        _pivot._graft_shim = True
        _pd.DataFrame.pivot = _pivot
    sys.dont_write_bytecode = True
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)


def import_pyabc():
    install()
    import pyabc  # noqa: E402
    return pyabc
