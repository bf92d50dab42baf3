"""Run a tools/ script against another build of libabc_hip.so (same-box A/B
of compile-time variants): python tools/lib_ab.py LIB SCRIPT [ARGS ...]"""
import runpy
import sys

sys.path.insert(0, ".")
from pyabc_amd import _native  # noqa: E402

_native.LIB_PATH = sys.argv[1]
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
