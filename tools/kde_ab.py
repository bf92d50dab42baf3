"""Same-box A/B of two builds of libabc_hip.so (e.g. a compiler-flag
variant): python tools/kde_ab.py LIB d N [variant specs as kde_variants]"""
import sys

sys.path.insert(0, ".")
from pyabc_amd import _native  # noqa: E402

_native.LIB_PATH = sys.argv[1]
sys.argv = [sys.argv[0]] + sys.argv[2:]
import kde_variants  # noqa: E402

kde_variants.main()
