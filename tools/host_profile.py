"""Host-side profile of the rank-slice generation loop: cProfile over
``bench.py --rank-slice R`` (default 8), the top functions by own time and
by cumulative time, to find the Python / host work that does not shrink
with R:

    python tools/host_profile.py [R] [steps]"""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

R = sys.argv[1] if len(sys.argv) > 1 else "8"
steps = sys.argv[2] if len(sys.argv) > 2 else "10"
sys.argv = ["bench.py", "--rank-slice", R, "--steps", steps, "--warmup", "3",
            "--no-cpu-baseline"]
import runpy  # noqa: E402

pr = cProfile.Profile()
pr.enable()
try:
    runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
finally:
    pr.disable()
    # the generation loop's own functions (imports filtered out): the
    # repo's modules and the numpy / torch calls they make
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        st = pstats.Stats(pr, stream=s).sort_stats(key)
        st.print_stats(r"pyabc_amd|bench\.py|linalg|torch/cuda|_native", 45)
        print(s.getvalue())
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(
            r"\{(method|built-in)", 25)
        print(s.getvalue())
