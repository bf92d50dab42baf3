"""Run the KDE issue-ceiling probe (tools/probes/issue_probe.hip) and print
ns per step per SIMD for each instruction mix at 1-3 waves per SIMD.

    python tools/issue_probe.py > profiles/r03_issue_probe.json"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIXES = {0: "d<=8 folded: 5 MFMA, 16 v_exp_f32, 23 v_add_f32",
         1: "d=20 split, bf16 pieces: 11 MFMA, 16 v_exp_f32, 40 v_add_f32",
         2: "d=20 split, f16 pieces: 9 MFMA, 16 v_exp_f32, 40 v_add_f32"}


def load():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probes", "libabc_probe.so"))
    lib.abc_probe_kde_mix.restype = ctypes.c_double
    lib.abc_probe_kde_mix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    return lib


def main():
    import torch
    torch.cuda.init()
    lib = load()
    out = []
    for v, desc in MIXES.items():
        for wps in (1, 2, 3):
            ns = lib.abc_probe_kde_mix(v, wps, 100000)
            out.append(dict(variant=v, mix=desc, waves_per_simd=wps,
                            ns_per_step_per_simd=ns))
            print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
