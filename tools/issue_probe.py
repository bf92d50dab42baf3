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
         2: "d=20 split, f16 pieces: 9 MFMA, 16 v_exp_f32, 40 v_add_f32",
         3: "d<=8 folded f16 (round 4): 4 MFMA, 16 v_exp_f32, 19 v_add_f32",
         4: "d=20 folded f16 (round 4): 9 MFMA, 16 v_exp_f32, 19 v_add_f32",
         5: "mix 3 + 2 ds_read_b128 per step",
         6: "mix 3 + 2 ds_read_b128 per step + barrier every 2 steps",
         7: "mix 3 + 2 ds_read_b128 + barrier + LDS-DMA refill every 2 steps",
         8: "mix 3 + 2 ds_read_b128 per step + barrier every 4 steps",
         9: "mix 3 + 2 ds_read_b128 + barrier + LDS-DMA refill every 4 steps",
         10: "mix 3 + 2 ds_read_b128 per step + barrier every 8 steps",
         11: "mix 3 + 2 ds_read_b128 + barrier + LDS-DMA refill every 8 steps",
         12: "d<=8 folded f16, PMC mix: 4 MFMA, 16 v_exp_f32, 22 v_add_f32",
         13: "d=20 folded f16, PMC mix: 9 MFMA, 16 v_exp_f32, 28 v_add_f32",
         14: "mix 13 + 5 ds_read_b128 per step",
         15: "mix 13 + 5 ds_read_b128 per step + barrier every 4 steps",
         16: "mix 13 + 5 ds_read_b128 + barrier + 18-KiB LDS-DMA refill every 4 steps",
         17: "mix 13 + 4 ds_read_b128 per step",
         18: "LocalTransition z form d=6 (lz_kernel): 3 MFMA, 2 v_exp_f32, 17 v_add_f32",
         19: "LocalTransition z form d=6: 3 MFMA, 2 v_exp_f32, 19 v_add_f32",
         20: "mix 13 as 16x16x32 f16: 4 tiles x (1 hi + 4 lo) = 20 MFMA, "
             "16 v_exp_f32, 28 v_add_f32 per 1024 pairs",
         21: "mix 12 as 16x16x32 f16: 4 tiles x (1 hi + 2 lo) = 12 MFMA, "
             "16 v_exp_f32, 22 v_add_f32 per 1024 pairs",
         22: "d<=8 folded f16, PMC mix without the MFMAs in VALU: 4 MFMA, "
             "16 v_exp_f32, 17 v_add_f32",
         23: "d<=8 folded f16: 4 MFMA, 16 v_exp_f32, 18 v_add_f32",
         24: "d=20 folded f16, PMC mix without the MFMAs in VALU: 9 MFMA, "
             "16 v_exp_f32, 18 v_add_f32"}


def parse():
    """--variants 13,14 --waves 2 (defaults: every mix, 1-4 waves)"""
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default=None)
    ap.add_argument("--waves", default="1,2,3,4")
    a = ap.parse_args()
    vs = [int(v) for v in a.variants.split(",")] if a.variants else list(MIXES)
    return vs, [int(w) for w in a.waves.split(",")]


def load():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probes", "libabc_probe.so"))
    lib.abc_probe_kde_mix.restype = ctypes.c_double
    lib.abc_probe_kde_mix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.abc_probe_last_clock_ghz.restype = ctypes.c_double
    lib.abc_probe_last_clock_ghz.argtypes = []
    return lib


def main():
    import torch
    torch.cuda.init()
    lib = load()
    variants, waves = parse()
    out = []
    for v in variants:
        desc = MIXES[v]
        for wps in waves:
            ns = lib.abc_probe_kde_mix(v, wps, 100000)
            ghz = lib.abc_probe_last_clock_ghz()
            out.append(dict(variant=v, mix=desc, waves_per_simd=wps,
                            ns_per_step_per_simd=ns,
                            clock_ghz=ghz if ghz > 0 else None))
            print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
