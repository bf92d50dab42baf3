"""Per-tile instruction counts of the MFMA KDE pass from rocprofv3 PMC passes.

    python tools/kde_pmc.py gpurun_out/r02a r02 [N M d]

Reads the ``pmcA`` / ``pmcB`` (and optional ``pmcC``) counter collections of
tools/gpu_job.sh profile (bench.py under ``rocprofv3 --pmc``), averages every
counter over the ``kde_mfma_kernel`` dispatches, divides by the 32x32 tiles
one launch computes (Mpad/32 * npad/32) and writes
``profiles/<tag>_kde_pmc.json``.  bench.py prices its live launch with these
per-tile counts (the issue ceiling):

    cycles per tile per SIMD = max(4 * VALU_plain + 8 * TRANS + 8 * MFMA,
                                   32 * MFMA)

with the MI355X_MICROARCH.md per-instruction SIMD issue costs (plain or
packed fp32 VALU 4 cycles per wave64 instruction -- the round-1 probe's
2.41 for v_fma_f32 timed SLP-packed pairs --, transcendental 8, an MFMA holding vector
issue for 8 of its 32 matrix-pipe cycles).  SQ_INSTS_VALU counts the MFMAs
too (round 6: the issue probe's own mix of 4 MFMA + 16 exp + 22 adds per
step reads 42.0 under --pmc), so VALU_plain = VALU - TRANS - MFMA; rounds
2-5 took VALU - TRANS and charged every MFMA twice.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


HEADLINE_KERNELS = ("kde_mfma_kernel", "kde_mfma_lds2g_kernel")


def load(path, kernel=HEADLINE_KERNELS):
    per = collections.defaultdict(dict)
    if not os.path.exists(path):
        return per
    names = (kernel,) if isinstance(kernel, str) else kernel
    for r in csv.DictReader(open(path)):
        if not any(k in r["Kernel_Name"] for k in names):
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        per[r["Dispatch_Id"]]["_ns"] = (int(r["End_Timestamp"])
                                        - int(r["Start_Timestamp"]))
    return per


def main(prof_dir, tag, N=1_000_000, M=1_000_000, d=8):
    from pyabc_amd import _native as nat
    lib = nat.lib()
    rp = lib.abc_kde_row_pad()
    npad = -(-N // rp) * rp
    mpad = lib.abc_kde_mfma_new_rows(M, d)
    tiles = (mpad // 32) * (npad // 32)
    counters = collections.defaultdict(list)
    for p in ("pmcA", "pmcB", "pmcC"):
        for disp in load(os.path.join(prof_dir, p,
                                      "run_counter_collection.csv")).values():
            for k, v in disp.items():
                counters[k].append(v)
    avg = {k: sum(v) / len(v) for k, v in counters.items()}
    per_tile = {k: v / tiles for k, v in avg.items()
                if k.startswith("SQ_INSTS") or k == "SQ_VALU_MFMA_BUSY_CYCLES"}
    valu = per_tile["SQ_INSTS_VALU"]
    trans = per_tile.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
    mfma = per_tile["SQ_INSTS_MFMA"]
    issue = 4 * (valu - trans - mfma) + 8 * trans + 8 * mfma
    cyc = max(issue, 32 * mfma)
    out = {
        "source": f"rocprofv3 --pmc passes over bench.py ({prof_dir}), "
                  f"MFMA KDE pass (kde_mfma_kernel / kde_mfma_lds2g_kernel), N={N} M={M} d={d}",
        "N": N, "M": M, "d": d, "npad": npad, "mpad": mpad,
        "tiles_per_launch": tiles,
        "counters_per_launch": avg,
        "per_tile": per_tile,
        "issue_cycles_per_tile": issue,
        "mfma_pipe_cycles_per_tile": 32 * mfma,
        "ceiling_cycles_per_tile": cyc,
        "cost_model": "plain VALU 4, TRANS 8, MFMA issue 8 / pipe 32 SIMD "
                      "cycles per wave64 instruction (MI355X_MICROARCH.md); "
                      "plain VALU = SQ_INSTS_VALU - TRANS - MFMA (the "
                      "counter includes the MFMAs)",
        "other_valu_per_tile": valu - trans - mfma,
    }
    if "GRBM_GUI_ACTIVE" in avg and "_ns" in avg:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs
        out["eff_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / avg["_ns"]
        sim_cycles = avg["GRBM_GUI_ACTIVE"] / 8 * 1024
        out["measured_cycles_per_tile"] = sim_cycles / tiles
        out["mfma_busy_frac"] = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / sim_cycles
        if "SQ_VALU_MFMA_COEXEC_CYCLES" in avg:
            out["coexec_frac"] = avg["SQ_VALU_MFMA_COEXEC_CYCLES"] / sim_cycles
    path = os.path.join(ROOT, "profiles", f"{tag}_kde_pmc.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], *(int(x) for x in a[2:]))
