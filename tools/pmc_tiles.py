"""Per-tile PMC summary of one kernel from rocprofv3 --pmc passes
(tools/gpu_job.sh pmc= steps): averages every counter over the kernel's
dispatches in each pass directory, divides by the tiles one launch computes
and writes a JSON with the derived clock and cycles per tile per SIMD.

    python tools/pmc_tiles.py OUT.json KERNEL TILES "DESCRIPTION" DIR [DIR ...]

GRBM_GUI_ACTIVE is summed over the 8 XCDs (cycles per XCD = value / 8);
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES cycles (MI355X_MICROARCH.md constants table)."""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(d, kernel):
    per = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            disp = per[r["Dispatch_Id"]]
            disp[r["Counter_Name"]] = disp.get(r["Counter_Name"], 0.0) + float(
                r["Counter_Value"])
            disp["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per


def main():
    out_path, kernel, tiles, desc = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    acc = collections.defaultdict(list)
    passes = {}
    for d in sys.argv[5:]:
        per = load(d, kernel)
        if not per:
            continue
        avg = collections.defaultdict(float)
        for disp in per.values():
            for k, v in disp.items():
                avg[k] += v / len(per)
        passes[os.path.basename(d.rstrip("/"))] = {
            "dispatches": len(per), "ns": avg["_ns"],
            "GRBM_GUI_ACTIVE": avg.get("GRBM_GUI_ACTIVE")}
        for k, v in avg.items():
            acc[k].append(v)
    mean = {k: sum(v) / len(v) for k, v in acc.items()}
    per_tile = {k: v / tiles for k, v in mean.items()
                if k.startswith("SQ_") and k not in ("SQ_WAVES", "SQ_BUSY_CYCLES")}
    # d from the file name (bench.py kde_pmc: rNN_kde_pmc.json is d = 8,
    # rNN_kde_dDD_pmc.json is d = DD)
    md = re.search(r"_kde_d(\d+)_pmc\.json$", out_path)
    out = {"kernel": kernel, "description": desc, "d": int(md.group(1)) if md else 8,
           "tiles_per_launch": tiles,
           "passes": passes, "per_tile": per_tile,
           "units": "per tile; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in "
                    "quad-cycles per wave, SQ_VALU_MFMA_BUSY_CYCLES in cycles"}
    if "GRBM_GUI_ACTIVE" in mean and mean.get("_ns"):
        xcd_cycles = mean["GRBM_GUI_ACTIVE"] / 8
        simd_cycles = xcd_cycles * 1024
        out["derived"] = {
            "launch_ms": mean["_ns"] / 1e6,
            "clock_GHz": xcd_cycles / mean["_ns"],
            "cycles_per_tile_per_simd": simd_cycles / tiles,
        }
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            out["derived"]["mfma_pipe_busy_frac"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        if "SQ_VALU_MFMA_COEXEC_CYCLES" in mean and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            out["derived"]["coexec_frac_of_mfma_busy"] = (
                mean["SQ_VALU_MFMA_COEXEC_CYCLES"] / mean["SQ_VALU_MFMA_BUSY_CYCLES"])
        if "FETCH_SIZE" in mean:
            # KB; x2 on gfx950 for wide coalesced reads (MI355X_MICROARCH.md)
            out["derived"]["fetch_GB_per_launch_raw"] = mean["FETCH_SIZE"] * 1024 / 1e9
            out["derived"]["fetch_GB_per_launch_x2"] = mean["FETCH_SIZE"] * 2048 / 1e9
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
