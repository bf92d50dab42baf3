"""Summarise rocprofv3 PMC passes (tools/gpu_job.sh profile) into per-kernel HBM
traffic and VALU counters, and write profiles/kde_traffic.json for bench.py.

    python tools/pmc_traffic.py gpurun_out/prof_r01 r01

FETCH_SIZE / WRITE_SIZE are kilobytes (rocprofiler-sdk counter_defs.yaml).
On gfx950 FETCH_SIZE reports half the bytes of a wide streaming read
(MI355X_MICROARCH.md, HBM section), so HBM read bytes = 2 * 1024 * FETCH_SIZE;
WRITE_SIZE is exact for streaming stores.  Infinity-Cache hits are counted as
fabric traffic, so for kernels whose working set stays on die this is an
upper bound on HBM bytes.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(prof_dir, tag):
    fetch = load(os.path.join(prof_dir, "fetch", "run_counter_collection.csv"))
    write = load(os.path.join(prof_dir, "write", "run_counter_collection.csv"))
    valu = load(os.path.join(prof_dir, "valu", "run_counter_collection.csv"))
    stats = {}
    sp = os.path.join(prof_dir, "stats", "run_kernel_stats.csv")
    if os.path.exists(sp):
        for r in csv.DictReader(open(sp)):
            stats[r["Name"]] = (int(r["Calls"]), float(r["AverageNs"]))
    rows = []
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, {}).get("FETCH_SIZE", [])
        w = write.get(k, {}).get("WRITE_SIZE", [])
        v = valu.get(k, {})
        rb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        row = {"kernel": k, "launches": len(f) or len(w),
               "hbm_read_bytes_per_launch": rb,
               "hbm_write_bytes_per_launch": wb,
               "avg_ns": stats.get(k, (None, None))[1]}
        for c in ("SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE",
                  "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU"):
            if c in v:
                row[c] = sum(v[c]) / len(v[c])
        if row["avg_ns"] and "GRBM_GUI_ACTIVE" in row:
            # effective clock: GRBM_GUI_ACTIVE summed over 8 XCDs / wall
            row["eff_clock_ghz"] = row["GRBM_GUI_ACTIVE"] / 8 / row["avg_ns"]
        rows.append(row)
    out_csv = os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.csv")
    keys = sorted({k for r in rows for k in r}, key=lambda x: (x != "kernel", x))
    with open(out_csv, "w", newline="") as fh:
        wr = csv.DictWriter(fh, fieldnames=keys)
        wr.writeheader()
        for r in rows:
            wr.writerow(r)
    kde = [r for r in rows if r["kernel"].startswith(("kde_mfma_kernel",
                                                      "kde_mfma_lds2g_kernel"))] or \
        [r for r in rows if r["kernel"].startswith("kde_main")]
    if kde:
        r = kde[0]
        traffic = {
            "kernel": r["kernel"],
            "hbm_bytes_per_launch": (r["hbm_read_bytes_per_launch"] or 0)
            + (r["hbm_write_bytes_per_launch"] or 0),
            "hbm_read_bytes_per_launch": r["hbm_read_bytes_per_launch"],
            "hbm_write_bytes_per_launch": r["hbm_write_bytes_per_launch"],
            "eff_clock_ghz": r.get("eff_clock_ghz"),
            "source": f"profiles/{tag}_pmc_summary.csv (rocprofv3 --pmc "
                      f"FETCH_SIZE / WRITE_SIZE passes over bench.py, "
                      f"FETCH_SIZE x2 gfx950 correction)"}
        with open(os.path.join(ROOT, "profiles", "kde_traffic.json"), "w") as fh:
            json.dump(traffic, fh, indent=1)
        print(json.dumps(traffic))
    for r in rows:
        print(r["kernel"][:40], r["hbm_read_bytes_per_launch"],
              r["hbm_write_bytes_per_launch"], r.get("eff_clock_ghz"))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r01")
