"""Per-generation kernel timeline of a rocprofv3 --kernel-trace run of
tools/bench_configs.py: kernel time between two launches of an anchor kernel
(C4: the LocalTransition density pass `lz_kernel`; C5: the MVN pass
`kde_mfma_lds2g_kernel`), by kernel, plus the device's idle gaps.

    python tools/gen_timeline.py STATS_DIR [ANCHOR_KERNEL]"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "lz_kernel"
    rows = []
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        rows += list(csv.DictReader(open(f)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0][:60]) for r in rows)
    ai = [i for i, e in enumerate(ev) if anchor in e[2]]
    for a, b in zip(ai, ai[1:]):
        busy = collections.defaultdict(float)
        idle = 0.0
        for i in range(a + 1, b + 1):
            s, e, n = ev[i]
            idle += max(0, s - max(x[1] for x in ev[a:i])) / 1e6
            if i < b:
                busy[n] += (e - s) / 1e6
        print(f"{anchor} {(ev[a][1] - ev[a][0]) / 1e6:.2f} ms; start-to-start "
              f"{(ev[b][0] - ev[a][0]) / 1e6:.2f} ms; kernels between "
              f"{sum(busy.values()):.2f} ms; device idle {idle:.2f} ms")
        for n, v in sorted(busy.items(), key=lambda x: -x[1])[:10]:
            print(f"   {v:7.3f} {n}")


if __name__ == "__main__":
    main()
