#!/usr/bin/env python3
"""Per-kernel totals of the last solver run in a rocprofv3 rocpd database (the default output
format of rocprofv3 --kernel-trace on ROCm 7; tools/prof_summary.py reads the CSV format).

    python tools/prof_db.py gpurun_out/roadprof/road_results.db [marker-kernel]

The last run starts at the last dispatch whose name contains the marker (default k_init).
Prints the kernels' total time, dispatch count, mean time, VGPRs and scratch, then the span of
the run and the idle time between its dispatches.
"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_init"
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, vgpr_count, scratch_size from kernels "
                     "order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if marker in r[0]]
    sub = rows[starts[-1]:] if starts else rows
    tot = collections.defaultdict(lambda: [0, 0.0, 0, 0])
    for name, s, e, vg, sc in sub:
        k = name.split("(")[0].replace("void ", "").replace("msbfs::bp::", "")[:60]
        t = tot[k]
        t[0] += 1
        t[1] += (e - s) / 1e6
        t[2], t[3] = vg, sc
    span = (sub[-1][2] - sub[0][1]) / 1e6
    gap = sum(max(0, sub[i + 1][1] - sub[i][2]) for i in range(len(sub) - 1)) / 1e6
    print("| kernel | ms | dispatches | us/dispatch | VGPR | scratch |")
    print("|---|---:|---:|---:|---:|---:|")
    for k, (n, ms, vg, sc) in sorted(tot.items(), key=lambda x: -x[1][1]):
        if ms >= 0.01:
            print(f"| {k} | {ms:.2f} | {n} | {1e3 * ms / n:.1f} | {vg} | {sc} |")
    print(f"\nrun span {span:.2f} ms, idle between dispatches {gap:.2f} ms")


if __name__ == "__main__":
    main()
