#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace and/or counter collection) as markdown.

    python tools/prof_summary.py gpurun_out/prof26 > profiles/rmat26_kernels.md

For a kernel trace it prints the per-kernel totals and the per-dispatch timeline of the LAST
solver run in the trace (the timed step); for counter collections it prints one row per
dispatch with every collected counter.
"""
import collections
import csv
import os
import sys


MAX_TIMELINE = 80


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "msbfs::bp::", "msbfs::dist::", "msbfs::(anonymous namespace)::",
              "msbfs::"):
        n = n.replace(p, "")
    return n[:48]


def trace_summary(d):
    p = os.path.join(d, "run_kernel_trace.csv")
    if not os.path.exists(p):
        return
    rows = load(p)
    tot = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        k = short(r["Kernel_Name"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        tot[k][0] += 1
        tot[k][1] += dur
    print(f"### Kernel totals ({d})\n")
    print("| kernel | calls | total ms |")
    print("|---|---|---|")
    for k, (c, ms) in sorted(tot.items(), key=lambda x: -x[1][1])[:25]:
        print(f"| `{k}` | {c} | {ms:.3f} |")
    # timeline of the last solver run: from the last init kernel on (PROF_START=<kernel>
    # PROF_NTH=<k>: from the k-th last dispatch of that kernel up to the next one, e.g. one
    # rank's hybrid phase C of tools/hybrid_sim.py: PROF_START=k_hybrid_setup PROF_NTH=8)
    marker = os.environ.get("PROF_START", "k_init")
    nth = int(os.environ.get("PROF_NTH", "1"))
    starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).startswith(marker)]
    if len(starts) >= nth:
        k = len(starts) - nth
        end = starts[k + 1] if k + 1 < len(starts) else len(rows)
        rows = rows[:end]
        starts = starts[:k + 1]
        run = rows[starts[-1]:]
        t0 = int(run[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in run)
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in run)
        print(f"\n### Timeline of the last solver run\n")
        print(f"{len(run)} dispatches, wall (first start to last end, under the profiler) "
              f"{(t1 - t0) / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms\n")
        print("| # | kernel | grid | VGPR | LDS B | ms |")
        print("|---|---|---|---|---|---|")
        shown = 0
        for i, r in enumerate(rows[starts[-1]:]):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            if dur < 0.01:
                continue
            shown += 1
            if shown > MAX_TIMELINE:
                print(f"| … | (timeline truncated at {MAX_TIMELINE} dispatches) | | | | |")
                break
            print(f"| {i} | `{short(r['Kernel_Name'])}` | {r.get('Grid_Size_X', r.get('Grid_Size', ''))} | "
                  f"{r.get('VGPR_Count', '')} | {r.get('LDS_Block_Size', '')} | {dur:.3f} |")
    print()


def counter_summary(d):
    p = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(p):
        return
    rows = load(p)
    agg = collections.OrderedDict()
    names = []
    for r in rows:
        key = r["Dispatch_Id"]
        e = agg.setdefault(key, {"kernel": short(r["Kernel_Name"]),
                                 "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
        if r["Counter_Name"] not in names:
            names.append(r["Counter_Name"])
    print(f"### Counters ({d}) — dispatches of the last run, > 0.2 ms\n")
    print("| kernel | ms | " + " | ".join(names) + " |")
    print("|---|---|" + "---|" * len(names))
    items = list(agg.values())
    for e in items[len(items) // 2:]:
        if e["ms"] < 0.2:
            continue
        vals = " | ".join(f"{e.get(n, 0):.4g}" for n in names)
        print(f"| `{e['kernel']}` | {e['ms']:.3f} | {vals} |")
    print()


if __name__ == "__main__":
    for d in sys.argv[1:]:
        trace_summary(d)
        counter_summary(d)
