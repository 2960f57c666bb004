#!/usr/bin/env python3
"""One-GPU solver time with the query groups in input order vs. sorted by lateness.

Lateness key of a group = the smallest degree-descending internal id among its sources (see
tools/hybrid_balance.py): late groups (every source of low degree) keep vertices open through the
late pull levels. Sorted ascending, the late groups share the last words of every row, so a
pull lane whose words are all covered (MSBFS_LANE_PRED builds) stops gathering while the lanes
of the late words continue. Prints ms per run (best of --reps) and the per-level ms; F is
checked against the input-order run.

    python tools/late_order.py --scale 26 --groups 1024
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--groups", type=int, default=1024)
    ap.add_argument("--group-size", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()

    import msbfs

    g = msbfs.DeviceGraph.rmat(args.scale, 16, 1, device=0, relabel=True)
    qs = msbfs.QuerySet.random(g.n, args.groups, args.group_size, 7)
    o2n = g.relabel_map()
    key = np.array([int(o2n[qs.group(k)].min()) for k in range(qs.K)], dtype=np.int64)
    order = np.argsort(key, kind="stable")
    plans = [("orig", np.arange(qs.K)), ("late_last", order)] * 2
    with msbfs.Solver(g, "bitpar", max_groups=qs.K) as s:
        s.prepare()
        ref = s.run(qs).F
        for name, perm in plans:
            q = qs.subset(perm)
            s.run(q)
            best, trace = 1e9, None
            for _ in range(args.reps):
                t = time.perf_counter()
                r = s.run(q)
                ms = (time.perf_counter() - t) * 1e3
                if ms < best:
                    best, trace = ms, s.level_trace()
            F = np.empty_like(r.F)
            F[perm] = r.F
            print(json.dumps({"order": name, "lib": os.environ.get("MSBFS_LIB", "in-tree"),
                              "correct": bool(np.array_equal(F, ref)), "ms": round(best, 3),
                              "level_ms": [round(t["ms"], 3) for t in trace]}), flush=True)
    g.close()


if __name__ == "__main__":
    main()
