#!/usr/bin/env python3
"""Where a bench step's wall time goes outside the levels (1 GPU, bench.py's config).

For each of --steps runs of the round-robin step it records the Python wall time of
Solver.run, the device time between the C API's events around it (stats device_ms) and the sum
of the per-level host ms (level_trace), and prints the medians and the spread: wall - device =
host-side launch / copy / sync overhead, device - sum(levels) = work outside the level loop
(batch start, F read-back).

    python tools/step_split.py [--scale 26] [--groups 1024] [--steps 30]
"""
import argparse
import json
import os
import sys
import time

import numpy as np


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--groups", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import msbfs

    g = msbfs.DeviceGraph.rmat(args.scale, 16, 1, device=0)
    g.relabel_by_degree()
    qs = msbfs.QuerySet.random(g.n, args.groups, 16, 7)
    s = msbfs.Solver(g, "bitpar", max_groups=qs.K)
    s.prepare()
    sub = qs.subset(np.arange(qs.K))
    for _ in range(3):
        s.run(sub)
    torch.cuda.synchronize()
    wall, dev, lev, gap = [], [], [], []
    t_prev = time.perf_counter()
    for _ in range(args.steps):
        t0 = time.perf_counter()
        r = s.run(sub)
        t1 = time.perf_counter()
        gap.append((t0 - t_prev) * 1e3)
        t_prev = t1
        wall.append((t1 - t0) * 1e3)
        dev.append(float(r.stats.get("device_ms", 0.0)))
        lev.append(sum(t["ms"] for t in s.level_trace()))
    out = {k: {"median": round(float(np.median(v)), 3), "min": round(float(np.min(v)), 3),
               "max": round(float(np.max(v)), 3)}
           for k, v in (("wall_ms", wall), ("device_ms", dev), ("levels_ms", lev),
                        ("between_ms", gap))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
