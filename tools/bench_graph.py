#!/usr/bin/env python3
"""Secondary benchmarks (BASELINE.json configs other than the RMAT-26 headline).

    python tools/bench_graph.py --graph grid:ROWS:COLS:KEEP --groups K --group-size S --algo A
    python tools/bench_graph.py --graph rmat:SCALE:EF --groups K ...
    python tools/bench_graph.py --graph uniform:N:M ...

Prints one JSON line: time per run of all K groups, TEPS (Graph500 edge accounting), levels.
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
    ap.add_argument("--graph", default="grid:4096:4096:0.7")
    ap.add_argument("--groups", type=int, default=256)
    ap.add_argument("--group-size", type=int, default=16)
    ap.add_argument("--algo", default="bitpar")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--relabel", type=int, default=0)
    ap.add_argument("--verify", type=int, default=0)
    ap.add_argument("--alpha", type=float, default=0.0)
    ap.add_argument("--beta", type=float, default=0.0)
    ap.add_argument("--force-dir", type=int, default=0)
    args = ap.parse_args()
    import torch
    import msbfs

    kind, *f = args.graph.split(":")
    t0 = time.perf_counter()
    if kind == "grid":
        r, c = int(f[0]), int(f[1])
        keep = float(f[2]) if len(f) > 2 else 1.0
        hg = msbfs.Graph.grid(r, c, keep, int(f[3]) if len(f) > 3 else 0, 1)
        g = hg.to_device(0)
    elif kind == "rmat":
        g = msbfs.DeviceGraph.rmat(int(f[0]), int(f[1]) if len(f) > 1 else 16, 1, device=0)
    elif kind == "uniform":
        g = msbfs.DeviceGraph.uniform(int(f[0]), int(f[1]), 1, device=0)
    else:
        raise SystemExit(f"unknown graph {kind}")
    if args.relabel:
        g.relabel_by_degree()
    qs = msbfs.QuerySet.random(g.n, args.groups, args.group_size, 7)
    with msbfs.Solver(g, args.algo, max_groups=qs.K, alpha=args.alpha, beta=args.beta,
                      force_dir=args.force_dir) as s:
        r0 = s.run(qs, count_edges=True)
        torch.cuda.synchronize()
        prep = time.perf_counter() - t0
        if args.verify:
            with msbfs.Solver(g, "dist") as d:
                rv = d.run(qs.subset(range(args.verify)))
            assert np.array_equal(rv.F, r0.F[:args.verify]), "verify failed"
        t1 = time.perf_counter()
        for _ in range(args.steps):
            r = s.run(qs)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t1) / args.steps
    edges = int(r0.edges.sum())
    print(json.dumps({"graph": args.graph, "algo": args.algo, "n": g.n, "m": g.m, "K": qs.K,
                      "ms": dt * 1e3, "teps": edges / dt, "traversed_edges": edges,
                      "stats": r.stats, "prep_s": round(prep, 3),
                      "min_k": int(msbfs.argmin_first(r.F)) + 1}), flush=True)


if __name__ == "__main__":
    main()
