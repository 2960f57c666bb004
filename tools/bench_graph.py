#!/usr/bin/env python3
"""Secondary benchmarks (BASELINE.json configs other than the RMAT-26 headline).

    python tools/bench_graph.py --graph grid:ROWS:COLS:KEEP --groups K --group-size S --algo A
    python tools/bench_graph.py --graph rmat:SCALE:EF --groups K ...
    python tools/bench_graph.py --graph uniform:N:M ...
    torchrun --nproc-per-node N tools/bench_graph.py ...   (one rank per GPU, RCCL)

Several ranks split the K groups round robin (main.cu:304-307), each on its own copy of the graph
(generated in place, no broadcast), and reduce the answer with the packed 8-byte all-reduce(MIN);
the time is the slowest rank's. BASELINE config 4 (road graph on 4 GPUs):
`torchrun --nproc-per-node 4 tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 64`;
config 5 (RMAT-30, 256 groups on 8 GPUs): `... --graph rmat:30:16 --relabel 1 --groups 256`.

Prints one JSON line (rank 0): time per run of all K groups, whole-job TEPS (Graph500 edge
accounting), levels of the slowest rank's last run.
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
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default RCCL)")
    ap.add_argument("--trace-out", default="", help="write rank 0's per-level records (JSON)")
    args = ap.parse_args()
    import torch
    import msbfs
    from msbfs.parallel import distributed as D

    ctx = D.init_from_env(backend=args.backend, use_gpu=True)
    dev = ctx.device
    kind, *f = args.graph.split(":")
    t0 = time.perf_counter()
    if kind == "grid":
        r, c = int(f[0]), int(f[1])
        keep = float(f[2]) if len(f) > 2 else 1.0
        hg = msbfs.Graph.grid(r, c, keep, int(f[3]) if len(f) > 3 else 0, 1)
        g = hg.to_device(dev)
    elif kind == "rmat":
        g = msbfs.DeviceGraph.rmat(int(f[0]), int(f[1]) if len(f) > 1 else 16, 1, device=dev)
    elif kind == "uniform":
        g = msbfs.DeviceGraph.uniform(int(f[0]), int(f[1]), 1, device=dev)
    else:
        raise SystemExit(f"unknown graph {kind}")
    if args.relabel:
        try:
            g.relabel_by_degree()
        except msbfs.native.MsbfsError as e:
            print(f"bench_graph: relabel skipped: {e}", file=sys.stderr)
    qs = msbfs.QuerySet.random(g.n, args.groups, args.group_size, 7)
    idx = D.round_robin(qs.K, ctx.rank, ctx.world)
    local = qs.subset(idx)
    with msbfs.Solver(g, args.algo, max_groups=max(1, local.K), alpha=args.alpha,
                      beta=args.beta, force_dir=args.force_dir) as s:
        r0 = s.run(local, count_edges=True)
        torch.cuda.synchronize(dev)
        prep = time.perf_counter() - t0
        edges = int(D.allreduce_sum_i64(np.array([int(r0.edges.sum())], np.int64), ctx)[0])
        D.barrier(ctx)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        r = r0
        for _ in range(args.steps):
            r = s.run(local)
        torch.cuda.synchronize(dev)
        D.barrier(ctx)
        dt = D.allreduce_max((time.perf_counter() - t1) / max(1, args.steps), ctx)
        # (untimed: solver time only; with --steps 0 the answer comes from the counting pass)
        min_k, min_f = D.packed_argmin(r.F, idx, qs.K, ctx)
        if args.verify and local.K:  # (untimed) the counting pass and the last timed run
            nv = min(args.verify, local.K)
            with msbfs.Solver(g, "dist") as d:
                rv = d.run(local.subset(range(nv)))
            assert np.array_equal(rv.F, r0.F[:nv]), "verify failed (counting pass)"
            assert np.array_equal(rv.F, r.F[:nv]), "verify failed (timed run)"
        if args.trace_out and ctx.rank == 0:
            with open(args.trace_out, "w") as f:
                json.dump(s.level_trace(), f)
    if ctx.rank == 0:
        print(json.dumps({"graph": args.graph, "algo": args.algo, "n": g.n, "m": g.m,
                          "K": qs.K, "n_gpus": ctx.world, "ms": dt * 1e3, "teps": edges / dt if dt > 0 else 0.0,
                          "traversed_edges": edges, "stats": r.stats, "prep_s": round(prep, 3),
                          "min_k": int(min_k) + 1, "min_f": int(min_f)}), flush=True)
    D.shutdown(ctx)


if __name__ == "__main__":
    main()
