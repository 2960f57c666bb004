#!/usr/bin/env python3
"""How many neighbour rows does a level-L pull gather per vertex, and how much of a wave's time
do its lanes idle? (CPU model of the pull levels, no GPU.)

Degree-relabelled RMAT (rows sorted: hubs first), K groups of `size` random sources, exact
per-group BFS distances (scipy). At pull level L a vertex v is active when some alive group j
has not visited it (dist_j(v) >= L); it ORs its neighbours' rows (groups with dist <= L - 1) in
row order until every such group is covered, or its row ends. The model counts the rows
gathered (k), the steps of the kernels (a first step of c1 rows, then steps of cs rows), and for
lock-step waves of `vpw` consecutive list vertices the busy fraction = mean steps / max steps
(k_bu_full with W <= 2 words runs 64 vertices per wave, one lane each).

    python tools/pull_steps_sim.py --scale 20 --groups 128 --level 3
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--groups", type=int, default=128)
    ap.add_argument("--size", type=int, default=16)
    ap.add_argument("--first-group", type=int, default=0,
                    help="groups [first, first + groups) of a 1024-group query set")
    ap.add_argument("--level", type=int, default=3)
    ap.add_argument("--c1", type=int, default=1)
    ap.add_argument("--cs", type=int, default=4)
    ap.add_argument("--vpw", type=int, default=64)
    ap.add_argument("--wide", type=int, default=1024, help="wider rows go to the chunk kernels")
    ap.add_argument("--push-frac", type=float, default=0.0,
                    help="groups whose level L-1 frontier holds fewer than this fraction of the "
                         "vertices are pushed (top-down) instead: the pull does not wait for them")
    args = ap.parse_args()

    import scipy.sparse as sp

    import msbfs
    g = msbfs.Graph.rmat(args.scale, 16, 1)
    deg = g.degrees()
    # degree relabelling (descending degree, ties by id) and sorted rows, as the solver does
    order = np.lexsort((np.arange(g.n), -deg))
    new_id = np.empty(g.n, np.int64)
    new_id[order] = np.arange(g.n)
    src = np.repeat(np.arange(g.n), deg)
    A = sp.csr_matrix((np.ones(len(g.col), np.int8), (new_id[src], new_id[g.col])),
                      shape=(g.n, g.n))
    A.sort_indices()
    rowptr, col = A.indptr.astype(np.int64), A.indices.astype(np.int64)
    d = np.diff(rowptr)
    qs = msbfs.QuerySet.random(g.n, 1024, args.size, 7)
    K = args.groups
    W = (K + 63) // 64
    L = args.level
    push_edges = 0
    npush = 0
    vis = np.zeros((g.n, W), np.uint64)     # groups with dist <= L - 1
    unv = np.zeros((g.n, W), np.uint64)     # alive groups with dist >= L
    for j in range(K):
        gj = args.first_group + j
        srcs = new_id[qs.ids[qs.off[gj]:qs.off[gj + 1]]]
        seen = np.zeros(g.n, bool)
        seen[srcs] = True
        fr = seen.copy()
        for _ in range(L - 1):  # levels 1 .. L-1 (boolean frontier expansion)
            nxt = (A @ fr.astype(np.int8)) > 0
            fr = nxt & ~seen
            seen |= fr
        bit = np.uint64(1) << np.uint64(j % 64)
        if not fr.any():
            continue  # group dead before level L (its frontier is empty)
        vis[seen, j // 64] |= bit
        if fr.sum() < args.push_frac * g.n:  # a push group: its frontier pushes along its edges
            npush += 1
            push_edges += int(d[fr].sum())
            continue
        unv[~seen, j // 64] |= bit
    active = np.nonzero((unv != 0).any(axis=1) & (d > 0) & (d <= args.wide))[0]
    k = np.zeros(len(active), np.int64)
    acc = np.zeros((len(active), W), np.uint64)
    need = unv[active]
    open_ = np.ones(len(active), bool)
    pos = 0
    while open_.any():
        idx = np.nonzero(open_ & (d[active] > pos))[0]
        if len(idx) == 0:
            break
        acc[idx] |= vis[col[rowptr[active[idx]] + pos]]
        k[idx] = pos + 1
        cov = ((acc[idx] & need[idx]) == need[idx]).all(axis=1)
        open_[idx[cov]] = False
        open_[np.nonzero(open_ & (d[active] <= pos + 1))[0]] = False
        pos += 1
    steps = np.where(k <= args.c1, 1, 1 + (k - args.c1 + args.cs - 1) // args.cs)
    nw = len(active) // args.vpw
    ws = steps[:nw * args.vpw].reshape(nw, args.vpw)
    busy = float(ws.mean() / ws.max(axis=1).mean()) if nw else 1.0
    hist = np.bincount(np.minimum(k, 16))
    print(json.dumps({
        "scale": args.scale, "groups": K, "first_group": args.first_group, "level": L,
        "active": int(len(active)), "rows_mean": round(float(k.mean()), 3),
        "first_row_covers": round(float((k == 1).mean()), 4),
        "steps_mean": round(float(steps.mean()), 3),
        "wave_steps_mean": round(float(ws.max(axis=1).mean()), 3) if nw else 0,
        "lane_busy": round(busy, 3),
        "push_groups": npush, "push_edges": push_edges, "rows_total": int(k.sum()),
        "rows_hist_0_16": hist.tolist()}))


if __name__ == "__main__":
    main()
