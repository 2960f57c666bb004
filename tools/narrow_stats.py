#!/usr/bin/env python3
"""Lane census of the per-vertex prefix pull (k_bu_narrow PFX, one lane per vertex at W = 1) on
an RMAT graph, host only (no GPU).

For sampled waves of 64 consecutive narrow active vertices (degree-relabelled ids, as the level-2
active list holds them) this counts the 4-entry steps each lane runs over its row prefix (ids <
H), with and without the early exit (every alive group covered), and the wave's step count (its
slowest lane): lane utilisation = mean steps / wave steps.

    python tools/narrow_stats.py --scale 26 --groups 16
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--groups", type=int, default=16)
    ap.add_argument("--group-size", type=int, default=16)
    ap.add_argument("--hub-bound", type=int, default=458752)
    ap.add_argument("--wide", type=int, default=128)
    ap.add_argument("--waves", type=int, default=400)
    ap.add_argument("--step", type=int, default=4)
    args = ap.parse_args()
    import msbfs
    t = time.time()
    g = msbfs.Graph.rmat(args.scale, 16, 1)
    n = g.n
    deg = np.diff(g.rowptr)
    order = np.argsort(-deg, kind="stable")
    rank = np.empty(n, np.int64)
    rank[order] = np.arange(n)
    print(f"graph n={n} nnz={g.nnz} {time.time() - t:.1f}s", flush=True)
    K = args.groups
    rng = np.random.default_rng(7)
    # visited bits after level 1 (ids = ranks): sources and their neighbours
    vis = np.zeros(n, np.uint64)
    for k in range(K):
        srcs = rng.choice(n, args.group_size, replace=False)  # ranks
        for s in srcs:
            vis[s] |= np.uint64(1) << np.uint64(k)
            o = order[s]
            nb = rank[g.col[g.rowptr[o]:g.rowptr[o + 1]]]
            vis[nb] |= np.uint64(1) << np.uint64(k)
    alive = np.uint64((1 << K) - 1) if K < 64 else np.uint64(~0 & ((1 << 64) - 1))
    H = args.hub_bound
    # narrow active vertices at level 2 (not done, 0 < degree <= wide), ascending rank
    dr = deg[order]
    act = np.nonzero((dr > 0) & (dr <= args.wide) & (vis != alive))[0]
    print(f"narrow active: {len(act)}", flush=True)
    C = args.step
    nwaves = len(act) // 64
    pick = rng.choice(nwaves, min(args.waves, nwaves), replace=False)
    tot_full = tot_exit = wave_full = wave_exit = 0
    plens = []
    for w in np.sort(pick):
        vs = act[w * 64:(w + 1) * 64]
        sf, se = [], []
        for v in vs:
            o = order[v]
            nb = np.sort(rank[g.col[g.rowptr[o]:g.rowptr[o + 1]]])
            pre = nb[nb < H]
            plens.append(len(pre))
            full = (len(pre) + C - 1) // C
            unv = ~vis[v] & alive
            acc = np.uint64(0)
            ex = full
            for s in range(full):
                for u in pre[s * C:(s + 1) * C]:
                    acc |= vis[u]
                if (acc & unv) == unv:
                    ex = s + 1
                    break
            sf.append(full)
            se.append(ex)
        tot_full += sum(sf)
        tot_exit += sum(se)
        wave_full += 64 * max(sf)
        wave_exit += 64 * max(se)
    pl = np.array(plens)
    print(f"prefix length: mean {pl.mean():.1f} median {np.median(pl):.0f} p90 "
          f"{np.percentile(pl, 90):.0f} max {pl.max()}")
    print(f"steps per lane: full {tot_full / len(pl):.2f}, with early exit {tot_exit / len(pl):.2f}")
    print(f"lane utilisation: full {tot_full / wave_full:.2f}, with early exit "
          f"{tot_exit / max(wave_exit, 1):.2f}")
    print(f"wave steps per vertex: full {wave_full / len(pl):.2f}, with early exit "
          f"{wave_exit / len(pl):.2f}")


if __name__ == "__main__":
    main()
