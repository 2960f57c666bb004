#!/usr/bin/env python3
"""Level-2 work census of the bit-parallel pull on an RMAT graph (host only, no GPU).

For the level-1 frontier X1 of K query groups (bits per vertex = groups whose sources are
adjacent), the level-2 pull gathers X1[u] for every edge (v, u) with u in the frontier. This
prints, by degree rank of u (the relabelled id) and by popcount of X1[u], how many such edge
endpoints there are and how many bytes a row gather / a sparse code of each width would move.

    python tools/level2_stats.py --scale 26 --groups 1024
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
    ap.add_argument("--groups", type=int, default=1024)
    ap.add_argument("--group-size", type=int, default=16)
    ap.add_argument("--qseed", type=int, default=7)
    ap.add_argument("--wide-rank", type=int, default=313845,
                    help="pullers below this rank use the hub-chunk kernel (0: skip the split)")
    ap.add_argument("--code-from", type=int, default=3000)
    args = ap.parse_args()
    import msbfs
    t = time.time()
    g = msbfs.Graph.rmat(args.scale, 16, 1)
    print(f"graph n={g.n} nnz={g.nnz} {time.time() - t:.1f}s", flush=True)
    deg = np.diff(g.rowptr)
    order = np.argsort(-deg, kind="stable")
    rank = np.empty(g.n, np.int64)
    rank[order] = np.arange(g.n)
    qs = msbfs.QuerySet.random(g.n, args.groups, args.group_size, args.qseed)
    # (u, group) pairs of the level-1 frontier
    us, gs = [], []
    for k in range(qs.K):
        for s in qs.group(k):
            nb = g.col[g.rowptr[s]:g.rowptr[s + 1]]
            us.append(nb)
            gs.append(np.full(len(nb), k, np.int32))
    u = np.concatenate(us)
    gg = np.concatenate(gs)
    src = np.zeros(g.n, bool)
    src[qs.ids] = True
    key = np.unique(u.astype(np.int64) * qs.K + gg)
    uu = key // qs.K
    pc = np.bincount(uu, minlength=g.n)
    # a source's own groups are visited at level 0: its row is not a level-1 frontier row
    pc[src] = 0
    infr = pc > 0
    print(f"level-1 frontier: {infr.sum()} vertices, {pc.sum()} (vertex, group) bits, "
          f"degree sum {deg[infr].sum()}")
    r = rank[infr]
    d = deg[infr].astype(np.int64)
    p = pc[infr]
    W = (qs.K + 63) // 64
    edges = d.sum()
    print(f"level-2 gathers (edge endpoints into the frontier): {edges:.4g}")
    bounds = [0, 1 << 6, 1 << 9, 1 << 11, 3000, 1 << 12, 1 << 13, 1 << 14, 18000, 1 << 15,
              1 << 16, 1 << 17, 1 << 18, 458752, 1 << 20, g.n]
    print("rank range | frontier ids | endpoints | mean bits | endpoints by bits "
          "(1 / 2-3 / 4-6 / 7-14 / 15-30 / >30)")
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        m = (r >= lo) & (r < hi)
        if not m.any():
            continue
        e = d[m]
        pb = p[m]
        cuts = [(1, 1), (2, 3), (4, 6), (7, 14), (15, 30), (31, 1 << 30)]
        parts = [e[(pb >= a) & (pb <= b)].sum() / 1e6 for a, b in cuts]
        print(f"[{lo:>8}, {hi:>9}) | {m.sum():>8} | {e.sum() / 1e6:8.1f}M | "
              f"{(pb * e).sum() / max(e.sum(), 1):6.1f} | " +
              " / ".join(f"{x:.1f}M" for x in parts))
    # bytes per scheme (gathers into u < H only: the prefix pull)
    for H in (458752,):
        m = r < H
        e, pb = d[m], p[m]
        dense = e.sum() * 8 * W
        print(f"H={H}: endpoints {e.sum() / 1e6:.1f}M, dense rows {dense / 1e9:.1f} GB")
        for slots, width in ((3, 4), (6, 8), (12, 16)):
            coded = pb <= slots
            b = (e[coded].sum() * width + e[~coded].sum() * 8 * W)
            print(f"  codes of {slots} slots ({width} B): coded endpoints "
                  f"{e[coded].sum() / 1e6:.1f}M, dense {e[~coded].sum() / 1e6:.1f}M, "
                  f"{b / 1e9:.1f} GB")
        lst = (e * np.minimum(2 * pb, 8 * W)).sum()
        print(f"  2-byte group lists: {lst / 1e9:.1f} GB")
    sd = -np.sort(-deg)
    print("first rank with degree < 16384:", int(np.searchsorted(-sd, -16384, side="left")))
    if args.wide_rank:
        # split the prefix-pull endpoints by the puller: wide (rank < wide_rank: hub chunks) or
        # narrow, and by what the gather reads (dense row: rank < code_from or > 3 bits; code)
        fr = np.flatnonzero(infr & (rank < 458752))
        cf = args.code_from
        tot = np.zeros((2, 2), np.int64)
        for i in range(0, len(fr), 4096):
            us = fr[i:i + 4096]
            lens = g.rowptr[us + 1] - g.rowptr[us]
            nb = np.concatenate([g.col[g.rowptr[x]:g.rowptr[x + 1]] for x in us])
            dense_u = (rank[us] < cf) | (pc[us] > 3)
            dn = np.repeat(dense_u, lens)
            wv = rank[nb] < args.wide_rank
            for a in (0, 1):
                for b in (0, 1):
                    tot[a, b] += int(((wv == bool(a)) & (dn == bool(b))).sum())
        print(f"pullers wide (rank < {args.wide_rank}): coded {tot[1, 0] / 1e6:.1f}M, dense "
              f"{tot[1, 1] / 1e6:.1f}M; narrow: coded {tot[0, 0] / 1e6:.1f}M, dense "
              f"{tot[0, 1] / 1e6:.1f}M (code_from {cf})")
        pl_w = pl_n = 0
        for i in range(0, g.n, 1 << 22):
            vs = np.arange(i, min(g.n, i + (1 << 22)))
            # prefix length = neighbours with rank < H
            for v0 in range(0, len(vs), 1 << 18):
                vv = vs[v0:v0 + (1 << 18)]
                lens = g.rowptr[vv + 1] - g.rowptr[vv]
                nb = g.col[g.rowptr[vv[0]]:g.rowptr[vv[-1] + 1]]
                hub = rank[nb] < 458752
                cs = np.r_[0, np.cumsum(hub, dtype=np.int64)]
                st = g.rowptr[vv] - g.rowptr[vv[0]]
                cnt = cs[st + lens] - cs[st]
                w = rank[vv] < args.wide_rank
                pl_w += int(cnt[w].sum())
                pl_n += int(cnt[~w].sum())
        print(f"prefix entries (neighbour rank < 458752): wide pullers {pl_w / 1e6:.1f}M, "
              f"narrow {pl_n / 1e6:.1f}M")


if __name__ == "__main__":
    main()
