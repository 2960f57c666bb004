#!/usr/bin/env python3
"""Census of the level-2 tail push (k_push_tail) on a degree-relabelled RMAT graph (host only).

Level 1 of K groups marks the sources' neighbours; the level-2 prefix pull covers row entries
with ids < H, and every level-1 frontier vertex u >= H pushes its groups to its neighbours
instead. This prints how many pushes that is (edges, and group bits = code slots), how many
distinct targets they hit, and how many of them land on big vertices (prefix longer than 1024
entries, the partial tiles) — the inputs for sizing a bucketed push.

    python tools/tail_push_stats.py --scale 24 --hub 114688
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--groups", type=int, default=1024)
    ap.add_argument("--group-size", type=int, default=16)
    ap.add_argument("--hub", type=int, default=458752, help="prefix bound H")
    args = ap.parse_args()
    import msbfs
    g = msbfs.Graph.rmat(args.scale, 16, 1)
    deg = np.diff(g.rowptr)
    order = np.lexsort((np.arange(g.n), -deg))
    new_id = np.empty(g.n, np.int64)
    new_id[order] = np.arange(g.n)
    qs = msbfs.QuerySet.random(g.n, args.groups, args.group_size, 7)
    src = np.unique(new_id[qs.ids[qs.ids >= 0]])
    # level-1 frontier and its group bits per vertex (counts only: bits = #groups adjacent)
    rp = g.rowptr
    ndeg = np.empty(g.n, np.int64)
    ndeg[new_id] = deg
    bits = np.zeros(g.n, np.int32)
    gid = np.repeat(np.arange(args.groups), np.diff(qs.off))
    for k in range(args.groups):
        s = new_id[qs.ids[qs.off[k]:qs.off[k + 1]]]
        nb = np.unique(np.concatenate([new_id[g.col[rp[o]:rp[o + 1]]] for o in order[s]]))
        bits[nb] += 1
    del gid
    f1 = np.nonzero(bits > 0)[0]
    f1 = f1[~np.isin(f1, src)]
    tail = f1[f1 >= args.hub]
    pushes = int(ndeg[tail].sum())
    slots = int((ndeg[tail] * np.minimum(bits[tail], 3)).sum())
    dense = int((ndeg[tail] * (bits[tail] > 3)).sum())
    # targets: neighbours of the tail pushers (new ids), and the share on big vertices
    old_tail = order[tail]
    tg = np.concatenate([new_id[g.col[rp[o]:rp[o + 1]]] for o in old_tail]) if len(tail) else \
        np.zeros(0, np.int64)
    # prefix length of a vertex = neighbours with id < H
    big_thresh = 1024
    uniq = np.unique(tg)
    pref = np.zeros(len(uniq), np.int64)
    for i, v in enumerate(uniq[: min(len(uniq), 200000)]):
        nb = new_id[g.col[rp[order[v]]:rp[order[v] + 1]]]
        pref[i] = int((nb < args.hub).sum())
    sample = min(len(uniq), 200000)
    big_frac_targets = float((pref[:sample] > big_thresh).mean()) if sample else 0.0
    cnt = np.bincount(np.searchsorted(uniq, tg), minlength=len(uniq))
    big_push_frac = float(cnt[:sample][pref[:sample] > big_thresh].sum() / max(1, cnt[:sample].sum()))
    print(json.dumps({"scale": args.scale, "H": args.hub, "frontier1": int(len(f1)),
                      "tail_pushers": int(len(tail)), "push_edges": pushes,
                      "push_code_slots": slots, "push_dense_edges": dense,
                      "distinct_targets": int(len(uniq)),
                      "big_target_frac(sampled)": round(big_frac_targets, 4),
                      "pushes_to_big_frac(sampled)": round(big_push_frac, 4)}))


if __name__ == "__main__":
    main()
