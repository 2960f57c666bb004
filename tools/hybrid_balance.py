#!/usr/bin/env python3
"""Does the group -> rank assignment change the hybrid mode's slowest phase C?

Phase C (levels >= 3 of a rank's own 64-group words) is the 8-rank floor
(profiles/hybrid_sim_rmat26.md: 3.1-4.8 ms per rank with the same code on every rank), and the
ranks differ only in which groups they hold. This tool re-runs the emulated hybrid job
(parallel/hybrid.py emulate_ranks) with the query groups permuted before the word split and
prints every rank's phase C for each ordering:

  orig     the groups in their input order (what bench.py runs)
  shuffle  random permutations
  snake    groups sorted by a lateness key, dealt to the ranks in snake order (balanced mix)
  cluster  the same sorted order, contiguous (late groups together)
  pair     sorted order, the last rank holding the 64 latest and the 64 earliest groups
  uneven   the cluster order with an uneven word split (--uneven, default 3,2,2,2,2,2,2,1 words
           for 8 ranks: fewer groups for the rank that holds the latest ones; it also receives
           less of the exchange, the earliest rank more)

Lateness key of a group = the smallest internal (degree-descending) id among its sources, i.e.
the degree rank of its best-connected source: a group whose every source has low degree reaches
the hubs one level later and keeps vertices open through levels 3-4.

    python tools/hybrid_balance.py --scale 26 --ranks 8
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def snake(order: np.ndarray, K: int, world: int, wbeg: np.ndarray) -> np.ndarray:
    """Deal `order` (sorted groups) to the ranks' word blocks in snake order."""
    slots = [list(range(64 * int(wbeg[r]), min(K, 64 * int(wbeg[r + 1])))) for r in range(world)]
    perm = np.empty(K, dtype=np.int64)
    r, d, fill = 0, 1, [0] * world
    for g in order:
        while fill[r] >= len(slots[r]):
            r = (r + d) % world
        perm[slots[r][fill[r]]] = g
        fill[r] += 1
        if (r == world - 1 and d == 1) or (r == 0 and d == -1):
            d = -d
        else:
            r += d
    return perm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--groups", type=int, default=1024)
    ap.add_argument("--group-size", type=int, default=16)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--orders", nargs="+", default=None, help="subset of the orderings to run")
    ap.add_argument("--uneven", default="3,2,2,2,2,2,2,1",
                    help="words per rank of the uneven split (sum = ceil(K/64))")
    args = ap.parse_args()

    import msbfs
    from msbfs.parallel import hybrid as H

    g = msbfs.DeviceGraph.rmat(args.scale, 16, 1, device=0, relabel=True)
    qs = msbfs.QuerySet.random(g.n, args.groups, args.group_size, 7)
    o2n = g.relabel_map()
    key = np.array([int(o2n[qs.group(k)].min()) for k in range(qs.K)], dtype=np.int64)
    K, N = qs.K, args.ranks
    wbeg = H.word_split(K, N)
    order = np.argsort(key, kind="stable")
    rng = np.random.default_rng(1)
    plans = {"orig": np.arange(K), "shuffle1": rng.permutation(K), "shuffle2": rng.permutation(K),
             "snake": snake(order, K, N, wbeg), "cluster": order,
             "pair": np.concatenate([order[64:K - 64], order[:64], order[K - 64:]]),
             "uneven": order}
    words = [int(x) for x in args.uneven.split(",")]
    wb_uneven = np.concatenate([[0], np.cumsum(words)]).astype(np.int32)
    with msbfs.Solver(g, "bitpar", max_groups=K) as s:
        ref = s.run(qs)
        H.emulate_ranks(s, qs, N)  # warm
        for name, perm in plans.items():
            if args.orders and name not in args.orders:
                continue
            sub = qs.subset(perm)
            best = None
            wb = wb_uneven if name == "uneven" else wbeg
            for _ in range(args.reps):
                tim = []
                F = H.emulate_ranks(s, sub, N, timings=tim, wbeg=wb)
                c = [x["phase_c_ms"] for x in tim]
                best = c if best is None else [min(a, b) for a, b in zip(best, c)]
            ok = bool(np.array_equal(F, ref.F[perm]))
            keys = [int(np.median(key[perm[64 * int(wb[r]):64 * int(wb[r + 1])]]))
                    if wb[r + 1] > wb[r] else -1 for r in range(N)]
            print(json.dumps({"order": name, "correct": ok, "phase_c_max": round(max(best), 3),
                              "phase_c_mean": round(float(np.mean(best)), 3),
                              "phase_c": [round(x, 3) for x in best],
                              "levels_c": [x["levels_c"] for x in tim],
                              "words": [int(wb[r + 1] - wb[r]) for r in range(N)],
                              "recv_MB": [round(x["recv_bytes"] / 2**20, 1) for x in tim],
                              "median_key": keys}), flush=True)
    g.close()


if __name__ == "__main__":
    main()
