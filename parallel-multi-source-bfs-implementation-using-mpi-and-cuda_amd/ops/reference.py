"""Independent oracles for F(U) (tests only; not used by the compute path).

`bfs_F_numpy` is a plain level-synchronous BFS in numpy; `bfs_F_scipy` uses
scipy.sparse.csgraph shortest paths from a super-source joined to every valid source (distance
to the super-source minus one = multi-source BFS distance). Both implement the reference's
semantics (main.cu:40-89): out-of-range sources ignored, unreachable vertices not counted.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np


def bfs_dist_numpy(n: int, rowptr: np.ndarray, col: np.ndarray, sources: Sequence[int]) -> np.ndarray:
    dist = np.full(n, -1, dtype=np.int64)
    src = np.asarray([s for s in sources if 0 <= s < n], dtype=np.int64)
    if len(src) == 0:
        return dist
    src = np.unique(src)
    dist[src] = 0
    frontier = src
    level = 0
    deg = np.diff(rowptr)
    while len(frontier):
        starts = rowptr[frontier]
        counts = deg[frontier]
        if counts.sum() == 0:
            break
        idx = np.repeat(starts - np.cumsum(np.concatenate([[0], counts[:-1]])), counts) + np.arange(counts.sum())
        nb = col[idx]
        nb = np.unique(nb[dist[nb] < 0])
        level += 1
        dist[nb] = level
        frontier = nb
    return dist


def bfs_F_numpy(n: int, rowptr: np.ndarray, col: np.ndarray, sources: Sequence[int]) -> Tuple[int, int]:
    """Returns (F, traversed_edges) for one group."""
    d = bfs_dist_numpy(n, rowptr, col, sources)
    reached = d >= 0
    return int(d[reached].sum()), int(np.diff(rowptr)[reached].sum() // 2)


def bfs_F_scipy(n: int, rowptr: np.ndarray, col: np.ndarray, sources: Sequence[int]) -> int:
    import scipy.sparse as sp
    from scipy.sparse.csgraph import shortest_path

    src = sorted({int(s) for s in sources if 0 <= s < n})
    if not src:
        return 0
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    r = np.concatenate([rows, np.full(len(src), n)])
    c = np.concatenate([col.astype(np.int64), np.asarray(src)])
    A = sp.csr_matrix((np.ones(len(r)), (r, c)), shape=(n + 1, n + 1))
    d = shortest_path(A, method="D", directed=False, unweighted=True, indices=n)
    d = d[:n]
    fin = np.isfinite(d)
    return int((d[fin] - 1).sum())
