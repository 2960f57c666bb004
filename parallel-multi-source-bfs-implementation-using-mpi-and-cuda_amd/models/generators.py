"""Graph and query generators (the reference ships none: SURVEY §2.1).

The native generators (host: csrc/src/gen_host.cpp, device: csrc/src/kernels/gen.hip) and
the vectorised numpy twins below evaluate the same counter-based RNG (splitmix64 finaliser,
csrc/include/msbfs/common.hpp), so a graph generated on the GPU is edge-for-edge identical to
the one written to a legacy .bin file on the host — tests pin that bit-exactly.

Graph500 RMAT: A=.57 B=.19 C=.19 D=.05, edge factor 16, vertex ids scrambled by a bijection.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _u64(x) -> np.ndarray:
    return np.asarray(x, dtype=np.uint64)


def mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = _u64(z) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _scalar_mix(x: int) -> int:
    return int(mix64(np.array([x & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64))[0])


def scramble_id(x: np.ndarray, scale: int, seed: int) -> np.ndarray:
    mask = np.uint64((1 << scale) - 1) if scale < 64 else M64
    k1 = np.uint64(_scalar_mix(seed ^ 0x51ED27) | 1)
    k2 = np.uint64(_scalar_mix(seed ^ 0xC0FFEE) | 1)
    a1 = np.uint64(_scalar_mix(seed ^ 0xA11CE))
    a2 = np.uint64(_scalar_mix(seed ^ 0xB0B))
    sh = np.uint64(scale // 2 + 1)
    with np.errstate(over="ignore"):
        x = (_u64(x) * k1 + a1) & mask
        x ^= x >> sh
        x = (x * k2 + a2) & mask
        x ^= x >> sh
        x = (x * k1 + a2) & mask
    return x


def _fx(p: float) -> int:
    s = p * 4294967296.0
    if s >= 4294967295.0:
        return 0xFFFFFFFF
    if s <= 0:
        return 0
    return int(s)


def rmat_edges_np(scale: int, edgefactor: int = 16, seed: int = 1, a: float = 0.57,
                  b: float = 0.19, c: float = 0.19, scramble: bool = True,
                  start: int = 0, count: int | None = None) -> Tuple[np.ndarray, np.ndarray]:
    """Edges [start, start+count) of the RMAT graph (numpy twin of common.hpp rmat_edge)."""
    n = 1 << scale
    m = n * edgefactor
    if count is None:
        count = m - start
    i = np.arange(start, start + count, dtype=np.uint64)
    tA, tAB, tABC = (np.uint64(_fx(a)), np.uint64(_fx(a + b)), np.uint64(_fx(a + b + c)))
    with np.errstate(over="ignore"):
        key = mix64(np.uint64(seed) ^ mix64(i + np.uint64(0x1234567)))
        u = np.zeros(count, dtype=np.uint64)
        v = np.zeros(count, dtype=np.uint64)
        for l in range(0, scale, 2):
            r = mix64(key + np.uint64(l))
            for h in range(2):
                if l + h >= scale:
                    break
                x = (r >> np.uint64(32 * h)) & np.uint64(0xFFFFFFFF)
                bu = (x >= tAB).astype(np.uint64)
                bv = (((x >= tA) & (x < tAB)) | (x >= tABC)).astype(np.uint64)
                u = (u << np.uint64(1)) | bu
                v = (v << np.uint64(1)) | bv
    if scramble:
        u = scramble_id(u, scale, seed)
        v = scramble_id(v, scale, seed)
    return u.astype(np.int32), v.astype(np.int32)


def uniform_edges_np(n: int, m: int, seed: int = 1) -> Tuple[np.ndarray, np.ndarray]:
    i = np.arange(m, dtype=np.uint64)
    with np.errstate(over="ignore"):
        r = mix64(np.uint64(seed) ^ mix64(i + np.uint64(0x9876543)))
        u = ((r & np.uint64(0xFFFFFFFF)) * np.uint64(n)) >> np.uint64(32)
        v = ((r >> np.uint64(32)) * np.uint64(n)) >> np.uint64(32)
    return u.astype(np.int32), v.astype(np.int32)


def query_groups_np(n: int, K: int, size: int, seed: int = 7):
    """K groups of `size` uniform vertex ids (twin of common.hpp query_vertex)."""
    k = np.repeat(np.arange(K, dtype=np.uint64), size)
    j = np.tile(np.arange(size, dtype=np.uint64), K)
    with np.errstate(over="ignore"):
        r = mix64(np.uint64(seed) ^ mix64((k << np.uint64(20)) ^ j ^ np.uint64(0xABCDEF)))
        ids = ((r >> np.uint64(32)) * np.uint64(n)) >> np.uint64(32)
    ids = ids.astype(np.int32).reshape(K, size) if K else np.zeros((0, size), np.int32)
    return [ids[i].copy() for i in range(K)]


def grid_edges_np(rows: int, cols: int, keep: float = 1.0, shortcuts: int = 0, seed: int = 1):
    """4-neighbour grid ("road-like", high diameter) — twin of gen_host.cpp gen_grid."""
    ids = np.arange(rows * cols, dtype=np.int64).reshape(rows, cols)
    thr = M64 if keep >= 1.0 else np.uint64(int(keep * 18446744073709551615.0))
    out_u, out_v = [], []
    # the native generator emits, per vertex id in row-major order, the right edge then the down edge
    right_ok = np.zeros((rows, cols), dtype=bool)
    down_ok = np.zeros((rows, cols), dtype=bool)
    with np.errstate(over="ignore"):
        hr = mix64(np.uint64(seed) ^ (np.uint64(2) * ids.astype(np.uint64).ravel()))
        hd = mix64(np.uint64(seed) ^ (np.uint64(2) * ids.astype(np.uint64).ravel() + np.uint64(1)))
    right_ok.ravel()[:] = hr <= thr
    down_ok.ravel()[:] = hd <= thr
    right_ok[:, -1] = False
    down_ok[-1, :] = False
    flat = ids.ravel()
    both = np.stack([right_ok.ravel(), down_ok.ravel()], axis=1)  # (n, 2) in emission order
    tgt = np.stack([flat + 1, flat + cols], axis=1)
    src = np.stack([flat, flat], axis=1)
    sel = both.ravel()
    u = src.ravel()[sel]
    v = tgt.ravel()[sel]
    if shortcuts:
        su, sv = uniform_edges_np(rows * cols, shortcuts, seed ^ 0x5107C075)
        u = np.concatenate([u, su])
        v = np.concatenate([v, sv])
    return u.astype(np.int32), v.astype(np.int32)
