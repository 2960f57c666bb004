"""TEPS accounting.

Per group: traversed edges = undirected input edges (duplicates and self-loops counted as in the
file) inside the connected components that contain >= 1 valid source = (sum of the degrees of the
reached vertices) / 2 — the Graph500 convention. Whole-node TEPS = sum over all K groups of
traversed edges / computation time (the reference's main.cu:301-400 phase).
"""
from __future__ import annotations

import numpy as np


def traversed_edges(rowptr: np.ndarray, dist: np.ndarray) -> int:
    deg = np.diff(rowptr)
    return int(deg[dist >= 0].sum() // 2)


def teps(total_edges: float, seconds: float) -> float:
    return float(total_edges) / seconds if seconds > 0 else 0.0


def fmt(x: float) -> str:
    for unit, s in (("T", 1e12), ("G", 1e9), ("M", 1e6), ("K", 1e3)):
        if x >= s:
            return f"{x / s:.3f} {unit}TEPS"
    return f"{x:.3f} TEPS"
