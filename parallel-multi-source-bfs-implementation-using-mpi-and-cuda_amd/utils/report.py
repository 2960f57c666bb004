"""The reference's 7-line stdout report and its two phase timers.

Report (main.cu:403-414, `fixed << setprecision(9)` only affects the doubles):
    Graph: <path>
    Query: <path>
    Query number (k) with minimum F value: <minK+1>     (1-based, main.cu:409)
    Minimum F value: <minF>                             (-1 when K == 0)
    GPU # : <numGPU> GPU                                (echoes -gn, main.cu:411)
    Preprocessing time: <s> s                           (main.cu:235-298)
    Computation time: <s> s                             (main.cu:301-400)
"""
from __future__ import annotations

import json
import time
from contextlib import contextmanager
from typing import Dict


def format_report(graph: str, query: str, min_k: int, min_f: int, num_gpu: int,
                  preprocessing_time: float, computation_time: float) -> str:
    return (f"Graph: {graph}\n"
            f"Query: {query}\n"
            f"Query number (k) with minimum F value: {min_k + 1}\n"
            f"Minimum F value: {min_f}\n"
            f"GPU # : {num_gpu} GPU\n"
            f"Preprocessing time: {preprocessing_time:.9f} s\n"
            f"Computation time: {computation_time:.9f} s\n")


def parse_report(text: str) -> Dict[str, str]:
    out = {}
    for line in text.splitlines():
        if ":" in line:
            k, v = line.split(":", 1)
            out[k.strip()] = v.strip()
    return out


class PhaseTimer:
    """Wall-clock phase timers (same boundaries as the reference) + optional JSON export."""

    def __init__(self):
        self.phases: Dict[str, float] = {}

    @contextmanager
    def phase(self, name: str, sync=None):
        if sync:
            sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if sync:
                sync()
            self.phases[name] = self.phases.get(name, 0.0) + time.perf_counter() - t0

    def to_json(self) -> str:
        return json.dumps(self.phases)
