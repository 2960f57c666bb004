"""Multi-source BFS operators: F(U_k) for every query group.

F(U) = sum over vertices v reachable from U of dist(U, v) (reference GPUMultiSourceBFS +
ComputeFofU, main.cu:40-89). Sources outside [0, n) are ignored (main.cu:49); unreachable
vertices contribute nothing (main.cu:84-85).

Algorithms (all give identical F — it is an exact integer sum):
  bitpar  — 64*W groups per pass, direction-optimising, per-group sums on chip (default, K > 1)
  dist    — per-group distance array, direction-optimising (default for K == 1)
  topdown — per-group, top-down only (queue + load-balanced edge expansion)
  sweep   — the reference algorithm (thread per vertex, full sweep per level), on-device sum
  cpu     — host threads (query-parallel), the "serial CPU BFS" config and oracle
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional, Union

import numpy as np

from . import native
from ..models.graph import DeviceGraph, Graph
from ..models.queries import QuerySet


@dataclass
class BfsResult:
    F: np.ndarray                      # int64[K]
    edges: Optional[np.ndarray] = None  # int64[K], Graph500 traversed edges per group (if asked)
    stats: dict = field(default_factory=dict)


class Solver:
    """Reusable device workspace for one graph + algorithm (allocated once, like the reference's
    one-time cudaMalloc of the distance array main.cu:294-295, but for all algorithms)."""

    def __init__(self, graph: DeviceGraph, algo: str = "auto", max_groups: int = 1024,
                 alpha: float = 0.0, beta: float = 0.0, wide_degree: int = 0,
                 force_dir: int = 0, max_words: int = 0, tuning=None):
        """tuning: algorithm tuning keys of the bit-parallel solver, a dict {"gamma2": 0.5, ...}
        or a "key=value,..." string (see msbfs_solver_tune in csrc/include/msbfs/msbfs.h);
        unknown keys raise MsbfsError."""
        if algo not in native.ALGOS or algo == "cpu":
            raise ValueError(f"unknown device algorithm {algo!r}")
        self.graph = graph
        self.algo = algo
        h = C.c_void_p()
        native.check(native.lib().msbfs_solver_create(graph.handle, native.ALGOS[algo],
                                                      max(1, int(max_groups)), C.byref(h)))
        self._h = h
        if alpha or beta or wide_degree or force_dir or max_words:
            o = native.Options(alpha, beta, wide_degree, force_dir, max_words)
            native.check(native.lib().msbfs_solver_set_options(self._h, C.byref(o)))
        if tuning:
            self.tune(tuning)

    def prepare(self, stream: Optional[int] = None) -> None:
        """Build the graph-derived tables and worst-case scratch now, not in the first run."""
        native.check(native.lib().msbfs_solver_prepare(self._h, C.c_void_p(stream) if stream
                                                       else None))

    def prepare_hybrid(self, part: int, nparts: int, stream: Optional[int] = None) -> None:
        """prepare() for the hybrid phase A of rank `part` of `nparts` (its own vertices)."""
        native.check(native.lib().msbfs_solver_prepare_hybrid(
            self._h, int(part), int(nparts), C.c_void_p(stream) if stream else None))

    def tune(self, tuning) -> None:
        spec = tuning if isinstance(tuning, str) else ",".join(
            f"{k}={v}" for k, v in dict(tuning).items())
        native.check(native.lib().msbfs_solver_tune(self._h, spec.encode()))

    def run(self, queries: QuerySet, count_edges: bool = False, stream: Optional[int] = None
            ) -> BfsResult:
        K = queries.K
        F = np.zeros(K, dtype=np.int64)
        E = np.zeros(K, dtype=np.int64) if count_edges else None
        st = native.Stats()
        if K:
            native.check(native.lib().msbfs_solver_run(
                self._h, K, native.ptr(queries.off, C.c_int64), native.ptr(queries.ids, C.c_int32),
                native.ptr(F, C.c_int64), native.ptr(E, C.c_int64) if E is not None else None,
                C.byref(st), C.c_void_p(stream) if stream else None))
        return BfsResult(F, None if E is None else E // 2, st.as_dict())

    def level_trace(self) -> list:
        """Per-level records of the last run / hybrid phase (bit-parallel solver): batch, level,
        dir ('T' push / 'B' pull), frontier size nf and degree sum ef entering the level, newly
        visited vertices nf_next, active (bottom-up) or touched (top-down) vertices, host ms."""
        L = native.lib()
        n = int(L.msbfs_solver_levels(self._h, None, 0))
        if n <= 0:
            return []
        buf = (native.Level * n)()
        L.msbfs_solver_levels(self._h, buf, n)
        return [r.as_dict() for r in buf]

    # ---- hybrid multi-GPU mode (parallel/hybrid.py drives these) ----
    def hybrid_max_groups(self) -> int:
        return int(native.lib().msbfs_solver_hybrid_max_groups(self._h))

    def hybrid_phase_a(self, queries: QuerySet, part: int, nparts: int, n_eff: int,
                       count_l1: bool, wbeg: np.ndarray, send_ptr: int,
                       stream: Optional[int] = None, coded: bool = False):
        """Levels 1-2 of all groups, level-2 pulls only for the vertices v = part + i*nparts
        below n_eff; packs their visited words into the device buffer at send_ptr (destination-
        major). Returns (out[2K+3], stats). coded: the send buffer gets one zero-word coded
        segment per destination instead (hybrid.encode_np), stats["coded_len"] their lengths."""
        K = queries.K
        wbeg = np.ascontiguousarray(wbeg, dtype=np.int32)
        out = np.zeros(2 * K + 3, dtype=np.int64)
        st = native.Stats()
        args = (self._h, K, native.ptr(queries.off, C.c_int64), native.ptr(queries.ids, C.c_int32),
                int(part), int(nparts), int(n_eff), int(bool(count_l1)),
                native.ptr(wbeg, C.c_int32), C.c_void_p(send_ptr), native.ptr(out, C.c_int64))
        strm = C.c_void_p(stream) if stream else None
        if coded:
            lens = np.zeros(int(nparts), dtype=np.int64)
            native.check(native.lib().msbfs_solver_hybrid_phase_a_coded(
                *args, native.ptr(lens, C.c_int64), C.byref(st), strm))
            d = st.as_dict()
            d["coded_len"] = lens
            return out, d
        native.check(native.lib().msbfs_solver_hybrid_phase_a(*args, C.byref(st), strm))
        return out, st.as_dict()

    def hybrid_chunk_bounds(self, part: int, nparts: int, n_eff: int, chunks: int) -> np.ndarray:
        """Own-vertex index ranges [b[c], b[c+1]) of a chunked phase A (chunks + 1 entries)."""
        b = np.zeros(int(chunks) + 1, dtype=np.int64)
        native.check(native.lib().msbfs_solver_hybrid_chunk_bounds(
            self._h, int(part), int(nparts), int(n_eff), int(chunks), native.ptr(b, C.c_int64)))
        return b

    def hybrid_phase_a_chunked(self, queries: QuerySet, part: int, nparts: int, n_eff: int,
                               count_l1: bool, wbeg: np.ndarray, send_ptr: int, chunks: int,
                               on_chunk, stream: Optional[int] = None):
        """hybrid_phase_a with the overlapped exchange: after each own-vertex range's words are
        packed (enqueued on the solver's stream), on_chunk(c, i0, i1) is called on this thread
        to start that piece of the all-to-all. Returns (out[2K+3], stats)."""
        K = queries.K
        wbeg = np.ascontiguousarray(wbeg, dtype=np.int32)
        out = np.zeros(2 * K + 3, dtype=np.int64)
        st = native.Stats()
        err = []

        def cb(_user, c, i0, i1):
            if err:
                return
            try:
                on_chunk(int(c), int(i0), int(i1))
            except BaseException as e:  # noqa: BLE001 (re-raised after the native call)
                err.append(e)

        fn = native.ChunkFn(cb)  # (kept alive for the call)
        rc = native.lib().msbfs_solver_hybrid_phase_a_chunked(
            self._h, K, native.ptr(queries.off, C.c_int64), native.ptr(queries.ids, C.c_int32),
            int(part), int(nparts), int(n_eff), int(bool(count_l1)), native.ptr(wbeg, C.c_int32),
            C.c_void_p(send_ptr), native.ptr(out, C.c_int64), int(chunks), fn, None,
            C.byref(st), C.c_void_p(stream) if stream else None)
        if err:
            raise err[0]
        native.check(rc)
        return out, st.as_dict()

    def hybrid_decode(self, coded_ptr: int, coded_len: np.ndarray, nparts: int, n_eff: int,
                      w_count: int, dense_ptr: int, stream: Optional[int] = None) -> None:
        """Expand the received coded segments (coded_len[r] u64 from each part r, back to back)
        into the dense layout hybrid_phase_c reads (asynchronous on the solver's stream)."""
        lens = np.ascontiguousarray(coded_len, dtype=np.int64)
        native.check(native.lib().msbfs_solver_hybrid_decode(
            self._h, C.c_void_p(coded_ptr), native.ptr(lens, C.c_int64), int(nparts), int(n_eff),
            int(w_count), C.c_void_p(dense_ptr), C.c_void_p(stream) if stream else None))

    def hybrid_phase_c(self, K: int, w_begin: int, w_count: int, nparts: int, n_eff: int,
                       recv_ptr: int, reduced: np.ndarray, stream: Optional[int] = None):
        """Levels >= 3 of the groups in words [w_begin, w_begin + w_count) from the exchanged
        words at recv_ptr (per source part, w_count u64 of each of its vertices). Returns
        (F_local[64 * w_count], stats)."""
        reduced = np.ascontiguousarray(reduced, dtype=np.int64)
        if len(reduced) != 2 * K + 3:
            raise ValueError("reduced must have 2K+3 entries")
        F = np.zeros(max(1, 64 * w_count), dtype=np.int64)
        st = native.Stats()
        native.check(native.lib().msbfs_solver_hybrid_phase_c(
            self._h, int(K), int(w_begin), int(w_count), int(nparts), int(n_eff),
            C.c_void_p(recv_ptr), native.ptr(reduced, C.c_int64), native.ptr(F, C.c_int64),
            C.byref(st), C.c_void_p(stream) if stream else None))
        return F, st.as_dict()

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            native.lib().msbfs_solver_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def cpu_bfs(graph: Graph, queries: QuerySet, threads: int = 0, count_edges: bool = False
            ) -> BfsResult:
    """Query-parallel host BFS (native C++ threads)."""
    K = queries.K
    F = np.zeros(K, dtype=np.int64)
    E = np.zeros(K, dtype=np.int64) if count_edges else None
    if K:
        native.check(native.lib().msbfs_cpu_run(
            graph.n, native.ptr(graph.rowptr, C.c_int64), native.ptr(graph.col, C.c_int32), K,
            native.ptr(queries.off, C.c_int64), native.ptr(queries.ids, C.c_int32),
            native.ptr(F, C.c_int64), native.ptr(E, C.c_int64) if E is not None else None,
            int(threads)))
    return BfsResult(F, E, {})


def multi_source_bfs(graph: Union[Graph, DeviceGraph], queries: QuerySet, algo: str = "auto",
                     device: int = 0, count_edges: bool = False, **opts) -> BfsResult:
    """One-shot convenience wrapper (creates and frees a Solver)."""
    if algo == "cpu":
        if isinstance(graph, DeviceGraph):
            graph = graph.download()
        return cpu_bfs(graph, queries, count_edges=count_edges)
    dg = graph if isinstance(graph, DeviceGraph) else DeviceGraph.from_host(graph, device)
    with Solver(dg, algo, max_groups=max(1, queries.K), **opts) as s:
        return s.run(queries, count_edges=count_edges)


def argmin_first(F: np.ndarray) -> int:
    """Reference tie-break (main.cu:381-397): first valid F, strict '<' => lowest index wins.
    Returns -1 for K == 0."""
    F = np.asarray(F)
    valid = np.nonzero(F >= 0)[0]
    if len(valid) == 0:
        return -1
    return int(valid[np.argmin(F[valid])])  # argmin returns the first minimum
