"""End-to-end distance-to-set job (the Python/torch.distributed twin of the native CLI).

Mirrors main() of the reference (main.cu:195-421) phase by phase:
  preprocessing  (main.cu:235-298): load graph on rank 0 -> distribute -> device CSR + solver
                   (or: every rank generates the identical RMAT graph in its own HBM)
  computation    (main.cu:301-400): round-robin local groups -> per-group F on the GPU ->
                   packed all-reduce(MIN) -> (minK, minF)
  report         (main.cu:402-414): the identical 7-line text
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from .models.graph import DeviceGraph, Graph
from .models.queries import QuerySet
from .ops.bfs import Solver, cpu_bfs
from .parallel import distributed as D
from .utils.report import format_report


@dataclass
class JobConfig:
    graph: Optional[str] = None     # legacy edge-list .bin path
    query: Optional[str] = None     # legacy / extended query .bin path
    gen: Optional[str] = None       # "rmat:SCALE:EF:SEED" | "uniform:N:M:SEED" | "grid:R:C:SEED"
    qgen: Optional[str] = None      # "K:SIZE:SEED"
    num_gpu: int = 1                # -gn (echoed in the report, used for device binding)
    algo: str = "auto"
    use_cache: bool = False
    count_edges: bool = False
    sort_rows: bool = False
    relabel: bool = True            # degree-descending internal ids (best effort)
    solver_opts: dict = field(default_factory=dict)


@dataclass
class JobResult:
    min_k: int
    min_f: int
    preprocessing_time: float
    computation_time: float
    F: Optional[np.ndarray] = None
    traversed_edges: Optional[int] = None
    stats: dict = field(default_factory=dict)


def _fill(args, defaults):
    return list(args[:len(defaults)]) + list(defaults[len(args):])


def _parse_gen(spec: str):
    f = spec.split(":")
    return f[0], [int(x) for x in f[1:]]


class Engine:
    def __init__(self, cfg: JobConfig, ctx: Optional[D.DistContext] = None):
        self.cfg = cfg
        self.ctx = ctx or D.DistContext()
        self.graph_host: Optional[Graph] = None
        self.dgraph: Optional[DeviceGraph] = None
        self.solver: Optional[Solver] = None
        self.queries: Optional[QuerySet] = None
        self.local_idx = np.zeros(0, np.int64)
        self.local_q: Optional[QuerySet] = None
        self.preprocessing_time = 0.0
        self.n = 0

    @property
    def on_gpu(self) -> bool:
        return self.cfg.algo != "cpu" and self.ctx.device >= 0

    def _sync(self):
        if self.on_gpu:
            import torch
            torch.cuda.synchronize(self.ctx.device)

    # ------------------------------------------------------------------ preprocessing
    def preprocess(self) -> float:
        cfg, ctx = self.cfg, self.ctx
        t0 = time.perf_counter()
        if cfg.gen:
            kind, a = _parse_gen(cfg.gen)
            if kind == "rmat":
                scale, ef, seed = _fill(a, [20, 16, 1])
                if self.on_gpu:
                    self.dgraph = DeviceGraph.rmat(scale, ef, seed, device=ctx.device)
                else:
                    self.graph_host = Graph.rmat(scale, ef, seed)
            elif kind == "uniform":
                n, m, seed = _fill(a, [1000, 0, 1])
                m = m or 10 * n
                if self.on_gpu:
                    self.dgraph = DeviceGraph.uniform(n, m, seed, device=ctx.device)
                else:
                    self.graph_host = Graph.uniform(n, m, seed)
            elif kind == "grid":
                r, c, seed = _fill(a, [100, 100, 1])
                self.graph_host = Graph.grid(r, c, 1.0, 0, seed)
                if self.on_gpu:
                    self.dgraph = DeviceGraph.from_host(self.graph_host, ctx.device)
            else:
                raise ValueError(f"unknown generator {kind}")
        else:
            g = Graph.from_file(cfg.graph, use_cache=cfg.use_cache) if ctx.rank == 0 else None
            res = D.broadcast_graph(g, ctx)
            if isinstance(res, tuple):  # RCCL: device tensors broadcast over xGMI
                rowptr_t, col_t, m = res
                self.dgraph = DeviceGraph.wrap(rowptr_t.numel() - 1, rowptr_t, col_t, ctx.device)
            else:
                self.graph_host = res
                if self.on_gpu:
                    self.dgraph = DeviceGraph.from_host(self.graph_host, ctx.device)
        if self.dgraph is not None and cfg.sort_rows:
            self.dgraph.sort_rows()
        if self.dgraph is not None and cfg.relabel and self.on_gpu:
            # the bit-parallel solver's prefix pulls rely on degree order; F does not depend on
            # the numbering, and each rank solves its own groups (round robin), so a rank without
            # room for the rebuild simply keeps the file's ids
            from .ops import native
            try:
                self.dgraph.relabel_by_degree()
            except native.MsbfsError as e:
                import sys
                print(f"msbfs: rank {ctx.rank} keeps the file's vertex ids: {e}", file=sys.stderr)
        self.n = self.dgraph.n if self.dgraph is not None else self.graph_host.n
        # queries
        if cfg.qgen:
            f = [int(x) for x in cfg.qgen.split(":")]
            K, size, seed = _fill(f, [64, 16, 7])
            self.queries = QuerySet.random(self.n, K, size, seed)
        else:
            q = QuerySet.from_file(cfg.query) if ctx.rank == 0 else None
            self.queries = D.broadcast_queries(q, ctx)
        self.local_idx = D.round_robin(self.queries.K, ctx.rank, ctx.world)
        self.local_q = self.queries.subset(self.local_idx)
        if self.on_gpu:
            self.solver = Solver(self.dgraph, cfg.algo, max_groups=max(1, self.local_q.K),
                                 **cfg.solver_opts)
        self._sync()
        self.preprocessing_time = time.perf_counter() - t0
        return self.preprocessing_time

    # ------------------------------------------------------------------ computation
    def run_local(self, count_edges: bool = False):
        if self.on_gpu:
            return self.solver.run(self.local_q, count_edges=count_edges)
        g = self.graph_host if self.graph_host is not None else self.dgraph.download()
        return cpu_bfs(g, self.local_q, count_edges=count_edges)

    def compute(self, gather: bool = False) -> JobResult:
        ctx = self.ctx
        t0 = time.perf_counter()
        res = self.run_local(count_edges=self.cfg.count_edges)
        min_k, min_f = D.packed_argmin(res.F, self.local_idx, self.queries.K, ctx)
        self._sync()
        dt = time.perf_counter() - t0
        F = D.gather_F(res.F, self.local_idx, self.queries.K, ctx) if gather else None
        edges = None
        if res.edges is not None:
            edges = int(D.allreduce_sum_i64(np.array([int(res.edges.sum())], np.int64), ctx)[0])
        return JobResult(min_k, min_f, self.preprocessing_time, dt, F, edges, res.stats)

    def report(self, r: JobResult) -> str:
        return format_report(self.cfg.graph or self.cfg.gen or "", self.cfg.query or self.cfg.qgen or "",
                             r.min_k, r.min_f, self.cfg.num_gpu, r.preprocessing_time,
                             r.computation_time)

    def close(self):
        if self.solver is not None:
            self.solver.close()
        if self.dgraph is not None:
            self.dgraph.close()
