"""Hybrid multi-GPU decomposition: vertex-partitioned levels 1-2, then query-partitioned.

Reference: the only decomposition in main.cu is static round-robin over query groups
(main.cu:304-307), each rank running whole BFSs on a full graph replica. The bit-parallel engine
keeps the replica but changes the split:

  phase A  every rank runs levels 1-2 for ALL groups (<= 1024, one pass), but the level-2
           bottom-up pull only for its own vertices v = rank + i*world (cyclic split: hubs and
           tail spread evenly, so pull work AND exchange volume are balanced). Level 2 is the
           explosive level: its row scans cost nearly the same for 128 groups as for 1024 (a
           scan stops only when every group is covered), so round-robin makes all N GPUs pay
           ~all of it.
  exchange one all-to-all of 64-bit visited words: rank j receives, for every vertex below
           n_eff (= 1 + the last vertex with an edge; a degree-relabelled graph keeps its
           isolated vertices in the suffix, which is never sent), the words of its own group
           block (1/N of the words); plus one small SUM all-reduce of the phase-A partial sums,
           "still alive" flags and frontier sizes.
  phase C  every rank continues its own groups from level 3 (bit-parallel, as in round-robin).

Result: F[k] = reduced[k] + F_C[k] for the own groups; the global argmin is the usual 8-byte
packed all-reduce(MIN) (distributed.packed_argmin). Groups are assigned in contiguous 64-group
words (rank j owns words [wbeg[j], wbeg[j+1]) of ceil(K/64)) instead of round-robin, so the
exchange moves whole words.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import distributed as D

# Largest world size one hybrid round supports (Solver::kHybridMaxParts in csrc device.hpp).
MAX_PARTS = 64


def word_split(K: int, world: int) -> np.ndarray:
    """wbeg[0..world]: rank j owns 64-group words [wbeg[j], wbeg[j+1]) of ceil(K/64)."""
    wt = (K + 63) // 64
    return np.array([j * wt // world for j in range(world + 1)], dtype=np.int32)


def own_groups(K: int, wbeg: np.ndarray, rank: int) -> np.ndarray:
    return np.arange(64 * int(wbeg[rank]), min(K, 64 * int(wbeg[rank + 1])), dtype=np.int64)


def part_count(n_eff: int, part: int, nparts: int) -> int:
    """Number of vertices v = part + i*nparts below n_eff."""
    return (n_eff - part + nparts - 1) // nparts if n_eff > part else 0


def part_vertices(n_eff: int, part: int, nparts: int) -> np.ndarray:
    return np.arange(part, n_eff, nparts, dtype=np.int64)


def split_sizes(n_eff: int, wbeg: np.ndarray, rank: int):
    """(input_split_sizes, output_split_sizes) of the all-to-all, in 64-bit words."""
    world = len(wbeg) - 1
    cnt = part_count(n_eff, rank, world)
    nw_me = int(wbeg[rank + 1] - wbeg[rank])
    send = [cnt * int(wbeg[j + 1] - wbeg[j]) for j in range(world)]
    recv = [part_count(n_eff, r, world) * nw_me for r in range(world)]
    return send, recv


# ---- numpy emulation of the device layout (tests; documents the kernels' contract) ----------
def pack_words_np(vis: np.ndarray, part: int, nparts: int, n_eff: int,
                  wbeg: np.ndarray) -> np.ndarray:
    """Twin of k_pack_words: vis[n, W] (uint64) -> destination-major send buffer."""
    wt = int(wbeg[-1])
    blk = vis[part_vertices(n_eff, part, nparts), :wt]
    return np.concatenate([blk[:, wbeg[j]:wbeg[j + 1]].reshape(-1)
                           for j in range(len(wbeg) - 1)]) if wt else np.zeros(0, vis.dtype)


def all_to_all_np(sends, n_eff: int, wbeg: np.ndarray):
    """Emulated all_to_all_single over all ranks: returns every rank's receive buffer."""
    world = len(wbeg) - 1
    outs = []
    for j in range(world):
        parts = []
        for r in range(world):
            s_sizes, _ = split_sizes(n_eff, wbeg, r)
            off = sum(s_sizes[:j])
            parts.append(sends[r][off:off + s_sizes[j]])
        outs.append(np.concatenate(parts) if parts else np.zeros(0, np.uint64))
    return outs


def unpack_np(recv: np.ndarray, n: int, n_eff: int, nparts: int, nw: int) -> np.ndarray:
    """Twin of k_hybrid_setup's indexing: recv -> rows[n, nw] (zero rows beyond n_eff)."""
    rows = np.zeros((n, nw), dtype=recv.dtype)
    off = 0
    for r in range(nparts):
        vs = part_vertices(n_eff, r, nparts)
        rows[vs] = recv[off:off + len(vs) * nw].reshape(len(vs), nw)
        off += len(vs) * nw
    return rows


@dataclass
class HybridResult:
    idx: np.ndarray          # global indices of this rank's groups
    F: np.ndarray            # their F(U)
    stats: dict = field(default_factory=dict)


class HybridRunner:
    """Reusable buffers + plan for one (solver, K, world) combination."""

    def __init__(self, solver, K: int, ctx: D.DistContext):
        import torch

        self.solver, self.K, self.ctx = solver, int(K), ctx
        g = solver.graph
        if self.K < 1 or self.K > solver.hybrid_max_groups():
            raise ValueError(f"hybrid mode handles 1..{solver.hybrid_max_groups()} groups per "
                             f"round, got {self.K}")
        if ctx.world > MAX_PARTS:
            raise ValueError(f"hybrid mode handles at most {MAX_PARTS} ranks, got {ctx.world}")
        self.n_eff = g.hybrid_extent()
        self.wbeg = word_split(self.K, ctx.world)
        self.idx = own_groups(self.K, self.wbeg, ctx.rank)
        self.send_sizes, self.recv_sizes = split_sizes(self.n_eff, self.wbeg, ctx.rank)
        self.nw = int(self.wbeg[ctx.rank + 1] - self.wbeg[ctx.rank])
        dev = torch.device("cuda", g.device)
        self.send = torch.empty(max(1, sum(self.send_sizes)), dtype=torch.int64, device=dev)
        self.recv = torch.empty(max(1, sum(self.recv_sizes)), dtype=torch.int64, device=dev)
        self._staged = ctx.distributed and ctx.backend != "nccl"

    def _exchange(self, out: np.ndarray) -> np.ndarray:
        import torch
        import torch.distributed as dist

        ctx = self.ctx
        if not ctx.distributed:
            self.recv[:sum(self.recv_sizes)].copy_(self.send[:sum(self.send_sizes)])
            return out
        if self._staged:  # gloo: through host memory
            s = self.send[:sum(self.send_sizes)].cpu()
            r = torch.empty(sum(self.recv_sizes), dtype=torch.int64)
            dist.all_to_all_single(r, s, self.recv_sizes, self.send_sizes)
            self.recv[:sum(self.recv_sizes)].copy_(r)
            t = torch.from_numpy(out)
        else:
            dist.all_to_all_single(self.recv[:sum(self.recv_sizes)],
                                   self.send[:sum(self.send_sizes)],
                                   self.recv_sizes, self.send_sizes)
            t = torch.from_numpy(out).to(self.send.device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        res = t.cpu().numpy()
        if not self._staged:
            # the native phase C runs on its own stream: make the received words visible first
            torch.cuda.current_stream(self.send.device).synchronize()
        return res

    def run(self, queries) -> HybridResult:
        if queries.K != self.K:
            raise ValueError("query count differs from the plan")
        ctx = self.ctx
        out, sa = self.solver.hybrid_phase_a(queries, ctx.rank, ctx.world, self.n_eff,
                                             ctx.rank == 0, self.wbeg, self.send.data_ptr())
        reduced = self._exchange(out)
        Fc, sc = self.solver.hybrid_phase_c(self.K, int(self.wbeg[ctx.rank]), self.nw, ctx.world,
                                            self.n_eff, self.recv.data_ptr(), reduced)
        F = reduced[self.idx] + Fc[:len(self.idx)]
        stats = {"levels": sa.get("levels", 0) + sc.get("levels", 0),
                 "td_levels": sa.get("td_levels", 0) + sc.get("td_levels", 0),
                 "bu_levels": sa.get("bu_levels", 0) + sc.get("bu_levels", 0),
                 "phase_a_ms": sa.get("device_ms"), "phase_c_ms": sc.get("device_ms"),
                 "part": (ctx.rank, ctx.world, self.n_eff), "words": self.nw}
        return HybridResult(self.idx, F, stats)


def hybrid_bfs(solver, queries, ctx: Optional[D.DistContext] = None) -> HybridResult:
    """One-shot hybrid run of all K groups over the ranks of ctx (single process if None)."""
    ctx = ctx or D.DistContext(device=solver.graph.device)
    return HybridRunner(solver, queries.K, ctx).run(queries)


def emulate_ranks(solver, queries, world: int, timings: Optional[list] = None) -> np.ndarray:
    """Run the hybrid algorithm for `world` ranks sequentially in ONE process on one GPU (no
    torch.distributed): phase A of every rank, a host-side all-to-all, phase C of every rank.
    Returns the full F vector. Used by the GPU tests and to time per-rank phases: with
    `timings` (a list) one dict per rank is appended (phase A / C device ms, send/recv bytes)."""
    import torch

    K = queries.K
    g = solver.graph
    n_eff = g.hybrid_extent()
    wbeg = word_split(K, world)
    dev = torch.device("cuda", g.device)
    sends, outs = [], []
    for r in range(world):
        ss, rs = split_sizes(n_eff, wbeg, r)
        buf = torch.empty(max(1, sum(ss)), dtype=torch.int64, device=dev)
        out, sa = solver.hybrid_phase_a(queries, r, world, n_eff, r == 0, wbeg, buf.data_ptr())
        if timings is not None:
            timings.append({"rank": r, "vertices": part_count(n_eff, r, world),
                            "phase_a_ms": sa["device_ms"], "send_bytes": 8 * sum(ss),
                            "recv_bytes": 8 * sum(rs), "phase_c_ms": 0.0})
        sends.append(buf[:sum(ss)].cpu().numpy().view(np.uint64))
        outs.append(out)
    reduced = np.sum(outs, axis=0)
    recvs = all_to_all_np(sends, n_eff, wbeg)
    F = np.zeros(K, dtype=np.int64)
    for j in range(world):
        nw = int(wbeg[j + 1] - wbeg[j])
        if nw == 0:
            continue
        rt = torch.from_numpy(recvs[j].view(np.int64)).to(dev)
        Fc, sc = solver.hybrid_phase_c(K, int(wbeg[j]), nw, world, n_eff, rt.data_ptr(), reduced)
        if timings is not None:
            timings[len(timings) - world + j]["phase_c_ms"] = sc["device_ms"]
            timings[len(timings) - world + j]["levels_c"] = sc["levels"]
        idx = own_groups(K, wbeg, j)
        F[idx] = reduced[idx] + Fc[:len(idx)]
    return F
