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
           "still alive" flags and frontier sizes. About half of those words are zero after
           level 2 (RMAT-26, 1024 groups, 8 ranks: 50.5 %): optionally (coded=True, bench
           candidate "hybrid-coded", CLI --dist hybrid-coded) each destination's share travels
           zero-word coded (encode_np: a bitmap word per 64 words + the nonzero words; the
           same all-reduce carries the N x N matrix of coded lengths) and the receiver expands
           it on the GPU (Solver.hybrid_decode); see coding_default for when that pays.
  phase C  every rank continues its own groups from level 3 (bit-parallel, as in round-robin).

Result: F[k] = reduced[k] + F_C[k] for the own groups; the global argmin is the usual 8-byte
packed all-reduce(MIN) (distributed.packed_argmin). Groups are assigned in contiguous 64-group
words (rank j owns words [wbeg[j], wbeg[j+1]) of ceil(K/64)) instead of round-robin, so the
exchange moves whole words.
"""
from __future__ import annotations

from dataclasses import dataclass, field
import os
import time
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


def coded_bound(words: int) -> int:
    """Largest zero-word coded size of a segment of `words` words (all nonzero)."""
    return int(words) + (int(words) + 63) // 64


def coding_default() -> bool:
    """Dense exchange by default (coded only when asked for: HybridRunner(coded=True), bench.py
    candidate "hybrid-coded", CLI --dist hybrid-coded; never from a per-rank environment
    variable, since every rank must size and call the same collectives). Measured (RMAT-26, 1024 groups, 8
    ranks emulated on one MI355X): 296 instead of 501 MB per GPU, but +0.8 ms of coding in phase
    A and +0.43 ms of decoding before phase C, so it pays only when the all-to-all runs below
    ~170 GB/s per GPU. bench.py measures it as a separate candidate ("hybrid-coded")."""
    return False


def encode_np(words: np.ndarray) -> np.ndarray:
    """Twin of k_code_bits/k_code_emit for one segment: ceil(L/64) bitmap words (bit i of word c
    set iff words[64c+i] != 0), then the nonzero words in order."""
    words = np.asarray(words, dtype=np.uint64)
    L = len(words)
    nch = (L + 63) // 64
    nz = np.zeros(nch * 64, dtype=bool)
    nz[:L] = words != 0
    bm = (nz.reshape(nch, 64).astype(np.uint64) << np.arange(64, dtype=np.uint64)).sum(
        axis=1, dtype=np.uint64)
    return np.concatenate([bm, words[nz[:L]]])


def decode_np(coded: np.ndarray, L: int) -> np.ndarray:
    """Twin of k_decode_pop/k_decode_emit: one coded segment back to its L dense words."""
    coded = np.asarray(coded, dtype=np.uint64)
    nch = (L + 63) // 64
    bits = ((coded[:nch, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)
    bits = bits.reshape(-1)[:L]
    if len(coded) != nch + int(bits.sum()):
        raise ValueError(f"coded segment has {len(coded)} words, expected {nch + int(bits.sum())}")
    out = np.zeros(L, dtype=np.uint64)
    out[bits] = coded[nch:]
    return out


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


def torch_sync(device) -> None:
    """Host wait for everything queued on the device's current stream (the native kernels run
    on the same null stream; collective pieces were made visible to it by Work.wait())."""
    import torch
    torch.cuda.current_stream(device).synchronize()


@dataclass
class HybridResult:
    idx: np.ndarray          # global indices of this rank's groups
    F: np.ndarray            # their F(U)
    stats: dict = field(default_factory=dict)


# Own-vertex ranges of the overlapped exchange (RCCL, dense layout): phase A hands each range's
# words to the all-to-all as soon as its level-2 pulls are done, while the next range computes.
# RMAT-26 / 8 ranks emulated: 4 pieces leave 0.34 of the 1.75 ms exchange exposed, 8 pieces
# ~0.01 ms (profiles/hybrid_sim_rmat26.md).
DEFAULT_CHUNKS = 8


def chunk_views(send, recv, cnt: int, wbeg: np.ndarray, rank: int, pcounts, bounds: np.ndarray,
                c: int):
    """(input list, output list) of chunk c for all_to_all: to rank j the words of own vertices
    [bounds[rank, c], bounds[rank, c+1]) from j's word block of send (destination-major); from
    rank r its range c, straight into r's block of recv (source-major, the layout phase C reads).
    bounds[r] are rank r's chunk bounds (every rank's, agreed at setup)."""
    P = len(wbeg) - 1
    nw_me = int(wbeg[rank + 1] - wbeg[rank])
    i0, i1 = int(bounds[rank, c]), int(bounds[rank, c + 1])
    ins, outs = [], []
    for j in range(P):
        nwj = int(wbeg[j + 1] - wbeg[j])
        base = cnt * int(wbeg[j])
        ins.append(send[base + i0 * nwj: base + i1 * nwj])
    rbase = 0
    for r in range(P):
        a, b = int(bounds[r, c]), int(bounds[r, c + 1])
        outs.append(recv[rbase + a * nw_me: rbase + b * nw_me])
        rbase += int(pcounts[r]) * nw_me
    return ins, outs


class PieceExchange:
    """The overlapped exchange's pieces as point-to-point operations, one batch per piece.

    Piece c sends to every peer j its words of this rank's own-vertex range c and receives
    from every peer r its range c (chunk_views). Each piece is one dist.batch_isend_irecv:
    grouped ncclSend/ncclRecv on RCCL's stream, or tagged isend/irecv under gloo. The local
    block is a copy on the current stream. Both backends issue the same calls in the same
    order, so the gloo tests run the sequence that the RCCL runs use. Gloo stages through host
    memory: a send is copied to the host when its piece starts, and a receive lands in a host
    buffer that finish() copies into recv.

    Pairing rule: every rank starts every piece, in the same order. Piece c's sizes depend
    only on the bounds agreed at setup, so a sender and its receiver agree on every size. A
    piece that is empty on both sides issues no operation. The reference gathers with blocking
    MPI_Gather + MPI_Gatherv after all compute (main.cu:340-365).
    """

    def __init__(self, ctx: D.DistContext, send, recv, cnt: int, wbeg: np.ndarray, pcounts,
                 bounds: np.ndarray, chunks: int):
        self.ctx, self.send, self.recv, self.cnt = ctx, send, recv, int(cnt)
        self.wbeg, self.pcounts, self.bounds, self.chunks = wbeg, pcounts, bounds, int(chunks)
        self.staged = ctx.distributed and ctx.backend != "nccl"
        self.reset()

    def reset(self) -> None:
        self.works, self.landing, self.started = [], [], []

    def order(self):
        """Issue order of the pieces: last range first (the tiled pull's order, tiles_pull)."""
        return list(range(self.chunks - 1, -1, -1))

    def start(self, c: int) -> None:
        import torch
        import torch.distributed as dist

        if c in self.started:
            raise RuntimeError(f"exchange piece {c} started twice")
        ctx = self.ctx
        ins, outs = chunk_views(self.send, self.recv, self.cnt, self.wbeg, ctx.rank,
                                self.pcounts, self.bounds, c)
        self.started.append(c)
        me = ctx.rank
        if outs[me].numel():
            outs[me].copy_(ins[me])
        if not ctx.distributed:
            return
        ops = []
        for j in range(ctx.world):
            if j == me:
                continue
            if ins[j].numel():
                ops.append(dist.P2POp(dist.isend, ins[j].cpu() if self.staged else ins[j], j,
                                      tag=c))
            if outs[j].numel():
                dst = outs[j]
                if self.staged:
                    dst = torch.empty(outs[j].numel(), dtype=outs[j].dtype)
                    self.landing.append((outs[j], dst))
                ops.append(dist.P2POp(dist.irecv, dst, j, tag=c))
        if ops:
            self.works.extend(dist.batch_isend_irecv(ops))

    def start_missing(self) -> None:
        """Start every piece not started yet, in issue order (after a failure partway through
        phase A: the peers still pair their calls with this rank's)."""
        for c in self.order():
            if c not in self.started:
                self.start(c)

    def finish(self) -> None:
        """Wait for every piece. The received words are then visible to the current stream,
        which the native kernels use too."""
        for w in self.works:
            w.wait()
        for dst, src in self.landing:
            dst.copy_(src)
        if self.recv.is_cuda:
            torch_sync(self.recv.device)
        self.reset()


class HybridRunner:
    """Reusable buffers + plan for one (solver, K, world) combination."""

    def __init__(self, solver, K: int, ctx: D.DistContext, coded: Optional[bool] = None,
                 chunks: Optional[int] = None):
        import torch

        self.solver, self.K, self.ctx = solver, int(K), ctx
        g = solver.graph
        if self.K < 1 or self.K > solver.hybrid_max_groups():
            raise ValueError(f"hybrid mode handles 1..{solver.hybrid_max_groups()} groups per "
                             f"round, got {self.K}")
        if ctx.world > MAX_PARTS:
            raise ValueError(f"hybrid mode handles at most {MAX_PARTS} ranks, got {ctx.world}")
        self.coded = coding_default() if coded is None else bool(coded)
        self.n_eff = g.hybrid_extent()
        self.wbeg = word_split(self.K, ctx.world)
        self.idx = own_groups(self.K, self.wbeg, ctx.rank)
        self.send_sizes, self.recv_sizes = split_sizes(self.n_eff, self.wbeg, ctx.rank)
        self.nw = int(self.wbeg[ctx.rank + 1] - self.wbeg[ctx.rank])
        dev = torch.device("cuda", g.device)
        ns = sum(coded_bound(x) for x in self.send_sizes) if self.coded else sum(self.send_sizes)
        self.send = torch.empty(max(1, ns), dtype=torch.int64, device=dev)
        self.recv = torch.empty(max(1, sum(self.recv_sizes)), dtype=torch.int64, device=dev)
        self.rcoded = (torch.empty(max(1, sum(coded_bound(x) for x in self.recv_sizes)),
                                   dtype=torch.int64, device=dev) if self.coded else None)
        self._staged = ctx.distributed and ctx.backend != "nccl"
        self.last_bytes = (0, 0)  # (sent, received) of the last exchange
        solver.prepare_hybrid(ctx.rank, ctx.world)  # (phase A's tables, outside timed runs)
        # overlapped exchange: the dense layout only (the coded segments exist only once the
        # whole phase A is done). Point-to-point pieces (PieceExchange): RCCL and gloo alike.
        if chunks is None:
            chunks = DEFAULT_CHUNKS if (ctx.distributed and not self.coded) else 1
        self.chunks = max(1, int(chunks)) if not self.coded else 1
        self.pcounts = [part_count(self.n_eff, r, ctx.world) for r in range(ctx.world)]
        self.bounds = None
        self.exchange = None
        if self.chunks > 1:
            b = solver.hybrid_chunk_bounds(ctx.rank, ctx.world, self.n_eff, self.chunks)
            full = np.zeros((ctx.world, self.chunks + 1), dtype=np.int64)
            full[ctx.rank] = b
            self.bounds = D.allreduce_sum_i64(full.reshape(-1), ctx).reshape(ctx.world, -1)
            self.exchange = PieceExchange(ctx, self.send, self.recv, self.pcounts[ctx.rank],
                                          self.wbeg, self.pcounts, self.bounds, self.chunks)

    def _all_to_all(self, recv, send, rsz, ssz) -> None:
        import torch
        import torch.distributed as dist

        if not self.ctx.distributed:
            recv[:sum(rsz)].copy_(send[:sum(ssz)])
        elif self._staged:  # gloo: through host memory
            s = send[:sum(ssz)].cpu()
            r = torch.empty(sum(rsz), dtype=torch.int64)
            dist.all_to_all_single(r, s, list(rsz), list(ssz))
            recv[:sum(rsz)].copy_(r)
        else:
            dist.all_to_all_single(recv[:sum(rsz)], send[:sum(ssz)], list(rsz), list(ssz))
        if self.ctx.distributed or recv.is_cuda:
            # the native kernels run on their own stream: make the received words visible first
            torch.cuda.current_stream(recv.device).synchronize()

    def _allreduce(self, vec: np.ndarray) -> np.ndarray:
        import torch
        import torch.distributed as dist

        if not self.ctx.distributed:
            return vec
        if not self._staged:  # (RCCL: through cached pinned buffers, see D._reduce_small)
            return D._reduce_small(np.ascontiguousarray(vec, dtype=np.int64), self.ctx,
                                   dist.ReduceOp.SUM)
        t = torch.from_numpy(vec)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()

    def run(self, queries, checked: bool = False) -> HybridResult:
        """One hybrid step. checked=True (bench.py's untimed selection pass): every rank-local
        phase is followed by an agreement all-reduce, so a failure on one rank raises on all of
        them instead of leaving the others in the exchange (distributed.checked)."""
        if queries.K != self.K:
            raise ValueError("query count differs from the plan")
        ctx, P = self.ctx, self.ctx.world

        def local(fn, what):
            return D.checked(fn, ctx, what) if checked else fn()

        t0 = time.perf_counter()
        if self.chunks > 1:
            ex = self.exchange
            ex.reset()
            err = None
            try:  # piece c starts as soon as phase A has packed range c (async)
                out, sa = self.solver.hybrid_phase_a_chunked(
                    queries, ctx.rank, P, self.n_eff, ctx.rank == 0, self.wbeg,
                    self.send.data_ptr(), self.chunks, lambda c, i0, i1: ex.start(c))
            except Exception as e:  # noqa: BLE001
                err = e
            if checked:
                # a failure partway: still start the remaining pieces (their words are junk), so
                # every peer's calls pair up, then fail on every rank together
                if err is not None:
                    ex.start_missing()
                if not D.agree_ok(err is None, ctx):
                    ex.finish()
                    if err is not None:
                        raise err
                    raise RuntimeError("hybrid phase A failed on another rank")
            elif err is not None:
                raise err
        else:
            out, sa = local(lambda: self.solver.hybrid_phase_a(
                queries, ctx.rank, P, self.n_eff, ctx.rank == 0, self.wbeg, self.send.data_ptr(),
                coded=self.coded), "hybrid phase A")
        t1 = time.perf_counter()  # (phase A returns host sums: its kernels are done)
        if self.coded:
            # one SUM all-reduce: phase-A partial sums + the P x P matrix of coded lengths
            ext = np.zeros(len(out) + P * P, dtype=np.int64)
            ext[:len(out)] = out
            ext[len(out) + ctx.rank * P:len(out) + (ctx.rank + 1) * P] = sa["coded_len"]
            ext = self._allreduce(ext)
            reduced = ext[:len(out)]
            M = ext[len(out):].reshape(P, P)
            ssz, rsz = [int(x) for x in M[ctx.rank]], [int(x) for x in M[:, ctx.rank]]
            self._all_to_all(self.rcoded, self.send, rsz, ssz)
            self.solver.hybrid_decode(self.rcoded.data_ptr(), np.array(rsz, np.int64), P,
                                      self.n_eff, self.nw, self.recv.data_ptr())
        elif self.chunks > 1:
            ssz, rsz = self.send_sizes, self.recv_sizes
            reduced = self._allreduce(out.copy())
            self.exchange.finish()  # (the pieces started during phase A)
        else:
            ssz, rsz = self.send_sizes, self.recv_sizes
            reduced = self._allreduce(out.copy())
            self._all_to_all(self.recv, self.send, rsz, ssz)
        self.last_bytes = (8 * sum(ssz), 8 * sum(rsz))
        t2 = time.perf_counter()  # (the exchange synchronises before returning)
        Fc, sc = local(lambda: self.solver.hybrid_phase_c(
            self.K, int(self.wbeg[ctx.rank]), self.nw, P, self.n_eff, self.recv.data_ptr(),
            reduced), "hybrid phase C")
        t3 = time.perf_counter()
        F = reduced[self.idx] + Fc[:len(self.idx)]
        stats = {"levels": sa.get("levels", 0) + sc.get("levels", 0),
                 "td_levels": sa.get("td_levels", 0) + sc.get("td_levels", 0),
                 "bu_levels": sa.get("bu_levels", 0) + sc.get("bu_levels", 0),
                 "phase_a_ms": sa.get("device_ms"), "phase_c_ms": sc.get("device_ms"),
                 "phase_a_wall_ms": (t1 - t0) * 1e3, "exchange_ms": (t2 - t1) * 1e3,
                 "phase_c_wall_ms": (t3 - t2) * 1e3,
                 "part": (ctx.rank, P, self.n_eff), "words": self.nw,
                 "sent_bytes": self.last_bytes[0], "coded": self.coded, "chunks": self.chunks}
        return HybridResult(self.idx, F, stats)


def hybrid_bfs(solver, queries, ctx: Optional[D.DistContext] = None) -> HybridResult:
    """One-shot hybrid run of all K groups over the ranks of ctx (single process if None)."""
    ctx = ctx or D.DistContext(device=solver.graph.device)
    return HybridRunner(solver, queries.K, ctx).run(queries)


def overlapped_exchange_ms(phase_a_ms: float, ready_ms, piece_bytes, gbps: float) -> float:
    """When the last piece of a rank's chunked exchange has left (ms after its phase A started):
    piece c can start once it is packed (ready_ms[c]) and the link is free; pieces go one after
    another at gbps. (Dense, non-chunked: one piece ready at phase_a_ms.)"""
    t = 0.0
    for r, b in zip(ready_ms, piece_bytes):
        t = max(t, r) + b / (gbps * 1e9) * 1e3
    return max(t, 0.0)


def emulate_ranks(solver, queries, world: int, timings: Optional[list] = None,
                  coded: Optional[bool] = None, chunks: int = 1,
                  wbeg: Optional[np.ndarray] = None, piece_hook=None) -> np.ndarray:
    """Run the hybrid algorithm for `world` ranks sequentially in ONE process on one GPU (no
    torch.distributed): phase A of every rank, a host-side all-to-all, phase C of every rank.
    Returns the full F vector. Used by the GPU tests and to time per-rank phases: with
    `timings` (a list) one dict per rank is appended (phase A / C device ms and host wall ms,
    send/recv bytes). coded: zero-word coded exchange (default: coding_default()), decoded on the
    GPU. chunks > 1 (dense only): phase A runs chunked like the overlapped exchange of
    HybridRunner; each piece's ready time (CUDA events after its pack) and bytes are recorded
    ("pieces") so that tools/hybrid_sim.py can price only the exchange phase A does not hide.
    wbeg: a custom word split (world + 1 non-decreasing entries from 0 to ceil(K/64); default
    word_split, the even one). piece_hook(c, nbytes): called after each piece is packed (e.g.
    to start a one-rank RCCL copy of that size and see what it does to phase A's kernels)."""
    import torch

    coded = coding_default() if coded is None else bool(coded)
    K = queries.K
    g = solver.graph
    n_eff = g.hybrid_extent()
    wt = (K + 63) // 64
    wbeg = word_split(K, world) if wbeg is None else np.asarray(wbeg, dtype=np.int32)
    if len(wbeg) != world + 1 or wbeg[0] != 0 or wbeg[-1] != wt or np.any(np.diff(wbeg) < 0):
        raise ValueError("wbeg: world + 1 non-decreasing word bounds from 0 to ceil(K/64)")
    dev = torch.device("cuda", g.device)
    sends, outs, lens = [], [], []
    chunks = 1 if coded else max(1, int(chunks))
    for r in range(world):
        ss, rs = split_sizes(n_eff, wbeg, r)
        nb = sum(coded_bound(x) for x in ss) if coded else sum(ss)
        buf = torch.empty(max(1, nb), dtype=torch.int64, device=dev)
        pieces = []
        torch.cuda.synchronize(dev)
        tw = time.perf_counter()
        if chunks > 1:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()

            def on_chunk(c, i0, i1):
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                pieces.append((e, 8 * (i1 - i0) * int(wbeg[-1])))
                if piece_hook is not None:
                    piece_hook(c, pieces[-1][1])

            out, sa = solver.hybrid_phase_a_chunked(queries, r, world, n_eff, r == 0, wbeg,
                                                    buf.data_ptr(), chunks, on_chunk)
            torch.cuda.synchronize(dev)
            pieces = [(ev0.elapsed_time(e), b) for e, b in pieces]
        else:
            out, sa = solver.hybrid_phase_a(queries, r, world, n_eff, r == 0, wbeg,
                                            buf.data_ptr(), coded=coded)
        wall_a = (time.perf_counter() - tw) * 1e3
        cl = [int(x) for x in sa["coded_len"]] if coded else list(ss)
        dense = buf[:sum(ss)].cpu().numpy().view(np.uint64) if not coded else None
        sends.append(buf[:sum(cl)].cpu().numpy().view(np.uint64))
        lens.append(cl)
        outs.append(out)
        if timings is not None:
            if coded:  # how much the coding saved: the dense twin of this rank's segments
                offs = np.concatenate([[0], np.cumsum(cl)])
                zero = sum(int(len(x) - np.count_nonzero(x)) for x in
                           (decode_np(sends[-1][offs[j]:offs[j + 1]], ss[j]) for j in range(world)))
            else:
                zero = int(len(dense) - np.count_nonzero(dense))
            timings.append({"rank": r, "vertices": part_count(n_eff, r, world),
                            "phase_a_ms": sa["device_ms"], "phase_a_wall_ms": wall_a,
                            "pieces": pieces, "send_bytes": 8 * sum(cl),
                            "dense_send_bytes": 8 * sum(ss), "recv_bytes": 0,
                            "send_zero_frac": zero / max(1, sum(ss)), "phase_c_ms": 0.0})
    reduced = np.sum(outs, axis=0)
    F = np.zeros(K, dtype=np.int64)
    for j in range(world):
        nw = int(wbeg[j + 1] - wbeg[j])
        rsz = [lens[r][j] for r in range(world)]
        parts = []
        for r in range(world):
            o = sum(lens[r][:j])
            parts.append(sends[r][o:o + lens[r][j]])
        rbuf = np.concatenate(parts) if parts else np.zeros(0, np.uint64)
        if timings is not None:
            timings[len(timings) - world + j]["recv_bytes"] = 8 * len(rbuf)
        if nw == 0:
            continue
        rt = torch.from_numpy(rbuf.view(np.int64)).to(dev) if len(rbuf) else \
            torch.zeros(1, dtype=torch.int64, device=dev)
        if coded:
            dense = torch.empty(max(1, sum(split_sizes(n_eff, wbeg, j)[1])), dtype=torch.int64,
                                device=dev)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            solver.hybrid_decode(rt.data_ptr(), np.array(rsz, np.int64), world, n_eff, nw,
                                 dense.data_ptr())
            torch.cuda.synchronize(dev)
            if timings is not None:  # wall time of the GPU decode (launches + kernels)
                timings[len(timings) - world + j]["decode_ms"] = (time.perf_counter() - t0) * 1e3
            rt = dense
        torch.cuda.synchronize(dev)
        tw = time.perf_counter()
        Fc, sc = solver.hybrid_phase_c(K, int(wbeg[j]), nw, world, n_eff, rt.data_ptr(), reduced)
        if timings is not None:
            timings[len(timings) - world + j]["phase_c_ms"] = sc["device_ms"]
            timings[len(timings) - world + j]["phase_c_wall_ms"] = (time.perf_counter() - tw) * 1e3
            timings[len(timings) - world + j]["levels_c"] = sc["levels"]
            # per level of phase C: direction, active (pull) / touched (push) vertices, ms
            timings[len(timings) - world + j]["levels_c_trace"] = [
                (t["dir"], t["level"], t["active"], round(t["ms"], 3))
                for t in solver.level_trace()]
        idx = own_groups(K, wbeg, j)
        F[idx] = reduced[idx] + Fc[:len(idx)]
    return F
