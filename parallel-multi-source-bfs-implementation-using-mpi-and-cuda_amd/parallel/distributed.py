"""Query-level data parallelism over torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

Reference distributed layer: MPI_Bcast of n, m, row_offsets, col_indices
(main.cu:242-255), 2K+1 MPI_Bcast for the queries (main.cu:257-280), static round-robin
kidx = rank, rank+P, ... (main.cu:304-307), MPI_Gather + MPI_Gatherv of (q, F) pairs with a custom
struct datatype (main.cu:324-368) and a serial argmin on rank 0 (main.cu:377-397).

MI355X design:
  * one process per GPU, `torch.distributed` with backend "nccl" (= RCCL);
  * the CSR is broadcast HBM -> HBM (device tensors, chunked) — or not at all when every rank
    generates the identical graph in its own HBM (deterministic counter-based generator);
  * queries travel as ONE packed (off, ids) blob;
  * the result is ONE 8-byte all-reduce(MIN) on a packed key (F << qbits | q): min F, and the
    lowest query index among ties — exactly the reference's strict-'<' first-wins argmin.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

CHUNK_BYTES = 1 << 30


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: int = -1          # GPU ordinal, -1 for CPU
    backend: str = "none"     # "nccl" (RCCL), "gloo" or "none" (single process)
    # a one-rank process group that still goes through every collective (MSBFS_FORCE_DIST=1):
    # exercises the RCCL code paths on a one-GPU box
    forced: bool = False

    @property
    def distributed(self) -> bool:
        return (self.world > 1 or self.forced) and self.backend != "none"

    def torch_device(self):
        import torch
        return torch.device("cuda", self.device) if self.device >= 0 else torch.device("cpu")


def pg_timeout_s() -> float:
    """Collective timeout of the process group: MSBFS_PG_TIMEOUT seconds (default 180)."""
    t = float(os.environ.get("MSBFS_PG_TIMEOUT", "180"))
    if not t > 0:
        raise ValueError(f"MSBFS_PG_TIMEOUT must be > 0, got {t}")
    return t


def init_from_env(backend: Optional[str] = None, gpus_per_node: Optional[int] = None,
                  use_gpu: Optional[bool] = None) -> DistContext:
    """Initialise from torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).

    Device binding follows the reference: device = local_rank % gpus_per_node (main.cu:227).

    A single process (world 1, not forced) never imports torch: the native engine drives the GPU
    alone, so the process holds one HIP runtime (the system's). torch's wheel bundles its own
    ROCm libraries; next to them rocprofv3's runtime tracer crashed in its exit-time finalizer
    (round 5: tools/exit_check.py, frames in librocprofiler-sdk -> libhsa-runtime64).
    """
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    forced = world == 1 and os.environ.get("MSBFS_FORCE_DIST") == "1"
    if world == 1 and not forced:
        from ..ops import native
        device = -1
        if use_gpu is None or use_gpu:
            ngpu = native.device_count()
            if use_gpu and ngpu < 1:
                raise RuntimeError("no GPU visible")
            if ngpu >= 1:
                device = 0
        return DistContext(0, 1, 0, device, "none")
    import torch
    import torch.distributed as dist

    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    device = -1
    if use_gpu:
        ngpu = torch.cuda.device_count()
        per_node = gpus_per_node or ngpu
        device = (local_rank % per_node) % max(ngpu, 1)
        torch.cuda.set_device(device)
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if world > 1 or forced:
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            # a hung or mismatched collective fails loudly after pg_timeout_s, well inside the
            # driver's lease, instead of blocking until the lease is killed
            kw = {"timeout": datetime.timedelta(seconds=pg_timeout_s())}
            if backend == "nccl" and device >= 0:
                kw["device_id"] = torch.device("cuda", device)
            dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
        return DistContext(rank, world, local_rank, device, backend, forced)
    return DistContext(0, 1, 0, device, "none")


def shutdown(ctx: DistContext) -> None:
    if not ctx.distributed:
        return
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def round_robin(K: int, rank: int, world: int) -> np.ndarray:
    """Static assignment of main.cu:304-307: kidx = rank, rank + world, ..."""
    return np.arange(rank, K, world, dtype=np.int64)


def _comm_device(ctx: DistContext):
    import torch
    return torch.device("cuda", ctx.device) if ctx.backend == "nccl" else torch.device("cpu")


_PINNED = {}


def _reduce_small(a: np.ndarray, ctx: DistContext, op) -> np.ndarray:
    """All-reduce of a small host array. Under RCCL the values travel through a cached pinned
    host buffer and device buffer (per device, dtype and length): pageable host<->device copies
    stage through the runtime and now and then stalled for milliseconds (the native solver's
    pageable source copies did, 1 step in 10-30 at +6 ms; tools/step_split.py)."""
    import torch
    import torch.distributed as dist
    dev = _comm_device(ctx)
    if dev.type != "cuda":
        t = torch.from_numpy(np.array(a, copy=True))
        dist.all_reduce(t, op=op)
        return t.numpy()
    key = (dev.index, a.dtype.str, a.shape[0])
    if key not in _PINNED:
        dt = torch.from_numpy(a[:0]).dtype
        _PINNED[key] = (torch.empty(a.shape[0], dtype=dt, pin_memory=True),
                        torch.empty(a.shape[0], dtype=dt, device=dev))
    h, d = _PINNED[key]
    h.numpy()[:] = a
    d.copy_(h, non_blocking=True)
    dist.all_reduce(d, op=op)
    h.copy_(d, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
    return h.numpy().copy()


def barrier(ctx: DistContext) -> None:
    if ctx.distributed:
        import torch.distributed as dist
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device])
        else:
            dist.barrier()


def broadcast_array(arr: Optional[np.ndarray], ctx: DistContext, dtype, count: int,
                    root: int = 0) -> np.ndarray:
    """Broadcast a host array from root (through device memory when the backend is RCCL)."""
    import torch
    import torch.distributed as dist

    if not ctx.distributed:
        return arr
    out = arr if ctx.rank == root else np.empty(count, dtype=dtype)
    dev = _comm_device(ctx)
    elems = max(1, CHUNK_BYTES // np.dtype(dtype).itemsize)
    for s in range(0, count, elems):
        e = min(count, s + elems)
        t = torch.from_numpy(np.ascontiguousarray(out[s:e])).to(dev)
        dist.broadcast(t, src=root)
        if ctx.rank != root:
            out[s:e] = t.cpu().numpy()
    return out


def broadcast_tensor_(t, ctx: DistContext, root: int = 0):
    """In-place chunked broadcast of a (device) tensor."""
    import torch.distributed as dist
    if not ctx.distributed:
        return t
    flat = t.view(-1)
    elems = max(1, CHUNK_BYTES // t.element_size())
    for s in range(0, flat.numel(), elems):
        dist.broadcast(flat[s:s + elems], src=root)
    return t


def broadcast_header(vals: Tuple[int, ...], ctx: DistContext, root: int = 0) -> Tuple[int, ...]:
    a = np.asarray(vals, dtype=np.int64) if ctx.rank == root else None
    return tuple(int(x) for x in broadcast_array(a, ctx, np.int64, len(vals), root))


def broadcast_queries(qs, ctx: DistContext, root: int = 0):
    """One packed blob instead of 2K+1 broadcasts (main.cu:257-280)."""
    from ..models.queries import QuerySet
    if not ctx.distributed:
        return qs
    K, nids = broadcast_header((qs.K, len(qs.ids)) if ctx.rank == root else (0, 0), ctx, root)
    off = broadcast_array(qs.off if ctx.rank == root else None, ctx, np.int64, K + 1, root)
    ids = broadcast_array(qs.ids if ctx.rank == root else None, ctx, np.int32, nids, root)
    return QuerySet(off, ids)


def broadcast_graph(g, ctx: DistContext, root: int = 0):
    """Replicate rank root's host Graph on every rank.

    RCCL backend: returns (rowptr, col) *device tensors* broadcast HBM -> HBM over xGMI;
    otherwise a host Graph. (The reference broadcasts pageable host vectors, main.cu:250,255.)
    """
    import torch
    from ..models.graph import Graph

    if not ctx.distributed:
        return g
    n, m, nnz = broadcast_header((g.n, g.m, g.nnz) if ctx.rank == root else (0, 0, 0), ctx, root)
    if ctx.backend == "nccl":
        dev = torch.device("cuda", ctx.device)
        if ctx.rank == root:
            rowptr = torch.from_numpy(g.rowptr).to(dev)
            col = torch.from_numpy(g.col).to(dev)
        else:
            rowptr = torch.empty(n + 1, dtype=torch.int64, device=dev)
            col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
        broadcast_tensor_(rowptr, ctx, root)
        if nnz:
            broadcast_tensor_(col, ctx, root)
        return rowptr, col, m
    rowptr = broadcast_array(g.rowptr if ctx.rank == root else None, ctx, np.int64, n + 1, root)
    col = broadcast_array(g.col if ctx.rank == root else None, ctx, np.int32, nnz, root)
    return Graph(n, rowptr, col, m=m)


def _qbits(K: int) -> int:
    b = 1
    while (1 << b) <= K:
        b += 1
    return b


def allreduce_max(x: float, ctx: DistContext) -> float:
    if not ctx.distributed:
        return float(x)
    import torch.distributed as dist
    return float(_reduce_small(np.array([float(x)], np.float64), ctx, dist.ReduceOp.MAX)[0])


def allreduce_sum_i64(a: np.ndarray, ctx: DistContext) -> np.ndarray:
    if not ctx.distributed:
        return a
    import torch.distributed as dist
    return _reduce_small(np.ascontiguousarray(a, dtype=np.int64), ctx, dist.ReduceOp.SUM)


def packed_argmin(F_local: np.ndarray, idx_local: np.ndarray, K: int, ctx: DistContext,
                  force_two_pass: bool = False) -> Tuple[int, int]:
    """Global (minK, minF) with the reference tie-break. (-1, -1) when K == 0 (main.cu:379-380).

    ONE all-reduce(MIN) of an int64 key 1 + (F << qbits | q). A rank whose F is too large to share
    62 bits with the query index sends key 0 instead, which every rank then sees as the MIN: all of
    them take the two-all-reduce fallback together.
    """
    F_local = np.asarray(F_local, dtype=np.int64)
    idx_local = np.asarray(idx_local, dtype=np.int64)
    qb = _qbits(K)
    NONE = np.iinfo(np.int64).max

    def allmin(v: int) -> int:
        if not ctx.distributed:
            return v
        import torch.distributed as dist
        return int(_reduce_small(np.array([v], np.int64), ctx, dist.ReduceOp.MIN)[0])

    maxF = int(F_local.max()) if len(F_local) else 0
    fits = qb < 62 and (maxF >> (62 - qb)) == 0
    key = 0 if force_two_pass else \
        allmin((1 + int(((F_local << qb) | idx_local).min()) if len(F_local) else NONE)
               if fits else 0)
    if key == NONE:
        return -1, -1
    if key > 0:
        key -= 1
        return int(key & ((1 << qb) - 1)), int(key >> qb)
    mf = allmin(int(F_local.min()) if len(F_local) else NONE)
    if mf == NONE:
        return -1, -1
    cand = idx_local[F_local == mf]
    mk = allmin(int(cand.min()) if len(cand) else NONE)
    return mk, mf


class AsyncArgmin:
    """packed_argmin in two halves: start() posts the step's 8-byte MIN all-reduce and returns at
    once; wait() gives (minK, minF). Between the two the next step's BFS runs (bench.py waits
    for step i's key after enqueueing step i + 1), so the reduction stays off the critical path.

    Under RCCL the key goes H2D, through the all-reduce and back D2H on a side stream of its own
    (non-blocking, never ordered against the solver's null-stream kernels). Two slots of pinned
    and device buffers alternate, so a new start() never rewrites a key still in flight. Under
    gloo it is an async host all-reduce. The reference runs MPI_Gather + MPI_Gatherv + a serial
    scan on rank 0 after all compute (main.cu:340-397).
    """

    def __init__(self, ctx: DistContext):
        self.ctx = ctx
        self.slot = 0
        self._bufs = None
        self._stream = None

    def start(self, F_local: np.ndarray, idx_local: np.ndarray, K: int):
        F_local = np.asarray(F_local, dtype=np.int64)
        idx_local = np.asarray(idx_local, dtype=np.int64)
        qb = _qbits(K)
        NONE = np.iinfo(np.int64).max
        maxF = int(F_local.max()) if len(F_local) else 0
        fits = qb < 62 and (maxF >> (62 - qb)) == 0
        key = ((1 + int(((F_local << qb) | idx_local).min())) if len(F_local) else NONE) \
            if fits else 0
        pend = {"F": F_local, "idx": idx_local, "K": K, "qb": qb, "key": key}
        if not self.ctx.distributed:
            return pend
        import torch
        import torch.distributed as dist

        dev = _comm_device(self.ctx)
        if dev.type != "cuda":
            t = torch.tensor([key], dtype=torch.int64)
            pend["work"] = dist.all_reduce(t, op=dist.ReduceOp.MIN, async_op=True)
            pend["t"] = t
            return pend
        if self._bufs is None:
            self._bufs = [(torch.empty(1, dtype=torch.int64, pin_memory=True),
                           torch.empty(1, dtype=torch.int64, device=dev)) for _ in range(2)]
            self._stream = torch.cuda.Stream(device=dev)
        h, d = self._bufs[self.slot]
        self.slot ^= 1
        h.numpy()[0] = key
        with torch.cuda.stream(self._stream):
            d.copy_(h, non_blocking=True)
            dist.all_reduce(d, op=dist.ReduceOp.MIN)
            h.copy_(d, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        pend["event"], pend["h"] = ev, h
        return pend

    def wait(self, pend) -> Tuple[int, int]:
        NONE = np.iinfo(np.int64).max
        key = pend["key"]
        if "event" in pend:
            pend["event"].synchronize()
            key = int(pend["h"].numpy()[0])
        elif "work" in pend:
            pend["work"].wait()
            key = int(pend["t"].numpy()[0])
        if key == NONE:
            return -1, -1
        if key > 0:
            key -= 1
            return int(key & ((1 << pend["qb"]) - 1)), int(key >> pend["qb"])
        # some rank's F does not fit next to the index: the two-pass form (every rank gets here)
        return packed_argmin(pend["F"], pend["idx"], pend["K"], self.ctx, force_two_pass=True)


def gather_F(F_local: np.ndarray, idx_local: np.ndarray, K: int, ctx: DistContext) -> np.ndarray:
    """Full F vector on every rank (replaces MPI_Gather + MPI_Gatherv, main.cu:340-365)."""
    full = np.zeros(K, dtype=np.int64)
    full[np.asarray(idx_local, dtype=np.int64)] = F_local
    return allreduce_sum_i64(full, ctx)


def allgather_int(x: int, ctx: DistContext) -> list:
    """Every rank's value of x, in rank order (e.g. the GPU ordinal each rank drives)."""
    if not ctx.distributed:
        return [int(x)]
    vec = np.zeros(ctx.world, dtype=np.int64)
    vec[ctx.rank] = int(x)
    return [int(v) for v in allreduce_sum_i64(vec, ctx)]


def agree_ok(ok: bool, ctx: DistContext) -> bool:
    """True on every rank iff ok is True on every rank (one MAX all-reduce)."""
    return allreduce_max(0.0 if ok else 1.0, ctx) == 0.0


def checked(fn, ctx: DistContext, what: str = "step"):
    """Run a rank-local piece of work (no collectives inside) and agree on its success before
    anyone moves on to the next collective: a failure on one rank raises on EVERY rank instead
    of leaving the others blocked in a collective the failed rank never joins."""
    err, out = None, None
    try:
        out = fn()
    except Exception as e:  # noqa: BLE001
        err = e
    if not agree_ok(err is None, ctx):
        if err is not None:
            raise err
        raise RuntimeError(f"{what} failed on another rank")
    return out


def evaluate_candidates(candidates, run, reference, ctx: DistContext, reps: int = 1,
                        required: str = "roundrobin", sync=None):
    """Time each decomposition candidate (untimed selection pass of bench.py) and drop the ones
    that fail, collectively: every rank reaches the same decisions, so no rank is ever left
    alone in a collective the others skipped.

    run(name) -> (F_full, stats) executes one step of candidate `name` and returns the GATHERED
    F vector (identical on every rank); reference is the F vector it must equal. run must wrap
    its rank-local work in checked() (between collectives), so that a failure surfaces on every
    rank at the same point. A candidate
    that raises on any rank, or whose F differs, is excluded and its reason recorded. Returns
    (ms, errors): ms[name] = best wall ms over `reps` runs (max over ranks), errors[name] =
    reason. The `required` candidate (round robin, the reference's own decomposition,
    main.cu:303-307) failing is reported to the caller, who must not time anything else.
    """
    import time
    ms, errors = {}, {}
    for name in candidates:
        for _ in range(max(1, reps)):
            err, dt, F = "", 0.0, None
            try:
                barrier(ctx)
                if sync:
                    sync()
                t = time.perf_counter()
                F, _ = run(name)
                if sync:
                    sync()
                dt = time.perf_counter() - t
            except Exception as e:  # noqa: BLE001 (any failure excludes the candidate)
                err = f"{type(e).__name__}: {e}"[:240]
            if not agree_ok(not err, ctx):
                errors[name] = err or "failed on another rank"
                break
            t_max = allreduce_max(dt, ctx) * 1e3
            if not np.array_equal(np.asarray(F), np.asarray(reference)):
                bad = np.flatnonzero(np.asarray(F) != np.asarray(reference))[:4]
                errors[name] = f"F differs from the round-robin pass at groups {bad.tolist()}"
                break
            ms[name] = min(ms.get(name, t_max), t_max)
        if name in errors:
            ms.pop(name, None)
    return ms, errors
