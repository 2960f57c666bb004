"""Multi-process (gloo, CPU) coverage of the torch.distributed layer and the end-to-end engine:
every world size must produce the identical report (round-robin invariance, main.cu:305)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, gp, qp, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import msbfs
    from msbfs.parallel import distributed as D
    ctx = D.init_from_env(backend="gloo", use_gpu=False)
    assert ctx.world == world and ctx.rank == rank
    # primitives
    qs = msbfs.QuerySet.from_file(qp) if rank == 0 else None
    qs = D.broadcast_queries(qs, ctx)
    g = msbfs.Graph.from_file(gp) if rank == 0 else None
    g = D.broadcast_graph(g, ctx)
    idx = D.round_robin(qs.K, rank, world)
    r = msbfs.cpu_bfs(g, qs.subset(idx), count_edges=True)
    k, f = D.packed_argmin(r.F, idx, qs.K, ctx)
    F = D.gather_F(r.F, idx, qs.K, ctx)
    # end-to-end engine
    eng = msbfs.Engine(msbfs.JobConfig(graph=gp, query=qp, algo="cpu", count_edges=True), ctx)
    eng.preprocess()
    res = eng.compute(gather=True)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), k=k, f=f, F=F, ek=res.min_k, ef=res.min_f,
             eF=res.F, edges=res.traversed_edges, n=g.n)
    D.shutdown(ctx)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_gloo_world_sizes(tmp_path, msbfs_pkg, world):
    m = msbfs_pkg
    g = m.Graph.rmat(10, 8, 1)
    qs = m.QuerySet.random(g.n, 7, 3, 2)
    gp, qp = str(tmp_path / "g.bin"), str(tmp_path / "q.bin")
    g.write(gp)
    qs.write(qp)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    mp.spawn(_worker, args=(world, _free_port(), gp, qp, str(tmp_path)), nprocs=world, join=True)
    k = m.argmin_first(ref.F)
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert int(z["n"]) == g.n
        assert int(z["k"]) == k and int(z["f"]) == ref.F[k]
        assert int(z["ek"]) == k and int(z["ef"]) == ref.F[k]
        assert np.array_equal(z["F"], ref.F) and np.array_equal(z["eF"], ref.F)
        assert int(z["edges"]) == int(ref.edges.sum())


def test_packed_argmin_tiebreak_and_fallback():
    from msbfs.parallel import distributed as D
    ctx = D.DistContext()
    assert D.packed_argmin(np.array([5, 3, 3, 9]), np.array([0, 1, 2, 3]), 4, ctx) == (1, 3)
    assert D.packed_argmin(np.array([], np.int64), np.array([], np.int64), 0, ctx) == (-1, -1)
    big = np.array([2 ** 61, 2 ** 61, 2 ** 62], np.int64)  # too large to pack next to q
    assert D.packed_argmin(big, np.array([7, 3, 1]), 8, ctx) == (3, 2 ** 61)
    assert list(D.round_robin(10, 2, 4)) == [2, 6]


def _argmin_worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from msbfs.parallel import distributed as D
    ctx = D.init_from_env(backend="gloo", use_gpu=False)
    K = 6
    F = np.array([9, 4, 2 ** 61, 4, 7, 4], np.int64)  # ties at q = 1, 3, 5
    res, pend = [], []
    amin = D.AsyncArgmin(ctx)
    for case in ("fit", "mixed", "empty-rank"):
        idx = D.round_robin(K, rank, world)
        Fl = F[idx].copy()
        if case == "fit":
            Fl[Fl > 100] = 50
        if case == "empty-rank" and rank == 1:
            idx, Fl = idx[:0], Fl[:0]
        res.append(D.packed_argmin(Fl, idx, K, ctx))
        pend.append(amin.start(Fl, idx, K))  # (several keys in flight at once)
    res += [amin.wait(p) for p in pend]
    np.save(os.path.join(out_dir, f"a{rank}.npy"), np.array(res, np.int64))
    D.shutdown(ctx)


def test_packed_argmin_gloo_mixed_fallback(tmp_path):
    """One rank's F too large to pack: every rank must take the fallback together (one MIN
    all-reduce decides it) and agree on the reference's lowest-index tie-break. The async form
    (AsyncArgmin, bench.py's timed loop) gives the same answers with several keys in flight."""
    mp.spawn(_argmin_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        got = [tuple(x) for x in np.load(tmp_path / f"a{r}.npy")]
        # rank 0 holds q = 0, 2, 4; rank 1 holds q = 1, 3, 5 (round robin)
        assert got == [(1, 4), (1, 4), (4, 7)] * 2, got


def test_async_argmin_single_process_and_pg_timeout(monkeypatch):
    from msbfs.parallel import distributed as D
    amin = D.AsyncArgmin(D.DistContext())
    p = amin.start(np.array([5, 3, 3, 9]), np.array([0, 1, 2, 3]), 4)
    assert amin.wait(p) == (1, 3)
    p = amin.start(np.array([2 ** 61, 2 ** 61]), np.array([7, 3]), 8)
    assert amin.wait(p) == (3, 2 ** 61)
    assert amin.wait(amin.start(np.array([], np.int64), np.array([], np.int64), 0)) == (-1, -1)
    monkeypatch.delenv("MSBFS_PG_TIMEOUT", raising=False)
    assert D.pg_timeout_s() == 180
    monkeypatch.setenv("MSBFS_PG_TIMEOUT", "30")
    assert D.pg_timeout_s() == 30
    monkeypatch.setenv("MSBFS_PG_TIMEOUT", "0")
    with pytest.raises(ValueError):
        D.pg_timeout_s()
