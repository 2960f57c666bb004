"""Hybrid multi-GPU decomposition (parallel/hybrid.py): levels 1-2 vertex-partitioned over ranks,
one all-to-all of visited words, the rest query-partitioned. Must give the exact F of the
single-process solver for every rank count, group count and graph shape.

CPU tests pin the exchange layout (numpy twins of the pack kernel and of all_to_all_single, and a
real gloo all_to_all_single with the same split sizes); GPU tests run all ranks' phases in one
process (emulate_ranks) and compare with the standard bit-parallel solver."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _H():
    from msbfs.parallel import hybrid
    return hybrid


@pytest.mark.parametrize("K,world", [(1024, 8), (1024, 3), (100, 4), (64, 8), (700, 5), (1, 1)])
def test_word_split_and_exchange_layout(K, world):
    H = _H()
    wbeg = H.word_split(K, world)
    wt = (K + 63) // 64
    assert wbeg[0] == 0 and wbeg[-1] == wt and np.all(np.diff(wbeg) >= 0)
    owned = np.concatenate([H.own_groups(K, wbeg, r) for r in range(world)])
    assert np.array_equal(owned, np.arange(K))  # every group exactly once, in order
    rng = np.random.default_rng(K + world)
    n = 257
    W = 1
    while W < wt:
        W *= 2
    vis = rng.integers(0, 2**63, size=(n, W), dtype=np.uint64)
    for n_eff in (n, n - 40, 3):  # rows >= n_eff (isolated-vertex suffix) are not exchanged
        sends = [H.pack_words_np(vis, r, world, n_eff, wbeg) for r in range(world)]
        assert sum(H.part_count(n_eff, r, world) for r in range(world)) == n_eff
        for r in range(world):
            ss, rs = H.split_sizes(n_eff, wbeg, r)
            assert sum(ss) == len(sends[r])
        recvs = H.all_to_all_np(sends, n_eff, wbeg)
        for j in range(world):
            nw = int(wbeg[j + 1] - wbeg[j])
            _, rs = H.split_sizes(n_eff, wbeg, j)
            assert len(recvs[j]) == sum(rs) == n_eff * nw
            # rank j holds its words of every vertex (the phase-C input, k_hybrid_setup order)
            rows = H.unpack_np(recvs[j], n, n_eff, world, nw)
            want = vis[:, wbeg[j]:wbeg[j + 1]].copy()
            want[n_eff:] = 0
            assert np.array_equal(rows, want)


@pytest.mark.parametrize("K,world,chunks", [(1024, 8, 4), (700, 3, 5), (64, 4, 2), (300, 1, 3)])
def test_chunked_exchange_layout(K, world, chunks):
    """The overlapped exchange's pieces (chunk_views: piece c carries every rank's own-vertex
    range c, any monotone split, some pieces empty) deliver exactly the dense all-to-all: every
    word lands where k_hybrid_setup reads it."""
    import torch
    H = _H()
    wbeg = H.word_split(K, world)
    wt = int(wbeg[-1])
    rng = np.random.default_rng(K + world + chunks)
    n, n_eff = 301, 290
    vis = rng.integers(0, 2**62, size=(n, 16), dtype=np.uint64)
    pc = [H.part_count(n_eff, r, world) for r in range(world)]
    # per-rank bounds: uneven, an empty piece in the middle where possible
    bounds = np.zeros((world, chunks + 1), dtype=np.int64)
    for r in range(world):
        cuts = np.sort(rng.integers(0, pc[r] + 1, size=chunks - 1))
        if chunks > 2:
            cuts[1] = cuts[0]
        bounds[r, 1:-1] = cuts
        bounds[r, -1] = pc[r]
    sends = [torch.from_numpy(H.pack_words_np(vis, r, world, n_eff, wbeg).view(np.int64))
             for r in range(world)]
    want = H.all_to_all_np([x.numpy().view(np.uint64) for x in sends], n_eff, wbeg)
    recvs = [torch.full((max(1, len(want[j])),), -1, dtype=torch.int64) for j in range(world)]
    for c in range(chunks):
        views = [H.chunk_views(sends[r], recvs[r], pc[r], wbeg, r, pc, bounds, c)
                 for r in range(world)]
        for j in range(world):  # emulated all_to_all of piece c
            for r in range(world):
                ins_r, _ = views[r]
                _, outs_j = views[j]
                assert outs_j[r].numel() == ins_r[j].numel()
                outs_j[r].copy_(ins_r[j])
    for j in range(world):
        got = recvs[j].numpy().view(np.uint64)[:len(want[j])]
        assert np.array_equal(got, want[j]), (j, wt)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _a2a_worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from msbfs.parallel import distributed as D
    from msbfs.parallel import hybrid as H
    ctx = D.init_from_env(backend="gloo", use_gpu=False)
    K, n, n_eff = 700, 101, 90
    wbeg = H.word_split(K, world)
    rng = np.random.default_rng(5)
    vis = rng.integers(0, 2**62, size=(n, 16), dtype=np.uint64)
    send = H.pack_words_np(vis, rank, world, n_eff, wbeg)
    ss, rs = H.split_sizes(n_eff, wbeg, rank)
    r = torch.empty(sum(rs), dtype=torch.int64)
    dist.all_to_all_single(r, torch.from_numpy(send.view(np.int64)), rs, ss)
    np.save(os.path.join(out_dir, f"a2a{rank}.npy"), r.numpy())
    D.shutdown(ctx)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_all_to_all_matches_emulation(tmp_path, world):
    H = _H()
    mp.spawn(_a2a_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    K, n, n_eff = 700, 101, 90
    wbeg = H.word_split(K, world)
    rng = np.random.default_rng(5)
    vis = rng.integers(0, 2**62, size=(n, 16), dtype=np.uint64)
    for j in range(world):
        nw = int(wbeg[j + 1] - wbeg[j])
        got = np.load(tmp_path / f"a2a{j}.npy").view(np.uint64)
        want = vis[:, wbeg[j]:wbeg[j + 1]].copy()
        want[n_eff:] = 0
        assert np.array_equal(H.unpack_np(got, n, n_eff, world, nw), want)


def _pieces_worker(rank, world, port, chunks, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    from msbfs.parallel import distributed as D
    from msbfs.parallel import hybrid as H
    ctx = D.init_from_env(backend="gloo", use_gpu=False)
    K, n, n_eff = 700, 301, 290
    wbeg = H.word_split(K, world)
    rng = np.random.default_rng(11)
    vis = rng.integers(0, 2**62, size=(n, 16), dtype=np.uint64)
    pc = [H.part_count(n_eff, r, world) for r in range(world)]
    bounds = np.zeros((world, chunks + 1), dtype=np.int64)  # (uneven, some pieces empty)
    for r in range(world):
        cuts = np.sort(rng.integers(0, pc[r] + 1, size=chunks - 1))
        if chunks > 2:
            cuts[1] = cuts[0]
        bounds[r, 1:-1] = cuts
        bounds[r, -1] = pc[r]
    send = torch.from_numpy(H.pack_words_np(vis, rank, world, n_eff, wbeg).view(np.int64))
    _, rs = H.split_sizes(n_eff, wbeg, rank)
    recv = torch.full((max(1, sum(rs)),), -1, dtype=torch.int64)
    ex = H.PieceExchange(ctx, send, recv, pc[rank], wbeg, pc, bounds, chunks)
    for step in range(2):
        recv.fill_(-1)
        order = ex.order()
        if step == 1 and rank == world - 1:
            for c in order[:2]:  # a rank that "failed" after two pieces makes up the rest
                ex.start(c)
            ex.start_missing()
        else:
            for c in order:
                ex.start(c)
        ex.finish()
        np.save(os.path.join(out_dir, f"p{rank}_{step}.npy"), recv.numpy()[:sum(rs)])
    D.shutdown(ctx)


@pytest.mark.parametrize("world,chunks", [(2, 4), (3, 8), (3, 1)])
def test_gloo_piece_exchange(tmp_path, world, chunks):
    """The overlapped exchange's point-to-point pieces (PieceExchange: batch_isend_irecv, the
    same calls under gloo as under RCCL) deliver exactly the dense all-to-all, also when one
    rank starts its last pieces through start_missing (the checked-mode recovery path)."""
    H = _H()
    mp.spawn(_pieces_worker, args=(world, _free_port(), chunks, str(tmp_path)), nprocs=world,
             join=True)
    K, n, n_eff = 700, 301, 290
    wbeg = H.word_split(K, world)
    rng = np.random.default_rng(11)
    vis = rng.integers(0, 2**62, size=(n, 16), dtype=np.uint64)
    want = H.all_to_all_np([H.pack_words_np(vis, r, world, n_eff, wbeg) for r in range(world)],
                           n_eff, wbeg)
    for j in range(world):
        for step in range(2):
            got = np.load(tmp_path / f"p{j}_{step}.npy").view(np.uint64)
            assert np.array_equal(got, want[j]), (j, step)


def test_word_codec_roundtrip():
    """Zero-word coding of one exchange segment: bitmap words + nonzero words, exact round trip,
    never larger than coded_bound (the buffer size the runner allocates)."""
    H = _H()
    rng = np.random.default_rng(1)
    for L in (0, 1, 5, 63, 64, 65, 127, 128, 129, 1000):
        for dens in (0.0, 0.02, 0.5, 1.0):
            w = rng.integers(1, 2**64 - 1, size=L, dtype=np.uint64, endpoint=True)
            w[rng.random(L) >= dens] = 0
            c = H.encode_np(w)
            nch = (L + 63) // 64
            assert len(c) == nch + np.count_nonzero(w) <= H.coded_bound(L)
            assert np.array_equal(H.decode_np(c, L), w)
    # the bitmap is little-endian within a word: word 64c + i -> bit i of bitmap word c
    w = np.zeros(70, np.uint64)
    w[[0, 63, 64, 69]] = [5, 6, 7, 8]
    c = H.encode_np(w)
    assert int(c[0]) == (1 | (1 << 63)) and int(c[1]) == (1 | (1 << 5))
    assert list(c[2:]) == [5, 6, 7, 8]
    with pytest.raises(ValueError):
        H.decode_np(c[:-1], 70)


def _coded_worker(rank, world, port, out_dir):
    """The runner's coded protocol over gloo with numpy twins of the kernels: one SUM all-reduce
    of the coded-length matrix, an all-to-all of the coded segments, per-source decode."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from msbfs.parallel import distributed as D
    from msbfs.parallel import hybrid as H
    ctx = D.init_from_env(backend="gloo", use_gpu=False)
    K, n, n_eff = 700, 301, 290
    wbeg = H.word_split(K, world)
    rng = np.random.default_rng(9)
    vis = rng.integers(0, 2**62, size=(n, 16), dtype=np.uint64)
    vis[rng.random((n, 16)) < 0.6] = 0
    dense = H.pack_words_np(vis, rank, world, n_eff, wbeg)
    ss, rs = H.split_sizes(n_eff, wbeg, rank)
    offs = np.concatenate([[0], np.cumsum(ss)])
    segs = [H.encode_np(dense[offs[j]:offs[j + 1]]) for j in range(world)]
    M = np.zeros((world, world), np.int64)
    M[rank] = [len(x) for x in segs]
    t = torch.from_numpy(M.reshape(-1))
    dist.all_reduce(t)
    M = t.numpy().reshape(world, world)
    ssz, rsz = [int(x) for x in M[rank]], [int(x) for x in M[:, rank]]
    r = torch.empty(sum(rsz), dtype=torch.int64)
    dist.all_to_all_single(r, torch.from_numpy(np.concatenate(segs).view(np.int64)), rsz, ssz)
    got, o = [], 0
    for src in range(world):
        got.append(H.decode_np(r.numpy()[o:o + rsz[src]].view(np.uint64), rs[src]))
        o += rsz[src]
    np.save(os.path.join(out_dir, f"c{rank}.npy"), np.concatenate(got))
    np.save(os.path.join(out_dir, f"b{rank}.npy"), np.array([sum(ssz), sum(ss)]))
    D.shutdown(ctx)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_coded_exchange(tmp_path, world):
    H = _H()
    mp.spawn(_coded_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    K, n, n_eff = 700, 301, 290
    wbeg = H.word_split(K, world)
    rng = np.random.default_rng(9)
    vis = rng.integers(0, 2**62, size=(n, 16), dtype=np.uint64)
    vis[rng.random((n, 16)) < 0.6] = 0
    for j in range(world):
        nw = int(wbeg[j + 1] - wbeg[j])
        got = np.load(tmp_path / f"c{j}.npy")
        want = vis[:, wbeg[j]:wbeg[j + 1]].copy()
        want[n_eff:] = 0
        assert np.array_equal(H.unpack_np(got, n, n_eff, world, nw), want)
        coded, dense = np.load(tmp_path / f"b{j}.npy")
        assert coded < 0.5 * dense  # 60 % zero words: the coded exchange moves < half the bytes


# ---------------------------------------------------------------------------------------------
# GPU: emulated ranks in one process vs the standard solver
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("K", [1024, 300, 64, 5])
def test_hybrid_matches_solver_rmat(msbfs_pkg, world, K):
    m = msbfs_pkg
    H = _H()
    dg = m.DeviceGraph.rmat(14, 16, 3, device=0, relabel=True)
    qs = m.QuerySet.random(dg.n, K, 16, seed=K + world)
    with m.Solver(dg, "bitpar", max_groups=K) as s:
        ref = s.run(qs).F
        got = H.emulate_ranks(s, qs, world)  # dense exchange (the default)
        assert np.array_equal(got, ref), (world, K)
        # zero-word coded exchange, decoded on the GPU
        assert np.array_equal(H.emulate_ranks(s, qs, world, coded=True), ref), (world, K)
        # buffers are reused: the standard path still works after hybrid phases
        assert np.array_equal(s.run(qs).F, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("wbeg", [[0, 3, 5, 7, 9, 11, 13, 15, 16], [0, 1, 1, 8, 9, 12, 14, 15, 16],
                                  [0, 0, 16, 16, 16, 16, 16, 16, 16]])
def test_hybrid_uneven_word_split(msbfs_pkg, wbeg):
    """Uneven word splits (tools/hybrid_balance.py 'uneven': fewer words for the rank with the
    latest groups), including ranks that own no word: every rank still runs phase A over its
    vertices and exchanges, the F is the solver's (dense and coded exchange, chunked pieces)."""
    m = msbfs_pkg
    H = _H()
    dg = m.DeviceGraph.rmat(14, 16, 3, device=0, relabel=True)
    qs = m.QuerySet.random(dg.n, 1024, 16, seed=41)
    with m.Solver(dg, "bitpar", max_groups=1024) as s:
        ref = s.run(qs).F
        wb = np.array(wbeg, dtype=np.int32)
        assert np.array_equal(H.emulate_ranks(s, qs, 8, wbeg=wb), ref)
        assert np.array_equal(H.emulate_ranks(s, qs, 8, wbeg=wb, coded=True), ref)
        assert np.array_equal(H.emulate_ranks(s, qs, 8, wbeg=wb, chunks=4), ref)
        with pytest.raises(ValueError):
            H.emulate_ranks(s, qs, 8, wbeg=wb[:-1])


@pytest.mark.gpu
@pytest.mark.parametrize("world,K", [(8, 1024), (3, 700), (2, 5)])
def test_hybrid_coded_send_matches_numpy_codec(msbfs_pkg, world, K):
    """k_code_bits/k_code_emit vs encode_np of the dense phase-A send segments, and the GPU
    decode of every rank's received segments vs the dense exchange."""
    import torch
    m = msbfs_pkg
    H = _H()
    dg = m.DeviceGraph.rmat(14, 16, 5, device=0, relabel=True)
    qs = m.QuerySet.random(dg.n, K, 16, seed=world)
    n_eff = dg.hybrid_extent()
    wbeg = H.word_split(K, world)
    dev = torch.device("cuda", 0)
    with m.Solver(dg, "bitpar", max_groups=K) as s:
        dense_sends, coded_sends, lens = [], [], []
        for r in range(world):
            ss, _ = H.split_sizes(n_eff, wbeg, r)
            bd = torch.empty(max(1, sum(ss)), dtype=torch.int64, device=dev)
            s.hybrid_phase_a(qs, r, world, n_eff, r == 0, wbeg, bd.data_ptr())
            bc = torch.empty(max(1, sum(H.coded_bound(x) for x in ss)), dtype=torch.int64,
                             device=dev)
            out, sa = s.hybrid_phase_a(qs, r, world, n_eff, r == 0, wbeg, bc.data_ptr(),
                                       coded=True)
            cl = [int(x) for x in sa["coded_len"]]
            d = bd[:sum(ss)].cpu().numpy().view(np.uint64)
            c = bc[:sum(cl)].cpu().numpy().view(np.uint64)
            do, co = np.concatenate([[0], np.cumsum(ss)]), np.concatenate([[0], np.cumsum(cl)])
            for j in range(world):
                assert np.array_equal(c[co[j]:co[j + 1]], H.encode_np(d[do[j]:do[j + 1]])), (r, j)
            dense_sends.append(d)
            coded_sends.append(c)
            lens.append(cl)
        recvs = H.all_to_all_np(dense_sends, n_eff, wbeg)
        for j in range(world):
            nw = int(wbeg[j + 1] - wbeg[j])
            if nw == 0:
                continue
            parts = [coded_sends[r][sum(lens[r][:j]):sum(lens[r][:j + 1])] for r in range(world)]
            rc = torch.from_numpy(np.concatenate(parts).view(np.int64)).to(dev)
            out = torch.full((max(1, len(recvs[j])),), -1, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            s.hybrid_decode(rc.data_ptr(), np.array([lens[r][j] for r in range(world)]), world,
                            n_eff, nw, out.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(out[:len(recvs[j])].cpu().numpy().view(np.uint64), recvs[j]), j


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_hybrid_matches_cpu_other_graphs(msbfs_pkg, world):
    """Small components, isolated vertices, invalid source ids, groups that finish before
    level 2, high-diameter grids."""
    m = msbfs_pkg
    H = _H()
    graphs = [m.Graph.uniform(5000, 2500, 4), m.Graph.grid(40, 60, 0.9, 5, 2),
              m.Graph.rmat(11, 4, 7)]
    for g in graphs:
        qs = m.QuerySet.random(g.n, 200, 3, seed=world)
        qs = m.QuerySet.from_groups([list(x) + [-1, g.n + 5] for x in qs.groups()] + [[-3], []])
        ref = m.cpu_bfs(g, qs)
        with m.Solver(g.to_device(0), "bitpar", max_groups=qs.K) as s:
            assert np.array_equal(H.emulate_ranks(s, qs, world), ref.F)


@pytest.mark.gpu
def test_hybrid_tiled_phase_a(msbfs_pkg):
    """Phase A's level 2 over the static tiles of each rank's strided vertex set (RMAT-23: large
    enough for the prefix pull; one tile set per emulated rank): F equal to the standard solver
    with the tiles on and off, for several rank counts in a row (cached tile sets reused)."""
    m = msbfs_pkg
    H = _H()
    dg = m.DeviceGraph.rmat(23, 16, 5, device=0, relabel=True)
    qs = m.QuerySet.random(dg.n, 1024, 16, seed=23)
    with m.Solver(dg, "bitpar", max_groups=1024, tuning={"tiles": 0}) as s:
        ref = s.run(qs).F
    with m.Solver(dg, "bitpar", max_groups=1024) as s:
        assert np.array_equal(s.run(qs).F, ref)
        for world in (2, 3, 8, 2):
            assert np.array_equal(H.emulate_ranks(s, qs, world), ref), world
        # the overlapped exchange: phase A's tiled level 2 in vertex ranges, each packed as soon
        # as it is final (the pieces' ready times are recorded, in order)
        for world, chunks in ((8, 4), (3, 7), (1, 2)):
            tim = []
            assert np.array_equal(H.emulate_ranks(s, qs, world, timings=tim, chunks=chunks),
                                  ref), (world, chunks)
            for x in tim:
                ready = [p[0] for p in x["pieces"]]
                assert len(ready) == chunks and ready == sorted(ready)
                assert sum(p[1] for p in x["pieces"]) == x["dense_send_bytes"]
            b = s.hybrid_chunk_bounds(0, world, dg.hybrid_extent(), chunks)
            assert b[0] == 0 and b[-1] == H.part_count(dg.hybrid_extent(), 0, world)
            assert np.all(np.diff(b) >= 0) and len(b) == chunks + 1
    # tiles from 4 words (tuning tiles_w = 4, 256 groups): the exchange ranges must start at
    # tile starts for that word count too (a range split inside a tile would send rows that the
    # next launch still changes), chunked and not
    qs4 = qs.subset(np.arange(256))
    with m.Solver(dg, "bitpar", max_groups=256, tuning={"tiles": 0}) as s:
        ref4 = s.run(qs4).F
    with m.Solver(dg, "bitpar", max_groups=256, tuning={"tiles_w": 4}) as s:
        s.prepare()
        for world, chunks in ((8, 4), (3, 5), (2, 1)):
            assert np.array_equal(H.emulate_ranks(s, qs4, world, chunks=chunks), ref4), (world,
                                                                                     chunks)
    dg.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,chunks", [(4, 3), (2, 5), (8, 2)])
def test_hybrid_chunked_small_graph(msbfs_pkg, world, chunks):
    """Chunked phase A on a graph too small for the tiled pull: the ranges are packed and handed
    out after the level (same callbacks, same answers)."""
    m = msbfs_pkg
    H = _H()
    dg = m.DeviceGraph.rmat(14, 16, 3, device=0, relabel=True)
    qs = m.QuerySet.random(dg.n, 700, 8, seed=9)
    with m.Solver(dg, "bitpar", max_groups=1024) as s:
        ref = s.run(qs).F
        tim = []
        assert np.array_equal(H.emulate_ranks(s, qs, world, timings=tim, chunks=chunks), ref)
        assert all(len(x["pieces"]) == chunks for x in tim)
        # one process, HybridRunner's own chunked path (local copies per piece)
        r = H.HybridRunner(s, qs.K, H.D.DistContext(device=0), chunks=chunks).run(qs)
        assert np.array_equal(r.F, ref) and r.stats["chunks"] == chunks


@pytest.mark.gpu
def test_hybrid_lazy_reset_with_stale_rows(msbfs_pkg):
    """Phase A skips the visited-buffer fill (k_zero_part_rows + the top-down anyvis guard): run
    it over buffers full of another query set's rows (a normal run, then other phases) and check
    every result against the filled variant (tuning lazy=0) and the standard solver; the coded
    exchange stages its dense segments in the other visited buffer, which the next runs must not
    depend on."""
    m = msbfs_pkg
    H = _H()
    dg = m.DeviceGraph.rmat(15, 16, 11, device=0, relabel=True)
    qa = m.QuerySet.random(dg.n, 1024, 16, seed=3)
    qb = m.QuerySet.random(dg.n, 700, 4, seed=4)
    with m.Solver(dg, "bitpar", max_groups=1024) as s:
        ref_a, ref_b = s.run(qa).F, s.run(qb).F
        for world in (8, 3, 8):
            assert np.array_equal(H.emulate_ranks(s, qa, world), ref_a), world
            assert np.array_equal(H.emulate_ranks(s, qb, world), ref_b), world
            assert np.array_equal(H.emulate_ranks(s, qa, world, coded=True), ref_a), world
        assert np.array_equal(s.run(qa).F, ref_a)
        assert np.array_equal(s.run(qb).F, ref_b)
    with m.Solver(dg, "bitpar", max_groups=1024, tuning={"lazy": 0}) as s:
        assert np.array_equal(H.emulate_ranks(s, qb, 4), ref_b)


@pytest.mark.gpu
def test_hybrid_runner_single_process(msbfs_pkg):
    m = msbfs_pkg
    H = _H()
    dg = m.DeviceGraph.rmat(13, 16, 2, device=0, relabel=True)
    qs = m.QuerySet.random(dg.n, 512, 8, seed=1)
    with m.Solver(dg, "bitpar", max_groups=qs.K) as s:
        ref = s.run(qs).F
        res = H.hybrid_bfs(s, qs)
        assert np.array_equal(res.idx, np.arange(qs.K))
        assert np.array_equal(res.F, ref)
        coded = H.HybridRunner(s, qs.K, H.D.DistContext(device=0), coded=True).run(qs)
        assert np.array_equal(coded.F, ref) and coded.stats["coded"]
