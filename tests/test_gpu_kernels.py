"""GPU numerics: every device algorithm against the CPU oracle (exact integer F and edges)."""
import numpy as np
import pytest

from golden import CASES

pytestmark = pytest.mark.gpu

DEVICE_ALGOS = ["bitpar", "dist", "topdown", "sweep"]


def _graphs(m):
    gs = [
        ("rmat10", m.Graph.rmat(10, 16, 3)),
        ("rmat12", m.Graph.rmat(12, 8, 5)),
        ("uniform", m.Graph.uniform(3000, 9000, 11)),
        ("grid", m.Graph.grid(40, 60, 0.9, 5, 2)),
        ("sparse", m.Graph.uniform(5000, 2500, 4)),  # many small components + isolated vertices
    ]
    return gs


@pytest.mark.parametrize("algo", DEVICE_ALGOS)
def test_golden_cases(msbfs_pkg, algo):
    m = msbfs_pkg
    for (n, edges), groups, F, k, minf in CASES:
        u = np.array([e[0] for e in edges], np.int32)
        v = np.array([e[1] for e in edges], np.int32)
        g = m.Graph.from_edges(n, u, v)
        qs = m.QuerySet.from_groups(groups)
        r = m.multi_source_bfs(g, qs, algo=algo)
        assert list(r.F) == F
        kk = m.argmin_first(r.F)
        assert kk + 1 == k and (r.F[kk] if kk >= 0 else -1) == minf


@pytest.mark.parametrize("algo", DEVICE_ALGOS)
def test_algos_match_cpu(msbfs_pkg, algo):
    m = msbfs_pkg
    for name, g in _graphs(m):
        qs = m.QuerySet.random(g.n, 70 if algo == "bitpar" else 9, 3, seed=len(name))
        ref = m.cpu_bfs(g, qs, count_edges=True)
        with m.Solver(g.to_device(0), algo, max_groups=qs.K) as s:
            r = s.run(qs, count_edges=True)
        assert np.array_equal(r.F, ref.F), (name, algo)
        assert np.array_equal(r.edges, ref.edges), (name, algo)


@pytest.mark.parametrize("K", [1, 63, 64, 65, 130, 300, 700, 1024, 1500])
def test_bitpar_batch_widths(msbfs_pkg, K):
    m = msbfs_pkg
    g = m.Graph.rmat(11, 16, 9)
    qs = m.QuerySet.random(g.n, K, 2, seed=K)
    ref = m.cpu_bfs(g, qs)
    with m.Solver(g.to_device(0), "bitpar", max_groups=K) as s:
        assert np.array_equal(s.run(qs).F, ref.F)


@pytest.mark.parametrize("force_dir,wide", [(1, 64), (2, 64), (0, 4), (2, 1), (0, 100000)])
def test_bitpar_direction_variants(msbfs_pkg, force_dir, wide):
    m = msbfs_pkg
    for name, g in _graphs(m)[:4]:
        qs = m.QuerySet.random(g.n, 200, 5, seed=3)
        ref = m.cpu_bfs(g, qs, count_edges=True)
        with m.Solver(g.to_device(0), "bitpar", max_groups=qs.K, force_dir=force_dir,
                      wide_degree=wide) as s:
            r = s.run(qs, count_edges=True)
        assert np.array_equal(r.F, ref.F), (name, force_dir, wide)
        assert np.array_equal(r.edges, ref.edges)


@pytest.mark.parametrize("wide", [2, 4, 16])
def test_bitpar_two_pass_chunks(msbfs_pkg, wide):
    """chunk2: the wide vertices of the early-exit pull levels pull their first chunk, then only
    the open ones the rest (k_chunk_first / k_chunk_rest_count / k_chunk_rest_desc). Small
    wide_degree thresholds put most vertices on the wide list (several chunks each with kChunk
    = 1024 only for the hubs); exact F against the CPU oracle, with the lean pass forced on."""
    m = msbfs_pkg
    for name, g in _graphs(m)[:4] + [("rmat14", m.Graph.rmat(14, 16, 5))]:
        qs = m.QuerySet.random(g.n, 300, 4, seed=wide)
        ref = m.cpu_bfs(g, qs)
        for tun in ({"chunk2": 1}, {"chunk2": 1, "lean_min": 0}, {"chunk2": 0}):
            with m.Solver(g.to_device(0), "bitpar", max_groups=qs.K, wide_degree=wide,
                          tuning=tun) as s:
                assert np.array_equal(s.run(qs).F, ref.F), (name, wide, tun)
                assert np.array_equal(s.run(qs).F, ref.F), (name, wide, tun)


def test_bitpar_first_pull_wide_threshold(msbfs_pkg):
    """wide_few: the first pull level's wide threshold for passes of <= 4 words while wide_degree
    is at its default, on graphs of >= 2^23 non-isolated vertices (a relabelled RMAT-24 here,
    prefix pull + tail push on level 2); 0 keeps wide_degree. Same F for every threshold at 1, 2
    and 4 words, equal to the distance solver on a sample."""
    m = msbfs_pkg
    g = m.DeviceGraph.rmat(24, 16, 3, device=0)
    g.relabel_by_degree()
    for K in (40, 100, 250):
        qs = m.QuerySet.random(g.n, K, 16, seed=K)
        out = {}
        for wf in (0, 8, 128, 1 << 20):
            with m.Solver(g, "bitpar", max_groups=K, tuning={"wide_few": wf}) as s:
                out[wf] = s.run(qs).F
                assert s.level_trace()[1]["dir"] == "B", (K, wf)  # level 2 pulls
            assert np.array_equal(out[wf], out[0]), (K, wf)
        with m.Solver(g, "dist") as ds:
            assert np.array_equal(ds.run(qs.subset(np.arange(0, K, 17))).F, out[128][::17])
    g.close()


@pytest.mark.parametrize("force_dir,wide", [(1, 64), (2, 64), (2, 2), (0, 8)])
def test_dist_direction_variants(msbfs_pkg, force_dir, wide):
    m = msbfs_pkg
    for name, g in _graphs(m)[:4]:
        qs = m.QuerySet.random(g.n, 6, 3, seed=5)
        ref = m.cpu_bfs(g, qs)
        with m.Solver(g.to_device(0), "dist", force_dir=force_dir, wide_degree=wide) as s:
            assert np.array_equal(s.run(qs).F, ref.F), (name, force_dir, wide)


def test_solver_reuse_is_deterministic(msbfs_pkg):
    m = msbfs_pkg
    g = m.DeviceGraph.rmat(13, 16, 2, device=0)
    qs = m.QuerySet.random(g.n, 256, 8, seed=1)
    with m.Solver(g, "bitpar", max_groups=qs.K) as s:
        a = s.run(qs).F
        b = s.run(qs).F
        c = s.run(qs.subset(range(100))).F
    assert np.array_equal(a, b) and np.array_equal(a[:100], c)


def test_device_rmat_matches_host_generator(msbfs_pkg):
    m = msbfs_pkg
    dg = m.DeviceGraph.rmat(12, 16, 42, device=0)
    hg = m.Graph.rmat(12, 16, 42)
    d = dg.download()
    assert d.n == hg.n and d.nnz == hg.nnz
    assert np.array_equal(d.rowptr, hg.rowptr)
    for v in range(0, hg.n, 7):
        a = np.sort(d.col[d.rowptr[v]:d.rowptr[v + 1]])
        b = np.sort(hg.col[hg.rowptr[v]:hg.rowptr[v + 1]])
        assert np.array_equal(a, b)
    dg.sort_rows()
    s = dg.download()
    for v in range(hg.n):
        assert np.all(np.diff(s.col[s.rowptr[v]:s.rowptr[v + 1]]) >= 0)
    assert dg.max_degree == int(np.diff(hg.rowptr).max())
    assert dg.isolated == int((np.diff(hg.rowptr) == 0).sum())


def test_device_uniform_and_wrap(msbfs_pkg):
    import torch
    m = msbfs_pkg
    hg = m.Graph.uniform(4000, 20000, 3)
    dg = m.DeviceGraph.uniform(4000, 20000, 3, device=0)
    assert np.array_equal(dg.download().rowptr, hg.rowptr)
    rp = torch.from_numpy(hg.rowptr).cuda()
    cl = torch.from_numpy(hg.col).cuda()
    wg = m.DeviceGraph.wrap(hg.n, rp, cl, device=0)
    qs = m.QuerySet.random(hg.n, 50, 4, 1)
    with m.Solver(wg, "bitpar", max_groups=50) as s:
        assert np.array_equal(s.run(qs).F, m.cpu_bfs(hg, qs).F)


@pytest.mark.parametrize("prep", ["none", "sorted"])
@pytest.mark.parametrize("scale,K", [(16, 1024), (18, 700)])
def test_bitpar_large_rmat_vs_cpu(msbfs_pkg, scale, K, prep):
    """Large enough that every block runs many tiles and flushes its LDS queues repeatedly:
    catches LDS init/flush races that 1-block toy graphs cannot. Sorted rows enable the
    XCD-labelled segment chunks of the first bottom-up level (rows are binary-searched)."""
    m = msbfs_pkg
    dg = m.DeviceGraph.rmat(scale, 16, 3, device=0)
    if prep == "sorted":
        dg.sort_rows()
    qs = m.QuerySet.random(dg.n, K, 16, seed=scale)
    ref = m.cpu_bfs(dg.download(), qs, count_edges=True)
    with m.Solver(dg, "bitpar", max_groups=K) as s:
        for _ in range(2):
            r = s.run(qs, count_edges=True)
            assert np.array_equal(r.F, ref.F)
            assert np.array_equal(r.edges, ref.edges)
    with m.Solver(dg, "dist") as s:
        assert np.array_equal(s.run(qs.subset(range(8))).F, ref.F[:8])


@pytest.mark.parametrize("algo", ["bitpar", "dist", "sweep"])
def test_relabelled_graph_same_answers(msbfs_pkg, algo):
    m = msbfs_pkg
    dg = m.DeviceGraph.rmat(14, 16, 5, device=0)
    host = dg.download()
    qs = m.QuerySet.random(dg.n, 300 if algo == "bitpar" else 5, 6, seed=2)
    qs = m.QuerySet.from_groups([list(g) + [-1, dg.n + 3] for g in qs.groups()])  # + invalid ids
    ref = m.cpu_bfs(host, qs, count_edges=True)
    dg.relabel_by_degree()
    assert dg.relabelled
    r = dg.download()
    deg = np.diff(r.rowptr)
    assert np.all(np.diff(deg) <= 0)  # degree-descending ids
    o2n = dg.relabel_map()
    assert np.array_equal(np.sort(o2n), np.arange(dg.n))
    assert np.array_equal(np.diff(host.rowptr), deg[o2n])
    for v in range(0, dg.n, 97):
        assert np.all(np.diff(r.col[r.rowptr[v]:r.rowptr[v + 1]]) >= 0)
    with m.Solver(dg, algo, max_groups=qs.K) as s:
        res = s.run(qs, count_edges=True)
    assert np.array_equal(res.F, ref.F)
    assert np.array_equal(res.edges, ref.edges)


@pytest.mark.parametrize("kind", ["rmat", "uniform"])
def test_relabel_by_regeneration_matches(msbfs_pkg, kind, monkeypatch):
    """The low-memory relabel path (device-generated graphs are regenerated straight into the
    new ids when a second column array does not fit, e.g. RMAT-30) gives the same CSR and map as
    the gather path."""
    m = msbfs_pkg
    make = ((lambda: m.DeviceGraph.rmat(15, 16, 9, device=0)) if kind == "rmat"
            else (lambda: m.DeviceGraph.uniform(30000, 250000, 4, device=0)))
    monkeypatch.delenv("MSBFS_RELABEL_REGEN", raising=False)
    a = make()
    a.relabel_by_degree()
    monkeypatch.setenv("MSBFS_RELABEL_REGEN", "1")
    b = make()
    b.relabel_by_degree()
    ga, gb = a.download(), b.download()
    assert np.array_equal(a.relabel_map(), b.relabel_map())
    assert np.array_equal(ga.rowptr, gb.rowptr)
    assert np.array_equal(ga.col, gb.col)


def test_bitpar_level_trace(msbfs_pkg):
    """Per-level records (msbfs_solver_levels): one per level, consistent with the stats and with
    the frontier chain (the next level starts from the previous level's new vertices)."""
    m = msbfs_pkg
    for g in (m.Graph.rmat(12, 16, 3), m.Graph.grid(60, 60, 0.9, 0, 2)):
        qs = m.QuerySet.random(g.n, 100, 4, seed=5)
        with m.Solver(g.to_device(0), "bitpar", max_groups=qs.K) as s:
            r = s.run(qs)
            tr = s.level_trace()
        assert len(tr) == r.stats["levels"]
        assert sum(t["dir"] == "B" for t in tr) == r.stats["bu_levels"]
        assert sum(t["dir"] == "T" for t in tr) == r.stats["td_levels"]
        assert [t["level"] for t in tr] == list(range(1, len(tr) + 1))
        for a, b in zip(tr, tr[1:]):
            assert b["nf"] == a["nf_next"]
        assert tr[-1]["nf_next"] == 0 and all(t["ms"] >= 0 for t in tr)


@pytest.mark.parametrize("K", [300, 1024])
def test_bitpar_sparse_codes_relabelled(msbfs_pkg, K):
    """First bottom-up level with sparse single-group row codes (k_build_codes) on a degree-
    relabelled device RMAT graph: identical F with the codes on, off, and against the CPU oracle."""
    m = msbfs_pkg
    g = m.DeviceGraph.rmat(14, 16, 5, device=0)
    qs = m.QuerySet.random(g.n, K, 8, seed=K)
    ref = m.cpu_bfs(g.download(), qs)  # original ids (download() after relabelling is internal)
    g.relabel_by_degree()
    out = {}
    for codes in ("1", "0"):
        # code_deg 0.5: codes for most ids, the dense fallback exercised
        with m.Solver(g, "bitpar", max_groups=K, tuning={"codes": codes, "code_deg": 0.5}) as s:
            out[codes] = s.run(qs).F
    assert np.array_equal(out["1"], ref.F)
    assert np.array_equal(out["0"], ref.F)
    g.close()


def test_bitpar_prefix_pull_tail_push(msbfs_pkg):
    """First bottom-up level as prefix pull (ids below the LDS hub bound) + tail push (k_push_tail)
    on a relabelled RMAT-23 (n = 8M, large enough for the 128-KB hub bitmap): identical F with
    the prefix mode on and off, and equal to the per-group distance solver on a sample."""
    m = msbfs_pkg
    g = m.DeviceGraph.rmat(23, 16, 3, device=0)
    g.relabel_by_degree()
    qs = m.QuerySet.random(g.n, 1024, 16, seed=11)
    out = {}
    for pfx in ("2", "0"):  # prefix bound 458752 / off (whole rows)
        with m.Solver(g, "bitpar", max_groups=qs.K, tuning={"pfx": pfx}) as s:
            out[pfx] = s.run(qs).F
            tr = s.level_trace()
        assert tr[0]["dir"] == "T" and tr[1]["dir"] == "B"  # the prefix level is level 2
    assert np.array_equal(out["2"], out["0"])
    sub = qs.subset(np.arange(0, 1024, 128))
    with m.Solver(g, "dist") as ds:
        assert np.array_equal(ds.run(sub).F, out["2"][::128])
    g.close()


@pytest.mark.parametrize("K", [16, 40, 128])
def test_bitpar_prefix_bound(msbfs_pkg, K):
    """The untiled prefix level (1-2 words) with its bound H chosen from the source count
    (BitparSolver::pfx_bound) or forced (tuning pfx_h): the per-vertex scans stop at the first id
    >= H, the hub chunks end there, the frontier vertices >= H push, and the frontier is left as
    a bitmap (materialised when a top-down level follows). Identical F for every bound, with a
    top-down level right after, and equal to the per-group distance solver on a sample."""
    m = msbfs_pkg
    g = m.DeviceGraph.rmat(23, 16, 5, device=0)
    g.relabel_by_degree()
    qs = m.QuerySet.random(g.n, K, 16, seed=K + 3)
    runs = {"auto": {}, "full": {"pfx_h": 458752}, "h1024": {"pfx_h": 1024},
            "h32768": {"pfx_h": 32768}, "h5000": {"pfx_h": 5000}, "off": {"pfx": 0},
            "td3": {"dirs": "TBT"}, "td3h1024": {"dirs": "TBT", "pfx_h": 1024},
            # every pull level filtered by the any-visited bitmap / none but the lazy first one
            "filter_all": {"filter_frac": 2}, "filter_none": {"filter_frac": 0}}
    out = {}
    for name, tun in runs.items():
        with m.Solver(g, "bitpar", max_groups=qs.K, tuning=tun) as s:
            s.prepare()
            out[name] = s.run(qs).F
            out[name + "2"] = s.run(qs).F
            tr = s.level_trace()
        assert "".join(t["dir"] for t in tr).startswith("TBT" if "td3" in name else "TB"), name
    for name in out:
        assert np.array_equal(out[name], out["off"]), name
    sub = qs.subset(np.arange(0, K, 7))
    with m.Solver(g, "dist") as ds:
        assert np.array_equal(ds.run(sub).F, out["auto"][::7])
    g.close()


@pytest.mark.parametrize("K", [1024, 900, 512, 200])
def test_bitpar_tiled_first_pull(msbfs_pkg, K):
    """The first pull level over static vertex tiles (k_pfx_tiles + big-vertex partial tiles +
    k_bu_wide_finalize, bitpar/tiles.hpp) on a relabelled RMAT-23, 16 / 8 / 4 words: identical F
    with the tiles on and off, with no / few / most ids coded, with a top-down level right after
    the tiled one (the frontier list comes from the tile bitmap), and equal to the per-group
    distance solver on a sample."""
    m = msbfs_pkg
    g = m.DeviceGraph.rmat(23, 16, 7, device=0)
    g.relabel_by_degree()
    qs = m.QuerySet.random(g.n, K, 16, seed=K)
    runs = {"tiles": {}, "plain": {"tiles": 0}, "nocodes": {"codes": 0},
            "fewcodes": {"tiles_code_deg": 1}, "manycodes": {"tiles_code_deg": 400},
            "td3": {"dirs": "TBT"}, "td3plain": {"dirs": "TBT", "tiles": 0},
            "pushbefore": {"push_after": 0}, "td3pushbefore": {"dirs": "TBT", "push_after": 0},
            "pushafter_nocodes": {"push_after": 1, "codes": 0}, "chunk2": {"chunk2": 1},
            "nolean": {"lean_min": 1 << 40},
            # tiles from 4 words on (K = 200: W = 4, no codes there)
            "tiles4": {"tiles_w": 4}, "tiles4_pushbefore": {"tiles_w": 4, "push_after": 0},
            "td3tiles4": {"dirs": "TBT", "tiles_w": 4}}
    out = {}
    for name, tun in runs.items():
        with m.Solver(g, "bitpar", max_groups=qs.K, tuning=tun) as s:
            s.prepare()
            out[name] = s.run(qs).F
            out[name + "2"] = s.run(qs).F  # reuse: the acc rows and stamps were left clean
            tr = s.level_trace()
        assert "".join(t["dir"] for t in tr).startswith("TBT" if "td3" in name else "TB")
    for name in out:
        assert np.array_equal(out[name], out["plain"]), name
    sub = qs.subset(np.arange(0, K, 97))
    with m.Solver(g, "dist") as ds:
        assert np.array_equal(ds.run(sub).F, out["tiles"][::97])
    g.close()


def test_bitpar_tiled_done_before_pull(msbfs_pkg):
    """Every group holds the top hub: all of its neighbours are visited by every group at level
    1, so they are done before the tiled level 2 (the tile epilogue and the big vertices'
    finalize still write their rows for the tail push after the tiles, which filters against
    them instead of probing the done bitmap). Same F with the push after / before the tiles and
    without tiles."""
    m = msbfs_pkg
    g = m.DeviceGraph.rmat(23, 16, 11, device=0)
    g.relabel_by_degree()
    top = int(np.nonzero(g.relabel_map() == 0)[0][0])  # user id of internal id 0
    base = m.QuerySet.random(g.n, 520, 6, seed=3)
    qs = m.QuerySet.from_groups([list(x) + [top] for x in base.groups()])
    out = {}
    for name, tun in {"after": {}, "before": {"push_after": 0}, "plain": {"tiles": 0}}.items():
        with m.Solver(g, "bitpar", max_groups=qs.K, tuning=tun) as s:
            s.prepare()
            out[name] = s.run(qs).F
            assert np.array_equal(s.run(qs).F, out[name]), name
    assert np.array_equal(out["after"], out["plain"])
    assert np.array_equal(out["before"], out["plain"])
    with m.Solver(g, "dist") as ds:
        assert np.array_equal(ds.run(qs.subset(np.arange(0, qs.K, 101))).F, out["plain"][::101])
    g.close()


@pytest.mark.parametrize("dirs", ["", "TBBBBBBBBBBBBBBBBBBB", "TBBTBBTBBTBBTBBT", "TBTBTBTBTBTBTBTB",
                                  "TTBBTTBBTTBB"])
def test_bitpar_forced_direction_plans(msbfs_pkg, dirs):
    """Forced per-level direction plans (tuning dirs): push levels right after pull levels read
    the frontier as the difference of the two visited buffers, pulls after pushes start from the
    top-down accumulator. Runs without the edge count (the fused-count kernels) on a relabelled
    RMAT, uniform and road-like graphs, several batches (K > 64 * W) included, and reuses the
    solver (stale rows of the previous run must not leak)."""
    m = msbfs_pkg
    dg = m.DeviceGraph.rmat(14, 16, 5, device=0)
    hg = dg.download()  # original ids (after relabelling download() gives internal ones)
    dg.relabel_by_degree()
    cases = [(dg, hg, 1024), (dg, hg, 300), (dg, hg, 1500)]
    for name, g in _graphs(m)[2:4]:
        cases.append((g.to_device(0), g, 200))
    for dev, host, K in cases:
        qs = m.QuerySet.random(host.n, K, 4, seed=K)
        ref = m.cpu_bfs(host, qs)
        for bu_max in (0, 1 << 30):  # host-driven / device-driven late pull levels
            tun = {"dirs": dirs, "bu_max": bu_max} if dirs else {"bu_max": bu_max}
            with m.Solver(dev, "bitpar", max_groups=min(K, 1024), tuning=tun) as s:
                r = s.run(qs)
                r2 = s.run(qs)
            assert np.array_equal(r.F, ref.F), (dirs, K, bu_max)
            assert np.array_equal(r2.F, ref.F), (dirs, K, bu_max)


@pytest.mark.parametrize("knobs", [{"lean_min": 0}, {"lean": 0}, {"lazy": 0},
                                   {"lazy": 0, "lean_min": 0}])
def test_bitpar_lean_and_lazy_paths(msbfs_pkg, knobs):
    """The lean first-row pass on late pull levels (k_bu_first + overflow pull; forced on small
    lists with tuning lean_min=0) and the lazy batches without the visited-buffer fill agree with
    the CPU oracle, with each switched on and off, over several batches and a reused solver."""
    m = msbfs_pkg
    dg = m.DeviceGraph.rmat(15, 16, 7, device=0)
    hg = dg.download()
    dg.relabel_by_degree()
    cases = [(dg, hg, 1024), (dg, hg, 2100), (dg, hg, 128)]
    for name, g in _graphs(m)[2:4]:
        cases.append((g.to_device(0), g, 300))
    for dev, host, K in cases:
        qs = m.QuerySet.random(host.n, K, 8, seed=K + 1)
        ref = m.cpu_bfs(host, qs)
        with m.Solver(dev, "bitpar", max_groups=min(K, 1024), tuning=knobs) as s:
            r = s.run(qs)
            r2 = s.run(qs)
        assert np.array_equal(r.F, ref.F), (knobs, K)
        assert np.array_equal(r2.F, ref.F), (knobs, K)


@pytest.mark.parametrize("tun", [{"bu_max": 1 << 30}, {"bu_max": 1 << 30, "batch": 2},
                                 {"bu_max": 1 << 30, "batch": 3, "lean": 0}])
def test_bitpar_device_pull_batches(msbfs_pkg, tun):
    """Late pull levels as device-driven batches (bu_batch: counter slots, BuGate per level,
    no-op levels after the frontier dies or the direction turns): answers equal the CPU oracle
    and the per-level records (level, direction, frontier size and degree sum, next frontier,
    new active lists) equal the host-driven levels' (tuning bu_max=0), so the device gate took
    every decision the host loop takes. Short batches (batch=2, 3) chain several per run; the
    uniform graph turns back to push within a batch; reused solvers; W = 1, 2, 16."""
    m = msbfs_pkg
    dg = m.DeviceGraph.rmat(15, 16, 7, device=0)
    hg = dg.download()
    cases = [(dg, hg)]
    rl = m.DeviceGraph.rmat(14, 16, 3, device=0)
    rh = rl.download()  # (original ids: the queries are mapped on the device)
    rl.relabel_by_degree()
    cases.append((rl, rh))
    u = m.Graph.uniform(30000, 300000, 9)
    cases.append((u.to_device(0), u))
    batched = 0
    for gi, (dev, host) in enumerate(cases):
        for K in (64, 100, 1024):
            qs = m.QuerySet.random(host.n, K, 6, seed=K + gi)
            ref = m.cpu_bfs(host, qs)
            recs = {}
            for name, t in (("dev", tun), ("host", {"bu_max": 0})):
                with m.Solver(dev, "bitpar", max_groups=K, tuning=t) as s:
                    r = s.run(qs)
                    assert np.array_equal(r.F, ref.F), (gi, K, name)
                    assert np.array_equal(s.run(qs).F, ref.F), (gi, K, name)
                    recs[name] = [(x["batch"], x["level"], x["dir"], x["nf"], x["ef"],
                                   x["nf_next"], x["active"]) for x in s.level_trace()]
            assert recs["dev"] == recs["host"], (gi, K)
            batched += sum(x[2] == "B" and x[1] >= 4 for x in recs["dev"])
    assert batched > 0


def _hyp_strategy():
    from hypothesis import strategies as st

    @st.composite
    def graphs_and_queries(draw):
        n = draw(st.integers(1, 60))
        m_ = draw(st.integers(0, 150))
        edges = draw(st.lists(st.tuples(st.integers(0, n - 1), st.integers(0, n - 1)),
                              min_size=m_, max_size=m_))
        K = draw(st.integers(1, 140))  # up to three 64-group words
        groups = draw(st.lists(st.lists(st.integers(-3, n + 3), max_size=6), min_size=K,
                               max_size=K))
        return n, edges, groups
    return graphs_and_queries()


def test_device_algos_property(msbfs_pkg):
    """SURVEY §4.2 item 3 on the GPU: hypothesis-generated graphs (self-loops, duplicate edges,
    isolated vertices) and query sets (empty groups, out-of-range ids) through every device
    algorithm, against the CPU path and the numpy oracle of the reference semantics."""
    from hypothesis import given, settings, HealthCheck
    from msbfs.ops import reference as R
    m = msbfs_pkg

    @settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck))
    @given(_hyp_strategy())
    def check(data):
        n, edges, groups = data
        u = np.array([e[0] for e in edges], np.int32)
        v = np.array([e[1] for e in edges], np.int32)
        g = m.Graph.from_edges(n, u, v)
        qs = m.QuerySet.from_groups(groups)
        ref = m.cpu_bfs(g, qs, count_edges=True)
        for k in range(min(qs.K, 5)):
            assert ref.F[k] == R.bfs_F_numpy(g.n, g.rowptr, g.col, qs.group(k))[0]
        dg = g.to_device(0)
        for algo in ("bitpar", "dist", "topdown", "sweep"):
            sub = qs if algo == "bitpar" else qs.subset(np.arange(min(qs.K, 6)))
            with m.Solver(dg, algo, max_groups=sub.K) as s:
                r = s.run(sub, count_edges=True)
            assert np.array_equal(r.F, ref.F[:sub.K]), algo
            assert np.array_equal(r.edges, ref.edges[:sub.K]), algo
        with m.Solver(dg, "bitpar", max_groups=qs.K) as s:  # fused-count (lazy) path
            assert np.array_equal(s.run(qs).F, ref.F)
        dg.close()

    check()


@pytest.mark.parametrize("fused", ["1", "0", "bitmap"])
def test_bitpar_fused_topdown_batches(msbfs_pkg, fused):
    """Low-degree graphs run device-driven top-down batches; by default each level is one
    k_td_fused kernel (claims bits with atomicOr on the visited row, keeps only vis[cur] current).
    Road-like grids stay top-down; the uniform graphs switch to pulls after fused levels (a level
    stops the device-driven batch on the host's test; the stale second buffer is restored
    first); repeated runs reuse the buffers; W = 1, 4, 16.
    "bitmap": the list/bitmap choice forced to the bitmap walk, short batches."""
    m = msbfs_pkg
    tun = {"td_fused": 0 if fused == "0" else 1}
    if fused == "bitmap":  # every level after a batch's first walks the frontier bitmap
        tun.update(td_bm=1, batch=5)
    graphs = [m.Graph.grid(90, 110, 0.65, 0, 3), m.Graph.grid(50, 50, 0.9, 20, 4),
              m.Graph.uniform(20000, 160000, 5), m.Graph.uniform(6000, 3500, 6),
              m.Graph.uniform(60000, 240000, 7)]
    for gi, g in enumerate(graphs):
        dg = g.to_device(0)
        for K in (1, 64, 200, 1024):
            qs = m.QuerySet.random(g.n, K, 3, seed=K + gi)
            ref = m.cpu_bfs(g, qs)
            with m.Solver(dg, "bitpar", max_groups=K, tuning=tun) as s:
                for _ in range(2):
                    r = s.run(qs)
                    assert np.array_equal(r.F, ref.F), (gi, K, fused)


def test_bitpar_fused_level_records_match(msbfs_pkg):
    """The fused levels take the frontier's degree sum from the next level's row offsets (and
    at a batch's last level from the appends): per-level frontier sizes and degree sums — the
    direction heuristic's inputs — equal the expand + finalize path's (push levels only: the
    fused batches also stop for a pull on their own estimate)."""
    m = msbfs_pkg
    g = m.Graph.grid(120, 130, 0.7, 0, 5)
    dg = g.to_device(0)
    for K in (64, 256):
        qs = m.QuerySet.random(g.n, K, 4, seed=K)
        recs = {}
        for fused in ("1", "0"):
            with m.Solver(dg, "bitpar", max_groups=K, force_dir=1,
                          tuning={"td_fused": fused, "batch": 7}) as s:
                s.run(qs)
                recs[fused] = [(r["level"], r["dir"], r["nf"], r["ef"], r["nf_next"])
                               for r in s.level_trace()]
        assert recs["1"] == recs["0"], K


@pytest.mark.parametrize("gamma2,want", [("0", "B"), ("100", "T")])
def test_bitpar_level2_direction_threshold(msbfs_pkg, gamma2, want):
    """Tuning gamma2 decides level 2's direction for few groups: a pull with the prefix pull + tail
    push (0) or a push that makes level 3 the first, whole-row pull (100). Both plans must give
    the oracle's F; the level records show which one ran."""
    m = msbfs_pkg
    tun = {"gamma2": gamma2, "gamma": 100}  # (gamma 100: the later levels' vertex test out of the way)
    dg = m.DeviceGraph.rmat(16, 16, 9, device=0)
    hg = dg.download()
    dg.relabel_by_degree()
    for K in (4, 32):
        qs = m.QuerySet.random(hg.n, K, 16, seed=K)
        ref = m.cpu_bfs(hg, qs)
        # a tiny alpha turns Beamer's edge test off: only the vertex test decides
        with m.Solver(dg, "bitpar", max_groups=K, alpha=1e-9, tuning=tun) as s:
            r = s.run(qs)
            dirs = "".join(t["dir"] for t in s.level_trace())
        assert np.array_equal(r.F, ref.F), (gamma2, K, dirs)
        assert dirs[:2] == "T" + want, (gamma2, K, dirs)


@pytest.mark.parametrize("gamma2,want", [("0", "B"), ("100", "T")])
@pytest.mark.parametrize("fused", [0, 1])
def test_bitpar_level2_threshold_in_device_batches(msbfs_pkg, gamma2, fused, want):
    """On a low-degree graph (max degree <= 64) levels 1-2 run inside a device-driven top-down
    batch, which stops itself where the host would pull: the stop must use gamma2 for level 2
    exactly like the host loop (0: level 2 pulls; 100: it pushes), with and without the fused
    one-kernel levels. F must equal the oracle's either way."""
    m = msbfs_pkg
    g = m.Graph.uniform(30000, 240000, 8)  # mean degree 16 > 8: the batches run expand+finalize
    g2 = m.Graph.uniform(60000, 200000, 9)  # mean degree 6.7: fused levels
    for host in (g, g2):
        assert int(np.diff(host.rowptr).max()) <= 64
        dg = host.to_device(0)
        qs = m.QuerySet.random(host.n, 64, 8, seed=3)
        ref = m.cpu_bfs(host, qs)
        with m.Solver(dg, "bitpar", max_groups=64, alpha=1e-9,
                      tuning={"gamma2": gamma2, "gamma": 100, "td_fused": fused}) as s:
            r = s.run(qs)
            dirs = "".join(t["dir"] for t in s.level_trace())
        assert np.array_equal(r.F, ref.F), (gamma2, dirs)
        assert dirs[:2] == "T" + want, (gamma2, fused, dirs)
        dg.close()


def test_bitpar_tuning_rejects_unknown_keys(msbfs_pkg):
    """Tuning is explicit and validated: an unknown key or a malformed value is an error, never a
    silently ignored setting (and the distance solver accepts no keys at all)."""
    m = msbfs_pkg
    g = m.Graph.grid(20, 20, 1.0, 0, 1).to_device(0)
    with m.Solver(g, "bitpar", max_groups=64) as s:
        for bad in ("gamma3=1", "gamma2", "pfx=1", "batch=0", "dirs=TX", "lean=x"):
            with pytest.raises(m.native.MsbfsError):
                s.tune(bad)
        s.tune("gamma2=0.5,lean=0,dirs=TB")
    with m.Solver(g, "dist") as s:
        with pytest.raises(m.native.MsbfsError):
            s.tune("gamma=1")
    g.close()


def test_dist_device_batches_and_reset(msbfs_pkg):
    """The per-group distance solver keeps every frontier in one visit-order array: low-degree
    graphs run device-driven batches of top-down levels (slice bounds in device slots, one host
    round trip per batch; uniform graphs stop a batch where the host pulls), and the distance
    array is reset by scattering -1 over the visited prefix after groups that reached few
    vertices (many small components) or refilled after large ones. F and the traversed-edge
    counts equal the CPU oracle's, for the distance solver and its top-down-only variant, over
    repeated runs of the same solver."""
    m = msbfs_pkg
    graphs = [m.Graph.grid(90, 110, 0.65, 0, 3), m.Graph.grid(60, 60, 0.9, 30, 2),
              m.Graph.uniform(20000, 160000, 5), m.Graph.uniform(6000, 3500, 6),
              m.Graph.rmat(12, 16, 3)]
    for gi, g in enumerate(graphs):
        dg = g.to_device(0)
        qs = m.QuerySet.random(g.n, 24, 2, seed=gi + 1)
        ref = m.cpu_bfs(g, qs, count_edges=True)
        for algo in ("dist", "topdown"):
            with m.Solver(dg, algo) as s:
                for _ in range(2):
                    r = s.run(qs, count_edges=True)
                    assert np.array_equal(r.F, ref.F), (gi, algo)
                    assert np.array_equal(r.edges, ref.edges), (gi, algo)
        dg.close()


@pytest.mark.parametrize("dirs", ["", "TBBTBBTBBTBBTBBT", "TBTBTBTBTBTBTBTB", "TBBBBBBBBBBBBBBT"])
@pytest.mark.parametrize("extra", [{}, {"lean_min": 0}, {"bu_max": 1 << 30}, {"full": 0},
                                   {"dskip3": 0}])
def test_bitpar_done_rows_skipped(msbfs_pkg, dirs, extra):
    """dskip (round 4): unfiltered pull levels never read done vertices' rows (a level-start
    snapshot of the done bitmap is probed, the alive mask ORed) and write none for the vertices
    they finish; a push level right after restores the skipped rows of its frontier. Forced
    pull -> push -> pull plans, the lean pass (lean_min=0), device-driven pull batches and the old
    per-vertex pulls (full=0: no skipping) all give the oracle's F, dskip on and off, over
    several batches and a reused solver."""
    m = msbfs_pkg
    dg = m.DeviceGraph.rmat(14, 16, 5, device=0)
    hg = dg.download()
    dg.relabel_by_degree()
    cases = [(dg, hg, 1024), (dg, hg, 1500), (dg, hg, 100)]
    for name, g in _graphs(m)[2:4]:
        cases.append((g.to_device(0), g, 300))
    for dev, host, K in cases:
        qs = m.QuerySet.random(host.n, K, 5, seed=K + 3)
        ref = m.cpu_bfs(host, qs)
        for dskip in (1, 0):
            tun = dict(extra, dskip=dskip)
            if dirs:
                tun["dirs"] = dirs
            with m.Solver(dev, "bitpar", max_groups=min(K, 1024), tuning=tun) as s:
                assert np.array_equal(s.run(qs).F, ref.F), (dirs, extra, K, dskip)
                assert np.array_equal(s.run(qs).F, ref.F), (dirs, extra, K, dskip)
