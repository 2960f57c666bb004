"""Reference semantics on the CPU path (golden table SURVEY §4.2) + property tests vs oracles."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from golden import CASES
from msbfs.ops import reference as R


def _graph(m, n, edges):
    u = np.array([e[0] for e in edges], np.int32)
    v = np.array([e[1] for e in edges], np.int32)
    return m.Graph.from_edges(n, u, v)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_golden_cpu(msbfs_pkg, case):
    m = msbfs_pkg
    (n, edges), groups, F, k, minf = CASES[case]
    g = _graph(m, n, edges)
    r = m.cpu_bfs(g, m.QuerySet.from_groups(groups))
    assert list(r.F) == F
    kk = m.argmin_first(r.F)
    assert kk + 1 == k
    assert (r.F[kk] if kk >= 0 else -1) == minf
    for grp, f in zip(groups, F):
        assert R.bfs_F_numpy(g.n, g.rowptr, g.col, grp)[0] == f
        assert R.bfs_F_scipy(g.n, g.rowptr, g.col, grp) == f


def test_argmin_matches_native(msbfs_pkg):
    import ctypes as C
    m = msbfs_pkg
    rng = np.random.default_rng(0)
    for _ in range(50):
        F = rng.integers(0, 5, size=rng.integers(0, 10)).astype(np.int64)
        got = m.native.lib().msbfs_argmin(m.native.ptr(F, C.c_int64), len(F))
        assert got == m.argmin_first(F)


@st.composite
def graphs_and_queries(draw):
    n = draw(st.integers(1, 40))
    m_ = draw(st.integers(0, 80))
    edges = draw(st.lists(st.tuples(st.integers(0, n - 1), st.integers(0, n - 1)),
                          min_size=m_, max_size=m_))
    K = draw(st.integers(0, 6))
    groups = draw(st.lists(st.lists(st.integers(-3, n + 3), max_size=5), min_size=K, max_size=K))
    return n, edges, groups


@settings(max_examples=150, deadline=None)
@given(graphs_and_queries())
def test_cpu_matches_oracles(msbfs_pkg, data):
    m = msbfs_pkg
    n, edges, groups = data
    g = _graph(m, n, edges)
    r = m.cpu_bfs(g, m.QuerySet.from_groups(groups), count_edges=True)
    for k, grp in enumerate(groups):
        f, e = R.bfs_F_numpy(g.n, g.rowptr, g.col, grp)
        assert r.F[k] == f == R.bfs_F_scipy(g.n, g.rowptr, g.col, grp)
        assert r.edges[k] == e


def test_cpu_against_networkx(msbfs_pkg):
    nx = pytest.importorskip("networkx")
    m = msbfs_pkg
    g = m.Graph.uniform(1000, 10000, 3)  # BASELINE config 1 shape: 1K vertices / 10K edges
    qs = m.QuerySet.random(g.n, 4, 1, 9)  # 4 single-source queries
    r = m.cpu_bfs(g, qs, threads=1)
    G = nx.Graph()
    G.add_nodes_from(range(g.n))
    src = np.repeat(np.arange(g.n), np.diff(g.rowptr))
    G.add_edges_from(zip(src.tolist(), g.col.tolist()))
    for k, grp in enumerate(qs.groups()):
        d = nx.multi_source_dijkstra_path_length(G, set(int(x) for x in grp))
        assert r.F[k] == sum(d.values())
