"""Device-side CSR build of a legacy graph file (SURVEY C5 "on GPU: atomic degree count + scan +
scatter"): DeviceGraph.from_file / msbfs_graph_from_edge_file stream the mapped
edge list to HBM and count / scatter it there. Checked against the host build row by row (as
multisets: the device scatter does not keep the file order) and through the solvers' F; the
reference's error paths (missing file, truncation, ids outside [0, n)) keep their messages."""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _write_raw_graph(path, n, edges):
    with open(path, "wb") as f:
        f.write(struct.pack("<iq", n, len(edges)))
        for u, v in edges:
            f.write(struct.pack("<ii", u, v))


def _rows(g):
    return [np.sort(g.col[g.rowptr[v]:g.rowptr[v + 1]]) for v in range(g.n)]


@pytest.mark.parametrize("scale,ef", [(10, 8), (14, 16)])
def test_device_file_build_matches_host(tmp_path, msbfs_pkg, scale, ef):
    m = msbfs_pkg
    g = m.Graph.rmat(scale, ef, 3)
    p = str(tmp_path / "g.bin")
    g.write(p)
    dg = m.DeviceGraph.from_file(p, device=0)
    d = dg.download()
    h = m.Graph.from_file(p)
    assert d.n == h.n and d.nnz == h.nnz and np.array_equal(d.rowptr, h.rowptr)
    for a, b in zip(_rows(d), _rows(h)):
        assert np.array_equal(a, b)
    qs = m.QuerySet.random(g.n, 200, 4, 5)
    with m.Solver(dg, "bitpar", max_groups=qs.K) as s:
        r = s.run(qs, count_edges=True)
    ref = m.cpu_bfs(h, qs, count_edges=True)
    assert np.array_equal(r.F, ref.F) and np.array_equal(r.edges, ref.edges)
    dg.close()


def test_device_file_build_duplicates_selfloops_isolated(tmp_path, msbfs_pkg):
    """Self-loops insert the vertex twice, duplicates stay (main.cu:113-115); isolated vertices."""
    m = msbfs_pkg
    p = str(tmp_path / "g.bin")
    _write_raw_graph(p, 6, [(0, 0), (0, 1), (0, 1), (1, 2), (3, 4)])
    d = m.DeviceGraph.from_file(p).download()
    assert list(np.diff(d.rowptr)) == [4, 3, 1, 1, 1, 0]
    assert sorted(d.col[0:4]) == [0, 0, 1, 1]
    qs = m.QuerySet.from_groups([[0], [3], [5]])
    with m.Solver(m.DeviceGraph.from_file(p, relabel=True), "bitpar") as s:
        assert list(s.run(qs).F) == [3, 1, 0]


def test_device_file_build_errors(tmp_path, msbfs_pkg):
    m = msbfs_pkg
    err = m.native.MsbfsError
    with pytest.raises(err, match="Could not open graph file"):
        m.DeviceGraph.from_file(str(tmp_path / "missing.bin"))
    p = str(tmp_path / "trunc.bin")
    _write_raw_graph(p, 5, [(0, 1), (1, 2)])
    open(p, "r+b").truncate(12 + 8 + 3)
    with pytest.raises(err, match="truncated"):
        m.DeviceGraph.from_file(p)
    p = str(tmp_path / "range.bin")
    _write_raw_graph(p, 3, [(0, 1), (1, 7), (2, -1)])
    with pytest.raises(err, match="edge 1 has a vertex id outside"):
        m.DeviceGraph.from_file(p)
    p = str(tmp_path / "empty.bin")
    _write_raw_graph(p, 4, [])
    d = m.DeviceGraph.from_file(p).download()
    assert d.n == 4 and d.nnz == 0
