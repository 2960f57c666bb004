"""Binary format contract (reference main.cu:92-164) — native loader vs pure-numpy twin."""
import os
import struct

import numpy as np
import pytest

from msbfs.utils import formats


def _write_raw_graph(path, n, edges):
    with open(path, "wb") as f:
        f.write(struct.pack("<iq", n, len(edges)))
        for u, v in edges:
            f.write(struct.pack("<ii", u, v))


def test_graph_roundtrip_bytes(tmp_path, msbfs_pkg):
    m = msbfs_pkg
    p = str(tmp_path / "g.bin")
    u = np.array([0, 1, 2, 3], np.int32)
    v = np.array([1, 2, 3, 4], np.int32)
    formats.write_graph_bin(p, 5, u, v)
    data = open(p, "rb").read()
    assert len(data) == 12 + 8 * 4
    assert struct.unpack_from("<iq", data) == (5, 4)
    p2 = str(tmp_path / "g2.bin")
    m.Graph.from_edges(5, u, v).write(p2)
    assert open(p2, "rb").read() == data


def test_native_and_numpy_csr_agree(tmp_path, msbfs_pkg):
    m = msbfs_pkg
    g = m.Graph.rmat(9, 8, 3)
    p = str(tmp_path / "r.bin")
    g.write(p)
    a = m.Graph.from_file(p, use_native=True)
    b = m.Graph.from_file(p, use_native=False)
    assert np.array_equal(a.rowptr, b.rowptr)
    for x in range(a.n):
        assert sorted(a.col[a.rowptr[x]:a.rowptr[x + 1]]) == sorted(b.col[b.rowptr[x]:b.rowptr[x + 1]])


def test_stable_csr_keeps_reference_neighbour_order(msbfs_pkg):
    m = msbfs_pkg
    u = np.array([0, 2, 0, 1, 0], np.int32)
    v = np.array([3, 0, 1, 1, 0], np.int32)
    g = m.Graph.from_edges(4, u, v, stable=True)
    # adj[0]: push order 3, 2 (from (2,0)), 1, 0, 0 (self loop twice)
    assert list(g.col[g.rowptr[0]:g.rowptr[1]]) == [3, 2, 1, 0, 0]
    assert list(g.col[g.rowptr[1]:g.rowptr[2]]) == [0, 1, 1]  # self loop (1,1) twice
    r2, c2 = formats.csr_from_edges(4, u, v)
    assert np.array_equal(r2, g.rowptr) and np.array_equal(c2, g.col)


@pytest.mark.parametrize("native", [True, False])
def test_graph_errors(tmp_path, msbfs_pkg, native):
    m = msbfs_pkg
    err = (m.native.MsbfsError, formats.FormatError)
    with pytest.raises(err, match="Could not open graph file"):
        m.Graph.from_file(str(tmp_path / "missing.bin"), use_native=native)
    p = str(tmp_path / "trunc.bin")
    _write_raw_graph(p, 5, [(0, 1), (1, 2)])
    open(p, "r+b").truncate(12 + 8 + 3)
    with pytest.raises(err, match="truncated"):
        m.Graph.from_file(p, use_native=native)
    p = str(tmp_path / "range.bin")
    _write_raw_graph(p, 3, [(0, 1), (1, 7)])
    with pytest.raises(err, match="outside"):
        m.Graph.from_file(p, use_native=native)


@pytest.mark.parametrize("native", [True, False])
def test_query_legacy_roundtrip(tmp_path, msbfs_pkg, native):
    m = msbfs_pkg
    groups = [[0], [2, 3, 4], [], [99, -1]]
    p = str(tmp_path / "q.bin")
    m.QuerySet.from_groups(groups).write(p, use_native=native)
    data = open(p, "rb").read()
    assert data[0] == 4 and data[1] == 1 and len(data) == 1 + (1 + 4) + (1 + 12) + 1 + (1 + 8)
    q = m.QuerySet.from_file(p, use_native=not native)
    assert [list(x) for x in q.groups()] == groups


def test_query_k0_is_one_byte(tmp_path, msbfs_pkg):
    p = str(tmp_path / "q0.bin")
    msbfs_pkg.QuerySet.from_groups([]).write(p)
    assert open(p, "rb").read() == b"\x00"
    assert msbfs_pkg.QuerySet.from_file(p).K == 0


@pytest.mark.parametrize("native", [True, False])
def test_query_extended_format(tmp_path, msbfs_pkg, native):
    m = msbfs_pkg
    qs = m.QuerySet.random(1000, 1024, 3, 5)  # K > 255 cannot be expressed in the legacy format
    p = str(tmp_path / "qx.bin")
    qs.write(p, use_native=native)
    data = open(p, "rb").read()
    assert data[:9] == b"\x00MSBFSQX1" and struct.unpack_from("<I", data, 9)[0] == 1024
    assert m.QuerySet.from_file(p, use_native=True) == qs
    assert m.QuerySet.from_file(p, use_native=False) == qs
    big = m.QuerySet.from_groups([list(range(300))])  # a set > 255
    big.write(p, use_native=native)
    assert m.QuerySet.from_file(p) == big


def test_query_truncated(tmp_path, msbfs_pkg):
    p = str(tmp_path / "qt.bin")
    with open(p, "wb") as f:
        f.write(bytes([2, 3]) + struct.pack("<ii", 1, 2))
    for native in (True, False):
        with pytest.raises((msbfs_pkg.native.MsbfsError, formats.FormatError), match="truncated"):
            msbfs_pkg.QuerySet.from_file(p, use_native=native)


def test_csr_cache(tmp_path, msbfs_pkg):
    m = msbfs_pkg
    g = m.Graph.rmat(8, 4, 1)
    p = str(tmp_path / "c.bin")
    g.write(p)
    a = m.Graph.from_file(p, use_cache=True)
    assert os.path.exists(p + ".csr")
    b = m.Graph.from_file(p, use_cache=True)  # served from the sidecar
    assert np.array_equal(a.rowptr, b.rowptr) and np.array_equal(a.col, b.col)
    # a changed source invalidates the cache
    m.Graph.rmat(8, 5, 1).write(p)
    os.utime(p, (1, 1))
    c = m.Graph.from_file(p, use_cache=True)
    assert c.m == 256 * 5
    # same n and m (same file size), rewritten within the same second, mtime forced back to the
    # cached value: the ctime / sampled-content key still tells the graphs apart
    st = os.stat(p)
    d_src = m.Graph.rmat(8, 5, 2)
    d_src.write(p)
    os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))
    assert os.path.getsize(p) == st.st_size
    d = m.Graph.from_file(p, use_cache=True)
    ref = m.Graph.from_file(p, use_cache=False)
    assert np.array_equal(np.diff(d.rowptr), np.diff(ref.rowptr))
    assert not np.array_equal(np.diff(d.rowptr), np.diff(c.rowptr))
    # a truncated / corrupted cache is rejected and rebuilt, not used
    with open(p + ".csr", "r+b") as f:
        f.seek(-4, os.SEEK_END)
        f.write(b"\xff\xff\xff\x7f")
    e = m.Graph.from_file(p, use_cache=True)
    assert np.array_equal(np.sort(e.col), np.sort(ref.col))
    with open(p + ".csr", "r+b") as f:
        f.truncate(os.path.getsize(p + ".csr") - 100)
    e = m.Graph.from_file(p, use_cache=True)
    assert np.array_equal(np.diff(e.rowptr), np.diff(ref.rowptr))
    # no temporary files are left behind
    assert sorted(os.listdir(tmp_path)) == ["c.bin", "c.bin.csr"]


def test_csr_cache_write_is_best_effort(tmp_path, msbfs_pkg):
    """A cache that cannot be written (here: a directory sits at <graph>.csr, which defeats the
    final rename even for root) does not fail the load and leaves no temporary file behind."""
    m = msbfs_pkg
    p = str(tmp_path / "g.bin")
    m.Graph.rmat(7, 4, 3).write(p)
    os.mkdir(p + ".csr")
    g = m.Graph.from_file(p, use_cache=True)
    assert g.m == 128 * 4
    assert sorted(os.listdir(tmp_path)) == ["g.bin", "g.bin.csr"]
    assert os.path.isdir(p + ".csr")
