"""The numpy twins of the native generators are bit-exact (the device generator is pinned to the
host one in tests/test_gpu_kernels.py)."""
import ctypes as C

import numpy as np

from msbfs.models import generators as G


def _native_rmat(m, scale, ef, seed, scramble=True):
    L = m.native.lib()
    pu, pv = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
    n, mm = C.c_int64(), C.c_int64()
    m.native.check(L.msbfs_gen_rmat_host(scale, ef, seed, 0.57, 0.19, 0.19, int(scramble),
                                         C.byref(pu), C.byref(pv), C.byref(n), C.byref(mm)))
    return m.native.take_array(pu, mm.value, np.int32), m.native.take_array(pv, mm.value, np.int32)


def test_rmat_twin_bit_exact(msbfs_pkg):
    for scale, ef, seed, scr in [(5, 4, 1, True), (10, 16, 7, True), (11, 2, 3, False)]:
        u, v = _native_rmat(msbfs_pkg, scale, ef, seed, scr)
        a, b = G.rmat_edges_np(scale, ef, seed, scramble=scr)
        assert np.array_equal(u, a) and np.array_equal(v, b)


def test_rmat_is_skewed_and_in_range(msbfs_pkg):
    g = msbfs_pkg.Graph.rmat(14, 16, 1)
    deg = g.degrees()
    assert g.n == 1 << 14 and g.m == 16 << 14
    assert deg.max() > 50 * deg.mean()          # power-law hubs
    assert (deg == 0).sum() > 0.05 * g.n        # RMAT leaves many isolated vertices


def test_scramble_is_bijective():
    for s in (1, 2, 7, 12):
        x = np.arange(1 << s, dtype=np.uint64)
        y = G.scramble_id(x, s, 99)
        assert len(np.unique(y)) == 1 << s and y.max() < (1 << s)


def test_queries_twin_bit_exact(msbfs_pkg):
    L = msbfs_pkg.native.lib()
    po, pi = C.POINTER(C.c_int64)(), C.POINTER(C.c_int32)()
    msbfs_pkg.native.check(L.msbfs_gen_queries(12345, 37, 5, 7, C.byref(po), C.byref(pi)))
    off = msbfs_pkg.native.take_array(po, 38, np.int64)
    ids = msbfs_pkg.native.take_array(pi, int(off[-1]), np.int32)
    q = msbfs_pkg.QuerySet.random(12345, 37, 5, 7)
    assert np.array_equal(q.off, off) and np.array_equal(q.ids, ids)


def test_uniform_and_grid_twins(msbfs_pkg):
    L = msbfs_pkg.native.lib()
    pu, pv = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
    msbfs_pkg.native.check(L.msbfs_gen_uniform_host(1000, 5000, 4, C.byref(pu), C.byref(pv)))
    u = msbfs_pkg.native.take_array(pu, 5000, np.int32)
    v = msbfs_pkg.native.take_array(pv, 5000, np.int32)
    a, b = G.uniform_edges_np(1000, 5000, 4)
    assert np.array_equal(u, a) and np.array_equal(v, b)
    n, mm = C.c_int64(), C.c_int64()
    msbfs_pkg.native.check(L.msbfs_gen_grid_host(7, 9, 0.8, 3, 5, C.byref(pu), C.byref(pv),
                                                 C.byref(n), C.byref(mm)))
    u = msbfs_pkg.native.take_array(pu, mm.value, np.int32)
    v = msbfs_pkg.native.take_array(pv, mm.value, np.int32)
    a, b = G.grid_edges_np(7, 9, 0.8, 3, 5)
    assert np.array_equal(u, a) and np.array_equal(v, b)
