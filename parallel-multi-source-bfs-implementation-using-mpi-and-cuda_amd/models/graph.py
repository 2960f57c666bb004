"""Graphs: host CSR (`Graph`) and HBM-resident CSR (`DeviceGraph`).

Reference: LoadGraphBin (main.cu:92-130) builds an int32-offset CSR on rank 0 from the binary
edge list; main.cu:282-291 copies it to the GPU. Here offsets are int64 (RMAT-26 ef16 has
2m = 2^31 adjacency entries, which overflows the reference), host loading is an mmap + parallel
count/scan/scatter in C++ with an optional CSR sidecar cache, and a DeviceGraph can also be
generated directly in HBM (no host edge list, no broadcast).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np

from ..ops import native
from ..utils import formats
from . import generators as gen


class Graph:
    """Symmetric CSR on the host: rowptr[n+1] int64, col[2m] int32."""

    def __init__(self, n: int, rowptr: np.ndarray, col: np.ndarray, m: Optional[int] = None,
                 edges: Optional[Tuple[np.ndarray, np.ndarray]] = None):
        self.n = int(n)
        self.rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        self.col = np.ascontiguousarray(col, dtype=np.int32)
        if len(self.rowptr) != self.n + 1 or self.rowptr[-1] != len(self.col):
            raise ValueError("inconsistent CSR")
        self.m = int(m) if m is not None else len(self.col) // 2
        self.edges = edges  # original edge list (u, v) if known, for writing .bin files

    @property
    def nnz(self) -> int:
        return len(self.col)

    def degrees(self) -> np.ndarray:
        return np.diff(self.rowptr)

    # ---- construction
    @classmethod
    def from_edges(cls, n: int, u, v, stable: bool = False, use_native: bool = True) -> "Graph":
        u = np.ascontiguousarray(u, dtype=np.int32)
        v = np.ascontiguousarray(v, dtype=np.int32)
        if use_native and native.available():
            L = native.lib()
            pr = C.POINTER(C.c_int64)()
            pc = C.POINTER(C.c_int32)()
            native.check(L.msbfs_build_csr(n, len(u), native.ptr(u, C.c_int32),
                                           native.ptr(v, C.c_int32), int(stable), C.byref(pr),
                                           C.byref(pc)))
            rowptr = native.take_array(pr, n + 1, np.int64)
            col = native.take_array(pc, int(rowptr[-1]), np.int32)
        else:
            if len(u) and (min(u.min(), v.min()) < 0 or max(u.max(), v.max()) >= n):
                raise formats.FormatError("edge has a vertex id outside [0, n)")
            rowptr, col = formats.csr_from_edges(n, u, v)
        return cls(n, rowptr, col, m=len(u), edges=(u, v))

    @classmethod
    def from_file(cls, path: str, use_cache: bool = False, use_native: bool = True) -> "Graph":
        if use_native and native.available():
            L = native.lib()
            n = C.c_int64()
            m = C.c_int64()
            pr = C.POINTER(C.c_int64)()
            pc = C.POINTER(C.c_int32)()
            native.check(L.msbfs_read_graph_csr(path.encode(), int(use_cache), C.byref(n),
                                                C.byref(m), C.byref(pr), C.byref(pc)))
            rowptr = native.take_array(pr, n.value + 1, np.int64)
            col = native.take_array(pc, int(rowptr[-1]), np.int32)
            return cls(n.value, rowptr, col, m=m.value)
        n, u, v = formats.read_graph_bin(path)
        return cls.from_edges(n, u, v, stable=True, use_native=False)

    @classmethod
    def rmat(cls, scale: int, edgefactor: int = 16, seed: int = 1, a: float = 0.57,
             b: float = 0.19, c: float = 0.19, scramble: bool = True) -> "Graph":
        if native.available():
            L = native.lib()
            pu = C.POINTER(C.c_int32)()
            pv = C.POINTER(C.c_int32)()
            n = C.c_int64()
            m = C.c_int64()
            native.check(L.msbfs_gen_rmat_host(scale, edgefactor, seed, a, b, c, int(scramble),
                                               C.byref(pu), C.byref(pv), C.byref(n), C.byref(m)))
            u = native.take_array(pu, m.value, np.int32)
            v = native.take_array(pv, m.value, np.int32)
            return cls.from_edges(n.value, u, v)
        u, v = gen.rmat_edges_np(scale, edgefactor, seed, a, b, c, scramble)
        return cls.from_edges(1 << scale, u, v, use_native=False)

    @classmethod
    def uniform(cls, n: int, m: int, seed: int = 1) -> "Graph":
        u, v = gen.uniform_edges_np(n, m, seed)
        return cls.from_edges(n, u, v)

    @classmethod
    def grid(cls, rows: int, cols: int, keep: float = 1.0, shortcuts: int = 0,
             seed: int = 1) -> "Graph":
        u, v = gen.grid_edges_np(rows, cols, keep, shortcuts, seed)
        return cls.from_edges(rows * cols, u, v)

    def write(self, path: str) -> None:
        """Write the legacy binary edge list (needs the original edges)."""
        if self.edges is None:
            # reconstruct one direction of every undirected edge from the CSR (u <= v rows),
            # self-loops appear twice in row u and are written once per pair
            src = np.repeat(np.arange(self.n, dtype=np.int64), self.degrees())
            dst = self.col.astype(np.int64)
            keep = src < dst
            loops = np.nonzero(src == dst)[0]
            u = np.concatenate([src[keep], src[loops[::2]]]).astype(np.int32)
            v = np.concatenate([dst[keep], dst[loops[::2]]]).astype(np.int32)
        else:
            u, v = self.edges
        if native.available():
            native.check(native.lib().msbfs_write_edge_list(
                path.encode(), self.n, len(u), native.ptr(np.ascontiguousarray(u), C.c_int32),
                native.ptr(np.ascontiguousarray(v), C.c_int32)))
        else:
            formats.write_graph_bin(path, self.n, u, v)

    def to_device(self, device: int = 0) -> "DeviceGraph":
        return DeviceGraph.from_host(self, device)

    def __repr__(self) -> str:
        return f"Graph(n={self.n}, m={self.m}, nnz={self.nnz})"


class DeviceGraph:
    """CSR resident in one GPU's HBM (native handle)."""

    def __init__(self, handle: C.c_void_p, device: int, keepalive=None):
        self._h = handle
        self.device = device
        self._keepalive = keepalive
        self._refresh()

    def _refresh(self) -> None:
        n, nnz, m, mx, iso = (C.c_int64() for _ in range(5))
        native.check(native.lib().msbfs_graph_info(self._h, C.byref(n), C.byref(nnz), C.byref(m),
                                                   C.byref(mx), C.byref(iso)))
        self.n, self.nnz, self.m = n.value, nnz.value, m.value
        self.max_degree, self.isolated = mx.value, iso.value

    @property
    def handle(self) -> C.c_void_p:
        if self._h is None:
            raise native.MsbfsError("DeviceGraph is closed")
        return self._h

    @classmethod
    def from_host(cls, g: Graph, device: int = 0) -> "DeviceGraph":
        h = C.c_void_p()
        native.check(native.lib().msbfs_graph_from_host_csr(
            device, g.n, native.ptr(g.rowptr, C.c_int64), native.ptr(g.col, C.c_int32),
            C.byref(h)))
        return cls(h, device)

    @classmethod
    def rmat(cls, scale: int, edgefactor: int = 16, seed: int = 1, a: float = 0.57,
             b: float = 0.19, c: float = 0.19, scramble: bool = True,
             device: int = 0, relabel: bool = False) -> "DeviceGraph":
        """Generate the RMAT graph directly in HBM (two-pass count/scatter, no edge list)."""
        h = C.c_void_p()
        native.check(native.lib().msbfs_graph_gen_rmat(device, scale, edgefactor, seed, a, b, c,
                                                       int(scramble), C.byref(h)))
        g = cls(h, device)
        return g.relabel_by_degree() if relabel else g

    @classmethod
    def from_file(cls, path: str, device: int = 0, relabel: bool = False) -> "DeviceGraph":
        """Build the CSR of a legacy graph file (main.cu:92-130) on the device: the mapped edge
        list is streamed to HBM and counted / scattered there (no host CSR build)."""
        h = C.c_void_p()
        native.check(native.lib().msbfs_graph_from_edge_file(device, str(path).encode(),
                                                             C.byref(h)))
        g = cls(h, device)
        return g.relabel_by_degree() if relabel else g

    @classmethod
    def uniform(cls, n: int, m: int, seed: int = 1, device: int = 0) -> "DeviceGraph":
        h = C.c_void_p()
        native.check(native.lib().msbfs_graph_gen_uniform(device, n, m, seed, C.byref(h)))
        return cls(h, device)

    @classmethod
    def wrap(cls, n: int, rowptr_t, col_t, device: int = 0) -> "DeviceGraph":
        """Borrow torch device tensors (int64 rowptr, int32 col) without copying."""
        h = C.c_void_p()
        native.check(native.lib().msbfs_graph_wrap_device(
            device, n, int(col_t.numel()), C.c_void_p(rowptr_t.data_ptr()),
            C.c_void_p(col_t.data_ptr()), C.byref(h)))
        return cls(h, device, keepalive=(rowptr_t, col_t))

    def device_ptrs(self) -> Tuple[int, int]:
        r = C.c_void_p()
        c = C.c_void_p()
        native.check(native.lib().msbfs_graph_device_ptrs(self.handle, C.byref(r), C.byref(c)))
        return r.value, c.value

    def sort_rows(self) -> "DeviceGraph":
        native.check(native.lib().msbfs_graph_sort_rows(self.handle))
        return self

    def relabel_by_degree(self) -> "DeviceGraph":
        """Renumber vertices by descending degree (hubs first, sorted rows) in place. Queries
        keep using the original ids — solvers map sources through the stored map; F(U) is
        label-invariant. download() then returns the relabelled CSR."""
        native.check(native.lib().msbfs_graph_relabel_by_degree(self.handle))
        self._refresh()
        return self

    @property
    def relabelled(self) -> bool:
        return bool(native.lib().msbfs_graph_is_relabelled(self.handle))

    def relabel_map(self) -> np.ndarray:
        """old2new[v] = internal id of user vertex v."""
        out = np.empty(self.n, dtype=np.int32)
        native.check(native.lib().msbfs_graph_relabel_map(self.handle, native.ptr(out, C.c_int32)))
        return out

    def hybrid_extent(self) -> int:
        """1 + the last vertex with deg > 0: the vertices the hybrid mode exchanges (after degree
        relabelling the isolated vertices form the suffix [extent, n))."""
        out = np.zeros(1, dtype=np.int64)
        native.check(native.lib().msbfs_hybrid_extent(self.handle, native.ptr(out, C.c_int64)))
        return int(out[0])

    def download(self) -> Graph:
        rowptr = np.empty(self.n + 1, dtype=np.int64)
        col = np.empty(self.nnz, dtype=np.int32)
        native.check(native.lib().msbfs_graph_download(self.handle, native.ptr(rowptr, C.c_int64),
                                                       native.ptr(col, C.c_int32)))
        return Graph(self.n, rowptr, col, m=self.m)

    def close(self) -> None:
        if self._h is not None:
            native.lib().msbfs_graph_free(self._h)
            self._h = None
        self._keepalive = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __repr__(self) -> str:
        return (f"DeviceGraph(n={self.n}, m={self.m}, nnz={self.nnz}, device={self.device}, "
                f"max_degree={self.max_degree}, isolated={self.isolated})")
