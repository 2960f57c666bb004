"""Query groups U_1..U_K packed as CSR (off[K+1] int64, ids int32).

Reference: LoadQueryBin (main.cu:134-164) returns vector<vector<int>>; the reference then issues
2K+1 MPI_Bcast calls to replicate it (main.cu:257-280). A packed QuerySet is one contiguous blob
(two arrays) and is broadcast in one shot by parallel.distributed.broadcast_queries.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, List, Sequence

import numpy as np

from ..ops import native
from ..utils import formats
from .generators import query_groups_np


class QuerySet:
    def __init__(self, off: np.ndarray, ids: np.ndarray):
        self.off = np.ascontiguousarray(off, dtype=np.int64)
        self.ids = np.ascontiguousarray(ids, dtype=np.int32)
        if self.off.ndim != 1 or len(self.off) < 1 or self.off[0] != 0:
            raise ValueError("QuerySet.off must start at 0")
        if self.off[-1] != len(self.ids):
            raise ValueError("QuerySet.off[-1] must equal len(ids)")

    # ---- construction
    @classmethod
    def from_groups(cls, groups: Iterable[Sequence[int]]) -> "QuerySet":
        groups = [np.asarray(g, dtype=np.int32).ravel() for g in groups]
        off = np.zeros(len(groups) + 1, dtype=np.int64)
        if groups:
            np.cumsum([len(g) for g in groups], out=off[1:])
            ids = np.concatenate(groups) if off[-1] else np.zeros(0, np.int32)
        else:
            ids = np.zeros(0, np.int32)
        return cls(off, ids)

    @classmethod
    def from_file(cls, path: str, use_native: bool = True) -> "QuerySet":
        if use_native and native.available():
            L = native.lib()
            K = C.c_int64()
            nids = C.c_int64()
            po = C.POINTER(C.c_int64)()
            pi = C.POINTER(C.c_int32)()
            native.check(L.msbfs_read_queries(path.encode(), C.byref(K), C.byref(po), C.byref(nids),
                                              C.byref(pi)))
            off = native.take_array(po, K.value + 1, np.int64)
            ids = native.take_array(pi, nids.value, np.int32)
            return cls(off, ids)
        return cls.from_groups(formats.read_query_bin(path))

    @classmethod
    def random(cls, n: int, K: int, size: int, seed: int = 7) -> "QuerySet":
        """K groups of `size` uniform vertex ids (bit-identical to the native --qgen)."""
        return cls.from_groups(query_groups_np(n, K, size, seed))

    # ---- access
    @property
    def K(self) -> int:
        return len(self.off) - 1

    def __len__(self) -> int:
        return self.K

    def group(self, k: int) -> np.ndarray:
        return self.ids[self.off[k]:self.off[k + 1]]

    def groups(self) -> List[np.ndarray]:
        return [self.group(k) for k in range(self.K)]

    def subset(self, indices: Sequence[int]) -> "QuerySet":
        return QuerySet.from_groups([self.group(int(k)) for k in indices])

    def write(self, path: str, force_extended: bool = False, use_native: bool = True) -> None:
        if use_native and native.available():
            native.check(native.lib().msbfs_write_queries(
                path.encode(), self.K, native.ptr(self.off, C.c_int64),
                native.ptr(self.ids, C.c_int32), int(force_extended)))
        else:
            formats.write_query_bin(path, self.groups(), force_extended)

    def __eq__(self, other) -> bool:
        return (isinstance(other, QuerySet) and np.array_equal(self.off, other.off)
                and np.array_equal(self.ids, other.ids))

    def __repr__(self) -> str:
        return f"QuerySet(K={self.K}, ids={len(self.ids)})"
