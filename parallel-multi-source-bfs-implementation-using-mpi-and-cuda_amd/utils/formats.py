"""Pure-numpy readers/writers for the reference's binary formats.

These are an independent implementation of the on-disk contract (used by tests to cross-check
the native mmap loader in csrc/src/io.cpp, and usable where the native library is absent).

Graph file (LoadGraphBin, reference main.cu:92-130): int32 n | int64 m | m x {int32 u, int32 v},
little endian, no magic. Edges are undirected; both directions are inserted (main.cu:113-115).

Query file (LoadQueryBin, reference main.cu:134-164): uint8 K | K x {uint8 size | size x int32}.
Extended format for K > 255 or sets > 255: byte 0 = 0 (a legacy K=0 file is
exactly one byte), magic b"MSBFSQX1", uint32 K, K x {uint32 size | size x int32}.
"""
from __future__ import annotations

import os
import struct
from typing import List, Sequence, Tuple

import numpy as np

QX_MAGIC = b"MSBFSQX1"


class FormatError(ValueError):
    pass


def write_graph_bin(path: str, n: int, u: np.ndarray, v: np.ndarray) -> None:
    u = np.asarray(u, dtype=np.int32)
    v = np.asarray(v, dtype=np.int32)
    if u.shape != v.shape:
        raise FormatError("u and v must have the same length")
    if n > np.iinfo(np.int32).max:
        raise FormatError("legacy graph format stores n as int32")
    e = np.empty((len(u), 2), dtype="<i4")
    e[:, 0] = u
    e[:, 1] = v
    with open(path, "wb") as f:
        f.write(struct.pack("<iq", int(n), len(u)))
        f.write(e.tobytes())


def read_graph_bin(path: str) -> Tuple[int, np.ndarray, np.ndarray]:
    """Returns (n, u, v). Validates truncation and id range (UB in the reference)."""
    try:
        size = os.path.getsize(path)
    except OSError:
        raise FormatError(f"Could not open graph file {path}")
    if size < 12:
        raise FormatError(f"graph file {path} is truncated (need 12-byte header)")
    with open(path, "rb") as f:
        n, m = struct.unpack("<iq", f.read(12))
        if n < 0 or m < 0:
            raise FormatError(f"graph file {path} has a negative n or m")
        if size < 12 + 8 * m:
            raise FormatError(f"graph file {path} is truncated: header says m={m}")
        e = np.frombuffer(f.read(8 * m), dtype="<i4").reshape(m, 2)
    u = e[:, 0].astype(np.int32)
    v = e[:, 1].astype(np.int32)
    if m and (u.min() < 0 or v.min() < 0 or u.max() >= n or v.max() >= n):
        raise FormatError(f"graph file {path} has a vertex id outside [0, n)")
    return int(n), u, v


def write_query_bin(path: str, groups: Sequence[Sequence[int]], force_extended: bool = False) -> None:
    K = len(groups)
    ext = force_extended or K > 255 or any(len(g) > 255 for g in groups)
    with open(path, "wb") as f:
        if not ext:
            f.write(bytes([K]))
            for g in groups:
                f.write(bytes([len(g)]))
                f.write(np.asarray(g, dtype="<i4").tobytes())
        else:
            f.write(b"\x00" + QX_MAGIC + struct.pack("<I", K))
            for g in groups:
                f.write(struct.pack("<I", len(g)))
                f.write(np.asarray(g, dtype="<i4").tobytes())


def read_query_bin(path: str) -> List[np.ndarray]:
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        raise FormatError(f"Could not open query file {path}")
    if not data:
        raise FormatError(f"query file {path} is empty")
    out: List[np.ndarray] = []
    if data[0] == 0 and len(data) >= 13 and data[1:9] == QX_MAGIC:
        (K,) = struct.unpack_from("<I", data, 9)
        pos = 13
        for _ in range(K):
            if pos + 4 > len(data):
                raise FormatError(f"query file {path} is truncated")
            (s,) = struct.unpack_from("<I", data, pos)
            pos += 4
            if pos + 4 * s > len(data):
                raise FormatError(f"query file {path} is truncated")
            out.append(np.frombuffer(data, dtype="<i4", count=s, offset=pos).astype(np.int32))
            pos += 4 * s
        return out
    K = data[0]
    pos = 1
    for _ in range(K):
        if pos + 1 > len(data):
            raise FormatError(f"query file {path} is truncated")
        s = data[pos]
        pos += 1
        if pos + 4 * s > len(data):
            raise FormatError(f"query file {path} is truncated")
        out.append(np.frombuffer(data, dtype="<i4", count=s, offset=pos).astype(np.int32))
        pos += 4 * s
    return out


def csr_from_edges(n: int, u: np.ndarray, v: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Symmetric CSR with int64 offsets; neighbour order = file order (main.cu:113-128)."""
    u = np.asarray(u, dtype=np.int64)
    v = np.asarray(v, dtype=np.int64)
    m = len(u)
    src = np.empty(2 * m, dtype=np.int64)
    dst = np.empty(2 * m, dtype=np.int32)
    # interleave (u->v, v->u) per edge, exactly the reference's push_back order
    src[0::2] = u
    src[1::2] = v
    dst[0::2] = v
    dst[1::2] = u
    order = np.argsort(src, kind="stable")
    col = dst[order]
    deg = np.bincount(src, minlength=n).astype(np.int64)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(deg, out=rowptr[1:])
    return rowptr, col.astype(np.int32)
