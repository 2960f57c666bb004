"""ctypes binding of the native engine ``_lib/libmsbfs.so`` (C API: csrc/include/msbfs/msbfs.h).

The compute path is native C++/HIP for gfx950; Python only marshals arrays. The library is
built in-tree by ``__graft_entry__.build()`` / ``make -C csrc``. On a machine with a GPU a
missing library is a hard error (no silent fallback to a Python path); on a CPU-only machine
host-side functions (I/O, generators, CPU BFS) still come from the same library.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional

import numpy as np

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MSBFS_LIB: load another build of the engine (A/B timing of two builds in one GPU session)
LIB_PATH = os.environ.get("MSBFS_LIB") or os.path.join(_PKG_DIR, "_lib", "libmsbfs.so")
CLI_PATH = os.path.join(_PKG_DIR, "_bin", "msbfs")

ALGOS = {"auto": 0, "bitpar": 1, "dist": 2, "topdown": 3, "sweep": 4, "cpu": 5}

_lock = threading.Lock()
_lib: Optional[C.CDLL] = None

i64p = C.POINTER(C.c_int64)
i32p = C.POINTER(C.c_int32)


class MsbfsError(RuntimeError):
    pass


# void (*)(void* user, int chunk, int64_t i0, int64_t i1): one range of a chunked hybrid phase A
ChunkFn = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int64, C.c_int64)


class Stats(C.Structure):
    _fields_ = [("levels", C.c_int64), ("td_levels", C.c_int64), ("bu_levels", C.c_int64),
                ("batches", C.c_int64), ("device_ms", C.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class Level(C.Structure):
    """One BFS level of a solver run (msbfs_level in msbfs.h)."""
    _fields_ = [("batch", C.c_int32), ("level", C.c_int32), ("dir", C.c_char),
                ("pad", C.c_char * 3), ("nf", C.c_int64), ("ef", C.c_int64),
                ("nf_next", C.c_int64), ("active", C.c_int64), ("ms", C.c_double)]

    def as_dict(self):
        return {"batch": self.batch, "level": self.level, "dir": self.dir.decode(),
                "nf": self.nf, "ef": self.ef, "nf_next": self.nf_next, "active": self.active,
                "ms": self.ms}


class Options(C.Structure):
    _fields_ = [("alpha", C.c_double), ("beta", C.c_double), ("wide_degree", C.c_int),
                ("force_dir", C.c_int), ("max_words", C.c_int)]


def _sig(lib):
    vp = C.c_void_p
    P = C.POINTER
    specs = {
        "msbfs_last_error": (C.c_char_p, []),
        "msbfs_version": (C.c_char_p, []),
        "msbfs_free": (None, [vp]),
        "msbfs_device_count": (C.c_int, [P(C.c_int)]),
        "msbfs_set_device": (C.c_int, [C.c_int]),
        "msbfs_device_sync": (C.c_int, []),
        "msbfs_read_graph_csr": (C.c_int, [C.c_char_p, C.c_int, i64p, i64p, P(i64p), P(i32p)]),
        "msbfs_read_edge_list": (C.c_int, [C.c_char_p, i64p, i64p, P(i32p), P(i32p)]),
        "msbfs_write_edge_list": (C.c_int, [C.c_char_p, C.c_int64, C.c_int64, i32p, i32p]),
        "msbfs_read_queries": (C.c_int, [C.c_char_p, i64p, P(i64p), i64p, P(i32p)]),
        "msbfs_write_queries": (C.c_int, [C.c_char_p, C.c_int64, i64p, i32p, C.c_int]),
        "msbfs_build_csr": (C.c_int, [C.c_int64, C.c_int64, i32p, i32p, C.c_int, P(i64p), P(i32p)]),
        "msbfs_gen_rmat_host": (C.c_int, [C.c_int, C.c_int64, C.c_uint64, C.c_double, C.c_double,
                                          C.c_double, C.c_int, P(i32p), P(i32p), i64p, i64p]),
        "msbfs_gen_uniform_host": (C.c_int, [C.c_int64, C.c_int64, C.c_uint64, P(i32p), P(i32p)]),
        "msbfs_gen_grid_host": (C.c_int, [C.c_int64, C.c_int64, C.c_double, C.c_int64, C.c_uint64,
                                          P(i32p), P(i32p), i64p, i64p]),
        "msbfs_gen_queries": (C.c_int, [C.c_int64, C.c_int64, C.c_int64, C.c_uint64, P(i64p),
                                        P(i32p)]),
        "msbfs_cpu_run": (C.c_int, [C.c_int64, i64p, i32p, C.c_int64, i64p, i32p, i64p, i64p,
                                    C.c_int]),
        "msbfs_graph_from_host_csr": (C.c_int, [C.c_int, C.c_int64, i64p, i32p, P(vp)]),
        "msbfs_graph_from_device_edges": (C.c_int, [C.c_int, C.c_int64, C.c_int64, vp, vp, P(vp)]),
        "msbfs_graph_wrap_device": (C.c_int, [C.c_int, C.c_int64, C.c_int64, vp, vp, P(vp)]),
        "msbfs_graph_gen_rmat": (C.c_int, [C.c_int, C.c_int, C.c_int64, C.c_uint64, C.c_double,
                                           C.c_double, C.c_double, C.c_int, P(vp)]),
        "msbfs_graph_gen_uniform": (C.c_int, [C.c_int, C.c_int64, C.c_int64, C.c_uint64, P(vp)]),
        "msbfs_graph_from_edge_file": (C.c_int, [C.c_int, C.c_char_p, P(vp)]),
        "msbfs_graph_sort_rows": (C.c_int, [vp]),
        "msbfs_graph_relabel_by_degree": (C.c_int, [vp]),
        "msbfs_graph_relabel_map": (C.c_int, [vp, i32p]),
        "msbfs_graph_is_relabelled": (C.c_int, [vp]),
        "msbfs_graph_info": (C.c_int, [vp, i64p, i64p, i64p, i64p, i64p]),
        "msbfs_graph_device_ptrs": (C.c_int, [vp, P(vp), P(vp)]),
        "msbfs_graph_download": (C.c_int, [vp, i64p, i32p]),
        "msbfs_graph_free": (None, [vp]),
        "msbfs_solver_create": (C.c_int, [vp, C.c_int, C.c_int64, P(vp)]),
        "msbfs_solver_set_options": (C.c_int, [vp, P(Options)]),
        "msbfs_solver_tune": (C.c_int, [vp, C.c_char_p]),
        "msbfs_solver_prepare": (C.c_int, [vp, vp]),
        "msbfs_solver_prepare_hybrid": (C.c_int, [vp, C.c_int, C.c_int, vp]),
        "msbfs_solver_run": (C.c_int, [vp, C.c_int64, i64p, i32p, i64p, i64p, P(Stats), vp]),
        "msbfs_solver_free": (None, [vp]),
        "msbfs_solver_levels": (C.c_int64, [vp, P(Level), C.c_int64]),
        "msbfs_argmin": (C.c_int64, [i64p, C.c_int64]),
        "msbfs_hybrid_extent": (C.c_int, [vp, i64p]),
        "msbfs_solver_hybrid_max_groups": (C.c_int64, [vp]),
        "msbfs_solver_hybrid_phase_a": (C.c_int, [vp, C.c_int64, i64p, i32p, C.c_int, C.c_int,
                                                  C.c_int64, C.c_int, i32p, vp, i64p, P(Stats),
                                                  vp]),
        "msbfs_solver_hybrid_phase_a_coded": (C.c_int, [vp, C.c_int64, i64p, i32p, C.c_int,
                                                        C.c_int, C.c_int64, C.c_int, i32p, vp,
                                                        i64p, i64p, P(Stats), vp]),
        "msbfs_solver_hybrid_decode": (C.c_int, [vp, vp, i64p, C.c_int, C.c_int64, C.c_int, vp,
                                                 vp]),
        "msbfs_solver_hybrid_chunk_bounds": (C.c_int, [vp, C.c_int, C.c_int, C.c_int64, C.c_int,
                                                       i64p]),
        "msbfs_solver_hybrid_phase_a_chunked": (C.c_int, [vp, C.c_int64, i64p, i32p, C.c_int,
                                                          C.c_int, C.c_int64, C.c_int, i32p, vp,
                                                          i64p, C.c_int, ChunkFn, vp, P(Stats),
                                                          vp]),
        "msbfs_solver_hybrid_phase_c": (C.c_int, [vp, C.c_int64, C.c_int, C.c_int, C.c_int,
                                                  C.c_int64, vp, i64p, i64p, P(Stats), vp]),
    }
    for name, (res, args) in specs.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def lib() -> C.CDLL:
    """Load (once) and return the native library; raises MsbfsError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise MsbfsError(
                    f"native engine not built: {LIB_PATH} is missing "
                    "(run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C csrc`)")
            l = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
            _sig(l)
            _lib = l
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except (MsbfsError, OSError):
        return False


def check(rc: int) -> None:
    if rc != 0:
        raise MsbfsError(lib().msbfs_last_error().decode(errors="replace"))


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def take_array(p, count: int, dtype) -> np.ndarray:
    """Copy a malloc'd native buffer into numpy and free it."""
    out = np.empty(count, dtype=dtype)
    if count:
        C.memmove(out.ctypes.data, p, count * out.itemsize)
    lib().msbfs_free(C.cast(p, C.c_void_p))
    return out


def device_count() -> int:
    n = C.c_int(0)
    check(lib().msbfs_device_count(C.byref(n)))
    return n.value


def version() -> str:
    return lib().msbfs_version().decode()
