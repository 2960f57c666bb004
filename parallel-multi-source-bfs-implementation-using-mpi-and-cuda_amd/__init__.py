"""msbfs — MI355X-native multi-source BFS / distance-to-set engine.

Capabilities of irmakerkol/Parallel-Multi-Source-BFS-Implementation-Using-MPI-and-CUDA (a single
CUDA/MPI file, main.cu), re-designed for AMD Instinct MI355X (gfx950):

  models/    Graph (host CSR, int64 offsets), DeviceGraph (HBM CSR, device RMAT generator),
             QuerySet, generators (RMAT / uniform / grid, query groups)
  ops/       native binding (libmsbfs.so: hand-written HIP kernels), multi-source BFS solvers
             (bit-parallel, per-group distance, top-down, reference sweep, CPU), oracles
  parallel/  query-level data parallelism over torch.distributed (RCCL over xGMI / gloo)
  utils/     binary formats, 7-line report, timers, TEPS accounting
  engine     end-to-end job with the reference's phase boundaries

The compute path is native (C++/HIP in csrc/); the native CLI `_bin/msbfs` is the drop-in for the
reference binary (`mpirun -np R msbfs -g G.bin -q Q.bin -gn N`).
"""
import importlib as _importlib
import sys as _sys

__version__ = "0.1.0"

from .ops import native  # noqa: E402
from .ops.bfs import BfsResult, Solver, argmin_first, cpu_bfs, multi_source_bfs  # noqa: E402
from .models.graph import DeviceGraph, Graph  # noqa: E402
from .models.queries import QuerySet  # noqa: E402
from .models import generators  # noqa: E402
from .utils import formats, report, teps  # noqa: E402
from .parallel import distributed  # noqa: E402
from . import engine  # noqa: E402
from .engine import Engine, JobConfig, JobResult  # noqa: E402

SUBMODULES = ["ops", "ops.native", "ops.bfs", "ops.reference", "models", "models.graph",
              "models.queries", "models.generators", "parallel", "parallel.distributed",
              "utils", "utils.formats", "utils.report", "utils.teps", "engine"]

for _m in SUBMODULES:
    _importlib.import_module(f"{__name__}.{_m}")
