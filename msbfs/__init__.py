"""Short import alias: `import msbfs` == the package in
`parallel-multi-source-bfs-implementation-using-mpi-and-cuda_amd/` (a directory name that is not a
Python identifier). Every submodule is registered under both names, so there is one module object
per file (one ctypes handle to libmsbfs.so)."""
import importlib
import os
import sys

_NAME = "parallel-multi-source-bfs-implementation-using-mpi-and-cuda_amd"
_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _root not in sys.path:
    sys.path.insert(0, _root)
_pkg = importlib.import_module(_NAME)
for _k, _v in list(sys.modules.items()):
    if _k == _NAME or _k.startswith(_NAME + "."):
        sys.modules["msbfs" + _k[len(_NAME):]] = _v
sys.modules[__name__] = _pkg
