"""Graph / query "models": the data the engine runs on (CSR graphs, query groups, generators)."""
from .graph import DeviceGraph, Graph  # noqa: F401
from .queries import QuerySet  # noqa: F401
from . import generators  # noqa: F401
