"""Distribution: query-level data parallelism over torch.distributed (RCCL / gloo)."""
from . import distributed  # noqa: F401
