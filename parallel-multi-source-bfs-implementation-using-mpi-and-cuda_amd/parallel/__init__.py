"""Distribution over torch.distributed (RCCL / gloo): query-level data parallelism
(distributed.py) and the hybrid vertex-then-query decomposition (hybrid.py)."""
from . import distributed  # noqa: F401
from . import hybrid  # noqa: F401
