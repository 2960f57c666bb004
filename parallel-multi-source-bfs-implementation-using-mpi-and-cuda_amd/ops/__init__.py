"""Compute operators: native binding + multi-source BFS solvers + test oracles."""
from . import native  # noqa: F401
