"""Formats, reporting, timing and TEPS accounting."""
from . import formats, report, teps  # noqa: F401
