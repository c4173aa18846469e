"""Goldens, metrics, Tecplot reader and timers."""
from .goldens import GOLDENS, golden  # noqa: F401
from .metrics import effective_bandwidth, glups, roofline_glups  # noqa: F401
from .tecplot import read_tecplot  # noqa: F401

__all__ = ["GOLDENS", "golden", "glups", "effective_bandwidth", "roofline_glups", "read_tecplot"]
