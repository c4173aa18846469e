"""Host timers (the reference timed the loop with MPI_Wtime, heat3D.cu:525-527, 1081)."""
from __future__ import annotations

import time


class Timer:
    def __init__(self):
        self.elapsed = 0.0

    def __enter__(self):
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.elapsed = time.perf_counter() - self._t0
        return False
