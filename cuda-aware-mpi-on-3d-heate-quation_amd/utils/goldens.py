"""Convergence goldens of the intended reference algorithm.

(N, eps) -> (0-based converged iteration, error %, iteration-0 norm).
``eps=None`` rows are ITER_MAX-limited runs.  Produced by an analysis-only
NumPy/OpenMP model of heat3D.cu with a working interior update; the native
CPU and GPU backends reproduce them exactly (tests/test_goldens.py).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

GOLDENS: Dict[Tuple[int, Optional[float]], Tuple[int, float, float]] = {
    (27, 1e-3): (938, 1.9155, 0.194872),
    (27, 1e-4): (1725, 0.1923, 0.194872),
    (27, 1e-5): (2513, 0.0192, 0.194872),
    (33, 1e-5): (3590, 0.0287, 0.195833),
    (64, 1e-3): (1915, 11.0449, 0.197884),
    (64, 1e-4): (6548, 1.0742, 0.197884),
    (64, 1e-5): (11173, 0.1077, 0.197884),
    (65, 1e-5): (11466, 0.1110, 0.197917),
    (129, 1e-3): (1929, 26.1990, 0.198958),
    (129, 1e-4): (15379, 4.2828, 0.198958),
    (129, 1e-5): (34324, 0.4359, 0.198958),
    (257, 1e-3): (2060, 36.4656, 0.199479),
    (257, 1e-4): (17957, 16.9804, 0.199479),
    (257, 1e-5): (91362, 1.7195, 0.199479),
    # round 3: the native CPU backend (OpenMP, exact FMA; the definition every
    # GPU kernel is bitwise-tested against), 513^3 fp64, 270 s on 6 threads
    (513, 1e-3): (2132, 42.7695, 0.199740),
    # round 5: the native CPU backend, 1024^3 fp64 (the headline grid), 3244 s
    # on 6 threads (profiles/golden_1024_cpu_r05.log)
    (1024, 1e-3): (2170, 46.2574, 0.199870),
}
# 27^3 with ITER_MAX = 100 (not converged): error 26.0129 %
ITERMAX_100_27 = 26.0129


def golden(n: int, eps: float) -> Tuple[int, float, float]:
    return GOLDENS[(n, eps)]
