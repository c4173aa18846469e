"""Performance metrics for the 7-point stencil."""
from __future__ import annotations

# measured HBM copy bandwidth of one MI355X (MI355X_MICROARCH.md: 6.29 TB/s float4 copy)
HBM_BW_BYTES_PER_S = 6.29e12


def glups(points: int, iterations: int, seconds: float) -> float:
    """Giga lattice-point updates per second."""
    return points * iterations / seconds / 1e9 if seconds > 0 else 0.0


def bytes_per_point(esize: int) -> int:
    """Compulsory HBM traffic per updated point: read once + write once."""
    return 2 * esize


def effective_bandwidth(glups_value: float, esize: int) -> float:
    """Effective HBM bandwidth in TB/s implied by a GLUPS figure."""
    return glups_value * 1e9 * bytes_per_point(esize) / 1e12


def roofline_glups(esize: int, n_gpus: int = 1, bw: float = HBM_BW_BYTES_PER_S) -> float:
    return n_gpus * bw / bytes_per_point(esize) / 1e9
