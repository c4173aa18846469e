"""Problem definitions (model families) for the heat3d engine.

Only one physical model exists in the reference (heat3D.cu): the 3D heat
equation with the Dirichlet steady state T = y.
"""
from .heat3d import HeatEquation3D, HeatSolver  # noqa: F401

__all__ = ["HeatEquation3D", "HeatSolver"]
