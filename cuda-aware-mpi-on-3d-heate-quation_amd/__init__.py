"""heat3d-mi355x: an MI355X-native 3D heat-equation (FTCS 7-point) solver.

Same capabilities as ``fredrickhang/Cuda-aware-MPI-on-3D-heate-quation``
(reference ``HeatEquation3D/src/heat3D.cu``): explicit forward-Euler 7-point
update on a vertex-centred unit cube, Dirichlet steady state ``T = y``,
relative per-step residual stop, 3D Cartesian domain decomposition with halo
exchange, global reductions, Tecplot output — re-designed for gfx950:
hand-written HIP kernels, RCCL over xGMI on device pointers, HIP streams for
comm/compute overlap, hipGraph-captured iterations, device-side convergence.

Import as ``heat3d_amd`` (repo-root alias module) — this directory's name is
not a Python identifier.

Sub-packages
------------
models    problem definitions and the high-level ``HeatSolver`` driver
ops       kernel-level ops on torch tensors (gfx950 kernels + torch references)
parallel  topology / decomposition mirrors, torch.distributed bootstrap of the
          native RCCL / socket communicators, a pure-torch distributed oracle
utils     goldens, metrics (GLUPS, roofline), Tecplot reader, timers
"""
from __future__ import annotations

__version__ = "0.1.0"

from . import _native  # noqa: F401  (the one HIP runtime of the process: _native.RUNTIME)
from ._native import available as native_available  # noqa: F401
from ._native import native, runtime  # noqa: F401
from . import models, parallel, utils  # noqa: F401,E402
from .models.heat3d import HeatEquation3D, HeatSolver  # noqa: F401

__all__ = ["HeatEquation3D", "HeatSolver", "native", "native_available", "runtime", "__version__"]


def __getattr__(name):
    # ops works on torch tensors: imported on first use, so that a torch-free
    # process (HEAT3D_RUNTIME=rocm) never loads torch
    if name == "ops":
        import importlib

        return importlib.import_module(__name__ + ".ops")
    raise AttributeError(name)
