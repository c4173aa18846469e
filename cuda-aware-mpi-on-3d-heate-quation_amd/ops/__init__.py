"""Kernel-level ops on torch tensors (gfx950 HIP kernels / OpenMP CPU kernels)."""
from .stencil import (PaddedField, ftcs_reference, ftcs_step, ftcs_step2, init_field, sweep3,  # noqa: F401
                      new_state, pack_box, residual_from_state, sweep, unpack_box)

__all__ = ["PaddedField", "ftcs_step", "ftcs_step2", "ftcs_reference", "init_field", "sweep3", "pack_box",
           "unpack_box", "new_state", "residual_from_state", "sweep"]
