"""Kernel-level ops on torch tensors.

The padded field layout of the native engine (csrc/kernels/layout.hpp: owned
block + one-cell ghost shell, z fastest, rows padded so the first owned z
point is 128-byte aligned) is allocated as a flat torch tensor; ``PaddedField``
exposes strided views of it.  ``ftcs_step`` launches the hand-written gfx950
kernel on torch's current HIP stream (or the OpenMP kernel for CPU tensors);
``ftcs_reference`` is the plain-PyTorch oracle of the same arithmetic
(heat3D.cu:128-131 with nvcc's FMA contraction, emulated exactly).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch

from .._native import native

_DT = {torch.float64: "fp64", torch.float32: "fp32"}


class PaddedField:
    """One subdomain field in the native padded layout."""

    def __init__(self, n: Sequence[int], dtype=torch.float64, device="cpu", gx: int = 1, gy: int = 1, gz: int = 1):
        if dtype not in _DT:
            raise TypeError(f"unsupported dtype {dtype}")
        self.n = tuple(int(v) for v in n)
        self.dtype = dtype
        self.gx = int(gx)  # ghost planes per x side (deep halos of the K-step slab schedule)
        self.gy, self.gz = int(gy), int(gz)  # ghost rows / columns (deep y / z halos of block splits)
        self.layout = native().layout(list(self.n), torch.tensor([], dtype=dtype).element_size(), self.gx,
                                      self.gy, self.gz)
        self.flat = torch.zeros(self.layout["elems"], dtype=dtype, device=device)

    @property
    def device(self):
        return self.flat.device

    @property
    def dt(self) -> str:
        return _DT[self.dtype]

    def ghosted(self) -> torch.Tensor:
        """View (n0+2, n1+2, n2+2) including the ghost shell."""
        L = self.layout
        off = L["origin"] - L["sx"] - L["sy"] - 1
        shape = tuple(v + 2 for v in self.n)
        return self.flat.as_strided(shape, (L["sx"], L["sy"], 1), off)

    def deep3(self) -> torch.Tensor:
        """View (n0+2gx, n1+2gy, n2+2gz): every ghost layer on every axis."""
        L = self.layout
        off = L["origin"] - self.gx * L["sx"] - self.gy * L["sy"] - self.gz
        shape = (self.n[0] + 2 * self.gx, self.n[1] + 2 * self.gy, self.n[2] + 2 * self.gz)
        return self.flat.as_strided(shape, (L["sx"], L["sy"], 1), off)

    def deep(self) -> torch.Tensor:
        """View (n0+2*gx, n1+2, n2+2): every ghost plane plus the y/z ghost shell."""
        L = self.layout
        off = L["origin"] - self.gx * L["sx"] - L["sy"] - 1
        shape = (self.n[0] + 2 * self.gx, self.n[1] + 2, self.n[2] + 2)
        return self.flat.as_strided(shape, (L["sx"], L["sy"], 1), off)

    def owned(self) -> torch.Tensor:
        L = self.layout
        return self.flat.as_strided(self.n, (L["sx"], L["sy"], 1), L["origin"])

    def data_ptr(self) -> int:
        return self.flat.data_ptr()


def _stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def ftcs_step(src: PaddedField, dst: PaddedField, D: Sequence[float],
              box: Optional[Sequence[int]] = None, kernel: str = "auto",
              state: Optional[torch.Tensor] = None, slot: int = 0) -> None:
    """dst[box] = FTCS(src) on the owned box (default: all owned points).

    ``state``: optional uint8/int64 tensor of ``DEVICE_STATE_BYTES`` that
    receives the fused max-residual (IEEE bits of a double in its first
    8 bytes for slot 0) and whose ``done`` word turns the kernel into a no-op.
    """
    if src.layout != dst.layout or src.dtype != dst.dtype or src.device != dst.device:
        raise ValueError("src and dst must share layout, dtype and device")
    n = src.n
    b = list(box) if box is not None else [0, n[0], 0, n[1], 0, n[2]]
    for a in range(3):
        if not (0 <= b[2 * a] <= b[2 * a + 1] <= n[a]):
            raise ValueError(f"box {b} outside owned extents {n}")
    sptr = 0
    if state is not None:
        if state.device != src.device or state.numel() * state.element_size() < native().DEVICE_STATE_BYTES:
            raise ValueError("state tensor too small or on the wrong device")
        sptr = state.data_ptr()
    ext = native()
    if src.device.type == "cuda":
        ext.hip.stencil(src.dt, src.data_ptr(), dst.data_ptr(), list(n), b, list(D), sptr, slot,
                        kernel, _stream_ptr(src.flat))
    else:
        ext.cpu.stencil(src.dt, src.data_ptr(), dst.data_ptr(), list(n), b, list(D), sptr, slot)


def ftcs_step2(src: PaddedField, dst: PaddedField, D: Sequence[float], kernel: str = "auto",
               state: Optional[torch.Tensor] = None, slot: int = 0) -> None:
    """dst = K FTCS steps of src in ONE temporally blocked sweep (gfx950).

    ``kernel`` picks the depth and variant: ``tl2`` .. ``tl6[:V:R:WZ:WY:L:Q]``
    (the lean K-step kernel, stencil_tbl.hip / stencil_tbp.hip); ``auto`` is
    ``tl2``.  The ghost shell of ``src`` is treated as constant (Dirichlet)
    for every step; the residual of step s lands in ``state`` slot
    ``slot + s``.  Bitwise identical to K ``ftcs_step`` calls.
    """
    if src.layout != dst.layout or src.dtype != dst.dtype or src.device != dst.device:
        raise ValueError("src and dst must share layout, dtype and device")
    if src.device.type != "cuda":
        raise ValueError("ftcs_step2 runs on the GPU")
    sptr = 0
    if state is not None:
        if state.device != src.device or state.numel() * state.element_size() < native().DEVICE_STATE_BYTES:
            raise ValueError("state tensor too small or on the wrong device")
        sptr = state.data_ptr()
    native().hip.stencil2(src.dt, src.data_ptr(), dst.data_ptr(), list(src.n), list(D), sptr, slot,
                          kernel, _stream_ptr(src.flat))


def sweep(src: PaddedField, dst: PaddedField, D: Sequence[float], box: Sequence[int],
          ux: Sequence[int] = (0, -1), kernel: str = "tl3", state: Optional[torch.Tensor] = None,
          slot: int = 0) -> None:
    """One K-step sweep (K from ``kernel``: tl2..tl6) on ``box``
    = (x0, x1, y0, y1, z0, z1) of a deep-ghost field, with the intermediate
    steps computed on the x range ``ux`` (the solver's x-slab schedule).
    GPU tensors run the gfx950 kernel, CPU tensors the K-single-steps
    definition (csrc/kernels/kernels_cpu.cpp)."""
    if src.layout != dst.layout or src.dtype != dst.dtype or src.device != dst.device:
        raise ValueError("src and dst must share layout, dtype and device")
    sptr = 0
    if state is not None:
        if state.device != src.device or state.numel() * state.element_size() < native().DEVICE_STATE_BYTES:
            raise ValueError("state tensor too small or on the wrong device")
        sptr = state.data_ptr()
    args = (src.dt, src.data_ptr(), dst.data_ptr(), list(src.n), src.gx, list(box), list(ux), list(D), sptr, slot,
            kernel)
    if src.device.type == "cuda":
        native().hip.stencil_sweep(*args, _stream_ptr(src.flat))
    else:
        native().cpu.stencil_sweep(*args)


def sweep3(src: PaddedField, dst: PaddedField, D: Sequence[float], box: Sequence[int], u: Sequence[int],
           kernel: str = "tl3", state: Optional[torch.Tensor] = None, slot: int = 0) -> None:
    """K-step sweep with deep ghosts on every axis (the block-decomposition
    schedule): ``u`` = (ux0, ux1, uy0, uy1, uz0, uz1) are the update ranges of
    the intermediate steps.  GPU tensors run the lean kernel, CPU tensors the
    K-single-steps definition."""
    if src.layout != dst.layout or src.dtype != dst.dtype or src.device != dst.device:
        raise ValueError("src and dst must share layout, dtype and device")
    sptr = 0
    if state is not None:
        if state.device != src.device or state.numel() * state.element_size() < native().DEVICE_STATE_BYTES:
            raise ValueError("state tensor too small or on the wrong device")
        sptr = state.data_ptr()
    args = (src.dt, src.data_ptr(), dst.data_ptr(), list(src.n), [src.gx, src.gy, src.gz], list(box), list(u),
            list(D), sptr, slot, kernel)
    if src.device.type == "cuda":
        native().hip.stencil_sweep3(*args, _stream_ptr(src.flat))
    else:
        native().cpu.stencil_sweep3(*args)


def init_field(f: PaddedField, gstart: Sequence[int], N: Sequence[int], h: Sequence[float]) -> None:
    """Analytic IC/BC into the padded field (reference heat3D.cu:408-453)."""
    ext = native()
    if f.device.type == "cuda":
        ext.hip.init_field(f.dt, f.data_ptr(), list(f.n), list(gstart), list(N), list(h), _stream_ptr(f.flat))
    else:
        ext.cpu.init_field(f.dt, f.data_ptr(), list(f.n), list(gstart), list(N), list(h))


def pack_box(f: PaddedField, box: Sequence[int], out: torch.Tensor) -> None:
    """Copy a local box (ghost indices allowed, -1..n) into a contiguous buffer (GPU)."""
    native().hip.pack_box(f.dt, f.data_ptr(), list(f.n), list(box), out.data_ptr(), _stream_ptr(f.flat))


def unpack_box(f: PaddedField, box: Sequence[int], buf: torch.Tensor) -> None:
    native().hip.unpack_box(f.dt, f.data_ptr(), list(f.n), list(box), buf.data_ptr(), _stream_ptr(f.flat))


def ftcs_reference(T: torch.Tensor, D: Sequence[float]) -> Tuple[torch.Tensor, float]:
    """Plain-PyTorch FTCS on a ghosted block; returns (new interior, max |dT|).

    Same arithmetic as the native backends (exactly rounded FMAs emulated with
    error-free transformations, utils/fma.py), so results compare bitwise."""
    from ..utils.fma import ftcs_update

    c = T[1:-1, 1:-1, 1:-1]
    new = ftcs_update(c, T[:-2, 1:-1, 1:-1], T[2:, 1:-1, 1:-1], T[1:-1, :-2, 1:-1], T[1:-1, 2:, 1:-1],
                      T[1:-1, 1:-1, :-2], T[1:-1, 1:-1, 2:], D)
    # residual in the field's precision (kernels.hpp resid_abs), widened for the max
    res = (new - c).abs().max().double().item() if new.numel() else 0.0
    return new, res


def residual_from_state(state: torch.Tensor, slot: int = 0) -> float:
    """Decode the fused residual (double bits) written by ftcs_step."""
    raw = state.detach().cpu().contiguous().view(torch.uint8)[8 * slot: 8 * slot + 8]
    return float(raw.view(torch.float64).item())


def new_state(device, eps: float = 0.0) -> torch.Tensor:
    """Zeroed DeviceState buffer with the residual slots at their initial value."""
    ext = native()
    st = torch.zeros(ext.DEVICE_STATE_BYTES // 8, dtype=torch.int64)
    init = ext.RESIDUAL_INIT_BITS
    st[: ext.RESIDUAL_SLOTS] = init if init < 2 ** 63 else init - 2 ** 64
    return st.to(device)
