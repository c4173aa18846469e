"""Pure-PyTorch distributed reference solver (oracle for tests).

Implements the *intended* reference algorithm with torch
tensor ops and torch.distributed point-to-point halos, independent of the
native code: same decomposition rule (interior points split evenly, one-cell
ghost shells), same per-point expression order (heat3D.cu:128-131), same
convergence logic (norm = iteration-0 global residual, stop when
global max residual / norm < eps).  The update's fused multiply-adds (nvcc's
contraction of heat3D.cu:128-131, as in the native backends) are emulated
exactly with error-free transformations (utils/fma.py), so on CPU the field
is bitwise identical to the native backends.  Works with gloo (CPU) and nccl (GPU).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .topology import decompose, dims_create


def ftcs_update(T: torch.Tensor, D: Sequence[float]) -> torch.Tensor:
    """New values of the interior of a ghosted block ``T`` (shape n+2)."""
    from ..utils.fma import ftcs_update as upd

    c = T[1:-1, 1:-1, 1:-1]
    return upd(c, T[:-2, 1:-1, 1:-1], T[2:, 1:-1, 1:-1], T[1:-1, :-2, 1:-1], T[1:-1, 2:, 1:-1],
               T[1:-1, 1:-1, :-2], T[1:-1, 1:-1, 2:], D)


def boundary_grid(N: Sequence[int], dtype=torch.float64) -> torch.Tensor:
    """Global initial field: Dirichlet values on the boundary, 0 inside
    (heat3D.cu:408-453 order)."""
    hy = 1.0 / (N[1] - 1.0)
    T = torch.zeros(tuple(N), dtype=torch.float64)
    T[:, N[1] - 1, :] = 1.0
    y = torch.arange(N[1], dtype=torch.float64) * hy
    T[0, :, :] = y[:, None]
    T[N[0] - 1, :, :] = y[:, None]
    T[:, :, 0] = y[None, :]
    T[:, :, N[2] - 1] = y[None, :]
    return T.to(dtype)


def physics(N: Sequence[int]):
    h = [1.0 / (n - 1.0) for n in N]
    dt = 0.4 * 1.0 / 6 * min(h) ** 2.0 / 1.0
    return h, dt, [dt * 1.0 / hh ** 2.0 for hh in h]


class TorchReferenceSolver:
    def __init__(self, N: Sequence[int], eps: float, iter_max: int, dims: Optional[Sequence[int]] = None,
                 dtype=torch.float64, device="cpu", group=None):
        import torch.distributed as dist

        self.N = tuple(N)
        self.eps, self.iter_max = eps, iter_max
        self.dist = dist.is_initialized() and dist.get_world_size() > 1
        self.rank = dist.get_rank() if self.dist else 0
        self.size = dist.get_world_size() if self.dist else 1
        self.group = group
        self.dims = tuple(dims) if dims else dims_create(self.size)
        self.sub = decompose(self.N, self.dims)[self.rank]
        self.h, self.dt, self.D = physics(self.N)
        g = boundary_grid(self.N, dtype)
        s = self.sub
        sl = tuple(slice(s.gstart[a] - 1, s.gstart[a] + s.n[a] + 1) for a in range(3))
        self.T = g[sl].clone().to(device)
        self.device = device

    def _exchange(self):
        import torch.distributed as dist

        if not self.dist:
            return
        ops, recvs = [], []
        for f, nb in enumerate(self.sub.neighbors):
            if nb < 0:
                continue
            a, side = divmod(f, 2)
            own = [slice(1, -1)] * 3
            ghost = [slice(1, -1)] * 3
            own[a] = slice(-2, -1) if side else slice(1, 2)
            ghost[a] = slice(-1, None) if side else slice(0, 1)
            sbuf = self.T[tuple(own)].contiguous()
            rbuf = torch.empty_like(sbuf)
            ops.append(dist.P2POp(dist.isend, sbuf, nb))
            ops.append(dist.P2POp(dist.irecv, rbuf, nb))
            recvs.append((tuple(ghost), rbuf))
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        for sl, buf in recvs:
            self.T[sl] = buf

    def _allmax(self, v: float) -> float:
        import torch.distributed as dist

        if not self.dist:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def run(self):
        norm = 1.0
        conv = -1
        it = 0
        for it in range(self.iter_max):
            self._exchange()
            new = ftcs_update(self.T, self.D)
            res = (new - self.T[1:-1, 1:-1, 1:-1]).abs().max().double().item()  # field precision
            self.T[1:-1, 1:-1, 1:-1] = new
            r = self._allmax(max(res, 2.2250738585072014e-308))
            if it == 0 and r != 0.0:
                norm = r
            if r / norm < self.eps:
                conv = it
                break
        return {"converged": conv >= 0, "conv_iter": conv,
                "iterations": conv + 1 if conv >= 0 else self.iter_max, "norm": norm}

    def interior(self) -> torch.Tensor:
        return self.T[1:-1, 1:-1, 1:-1]

    def error_sum(self):
        y = (torch.arange(self.sub.n[1], dtype=torch.float64) + self.sub.gstart[1]) * self.h[1]
        e = (self.interior().double().cpu() - y[None, :, None]).abs().sum().item()
        return e, self.sub.n[0] * self.sub.n[1] * self.sub.n[2]
