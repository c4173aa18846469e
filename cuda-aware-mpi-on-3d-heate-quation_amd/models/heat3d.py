"""The 3D heat equation model and its high-level solver driver.

``HeatEquation3D`` is the problem definition of the reference
(heat3D.cu:1-37 physics header, 331-367 constants, 408-453 IC/BC, 1093-1106
analytic steady state T = y).  ``HeatSolver`` drives the native MI355X engine
(csrc/runtime/solver.cpp) from Python: it picks the backend (gfx950 HIP or
OpenMP CPU), the communicator (RCCL over xGMI for one-process-per-GPU jobs,
sockets for multi-process CPU jobs, LocalComm for virtual ranks) and the
process grid, and exposes run / step / gather / checkpoint.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .._native import native


@dataclass(frozen=True)
class HeatEquation3D:
    """T_t = alpha * lap(T) on [0,1]^3, vertex-centred grid of n[0] x n[1] x n[2]."""

    n: Tuple[int, int, int]
    alpha: float = 1.0
    cfl: float = 0.4

    @property
    def h(self) -> Tuple[float, float, float]:
        return tuple(1.0 / (float(k) - 1.0) for k in self.n)  # type: ignore[return-value]

    @property
    def dt(self) -> float:
        return self.cfl * 1.0 / 6 * min(self.h) ** 2.0 / self.alpha

    @property
    def D(self) -> Tuple[float, float, float]:
        return tuple(self.dt * self.alpha / hh ** 2.0 for hh in self.h)  # type: ignore[return-value]

    @property
    def interior_points(self) -> int:
        return (self.n[0] - 2) * (self.n[1] - 2) * (self.n[2] - 2)

    def boundary_value(self, i: int, j: int, k: int) -> float:
        N = self.n
        if i == 0 or i == N[0] - 1 or k == 0 or k == N[2] - 1:
            return float(j) * self.h[1]
        if j == N[1] - 1:
            return 1.0
        return 0.0

    def initial_field(self, dtype=np.float64) -> np.ndarray:
        """Global initial condition: 0 inside, Dirichlet values on the boundary."""
        N = self.n
        y = np.arange(N[1], dtype=np.float64) * self.h[1]
        T = np.zeros(N, dtype=np.float64)
        T[:, N[1] - 1, :] = 1.0
        T[0, :, :] = y[:, None]
        T[-1, :, :] = y[:, None]
        T[:, :, 0] = y[None, :]
        T[:, :, -1] = y[None, :]
        return T.astype(dtype)

    def steady_state(self) -> np.ndarray:
        """Analytic steady state T = y (heat3D.cu:1096-1102)."""
        y = np.arange(self.n[1], dtype=np.float64) * self.h[1]
        return np.broadcast_to(y[None, :, None], self.n).copy()

    def error_percent(self, T: np.ndarray) -> float:
        """100 * mean |T - y| over interior points (the reference's 'L2-norm error')."""
        y = self.steady_state()
        d = np.abs(T[1:-1, 1:-1, 1:-1] - y[1:-1, 1:-1, 1:-1])
        return 100.0 * float(d.mean())


def _fmt(x) -> str:
    return repr(float(x)) if isinstance(x, float) else str(x)


class HeatSolver:
    """Python driver of the native engine.

    Parameters mirror the CLI (``heat3d NX NY NZ ITER_MAX EPS --flags``).  In a
    torch.distributed job (``WORLD_SIZE > 1``) the native communicator is
    bootstrapped through torch.distributed: RCCL for the HIP backend,
    sockets for the CPU backend.
    """

    def __init__(self, n: Sequence[int], iter_max: int = 1000, eps: float = 1e-5, *,
                 dtype: str = "fp64", backend: str = "auto", comm: str = "auto",
                 decomp: Optional[Sequence[int]] = None, virtual_ranks: int = 1,
                 kernel: str = "auto", graph: bool = True, overlap: bool = True,
                 check_every: int = 64, graph_chunk: int = 0, device: Optional[int] = None,
                 threads: int = 0, extra_args: Sequence[str] = (), group=None,
                 phantom: Optional[Sequence[int]] = None):
        ext = native()
        self.model = HeatEquation3D(tuple(int(v) for v in n))  # type: ignore[arg-type]
        args: List[str] = [str(int(v)) for v in n] + [str(int(iter_max)), _fmt(eps)]
        args += ["--dtype", dtype, "--kernel", kernel, "--check-every", str(check_every),
                 "--graph-chunk", str(graph_chunk)]
        if backend != "auto":
            args += ["--backend", backend]
        if decomp:
            args += ["--decomp", "x".join(str(int(d)) for d in decomp)]
        if virtual_ranks > 1:
            args += ["--virtual-ranks", str(virtual_ranks)]
        if not graph:
            args.append("--no-graph")
        if not overlap:
            args.append("--no-overlap")
        if threads:
            args += ["--threads", str(threads)]
        args += list(extra_args)
        self.args = args

        from ..parallel.distributed import env_info, native_comm_args

        info = env_info()
        use_gpu = backend == "hip" or (backend == "auto" and ext.device_count() > 0)
        if comm == "auto":
            if info.world_size > 1:
                comm = "rccl" if use_gpu else "socket"
            else:
                comm = "local"
        if phantom is not None:
            comm = "phantom"
        dev = -1 if device is None else int(device)
        if use_gpu and device is None and info.world_size > 1:
            dev = info.local_rank % max(1, ext.device_count())
        self.comm_kind = comm

        def make(extra=()):
            from ..parallel.distributed import NativeCommArgs

            if phantom is not None:
                # performance proxy: rank phantom[0] of a phantom[1]-rank job, peers emulated
                cargs = NativeCommArgs(int(phantom[0]), int(phantom[1]), "phantom")
            elif comm in ("rccl", "socket", "staged"):
                cargs = native_comm_args(comm, group=group)  # collective: every rank calls it
            else:
                cargs = NativeCommArgs()
            return ext.Solver(args + list(extra), device=dev, **cargs.kwargs())

        self._make = make
        self._s = make()
        self._initialized = False
        self.stream_graphs_retried = False

    # -- lifecycle -------------------------------------------------------------
    def initialize(self) -> "HeatSolver":
        """(Re)initialise the fields.  If the start-up canary of the
        overlapped schedule's per-stream hipGraphs deadlocks (the solver aborts
        its communicators and raises; every rank alike), the native solver is
        rebuilt once with the graphs off — a new communicator — and
        initialised again: the run continues eagerly in this process."""
        try:
            self._s.initialize()
        except RuntimeError as e:
            if "stream-graph canary deadlock" not in str(e) or self.stream_graphs_retried:
                raise
            import sys

            print(f"heat3d: {e}; rebuilding the solver with --stream-graphs off", file=sys.stderr, flush=True)
            self.stream_graphs_retried = True
            self._s = None
            self._s = self._make(["--stream-graphs", "off"])
            self._s.initialize()
        self._initialized = True
        return self

    def _ensure(self):
        if not self._initialized:
            self.initialize()

    def run(self) -> Dict:
        """Iterate until converged or ITER_MAX; returns the run report."""
        self._ensure()
        r = dict(self._s.run())
        g, loc = self._s.compute_error()
        r["error_percent"] = 100.0 * g
        r["error_percent_local"] = 100.0 * loc
        return r

    def step(self, n: int) -> None:
        """Enqueue exactly ``n`` iterations (asynchronous on the GPU)."""
        self._ensure()
        self._s.step(int(n))

    def synchronize(self) -> None:
        self._s.synchronize()

    def prepare_steps(self, n: int) -> None:
        """Capture (untimed) the hipGraph that ``step(n)`` will replay."""
        self._ensure()
        self._s.prepare_steps(int(n))

    def state(self) -> Dict:
        """Convergence state (iter, conv_iter, done, fault, norm, last_residual, ...).

        With the monotone check (Solver::resolve_coarse) the first call after a
        multi-rank run converged inside a sweep that computed only its last
        residual replays that sweep and all-reduces its residuals: call it on
        every rank then (``run()`` already does)."""
        return dict(self._s.state())

    # -- data ------------------------------------------------------------------
    def gather(self) -> Optional[np.ndarray]:
        """Global field (N0, N1, N2) as float64 on the root process, else None."""
        return self._s.gather_global()

    def local_field(self, idx: int = 0, ghosts: bool = False) -> np.ndarray:
        return self._s.local_field(idx, ghosts)

    def error_percent(self) -> Tuple[float, float]:
        g, loc = self._s.compute_error()
        return 100.0 * g, 100.0 * loc

    def write_tecplot(self, path: str = "output/out.dat", layout: str = "auto") -> None:
        self._s.write_tecplot(path, layout)

    def save_checkpoint(self, path: str) -> None:
        self._s.save_checkpoint(path)

    def load_checkpoint(self, path: str) -> None:
        self._s.load_checkpoint(path)

    # -- introspection -----------------------------------------------------------
    @property
    def native(self):
        return self._s

    @property
    def dims(self):
        return tuple(self._s.dims)

    @property
    def backend(self) -> str:
        return self._s.backend_name

    @property
    def kernel(self) -> str:
        return self._s.kernel_name

    @property
    def is_root(self) -> bool:
        return self._s.is_root

    @property
    def interior_points(self) -> int:
        return self._s.interior_points
