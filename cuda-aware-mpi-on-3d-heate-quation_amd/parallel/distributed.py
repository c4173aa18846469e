"""Process bootstrap for the native communicators through torch.distributed.

One process per GPU (torchrun / ``python -m torch.distributed.run``).
torch.distributed is used only to *bootstrap* and for host-side barriers /
timing reductions; all per-iteration traffic goes through the native
communicators:

* ``rccl``   — rank 0 creates an ``ncclUniqueId`` (native), it is broadcast
  over a gloo group, every rank calls ``ncclCommInitRank`` in C++.  Halos are
  ncclSend/ncclRecv on device pointers over xGMI; the residual is an
  ncclAllReduce(max) on the device (replaces heat3D.cu:610-755, 1037-1063).
* ``socket`` — CPU backend: each rank opens a listening TCP socket, the
  address table is all-gathered, the native SocketComm builds a mesh.  With
  the HIP backend the same transport is wrapped in StagedComm (device buffers
  staged through host memory, as the reference's MPI path does); ``staged``
  forces that wrapper on the CPU backend as well.
"""
from __future__ import annotations

import json
import os
import socket
import sys
from dataclasses import dataclass, field
from typing import List, Optional

from .._native import native


@dataclass
class ProcessInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    master_addr: str = "127.0.0.1"


def env_info() -> ProcessInfo:
    def geti(*names, default):
        for n in names:
            v = os.environ.get(n)
            if v not in (None, ""):
                return int(v)
        return default

    rank = geti("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", default=0)
    ws = geti("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", default=1)
    lr = geti("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", default=rank)
    return ProcessInfo(rank, ws, lr, os.environ.get("MASTER_ADDR", "127.0.0.1"))


def init_process_group(backend: Optional[str] = None):
    """Initialise torch.distributed from the torchrun env (idempotent).

    Returns ``(info, bootstrap_group)``: the gloo group used for object
    collectives (a separate gloo group when the default backend is nccl).
    """
    import torch
    import torch.distributed as dist

    info = env_info()
    if info.world_size <= 1:
        return info, None
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if native().device_count() > 0 else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(info.local_rank % max(1, torch.cuda.device_count()))
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, init_method="env://", **kw)
    group = None
    if dist.get_backend() != "gloo":
        group = dist.new_group(backend="gloo")
    return info, group


@dataclass
class NativeCommArgs:
    rank: int = 0
    size: int = 1
    comm: str = "local"
    unique_id: bytes = b""
    listen_fd: int = -1
    addrs: List[str] = field(default_factory=list)

    def kwargs(self):
        return dict(rank=self.rank, size=self.size, comm=self.comm, unique_id=self.unique_id,
                    listen_fd=self.listen_fd, addrs=list(self.addrs))


def _route_ip(master: str) -> str:
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.connect((master, 9))
        ip = s.getsockname()[0]
        s.close()
        return ip
    except OSError:
        return "127.0.0.1"


class HostGroup:
    """Torch-free host collectives of a job (one process per rank).

    A star of TCP connections to rank 0 held open for the job (native
    ``net::Bootstrap``, the CLI's bootstrap, heat3D.cu:203-205's MPI_Init
    analogue).  bench.py's ranks use it instead of torch.distributed so that
    the process never loads torch, whose bundled HIP 7.0 runtime / RCCL 2.26
    would otherwise be the ones the solver binds to (one runtime per process:
    /opt/rocm's).  Objects travel as JSON.
    """

    def __init__(self, rank: int, size: int, master: str = "127.0.0.1", port: Optional[int] = None,
                 timeout_s: float = 600.0):
        self.rank, self.size = int(rank), int(size)
        if port is None:
            port = host_group_port()
        self._b = native().HostGroup(self.rank, self.size, master, int(port), float(timeout_s)) if size > 1 else None

    @classmethod
    def from_env(cls, timeout_s: float = 600.0) -> "HostGroup":
        info = env_info()
        return cls(info.rank, info.world_size, info.master_addr, None, timeout_s)

    def allgather(self, obj) -> list:
        if self._b is None:
            return [obj]
        blobs = self._b.allgather(json.dumps(obj).encode())
        return [json.loads(b.decode()) for b in blobs]

    def allgather_bytes(self, blob: bytes) -> List[bytes]:
        return [blob] if self._b is None else list(self._b.allgather(blob))

    def barrier(self) -> None:
        if self._b is not None:
            self._b.barrier()

    def max(self, value: float) -> float:
        return max(float(v) for v in self.allgather(float(value)))


def host_group_port() -> int:
    """HEAT3D_HOSTGROUP_PORT, else MASTER_PORT + 2 (torchrun's agent store owns
    MASTER_PORT, the native CLI bootstrap MASTER_PORT + 1)."""
    v = os.environ.get("HEAT3D_HOSTGROUP_PORT")
    if v:
        return int(v)
    return int(os.environ.get("MASTER_PORT", "29500")) + 2


def native_comm_args(kind: str, group=None) -> NativeCommArgs:
    """Bootstrap arguments for ``_heat3d.Solver``: through a :class:`HostGroup`
    (torch-free), else through torch.distributed."""
    if isinstance(group, HostGroup):
        if group.size == 1:
            return NativeCommArgs()
        rank, size = group.rank, group.size
        if kind == "rccl":
            uid = group.allgather_bytes(native().rccl_unique_id() if rank == 0 else b"")[0]
            return NativeCommArgs(rank, size, "rccl", unique_id=uid)
        if kind in ("socket", "staged"):
            fd, port = native().socket_listen()
            me = f"{_route_ip(os.environ.get('MASTER_ADDR', '127.0.0.1'))}:{port}"
            return NativeCommArgs(rank, size, kind, listen_fd=fd, addrs=[str(a) for a in group.allgather(me)])
        raise ValueError(f"unknown native comm kind {kind!r}")
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return NativeCommArgs()
    rank, size = dist.get_rank(), dist.get_world_size()
    if kind == "rccl":
        obj = [native().rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return NativeCommArgs(rank, size, "rccl", unique_id=obj[0])
    if kind in ("socket", "staged"):
        fd, port = native().socket_listen()
        me = f"{_route_ip(os.environ.get('MASTER_ADDR', '127.0.0.1'))}:{port}"
        table: List[Optional[str]] = [None] * size
        dist.all_gather_object(table, me, group=group)
        return NativeCommArgs(rank, size, kind, listen_fd=fd, addrs=[str(a) for a in table])
    raise ValueError(f"unknown native comm kind {kind!r}")


def _torch_dist():
    """torch.distributed if this process initialised it, else None — without
    importing torch (a torch-free rank must not load torch's HIP runtime)."""
    dist = sys.modules.get("torch.distributed")
    return dist if dist is not None and dist.is_initialized() else None


def barrier(group=None):
    if isinstance(group, HostGroup):
        group.barrier()
        return
    dist = _torch_dist()
    if dist is not None:
        dist.barrier(group=group)


def all_gather_objects(obj, group=None) -> list:
    """Host-side all-gather of an object (HostGroup: JSON; torch gloo group:
    pickle); [obj] alone."""
    if isinstance(group, HostGroup):
        return group.allgather(obj)
    dist = _torch_dist()
    if dist is None or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj, group=group)
    return out


def max_over_ranks(value: float, group=None) -> float:
    """Host-side max of a scalar over ranks (HostGroup or gloo bootstrap group)."""
    if isinstance(group, HostGroup):
        return group.max(value)
    dist = _torch_dist()
    if dist is None or dist.get_world_size() == 1:
        return value
    import torch

    dev = "cpu"
    if group is None and dist.get_backend() == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
