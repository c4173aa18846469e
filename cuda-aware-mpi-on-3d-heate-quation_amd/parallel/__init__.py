"""Topology, decomposition and communicator bootstrap.

Per-iteration traffic is native (RCCL over xGMI / sockets, csrc/comm);
torch.distributed only bootstraps it (distributed.py).  torch_reference.py is
an independent pure-PyTorch distributed oracle used by the tests.
"""
from .topology import (SLAB_MIN_LINK_GBPS, best_dims_for, choose_dims, decompose, dims_create,  # noqa: F401
                       field_bytes_per_rank, halo_bytes_per_iteration, reference_legal)

__all__ = ["dims_create", "decompose", "reference_legal", "halo_bytes_per_iteration",
           "field_bytes_per_rank", "best_dims_for", "choose_dims", "SLAB_MIN_LINK_GBPS"]
