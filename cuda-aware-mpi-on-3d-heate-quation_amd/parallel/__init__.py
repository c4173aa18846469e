"""Topology, decomposition and communicator bootstrap.

Per-iteration traffic is native (RCCL over xGMI / sockets, csrc/comm);
torch.distributed or the native HostGroup only bootstraps it (distributed.py).  torch_reference.py is
an independent pure-PyTorch distributed oracle used by the tests.
"""
from .topology import (SLAB_MIN_LINK_GBPS, best_dims_for, choose_dims, decomp_candidates, decompose,  # noqa: F401
                       dims_create, field_bytes_per_rank, halo_bytes_per_iteration, pick_measured, reference_legal)

__all__ = ["dims_create", "decompose", "reference_legal", "halo_bytes_per_iteration",
           "field_bytes_per_rank", "best_dims_for", "choose_dims", "SLAB_MIN_LINK_GBPS", "decomp_candidates",
           "pick_measured"]
