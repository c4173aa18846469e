"""Torch-free rank of a multi-process CPU job (tests/test_hostgroup.py).

Bootstraps through the native HostGroup (no torch.distributed), solves with
the socket transport, and checks the process never loaded torch
(HEAT3D_RUNTIME=rocm, the bench's runtime policy).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HEAT3D_RUNTIME"] = "rocm"

import numpy as np  # noqa: E402

import heat3d_amd  # noqa: E402
from heat3d_amd.parallel.distributed import HostGroup, all_gather_objects, barrier, max_over_ranks  # noqa: E402


def main():
    out, n, eps, decomp = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), sys.argv[4]
    g = HostGroup.from_env(timeout_s=120)
    rank = g.rank
    s = heat3d_amd.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", comm="socket", group=g,
                              decomp=[int(v) for v in decomp.split("x")],
                              extra_args=["--temporal", "3"])
    r = s.run()
    field = s.gather()
    objs = all_gather_objects({"rank": rank, "iter": int(r["conv_iter"])}, g)
    mx = max_over_ranks(float(rank), g)
    barrier(g)
    assert "torch" not in sys.modules, "a HEAT3D_RUNTIME=rocm rank imported torch"
    if rank == 0:
        np.save(os.path.join(out, "field.npy"), field)
        with open(os.path.join(out, "result.json"), "w") as f:
            json.dump({"iter": int(r["conv_iter"]), "objs": objs, "max": mx,
                       "runtime_policy": heat3d_amd._native.RUNTIME}, f)


if __name__ == "__main__":
    main()
