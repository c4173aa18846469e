#!/usr/bin/env python3
"""Check of hipGraph replays of the overlapped multi-stream schedule.

The overlapped schedules replay one linear graph per stream (compute, comm,
reduce), each launched on its own stream, with device-side signal / wait
kernels for the cross-stream dependencies (csrc/runtime/hip_backend.cpp).
Runs the same solve twice on one GPU — eager (--no-graph) and graph-captured —
with P virtual ranks (LocalComm: halo copies on the comm stream, boundary slabs
on the comm stream, residual check on the reduce stream, interior on the
compute stream), or as a phantom rank (PhantomComm: delay kernels standing in
for RCCL), and compares the fields bitwise.

  python tools/graph_multistream_probe.py --n 96 --ranks 8 --decomp 8x1x1 --steps 60
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=96)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--decomp", default="8x1x1")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--phantom", default="", help="R/P: run rank R of a P-rank job (PhantomComm)")
    args = ap.parse_args()

    import numpy as np

    import heat3d_amd
    from heat3d_amd import HeatSolver

    dims = tuple(int(v) for v in args.decomp.split("x"))
    N = (args.n,) * 3

    def solve(graph: bool):
        # the overlapped schedules' per-stream graphs are opt-in (--stream-graphs on)
        kw = dict(dtype=args.dtype, backend="hip", decomp=dims, graph=graph, graph_chunk=36, device=0,
                  extra_args=["--stream-graphs", "on"])
        if args.phantom:
            r, p = (int(v) for v in args.phantom.split("/"))
            s = HeatSolver(N, iter_max=1 << 30, eps=0.0, phantom=(r, p), **kw)
        else:
            s = HeatSolver(N, iter_max=1 << 30, eps=0.0, virtual_ranks=args.ranks, **kw)
        s.initialize()
        s.prepare_steps(args.steps)
        s.step(args.steps)
        s.synchronize()
        st = s.state()
        out = [s.local_field(i) for i in range(s.native.num_local)]
        info = dict(graph_launches=s.native.graph_launches, K=s.native.temporal_steps,
                    nbuf=s.native.field_buffers, kernel=s.kernel, iter=st["iter"], done=st["done"])
        return out, info

    eager, ie = solve(False)
    print("eager:", ie, flush=True)
    graph, ig = solve(True)
    print("graph:", ig, flush=True)
    same = all(np.array_equal(a.view(np.uint64), b.view(np.uint64)) for a, b in zip(eager, graph))
    print("bitwise_equal:", same, "graph_used:", ig["graph_launches"] > 0, flush=True)
    return 0 if same and ig["graph_launches"] > 0 and ie["iter"] == ig["iter"] else 1


if __name__ == "__main__":
    sys.exit(main())
