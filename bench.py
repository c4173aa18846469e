#!/usr/bin/env python3
"""Headline benchmark: GLUPS of the FTCS 7-point heat solver, 1024^3 fp64.

BASELINE.json metric "GLUPS (cell-updates/sec, whole node) + time-to-converge,
1024^3 fp64 grid".  One process per GPU (torchrun); the global grid is fixed
(strong scaling): 1 GPU -> 1x1x1, N GPUs -> N x 1 x 1 slabs (BASELINE config
3: 1D slab decomposition + 2-neighbour halo over xGMI, RCCL on device
pointers).  Every timed step is a full iteration of the production loop:
interior sweep || (halo exchange -> boundary shell), fused residual, RCCL
all-reduce(max) of the residual and the device-side convergence check
(eps = 0 so it never stops early).  Synthetic data = the reference's analytic
initial/boundary condition.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GLUPS (cell-updates/sec, whole node) + time-to-converge, 1024^3 fp64 grid"


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--weak-block", type=int, default=0,
                    help="weak scaling: each GPU owns B^3 interior points, global grid = dims*B + 2 "
                         "(BASELINE config 5: B=2047 fp32 gives 4096^3 on 8 GPUs)")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--decomp", default="auto", help="auto | slab | block | AxBxC")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--graph-chunk", type=int, default=32)
    ap.add_argument("--converge-eps", type=float, default=1e-3,
                    help="also measure time-to-converge at this EPS (0 disables)")
    ap.add_argument("--temporal", type=int, default=0, help="0 auto | 1 single-step | K (2..6) K-step temporally blocked sweeps")
    ap.add_argument("--kernel2", default="auto", help="temporally blocked sweep kernel (tbK / trK[:V:R:WZ:WY:L:Q])")
    ap.add_argument("--virtual-ranks", type=int, default=1,
                    help="diagnostic: split the grid into this many subdomains on one GPU (not the headline)")
    ap.add_argument("--comm", default="auto", choices=["auto", "rccl", "socket"],
                    help="multi-process transport: auto = RCCL over xGMI; socket = host-staged TCP "
                         "(rehearses the N>1 launch with several ranks on one GPU, which RCCL refuses)")
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()

    import torch

    import heat3d_amd
    from heat3d_amd import HeatSolver
    from heat3d_amd.parallel import best_dims_for, dims_create
    from heat3d_amd.parallel.distributed import barrier, init_process_group, max_over_ranks
    from heat3d_amd.utils.metrics import roofline_glups

    ext = heat3d_amd.native()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with "
              f"python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}",
              file=sys.stderr)
        return 2
    info, group = init_process_group(("gloo" if args.comm == "socket" else "nccl") if world > 1 else None)
    rank = info.rank
    if ext.device_count() < 1:
        print("bench.py: no HIP device visible", file=sys.stderr)
        return 2
    dev = info.local_rank % ext.device_count()
    torch.cuda.set_device(dev)

    G = args.grid
    N = (G, G, G)
    nparts = world * args.virtual_ranks
    if args.virtual_ranks > 1:
        assert world == 1, "--virtual-ranks is a single-process diagnostic"
    if args.decomp in ("auto", "slab", "block"):
        dims = best_dims_for(N, nparts, None if args.decomp == "auto" else args.decomp)
    else:
        dims = tuple(int(v) for v in args.decomp.lower().split("x"))
    assert dims[0] * dims[1] * dims[2] == nparts, (dims, nparts)
    if args.weak_block:
        N = tuple(d * args.weak_block + 2 for d in dims)
        G = N[0]

    def make(eps, iter_max):
        return HeatSolver(N, iter_max=iter_max, eps=eps, dtype=args.dtype, backend="hip",
                          decomp=dims, kernel=args.kernel, graph=not args.no_graph,
                          overlap=not args.no_overlap, graph_chunk=args.graph_chunk,
                          device=dev, group=group, virtual_ranks=args.virtual_ranks, comm=args.comm,
                          extra_args=["--temporal", str(args.temporal), "--kernel2", args.kernel2])

    s = make(0.0, 1 << 40)
    s.initialize()
    s.step(args.warmup)
    s.synchronize()
    barrier(group)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.step(args.steps)
    s.synchronize()
    torch.cuda.synchronize()
    barrier(group)
    t1 = time.perf_counter()
    dt = max_over_ranks(t1 - t0, group)
    st = s.state()
    # every issued iteration must have been checked and none skipped
    assert st["iter"] == args.warmup + args.steps and st["done"] == 0, st
    points = s.interior_points
    value = points * args.steps / dt / 1e9
    esize = 8 if args.dtype == "fp64" else 4
    kernel = s.kernel
    comm_name = s.native.comm_name
    del s

    ttc = None
    if args.converge_eps and args.converge_eps > 0:
        c = make(args.converge_eps, 10 ** 7)
        c.initialize()
        barrier(group)
        r = c.run()
        ttc = {"eps": args.converge_eps, "converged": bool(r["converged"]),
               "iterations": int(r["conv_iter"]), "seconds": max_over_ranks(r["seconds"], group),
               "error_percent": r["error_percent"]}
        del c

    par = "x".join(str(d) for d in dims)
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GLUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.weak_block else "strong",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (analytic Dirichlet IC/BC of the reference, random-free)",
        "config": {"model": f"heat3d FTCS 7-point, {'x'.join(map(str, N)) if len(set(N)) > 1 else f'{G}^3'} {args.dtype} grid",
                   "grid": list(N),
                   "global_batch": 1, "seq_len": G, "parallelism": f"{'slab' if dims[1] == dims[2] == 1 and dims[0] > 1 else 'block'} {par}"
                   + (f" ({args.virtual_ranks} virtual ranks on 1 GPU)" if args.virtual_ranks > 1 else ""),
                   "kernel": kernel, "graph": not args.no_graph, "overlap": not args.no_overlap,
                   "comm": comm_name},
        "glups_per_gpu": round(value / world, 3),
        "effective_hbm_tbps_per_gpu": round(value / world * 2 * esize / 1e3, 3),
        "vs_roofline": round(value / roofline_glups(esize, world), 4),
        "time_to_converge": ttc,
        "baseline_note": "reference publishes no numbers (BASELINE.md); roofline = 6.29 TB/s / (2*esize) per GPU",
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
