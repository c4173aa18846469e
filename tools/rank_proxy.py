#!/usr/bin/env python3
"""Per-GPU time of the multi-GPU bench, measured on one GPU (performance proxy).

Runs rank R of a P-rank decomposition of the bench grid alone on the device
(PhantomComm, csrc/comm/phantom_comm.cpp): that rank's own kernels, streams and
schedule — interior sweep || (emulated halo exchange -> boundary slabs),
lagged all-reduce — with the peers' traffic replaced by a D2D copy plus a
one-workgroup delay of bytes / --gbps per exchange and --ar-us per all-reduce.
The projected node GLUPS assumes every rank takes as long as this one.  It
is a model input, not a measurement of xGMI; the driver's multi-GPU bench run
is the real number.

  python tools/rank_proxy.py --ranks 8 [--rank 1] [--grid 1024] [--gbps 50] [--ar-us 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--rank", type=int, default=-1, help="default: an inner rank (two neighbours)")
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--decomp", default="auto")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--gbps", type=float, default=50.0, help="emulated halo bandwidth per peer (GB/s)")
    ap.add_argument("--ar-us", type=float, default=20.0, help="emulated all-reduce latency (us)")
    ap.add_argument("--wire", default="serial", choices=["serial", "overlap", "paced"],
                    help="serial: an exchange is bytes / gbps, then the stand-in D2D copies; overlap: the "
                         "copies run inside the wire time (a transport moving data while on the wire); paced: "
                         "the copies move the data at the wire rate over the wire time (RCCL-like channels, "
                         "no burst)")
    ap.add_argument("--footprint", default="small", choices=["rccl", "small"],
                    help="stand-in comm kernels sized as RCCL's device kernel (256 threads, 140 VGPRs, 20 KB "
                         "LDS: they wait for CUs as RCCL does) or small (64 threads, round 4's proxy)")
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--extra", default="", help="extra solver flags, e.g. '--no-overlap'")
    ap.add_argument("--preheat-ms", type=float, default=0.0,
                    help="as bench.py --preheat-ms: untimed idempotent sweeps right before the timed window "
                         "(the driver-config rehearsal: --steps 20 --warmup 5 --preheat-ms 20)")
    ap.add_argument("--idle-ms", type=float, default=0.0,
                    help="diagnostic: host sleep between the synchronised warm-up / preheat and the timed window "
                         "(the GPU idles that long; does the first timed sweep slow down?)")
    ap.add_argument("--no-sync", action="store_true",
                    help="diagnostic: do not synchronise between the preheat and the timed window (the timed window "
                         "then also waits for the preheat's tail: not a valid timing, a trace-shape probe)")
    ap.add_argument("--trace-schedule", action="store_true",
                    help="print the start-up schedule tuner's candidate timings (HEAT3D_TRACE, read once: on for the whole run)")
    args = ap.parse_args()

    import heat3d_amd
    from heat3d_amd import HeatSolver
    from heat3d_amd.parallel import best_dims_for

    N = (args.grid,) * 3
    P = args.ranks
    if args.decomp in ("auto", "slab", "block"):
        dims = best_dims_for(N, P, None if args.decomp == "auto" else args.decomp)
    else:
        dims = tuple(int(v) for v in args.decomp.lower().split("x"))
    r = args.rank if args.rank >= 0 else min(1, P - 1)
    gb = lambda b: None if b is None else round(b / 1e9, 2)
    s = HeatSolver(N, iter_max=1 << 40, eps=0.0, dtype=args.dtype, backend=args.backend, decomp=dims,
                   device=0 if args.backend == "hip" else None, phantom=(r, P),
                   extra_args=["--phantom-gbps", str(args.gbps), "--phantom-allreduce-us", str(args.ar_us),
                               "--phantom-wire", args.wire, "--phantom-footprint", args.footprint]
                   + (args.extra.split() if args.extra else []))
    if args.trace_schedule:
        os.environ["HEAT3D_TRACE"] = "1"
    s.initialize()
    os.environ.pop("HEAT3D_TRACE", None)
    free_after, total = s.native.mem_info()
    s.step(args.warmup)
    s.prepare_steps(args.steps)
    s.synchronize()
    preheat = 0
    if args.preheat_ms > 0:
        K = s.native.temporal_steps
        est_ms = s.interior_points / P * max(1, K) / (800e9 if args.dtype == "fp64" else 1400e9) * 1e3
        preheat = s.native.preheat(max(1, min(64, int(args.preheat_ms / max(est_ms, 1e-3)) + 1)))
        if not args.no_sync:
            s.synchronize()
    if args.idle_ms > 0:
        time.sleep(args.idle_ms / 1e3)
    t0 = time.perf_counter()
    s.step(args.steps)
    s.synchronize()
    dt = time.perf_counter() - t0
    st = s.state()
    assert st["iter"] == args.warmup + args.steps, st
    # the schedule's phases per sweep (after the timed window, as bench.py's 'phases')
    phases = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in s.native.profile_sweeps(8).items()}
    out = {"proxy": "phantom rank", "rank": r, "ranks": P, "dims": list(dims), "grid": args.grid,
           "dtype": args.dtype, "gbps": args.gbps, "wire": args.wire, "footprint": args.footprint, "ar_us": args.ar_us, "extra": args.extra,
           "steps": args.steps, "warmup": args.warmup, "preheat_sweeps": preheat,
           "ms_per_step": round(dt / args.steps * 1e3, 4), "kernel": s.kernel,
           "reserved_cus": s.native.reserved_cus, "graph_launches": s.native.graph_launches,
           "projected_node_glups": round(s.interior_points * args.steps / dt / 1e9, 2),
           "rank_glups": round(s.interior_points / P * args.steps / dt / 1e9, 2),
           "temporal_K": s.native.temporal_steps, "field_buffers": s.native.field_buffers,
           # memory preflight (solver.cpp preflight_memory) and hipMemGetInfo
           # before the solver's allocations / after initialize()
           "mem_planned_gb": gb(s.native.planned_bytes), "mem_free_before_gb": gb(s.native.mem_free_before),
           "mem_free_after_gb": gb(free_after), "mem_total_gb": gb(total),
           "mem_used_gb": gb(s.native.mem_free_before - free_after) if free_after is not None else None,
           "phases": phases,
           "long_remainders": list(s.native.long_remainders),
           "long_major": bool(s.native.long_major),
           "sweep_costs_ms": {k: round(v, 4) for k, v in s.native.sweep_costs.items()},
           "x_schedules": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in t.items()}
                           for t in heat3d_amd.native().tuned_schedules()]}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
