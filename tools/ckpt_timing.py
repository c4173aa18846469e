#!/usr/bin/env python3
"""Checkpoint save / restart seconds on one GPU.

Saves the field of an N^3 run after a few steps (Solver::save_checkpoint:
streamed device -> pinned host -> pwrite, fsync, rename, meta.json), then
restarts a fresh solver from it (load_checkpoint inside initialize():
contiguous preads, checksum, H2D), and checks the restarted field is bitwise
the saved one.

  python tools/ckpt_timing.py [--grid 1024] [--dtype fp64] [--dir /tmp/h3d_ckpt]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "h3d_ckpt"))
    ap.add_argument("--backend", default="hip")
    args = ap.parse_args()

    from heat3d_amd import HeatSolver

    N = (args.grid,) * 3
    dev = 0 if args.backend == "hip" else None
    shutil.rmtree(args.dir, ignore_errors=True)
    a = HeatSolver(N, iter_max=1 << 40, eps=0.0, dtype=args.dtype, backend=args.backend, device=dev)
    a.initialize()
    a.step(args.steps)
    a.synchronize()
    t0 = time.perf_counter()
    a.save_checkpoint(args.dir)
    t_save = time.perf_counter() - t0
    del a
    meta = lambda d: json.load(open(os.path.join(d, "meta.json")))
    saved = meta(args.dir)
    nbytes = sum(os.path.getsize(os.path.join(args.dir, f)) for f in os.listdir(args.dir))
    b = HeatSolver(N, iter_max=1 << 40, eps=0.0, dtype=args.dtype, backend=args.backend, device=dev,
                   extra_args=["--restart", args.dir])
    t0 = time.perf_counter()
    b.initialize()
    b.synchronize()
    t_load = time.perf_counter() - t0
    it = b.state()["iter"]
    shutil.rmtree(args.dir, ignore_errors=True)
    # the restarted field, saved again, must carry the same checksum (sum of
    # the value bit patterns over the whole grid)
    t0 = time.perf_counter()
    b.save_checkpoint(args.dir)
    t_save2 = time.perf_counter() - t0
    same = meta(args.dir)["checksum"] == saved["checksum"]
    del b
    shutil.rmtree(args.dir, ignore_errors=True)
    print(json.dumps({"grid": args.grid, "dtype": args.dtype, "bytes": nbytes, "save_s": round(t_save, 3),
                      "save_GBps": round(nbytes / t_save / 1e9, 3), "restart_s_incl_init": round(t_load, 3),
                      "restart_GBps": round(nbytes / t_load / 1e9, 3), "restart_iter": it, "save2_s": round(t_save2, 3),
                      "checksum": saved["checksum"],
                      "bitwise_equal": same}), flush=True)
    return 0 if same and it == args.steps else 1


if __name__ == "__main__":
    sys.exit(main())
