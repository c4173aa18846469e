#!/usr/bin/env python3
"""Run one native solve with explicit options (GPU debugging aid).

  HEAT3D_TRACE=1 HEAT3D_SEGV_TRACE=1 python tools/debug_solver.py --n 37 --vr 2 --graph 0
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=37)
    ap.add_argument("--eps", type=float, default=1e-4)
    ap.add_argument("--iters", type=int, default=10 ** 6)
    ap.add_argument("--vr", type=int, default=1)
    ap.add_argument("--decomp", default="")
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--overlap", type=int, default=1)
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--check-every", type=int, default=64)
    ap.add_argument("--graph-chunk", type=int, default=32)
    a = ap.parse_args()
    import heat3d_amd

    dec = tuple(int(v) for v in a.decomp.split("x")) if a.decomp else None
    s = heat3d_amd.HeatSolver((a.n,) * 3, a.iters, a.eps, backend=a.backend, virtual_ranks=a.vr,
                              decomp=dec, graph=bool(a.graph), overlap=bool(a.overlap),
                              check_every=a.check_every, graph_chunk=a.graph_chunk)
    print("created", flush=True)
    s.initialize()
    print("initialized", flush=True)
    r = s.run()
    print("run:", r, flush=True)
    g = s.gather()
    print("gathered", g.shape, float(g.sum()), flush=True)


if __name__ == "__main__":
    main()
