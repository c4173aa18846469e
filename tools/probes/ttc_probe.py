#!/usr/bin/env python3
"""Where does time-to-converge go?  1024^3 fp64 on one GPU: run() at eps 1e-3
against fixed-length runs (eps = 0) of 60 / 600 / 2220 iterations, so the fixed
cost of run() is the intercept.  python tools/probes/ttc_probe.py [--grid N]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--extra", nargs="*", default=[])
    ap.add_argument("--bench-like", action="store_true", help="the arguments bench.py's convergence run uses")
    a = ap.parse_args()
    from heat3d_amd import HeatSolver

    N = (a.grid,) * 3
    for eps, it in ((0.0, 60), (0.0, 600), (0.0, 2220), (1e-3, 10 ** 7), (1e-3, 10 ** 7)):
        t0 = time.perf_counter()
        kw = {}
        if a.bench_like:
            kw = dict(decomp=(1, 1, 1), kernel="auto", graph=True, overlap=True, graph_chunk=32, device=0,
                      virtual_ranks=1, comm="auto")
            extra = ["--temporal", "0", "--kernel2", "auto", "--watchdog", "300"] + list(a.extra)
        else:
            extra = list(a.extra)
        s = HeatSolver(N, it, eps, backend="hip", extra_args=extra, **kw)
        t1 = time.perf_counter()
        s.initialize()
        t2 = time.perf_counter()
        r = s.run()
        t3 = time.perf_counter()
        print(f"eps {eps:g} iter_max {it}: construct {t1 - t0:.3f} s, initialize {t2 - t1:.3f} s, run() "
              f"{t3 - t2:.3f} s wall / {r['seconds']:.3f} s reported, issued {r['issued']}, "
              f"conv_iter {r['conv_iter']}, per issued it {1e3 * r['seconds'] / max(1, r['issued']):.3f} ms",
              flush=True)
        del s


if __name__ == "__main__":
    main()
