#!/usr/bin/env python3
"""Print the start-up schedule tuner's candidate timings and choice for a
single-GPU grid (HEAT3D_TRACE during initialize).

  python tools/probes/schedule_probe.py --grid 1024 --dtype fp64
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs="+", default=[1024])
    ap.add_argument("--dtype", default="fp64")
    a = ap.parse_args()
    import heat3d_amd
    from heat3d_amd import HeatSolver

    for g in a.grid:
        os.environ["HEAT3D_TRACE"] = "1"
        s = HeatSolver((g, g, g), 10, 0.0, dtype=a.dtype, backend="hip")
        s.initialize()
        os.environ.pop("HEAT3D_TRACE", None)
        del s
    print(json.dumps(heat3d_amd.native().tuned_schedules()), flush=True)


if __name__ == "__main__":
    main()
