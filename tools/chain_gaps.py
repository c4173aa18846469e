#!/usr/bin/env python3
"""Comm-chain gaps of the overlapped multi-rank sweep in a rocprofv3 kernel trace.

For a phantom-rank (tools/rank_proxy.py) or RCCL rank trace, per sweep on the
comm stream: the halo (emulated wire delay + stand-in copies, or RCCL kernels),
the idle gap before the boundary slabs, the slabs, the gap after them; the
cross-stream dependency kernels (graph_wait / graph_signal of the per-stream
graphs) on that chain; and the sweep period from interior start to interior
start on the compute stream.

  python tools/chain_gaps.py TRACE_DIR > profiles/...md
"""
import argparse
import csv
import glob
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    a = ap.parse_args()
    f = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["k"] = r["Kernel_Name"]
    rows.sort(key=lambda r: r["s"])
    # the compute stream runs the interior sweeps (the widest stencil grid among
    # the stencil kernels with the most dispatches on one stream); the comm stream
    # the boundary slabs (swapped-axis thin-slab tiles, ", true>")
    slab = [r for r in rows if "stencil_tbl" in r["k"] and ", true>" in r["k"]]
    if not slab:
        print("no boundary-slab dispatches")
        return
    comm = slab[0]["Stream_Id"]
    inter = [r for r in rows if "stencil" in r["k"] and r["Stream_Id"] != comm and ", true>" not in r["k"]]
    comp = max({r["Stream_Id"] for r in inter}, key=lambda s: sum(1 for r in inter if r["Stream_Id"] == s))
    ints = [r for r in inter if r["Stream_Id"] == comp]
    crows = [r for r in rows if r["Stream_Id"] == comm]
    sweeps = []
    i = 0
    while i < len(crows):
        # a sweep on the comm stream: halo kernels, then the two boundary slabs
        j = i
        while j < len(crows) and ", true>" not in crows[j]["k"]:
            j += 1
        if j + 1 >= len(crows) or ", true>" not in crows[j + 1]["k"]:
            break
        halo = [r for r in crows[i:j] if "graph_" not in r["k"]]
        sync = [r for r in crows[i:j] if "graph_" in r["k"]]
        if halo:
            sweeps.append(dict(halo_start=halo[0]["s"], halo_end=halo[-1]["e"], bnd_start=crows[j]["s"],
                               bnd_end=crows[j + 1]["e"], sync_kernels=len(sync),
                               sync_us=sum(r["e"] - r["s"] for r in sync) / 1e3,
                               graph=any("graph_" in r["k"] for r in crows[max(0, i - 3):j + 3])))
        i = j + 2
    periods = [(b["s"] - a["s"]) / 1e3 for a, b in zip(ints, ints[1:])]
    print(f"# Comm-chain gaps: {os.path.relpath(a.dir)}\n")
    print(f"compute stream {comp} ({len(ints)} interior sweeps), comm stream {comm} ({len(sweeps)} sweeps)\n")
    print("| sweep | mode | halo µs | gap halo→slabs µs | slabs µs | gap slabs→next halo µs | graph wait/signal kernels on the chain (µs) |")
    print("|---|---|---|---|---|---|---|")
    for n, (sw, nx) in enumerate(zip(sweeps, sweeps[1:] + [None])):
        g2 = (nx["halo_start"] - sw["bnd_end"]) / 1e3 if nx else float("nan")
        print(f"| {n} | {'graph' if sw['graph'] else 'eager'} | {(sw['halo_end'] - sw['halo_start']) / 1e3:.1f} | "
              f"{(sw['bnd_start'] - sw['halo_end']) / 1e3:.1f} | {(sw['bnd_end'] - sw['bnd_start']) / 1e3:.1f} | "
              f"{g2:.1f} | {sw['sync_kernels']} ({sw['sync_us']:.1f}) |")
    for mode in ("graph", "eager"):
        ss = [s for s in sweeps if s["graph"] == (mode == "graph")]
        if len(ss) < 2:
            continue
        g1 = [(s["bnd_start"] - s["halo_end"]) / 1e3 for s in ss]
        print(f"\n{mode}: median gap halo→slabs {statistics.median(g1):.1f} µs over {len(ss)} sweeps")
    if periods:
        print(f"\ninterior start-to-start: median {statistics.median(periods):.1f} µs over {len(periods)} sweeps")


if __name__ == "__main__":
    main()
