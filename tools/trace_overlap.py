#!/usr/bin/env python3
"""Concurrency report of a multi-process rocprofv3 kernel trace.

For every ``*kernel_trace.csv`` under DIR (one per traced process, e.g. the
ranks of ``bench.py --gpus 2 --comm rccl``) the dispatches are classified as

  interior  the sweep kernel on the compute stream (the widest stencil grid)
  boundary  the other stencil dispatches (x-slab / shell pieces, comm stream)
  rccl      RCCL kernels (halo send/recv groups, all-reduce)
  check     the convergence check kernel
  wait      graph_wait_kernel: a per-stream graph's device-side wait for another stream
  signal    graph_signal_kernel: the signal it waits for
  other     pack / unpack / copies / anything else

and the report gives, per process: count, median duration and the hardware
queue(s) of each class, and how much of the boundary / rccl / check time ran
while an interior dispatch of the same process was executing (wall-clock
overlap of [start, end) intervals).  A class that shares its queue with the
interior can only run between interior dispatches: its overlap is 0.

  python tools/trace_overlap.py gpurun_out/rccl2 > profiles/rccl2_overlap.md
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def classify(name, interior_grid, grid):
    n = name.lower()
    if "nccl" in n:
        return "rccl"
    if "check_convergence" in n or "check_kernel" in n:
        return "check"
    if "graph_wait" in n:
        return "wait"
    if "graph_signal" in n:
        return "signal"
    if "stencil" in n:
        return "interior" if grid == interior_grid else "boundary"
    return "other"


def overlap(iv, others):
    """total length of iv's intersection with the union of intervals `others` (sorted)"""
    a, b = iv
    tot, cur_hi = 0, a
    for s, e in others:
        if e <= cur_hi:
            continue
        if s >= b:
            break
        lo, hi = max(s, cur_hi), min(e, b)
        if hi > lo:
            tot += hi - lo
            cur_hi = hi
    return tot


def report(path):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        return
    for r in rows:
        r["_s"], r["_e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["_g"] = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    st = [r for r in rows if "stencil" in r["Kernel_Name"].lower()]
    interior_grid = max((r["_g"] for r in st), default=-1)
    by = collections.defaultdict(list)
    for r in rows:
        r["_c"] = classify(r["Kernel_Name"], interior_grid, r["_g"])
        by[r["_c"]].append(r)
    ints = sorted((r["_s"], r["_e"]) for r in by.get("interior", []))
    print(f"## {os.path.relpath(path)}\n")
    print(f"{len(rows)} dispatches; interior = stencil dispatches with grid {interior_grid}\n")
    print("| class | dispatches | median µs | total ms | queue ids | stream ids | time under an interior dispatch |")
    print("|---|---|---|---|---|---|---|")
    for c in ("interior", "boundary", "rccl", "check", "wait", "signal", "other"):
        rs = by.get(c, [])
        if not rs:
            continue
        durs = [(r["_e"] - r["_s"]) / 1e3 for r in rs]
        q = sorted({r.get("Queue_Id", "?") for r in rs})
        s = sorted({r.get("Stream_Id", "?") for r in rs})
        tot = sum(r["_e"] - r["_s"] for r in rs)
        if c == "interior":
            ov = "—"
        else:
            o = sum(overlap((r["_s"], r["_e"]), ints) for r in rs)
            ov = f"{100.0 * o / max(1, tot):.1f} %"
        print(f"| {c} | {len(rs)} | {statistics.median(durs):.1f} | {tot / 1e6:.3f} | {', '.join(q)} | "
              f"{', '.join(s)} | {ov} |")
    # stream -> hardware queue: a device-side wait must not share a queue with
    # the stream that signals it (its signal would queue behind the spin)
    sq = collections.defaultdict(set)
    scls = collections.defaultdict(collections.Counter)
    for r in rows:
        sq[r.get("Stream_Id", "?")].add(r.get("Queue_Id", "?"))
        scls[r.get("Stream_Id", "?")][r["_c"]] += 1
    print("\n| stream id | queue ids | dispatches by class |\n|---|---|---|")
    for s_id in sorted(sq):
        print(f"| {s_id} | {', '.join(sorted(sq[s_id]))} | "
              f"{', '.join(f'{c} {n}' for c, n in sorted(scls[s_id].items()))} |")
    sync_streams = [s_id for s_id in sq if scls[s_id]["wait"] or scls[s_id]["signal"]]
    shared = [(a, b) for i, a in enumerate(sync_streams) for b in sync_streams[i + 1:] if sq[a] & sq[b]]
    if sync_streams:
        print(f"\nstreams with graph waits / signals: {', '.join(sorted(sync_streams))}; "
              + ("**share a hardware queue: " + "; ".join(f"{a} & {b}" for a, b in shared) + "**" if shared
                 else "each on hardware queues of its own (no wait can queue behind its signaller)"))
    names = collections.Counter((r["_c"], r["Kernel_Name"][:110]) for r in rows)
    print("\n| class | kernel | dispatches |\n|---|---|---|")
    for (c, k), n in sorted(names.items()):
        print(f"| {c} | `{k}` | {n} |")
    print()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True))
    print(f"# Kernel concurrency: {a.dir}\n")
    if not files:
        print("no kernel_trace.csv found")
    for f in files:
        report(f)


if __name__ == "__main__":
    main()
