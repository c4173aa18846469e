#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats / kernel trace / PMC counters) as markdown.

  python tools/summarize_rocprof.py gpurun_out/prof_bench [--title T] > profiles/x.md
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def short(name, n=90):
    name = name.replace("void ", "").replace("heat3d::hip::", "")
    return name if len(name) <= n else name[:n] + "…"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    print(f"# {a.title or os.path.basename(a.dir.rstrip('/'))}\n")
    for f in sorted(glob.glob(os.path.join(a.dir, "*kernel_stats.csv"))):
        print("## Kernel statistics (rocprofv3 --kernel-trace --stats)\n")
        print("| kernel | calls | avg µs | min µs | max µs | % time |")
        print("|---|---|---|---|---|---|")
        for r in csv.DictReader(open(f)):
            print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                  f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.2f} |")
        print()
    for f in sorted(glob.glob(os.path.join(a.dir, "*kernel_trace.csv"))):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        by = collections.defaultdict(list)
        for r in rows:
            by[r["Kernel_Name"]].append(r)
        print("## Dispatch geometry and inter-kernel gaps\n")
        print("| kernel | grid | block | VGPR | LDS B | median µs |")
        print("|---|---|---|---|---|---|")
        for k, rs in by.items():
            d = statistics.median((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs)
            r0 = rs[0]
            print(f"| `{short(k)}` | {r0['Grid_Size_X']} | {r0['Workgroup_Size_X']} | {r0['VGPR_Count']} | "
                  f"{r0['LDS_Block_Size']} | {d:.1f} |")
        st = [r for r in rows if "stencil" in r["Kernel_Name"]]
        if len(st) > 2:
            gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(st, st[1:])]
            print(f"\nstencil-to-stencil gap: median {statistics.median(gaps):.1f} µs over {len(gaps)} pairs\n")
    for f in sorted(glob.glob(os.path.join(a.dir, "*counter_collection.csv"))):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, k, c), v in per.items():
            agg[k][c].append(v)
        print("## PMC counters (per dispatch, median)\n")
        print("| kernel | counter | value |")
        print("|---|---|---|")
        for k, cs in agg.items():
            if "at::native" in k or "rocclr" in k:
                continue
            for c, vs in cs.items():
                print(f"| `{short(k)}` | {c} | {statistics.median(vs):.4g} |")
        print()


if __name__ == "__main__":
    main()
