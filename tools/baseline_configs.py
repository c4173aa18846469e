#!/usr/bin/env python3
"""Run the five BASELINE.json configs and tabulate them (profiles/baseline_configs.md).

  1  64^3 fp64, 1-rank CPU Jacobi (OpenMP backend, no GPU, no MPI)
  2  512^3 fp64, 1 MI355X, single-GPU stencil (no halo exchange)
  3  1024^3 fp64, 8 GPUs, 1D slab 8x1x1 + 2-neighbour halo
  4  2048^3 fp32, 8 GPUs, 2x2x2 blocks + 6-neighbour halo, comm/compute overlap
  5  4096^3 fp32 (2047^3 interior points per GPU), hipGraph, weak scaling 1 -> 8

Configs 3-5 need an 8-GPU node (``--gpus 8`` runs bench.py under
torch.distributed.run).  With fewer GPUs they run as *proxies* on one GPU:
3 and 4 split the same global grid into 8 virtual ranks (LocalComm, device
copies instead of xGMI), 5 runs its one-GPU weak-scaling point.  Every row
says which it is.

  python tools/baseline_configs.py [--configs 1 2 3 4 5] [--gpus 1|8] [--steps K]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_bench(args, gpus, timeout):
    if gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
               "--gpus", str(gpus)] + args
    else:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    t0 = time.time()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    if p.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd)} failed ({p.returncode}):\n{p.stderr[-3000:]}")
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    out["wall_s"] = round(time.time() - t0, 1)
    return out


def run_proxy(args, timeout):
    """tools/rank_proxy.py: one inner rank of the 8-rank job alone on the GPU."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "rank_proxy.py")] + args
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    if p.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd)} failed ({p.returncode}):\n{p.stderr[-3000:]}")
    return json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])


def config1(steps):
    import heat3d_amd
    from heat3d_amd.utils import golden

    n, eps = 64, 1e-5
    s = heat3d_amd.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu")
    r = s.run()
    it, err, _ = golden(n, eps)
    pts = (n - 2) ** 3
    return {"config": 1, "name": "64^3 fp64 CPU 1 rank", "mode": "measured",
            "glups": round(pts * (r["conv_iter"] + 1) / r["seconds"] / 1e9, 3),
            "time_to_converge_s": round(r["seconds"], 3), "eps": eps, "iterations": r["conv_iter"],
            "golden_iterations": it, "error_percent": round(r["error_percent"], 4), "golden_error": err}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--configs", nargs="+", type=int, default=[1, 2, 3, 4, 5])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--timeout", type=int, default=900)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--md-out", default="", help="also write the markdown table (profiles/baseline_configs.md)")
    a = ap.parse_args()
    rows = []
    real = a.gpus >= 8
    for c in a.configs:
        if c == 1:
            row = config1(a.steps)
        elif c == 2:
            b = run_bench(["--grid", "512", "--steps", str(4 * a.steps), "--converge-eps", "1e-3"], 1, a.timeout)
            row = {"config": 2, "name": "512^3 fp64 1 GPU", "mode": "measured", "bench": b}
        elif c == 3:
            extra = ["--grid", "1024", "--decomp", "8x1x1", "--steps", str(a.steps), "--converge-eps", "1e-3"]
            if real:
                row = {"config": 3, "name": "1024^3 fp64 8 GPUs slab", "mode": "measured",
                       "bench": run_bench(extra, 8, a.timeout)}
            else:
                row = {"config": 3, "name": "1024^3 fp64 slab 8x1x1", "mode": "proxy: 8 virtual ranks on 1 GPU",
                       "bench": run_bench(extra + ["--virtual-ranks", "8"], 1, a.timeout),
                       "phantom": run_proxy(["--ranks", "8", "--grid", "1024", "--decomp", "8x1x1",
                                             "--gbps", "64", "--steps", str(4 * a.steps)], a.timeout)}
        elif c == 4:
            extra = ["--grid", "2048", "--dtype", "fp32", "--decomp", "2x2x2", "--steps", str(a.steps // 2),
                     "--warmup", "4", "--converge-eps", "0"]
            if real:
                row = {"config": 4, "name": "2048^3 fp32 8 GPUs 2x2x2", "mode": "measured",
                       "bench": run_bench(extra, 8, a.timeout)}
            else:
                row = {"config": 4, "name": "2048^3 fp32 block 2x2x2", "mode": "proxy: 8 virtual ranks on 1 GPU",
                       "bench": run_bench(extra + ["--virtual-ranks", "8"], 1, a.timeout),
                       "phantom": run_proxy(["--ranks", "8", "--grid", "2048", "--dtype", "fp32", "--decomp", "2x2x2",
                                             "--gbps", "64", "--steps", str(2 * a.steps)], a.timeout)}
        elif c == 5:
            pts = []
            for g in ([1, 2, 4, 8] if real else [1]):
                pts.append(run_bench(["--weak-block", "2047", "--dtype", "fp32", "--steps", str(a.steps // 2),
                                      "--warmup", "4", "--converge-eps", "0"], g, a.timeout))
            row = {"config": 5, "name": "4096^3 fp32 weak scaling (2047^3 per GPU)",
                   "mode": "measured 1->8" if real else "measured: 1-GPU point only", "bench": pts}
        else:
            raise SystemExit(f"unknown config {c}")
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(rows, f, indent=1)
    if a.md_out:
        with open(a.md_out, "w") as f:
            f.write(markdown(rows))


def markdown(rows):
    out = ["| # | config | mode | dtype | grid | parallelism | kernel | GLUPS | ms/step | time-to-converge |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        if r["config"] == 1:
            out.append(f"| 1 | {r['name']} | {r['mode']} | fp64 | 64^3 | 1 rank, OpenMP | cpu | {r['glups']} | — | "
                       f"{r['iterations']} it (golden {r['golden_iterations']}) in {r['time_to_converge_s']} s at "
                       f"eps {r['eps']:g}, error {r['error_percent']} % (golden {r['golden_error']}) |")
            continue
        for b in (r["bench"] if isinstance(r["bench"], list) else [r["bench"]]):
            c = b["config"]
            t = b.get("time_to_converge")
            ttc = (f"{t['iterations']} it in {t['seconds']:.3f} s at eps {t['eps']:g}" if t else "—")
            out.append(f"| {r['config']} | {r['name']} | {r['mode']} | {b['dtype']} | {'x'.join(map(str, c['grid']))} | "
                       f"{c['parallelism']} | `{c['kernel']}` | {b['value']} | {b['ms_per_step']} | {ttc} |")
        ph = r.get("phantom")
        if ph:
            g = ph["grid"]
            out.append(f"| {r['config']} | {r['name']} | proxy: phantom rank {ph['rank']} of {ph['ranks']} alone on 1 GPU, "
                       f"{ph['gbps']:g} GB/s emulated links (projected node GLUPS) | {ph['dtype']} | {g}^3 | "
                       f"{'x'.join(map(str, ph['dims']))} | `{ph['kernel']}` | {ph['projected_node_glups']} | "
                       f"{ph['ms_per_step']} | — |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    main()
