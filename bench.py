#!/usr/bin/env python3
"""Headline benchmark: GLUPS of the FTCS 7-point heat solver, 1024^3 fp64.

BASELINE.json metric "GLUPS (cell-updates/sec, whole node) + time-to-converge,
1024^3 fp64 grid".  One process per GPU; the global grid is fixed (strong
scaling): 1 GPU -> 1x1x1, N GPUs -> N x 1 x 1 slabs (BASELINE config 3: 1D
slab decomposition + 2-neighbour halo over xGMI, RCCL send/recv on device
pointers).  Every timed step is a full iteration of the production loop:
interior sweep || (halo exchange -> boundary slabs), fused residual, RCCL
all-reduce(max) of the residual and the device-side convergence check
(eps = 0 so it never stops early).  Synthetic data = the reference's analytic
initial/boundary condition (heat3D.cu:408-453).

Launch (the reference: ``mpirun -n P ./heat3D ...``, heat3D.cu:203-205):

  python bench.py [--gpus N] [--steps K] [--warmup W]
      N > 1 without a launcher: this process starts N fresh worker processes
      (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment) before
      touching the GPU, waits for them under a watchdog and exits with the
      worst return code; rank 0 prints the JSON line.
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
      one rank per process as launched (RANK / WORLD_SIZE from torchrun).

The ranks never import torch: one HIP runtime per process, /opt/rocm's HIP 7.2
and RCCL 2.27 (the native CLI's), not the HIP 7.0 / RCCL 2.26 copies PyTorch
bundles under the same sonames (HEAT3D_RUNTIME=rocm, _native.py; the JSON's
"runtime" block records the versions and library files each rank bound).
The host bootstrap is native too (HostGroup: the ncclUniqueId broadcast, host
barriers, the max-over-ranks of the timed interval).  All per-iteration
traffic goes through the native RCCL communicator.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "GLUPS (cell-updates/sec, whole node) + time-to-converge, 1024^3 fp64 grid"


def metric_name(grid: str, dtype: str) -> str:
    return f"GLUPS (cell-updates/sec, whole node) + time-to-converge, {grid} {dtype} grid"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--weak-block", type=int, default=0,
                    help="weak scaling: each GPU owns B^3 interior points, global grid = dims*B + 2 "
                         "(BASELINE config 5: B=2047 fp32 gives 4096^3 on 8 GPUs)")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--decomp", default="auto",
                    help="auto | slab | block | AxBxC.  auto (N > 1): each candidate grid (x slabs, 2D and 3D "
                         "blocks: parallel.decomp_candidates) runs --decomp-trial-steps timed steps of the "
                         "production schedule through the job's transport at start-up; the fastest by its "
                         "slowest rank is kept (JSON decomp_auto)")
    ap.add_argument("--decomp-trial-steps", type=int, default=36,
                    help="steps per timed window of each --decomp auto candidate (best of 3; 0: slabs untimed)")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--stream-graphs", default="auto", choices=["auto", "on", "off"],
                    help="the overlapped multi-rank schedule as per-stream hipGraphs (auto: unless more than 4 "
                         "ranks share a GPU); a start-up canary with a short device-wait timeout falls back to "
                         "eager replay in-process when they do not hold")
    ap.add_argument("--graph-canary", type=float, default=2.0,
                    help="device-wait timeout (s) of the start-up canary replay (0: no canary)")
    ap.add_argument("--graph-chunk", type=int, default=0,
                    help="iterations per hipGraph (0 = the solver's choice: 32, 96 for the overlapped N > 1 schedule)")
    ap.add_argument("--converge-eps", type=float, default=1e-5,
                    help="also measure time-to-converge at this EPS (0 disables).  Default: the reference's "
                         "tolerance 1e-5 (1024^3 fp64: 186188 iterations, 240 s on one MI355X, 21.5%% off the "
                         "steady state; profiles/converge_1024_r04.md)")
    ap.add_argument("--converge-time-limit", type=float, default=360.0,
                    help="wall budget (s) of the time-to-converge run: past it the run stops unconverged and "
                         "the JSON says so (bounds the driver's bench on a slow box; 0 = none)")
    ap.add_argument("--temporal", type=int, default=0, help="0 auto | 1 single-step | K (2..6) K-step temporally blocked sweeps")
    ap.add_argument("--reserve-cus", type=int, default=-1,
                    help="CUs kept free of the interior sweep for the comm kernels (-1 auto: 8 under the "
                         "overlapped multi-rank schedule, 0 under a long x-slab interior)")
    ap.add_argument("--kernel2", default="auto", help="temporally blocked sweep kernel (tbK / trK[:V:R:WZ:WY:L:Q])")
    ap.add_argument("--virtual-ranks", type=int, default=1,
                    help="diagnostic: split the grid into this many subdomains on one GPU (not the headline)")
    ap.add_argument("--comm", default="auto", choices=["auto", "rccl", "socket"],
                    help="multi-process transport: auto = RCCL over xGMI; socket = host-staged TCP "
                         "(rehearses the N>1 launch with several ranks on one GPU)")
    ap.add_argument("--rccl-host-split", action="store_true",
                    help="testing: give every rank its own NCCL_HOSTID so that RCCL accepts several "
                         "ranks on one GPU (its traffic then takes RCCL's network transport over "
                         "loopback); exercises the real RCCL send/recv/all-reduce path on a 1-GPU box")
    ap.add_argument("--timeout", type=float, default=1500.0,
                    help="watchdog (s): a launched job that runs longer is killed and exits non-zero")
    ap.add_argument("--profile-sweeps", type=int, default=8,
                    help="after the timed window, profile this many more sweeps per rank with timing "
                         "events at the schedule's phase boundaries (JSON 'phases'; 0 disables)")
    ap.add_argument("--watchdog", type=float, default=300.0,
                    help="native watchdog (s): a rank whose peers stop making progress aborts its communicators")
    ap.add_argument("--preheat-ms", type=float, default=20.0,
                    help="untimed GPU warm-up right before the timed window: repetitions of the next sweep's "
                         "interior into the buffer it will overwrite, without residual state (the solver state "
                         "is untouched), so the timed steps do not start on a GPU idled by the graph capture "
                         "(0 disables)")
    ap.add_argument("--progress", type=float, default=30.0,
                    help="time-to-converge run: stderr heartbeat (iteration, relative residual, GLUPS) every S "
                         "seconds (0 disables)")
    ap.add_argument("--verbose", type=int, default=0,
                    help="time-to-converge run: print the residual every N iterations (stdout, rank 0)")
    ap.add_argument("--solver-flags", default="",
                    help="extra native solver flags for A/B runs, e.g. \"--no-fused-check --lag off\"")
    ap.add_argument("--json-out", default="")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher: N fresh worker processes, started before anything touches the GPU

def _free_port() -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args, argv) -> int:
    n = args.gpus
    port = _free_port()
    hg_port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HEAT3D_HOSTGROUP_PORT=str(hg_port), HEAT3D_BENCH_WORKER="1")
        if args.rccl_host_split:
            env.update(NCCL_HOSTID=f"heat3d-bench-rank{r}", NCCL_SOCKET_IFNAME="lo")
        # each worker leads its own process group so that the watchdog can end
        # it together with anything it started
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv),
                                      env=env, start_new_session=True))
    deadline = time.monotonic() + args.timeout
    rc = 0
    failed_at = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and failed_at is None:
            failed_at = time.monotonic()
            rc = bad[0]
        if all(c is not None for c in codes):
            break
        now = time.monotonic()
        # one rank failed: give its peers 20 s to notice (their native watchdogs
        # abort the communicators), then end them
        if now > deadline or (failed_at is not None and now - failed_at > 20):
            if now > deadline:
                print(f"bench.py: watchdog: job exceeded {args.timeout:.0f} s, killing workers",
                      file=sys.stderr, flush=True)
                rc = rc or 124
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
            for p in procs:
                p.wait()
            break
        time.sleep(0.1)
    for p in procs:
        c = p.returncode
        if c not in (0, None) and rc == 0:
            rc = c
    if rc < 0:
        rc = 128 - rc
    return rc


# ---------------------------------------------------------------------------
# one rank

def run_rank(args) -> int:
    # one HIP runtime per process, /opt/rocm's: never import torch here
    os.environ.setdefault("HEAT3D_RUNTIME", "rocm")
    import heat3d_amd
    from heat3d_amd import HeatSolver
    from heat3d_amd.parallel import best_dims_for, decomp_candidates, pick_measured
    from heat3d_amd.parallel.distributed import (HostGroup, all_gather_objects, barrier, env_info,
                                                 max_over_ranks)
    from heat3d_amd.utils.metrics import roofline_glups

    ext = heat3d_amd.native()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    # host bootstrap (native TCP star, no torch): the ncclUniqueId broadcast,
    # barriers and the max over ranks; the per-iteration halo and all-reduce
    # traffic goes through the native RCCL communicator
    info = env_info()
    group = HostGroup.from_env(timeout_s=args.timeout) if world > 1 else None
    rank = info.rank
    if args.rccl_host_split and world > 1 and "NCCL_HOSTID" not in os.environ:
        # under an external launcher (torchrun): every rank its own RCCL "host"
        # before the communicator exists (RCCL reads these at initialisation)
        os.environ["NCCL_HOSTID"] = f"heat3d-bench-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    ndev = ext.device_count()
    if ndev < 1:
        print("bench.py: no HIP device visible", file=sys.stderr)
        return 2
    dev = info.local_rank % ndev
    runtime = heat3d_amd.runtime()

    G = args.grid
    N = (G, G, G)
    nparts = world * args.virtual_ranks
    if args.virtual_ranks > 1:
        assert world == 1, "--virtual-ranks is a single-process diagnostic"
    trials = None
    if args.decomp == "auto" and world > 1 and args.virtual_ranks == 1 and args.decomp_trial_steps > 0 \
            and not args.weak_block:
        dims, trials = None, []
    elif args.decomp in ("auto", "slab", "block"):
        dims = best_dims_for(N, nparts, None if args.decomp == "auto" else args.decomp)
    else:
        dims = tuple(int(v) for v in args.decomp.lower().split("x"))

    # the per-stream graphs' mode: a canary deadlock (HeatSolver.initialize
    # rebuilt that solver eagerly) turns them off for the later solvers too
    sg_mode = [args.stream_graphs]

    def make(eps, iter_max, extra=(), decomp=None):
        return HeatSolver(N, iter_max=iter_max, eps=eps, dtype=args.dtype, backend="hip",
                          decomp=decomp or dims, kernel=args.kernel, graph=not args.no_graph,
                          overlap=not args.no_overlap, graph_chunk=args.graph_chunk,
                          device=dev, group=group, virtual_ranks=args.virtual_ranks, comm=args.comm,
                          extra_args=["--stream-graphs", sg_mode[0], "--graph-canary", str(args.graph_canary),
                                      "--temporal", str(args.temporal), "--kernel2", args.kernel2,
                                      "--watchdog", str(args.watchdog), "--reserve-cus", str(args.reserve_cus)]
                          + args.solver_flags.split() + list(extra))

    if trials is not None:
        # --decomp auto: time each candidate process grid (x slabs, 2D, 3D
        # blocks) through the job's own transport — the production schedule
        # (overlapped sweeps, graphs as configured) from the initial state —
        # and keep the fastest by the slowest rank's time (one decision: every
        # rank gets the same maxima).  The reference takes MPI_Dims_create's
        # grid by rank count alone (heat3D.cu:243).
        esteps = args.decomp_trial_steps
        cands = decomp_candidates(N, nparts, args.temporal if args.temporal >= 2 else 3)
        if len(cands) == 1:
            dims, trials = cands[0], None
            cands = []
        for d in cands:
            t = make(0.0, 1 << 40, decomp=d)
            t.initialize()
            if t.stream_graphs_retried:
                sg_mode[0] = "off"
            t.step(esteps)
            t.prepare_steps(esteps)
            t.synchronize()
            best = None
            for _ in range(3):
                barrier(group)
                t0 = time.perf_counter()
                t.step(esteps)
                t.synchronize()
                dt1 = time.perf_counter() - t0
                best = dt1 if best is None else min(best, dt1)
            ms = max_over_ranks(best, group) / esteps * 1e3
            trials.append({"dims": list(d), "ms_per_step": round(ms, 4),
                           "stream_graphs": t.native.stream_graphs_state})
            del t
        if trials:
            dims = pick_measured(trials)
    assert dims[0] * dims[1] * dims[2] == nparts, (dims, nparts)
    if args.weak_block:
        N = tuple(d * args.weak_block + 2 for d in dims)
        G = N[0]

    phase_log = os.environ.get("HEAT3D_BENCH_PHASES") == "1"
    tp = [time.perf_counter()]

    def phase(name):
        if phase_log:
            tp.append(time.perf_counter())
            print(f"bench.py phase {name}: {1e3 * (tp[-1] - tp[-2]):.2f} ms", file=sys.stderr, flush=True)

    s = make(0.0, 1 << 40)
    s.initialize()
    if s.stream_graphs_retried:
        sg_mode[0] = "off"
    phase("initialize")
    s.step(max(1, args.warmup))
    phase("warmup enqueued")
    # capture the graphs the timed steps replay (untimed) while the GPU still
    # runs the warm-up, so that it does not idle (and clock down) between the
    # warm-up and the timed steps
    s.prepare_steps(args.steps)
    phase("graphs prepared")
    s.synchronize()
    ext.device_synchronize(dev)
    phase("warmup synchronized")
    # race detection before timing: every face sent by the warm-up exchange
    # must match, bit for bit, the ghost layer the neighbour received
    bad_faces = s.native.verify_halos()
    if bad_faces:
        print(f"bench.py: rank {rank}: {bad_faces} halo face(s) differ after warm-up", file=sys.stderr)
        return 3
    phase("halos verified")
    warm = s.native.iterations_issued
    g0 = s.native.graph_launches
    # The graph capture above (12 ms for the 1024^3 timed graph) outlasts a
    # short warm-up on the GPU, which then idles and clocks down: the first
    # timed sweeps of the driver's 20-step run ran 7-12% slow (kernel trace,
    # profiles/bench_r03_preheat.md).  Keep the GPU at work until the timed
    # window with sweeps that leave the solver state as it is.
    K = s.native.temporal_steps
    est_ms = s.interior_points / world * max(1, K) / ((800e9 if args.dtype == "fp64" else 1400e9)) * 1e3
    preheat = (s.native.preheat(max(1, min(64, int(args.preheat_ms / max(est_ms, 1e-3)) + 1)))
               if args.preheat_ms > 0 else 0)
    phase("preheat enqueued")
    # nothing between the preheat and the timed window may take host time: a
    # barrier that imported torch (~1.4 s, the single-process path of the
    # host collectives before round 6's fix) idled the GPU, which clocked
    # down, and the first timed sweeps ran ~10 % slow (gpurun_out/r6h trace,
    # r6i-r6k phases; tools/probes/sync_wake_probe.hip: the waits themselves
    # wake on time)
    barrier(group)
    s.synchronize()
    ext.device_synchronize(dev)
    phase("barrier")
    t0 = time.perf_counter()
    s.step(args.steps)
    phase("timed steps enqueued")
    s.synchronize()
    ext.device_synchronize(dev)
    barrier(group)
    t1 = time.perf_counter()
    dt = max_over_ranks(t1 - t0, group)
    graph_launches = s.native.graph_launches - g0
    st = s.state()
    # every issued iteration must have been checked and none skipped
    assert st["iter"] == warm + args.steps and st["done"] == 0, st
    points = s.interior_points
    value = points * args.steps / dt / 1e9
    esize = 8 if args.dtype == "fp64" else 4
    kernel = s.kernel
    runtime = heat3d_amd.runtime()  # after the backend set the device's host-wait mode
    sg_state, sg_note = s.native.stream_graphs_state, s.native.stream_graphs_note
    if s.stream_graphs_retried or (args.stream_graphs != "off" and sg_mode[0] == "off"):
        sg_state, sg_note = "fallback", "canary deadlock: the solver was rebuilt with --stream-graphs off"
    per_dev = s.native.ranks_per_device
    comm_name = s.native.comm_name
    comm_ranks = s.native.comm_transport_ranks
    nbuf = s.native.field_buffers
    reserved = s.native.reserved_cus
    # the x schedules timed at start-up (Config autotune): L = -3 is the
    # dispatch model's plan, L > 0 fixed x segments of L planes
    xs = [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in t.items()} for t in ext.tuned_schedules()]
    # remainder policy (Solver::calibrate_remainders): which n mod K end in
    # K+1-step sweeps, from the start-up sweep timings (ms)
    placement = all_gather_objects({"rank": rank, "device": dev, "host": socket.gethostname(),
                                    "hip_library": runtime["hip_library"], "rccl_library": runtime["rccl_library"],
                                    "dims": list(dims), "rccl_p2p_channels": s.native.rccl_p2p_channels or None,
                                    "subdomain": list(s.native.local_subdomain(0)["n"]), "x_schedules": xs,
                                    "long_remainders": list(s.native.long_remainders),
                                    "long_major": bool(s.native.long_major),
                                    "sweep_costs_ms": {k: round(v, 4) for k, v in s.native.sweep_costs.items()}},
                                   group)
    # per-rank schedule profile, after (outside) the timed window: a few more
    # sweeps of the same pipeline with timing events at its phase boundaries
    # (interior / halo / boundary / all-reduce / check, compute-stream idle,
    # how much of the halo + boundary chain ran under the interior)
    prof = {}
    if args.profile_sweeps > 0:
        prof = {k: (round(v, 4) if isinstance(v, float) else v)
                for k, v in s.native.profile_sweeps(args.profile_sweeps).items()}
    phases = all_gather_objects(dict(rank=rank, **prof), group)
    del s

    ttc = None
    if args.converge_eps and args.converge_eps > 0:
        c = make(args.converge_eps, 10 ** 7,
                 ["--progress", str(args.progress), "--time-limit", str(args.converge_time_limit)]
                 + (["--verbose", str(args.verbose)] if args.verbose > 0 else []))
        c.initialize()
        barrier(group)
        r = c.run()
        ttc = {"eps": args.converge_eps, "converged": bool(r["converged"]),
               "iterations": int(r["conv_iter"]) if r["converged"] else int(r["iterations"]),
               "seconds": max_over_ranks(r["seconds"], group),
               "error_percent": r["error_percent"], "time_limit_s": args.converge_time_limit,
               "relative_residual": r["last_residual"] / r["norm"] if r["norm"] else None}
        del c

    par = "x".join(str(d) for d in dims)
    grid_txt = "x".join(map(str, N)) if len(set(N)) > 1 else f"{G}^3"
    metric = metric_name(grid_txt, args.dtype)
    is_headline = metric == BASELINE_METRIC and args.virtual_ranks == 1 and not args.weak_block
    out = {
        "metric": metric,
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
        "config": {"model": f"heat3d FTCS 7-point, {grid_txt} {args.dtype} grid",
                   "grid": list(N),
                   "global_batch": 1, "seq_len": G,
                   "parallelism": f"{'slab' if dims[1] == dims[2] == 1 and dims[0] > 1 else 'block'} {par}"
                   + (f" ({args.virtual_ranks} virtual ranks on 1 GPU)" if args.virtual_ranks > 1 else ""),
                   "kernel": kernel, "temporal_K": K, "field_buffers": nbuf,
                   "graph_requested": not args.no_graph, "graph_used": graph_launches > 0,
                   # the overlapped schedule's per-stream graphs as the start-up canary
                   # left them (on / fallback / off / n/a; Solver::canary_stream_graphs)
                   "stream_graphs": sg_state, "stream_graphs_canary": sg_note,
                   "ranks_per_device": per_dev,
                   "graph_launches": graph_launches,
                   "overlap": not args.no_overlap, "comm": comm_name, "reserved_cus": reserved,
                   "solver_flags": args.solver_flags or None,
                   "preheat_sweeps": preheat},
        "comm_ranks": comm_ranks,
        # --decomp auto: every candidate grid's timed ms/step (slowest rank)
        # and the one kept
        "decomp_auto": None if not trials else {"trials": trials, "dims": list(dims),
                                                "trial_steps": args.decomp_trial_steps},
        "placement": placement,
        "halo_verified": True,
        "headline_config": is_headline,
        "glups_per_gpu": round(value / world, 3),
        # the single-step-equivalent traffic rate (16 B / 8 B per point update);
        # the real HBM traffic is about 1/K of it with K-step temporal blocking
        "single_step_equiv_tbps_per_gpu": round(value / world * 2 * esize / 1e3, 3),
        "vs_single_step_roofline": round(value / roofline_glups(esize, world), 4),
        # K-step roofline: one read + one write of the field per K steps (no
        # tile overlap) at the float4-copy rate measured on these boxes
        # (5.6 TB/s, profiles/hbm_probes_r02.md); the fp64 sweep's measured
        # traffic is 19.1 B per point per 3 steps (profiles/pmc_tl3_nt_r02.md)
        "temporal_roofline_glups_per_gpu": round(5.6e12 / (2 * esize / max(1, K)) / 1e9, 1),
        "vs_temporal_roofline": round(value / world / (5.6e12 / (2 * esize / max(1, K)) / 1e9), 4),
        "time_to_converge": ttc,
        # the HIP runtime / RCCL the ranks ran on (rank 0; every rank's files in placement)
        "runtime": dict(runtime, torch_loaded="torch" in sys.modules),
        "phases": phases,
        "baseline_note": "reference publishes no numbers (BASELINE.md); single-step roofline = "
                         "6.29 TB/s / (2*esize) per GPU",
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        barrier(group)
    return 0


def main() -> int:
    argv = sys.argv[1:]
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the ranks ourselves (nothing here has touched HIP)
        return launch(args, argv)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
