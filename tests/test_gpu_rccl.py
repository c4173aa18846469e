"""RCCL on the one-GPU box (SURVEY.md §5 "Distributed communication backend").

* ``rccl_self_exchange``: RcclComm::exchange / allreduce on a one-rank
  communicator — ncclSend / ncclRecv to self inside one group, byte counts
  that are and are not multiples of 8, a padded K-deep x halo plane moved in
  place between two ghosted fields (the solver's x-face message), all-reduce
  identities.
* Real multi-rank RCCL: 2 and 4 processes on the one GPU, each with its own
  NCCL_HOSTID (RCCL refuses two ranks per device of one host; as separate
  "hosts" its traffic takes the network transport over loopback).  The halo
  exchange, the all-reduce of the residual slots, the halo checksums and the
  gather all run through RcclComm with real peers; the gathered field must be
  bitwise equal to the single-process solve, the iteration count identical.
  Reference: heat3D.cu:619-641, 724-755 (halo), 1062-1063 (reduction),
  1112-1162 (gather).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, free_port
from _mp_workers import native_rccl_gpu_worker

pytestmark = pytest.mark.gpu


def test_rccl_self_exchange(ext, gpu):
    r = ext.rccl_self_exchange(0, [8, 24, 1000, 4093, 1 << 20, 3 * (1 << 20) + 5], (6, 7, 9), 3)
    assert all(r["ok"]), r
    assert r["touched_outside"] == 0
    assert r["transport_ranks"] == 1
    assert r["allreduce_u64"] == (7, 0x7FF0000000000000, 3)
    assert r["allreduce_f64"] == (1.5, -2.25)


@pytest.mark.parametrize("world,decomp,extra", [
    (2, (2, 1, 1), None),
    (2, (2, 1, 1), ["--rccl-shared"]),               # one communicator for halos and all-reduce
    (4, (2, 2, 1), None),                             # block: deep y halos, axis-ordered phases
    (3, (3, 1, 1), None),
])
def test_rccl_multirank_bitwise(h3d, gpu, tmp_path, world, decomp, extra):
    n, eps = 33, 1e-4
    mp.start_processes(native_rccl_gpu_worker,
                       args=(world, free_port(), str(tmp_path), n, eps, decomp, "fp64", extra or []),
                       nprocs=world, join=True, start_method="spawn")
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="hip", device=0)
    r1 = single.run()
    it, err, name, graphs = open(tmp_path / "result.txt").read().split()
    assert int(it) == r1["conv_iter"]  # the same stopping iteration as one rank
    assert name == ("rccl(shared)" if extra and "--rccl-shared" in extra else "rccl")
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


def test_bench_self_launch_rccl(gpu, tmp_path):
    """``bench.py --gpus 2`` without torchrun: the launcher starts two workers,
    RCCL spans both (comm_ranks from ncclCommCount), halos verified before timing."""
    out = tmp_path / "b.json"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--comm", "rccl",
                        "--rccl-host-split", "--grid", "96", "--steps", "6", "--warmup", "3",
                        "--converge-eps", "0", "--timeout", "100", "--json-out", str(out)],
                       capture_output=True, text=True, timeout=110, cwd=ROOT,
                       env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    j = json.loads(lines[0])
    assert j == json.loads(out.read_text())
    assert j["n_gpus"] == 2 and j["comm_ranks"] == 2 and j["halo_verified"]
    assert j["config"]["comm"] == "rccl" and j["config"]["parallelism"] == "slab 2x1x1"
    assert j["value"] > 0 and j["steps"] == 6 and [q["rank"] for q in j["placement"]] == [0, 1]
    # the per-rank phase block the N-GPU JSON carries:
    # every rank reports its overlapped schedule's phases per sweep
    ph = j["phases"]
    assert [q["rank"] for q in ph] == [0, 1], ph
    for q in ph:
        for key in ("interior_ms", "halo_ms", "boundary_ms", "allreduce_ms", "check_ms", "compute_idle_ms",
                    "sweep_ms", "chain_overlap_fraction"):
            assert key in q, (key, q)
        assert q["sweeps"] > 0 and q["steps_per_sweep"] == 3 and q["interior_ms"] > 0 and q["halo_ms"] > 0
        assert 0.0 <= q["chain_overlap_fraction"] <= 1.0 and q["sweep_ms"] >= q["interior_ms"] * 0.5, q


def test_bench_under_torchrun_rccl(gpu, tmp_path):
    """The driver's N-GPU launch line, ``python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P
    bench.py --gpus 2 ...``: ranks from torchrun's environment, the gloo
    bootstrap, real RCCL (each rank its own NCCL_HOSTID, set by bench.py
    itself under --rccl-host-split), one JSON line from rank 0."""
    out = tmp_path / "t.json"
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--comm", "rccl", "--rccl-host-split",
                        "--grid", "96", "--steps", "6", "--warmup", "3", "--converge-eps", "0",
                        "--json-out", str(out)],
                       capture_output=True, text=True, timeout=150, cwd=ROOT,
                       env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["comm_ranks"] == 2 and j["config"]["comm"] == "rccl" and j["halo_verified"]
    assert [q["rank"] for q in j["phases"]] == [0, 1] and j == json.loads(out.read_text())


def test_bench_self_launch_socket(gpu, tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--comm", "socket",
                        "--grid", "128", "--steps", "6", "--warmup", "3", "--converge-eps", "0",
                        "--timeout", "100"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT,
                       env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert j["n_gpus"] == 2 and j["comm_ranks"] == 2 and j["config"]["comm"] == "staged-socket"
    assert j["metric"].endswith("128^3 fp64 grid") and j["config"]["model"].endswith("128^3 fp64 grid")


@pytest.mark.parametrize("world,decomp,schedule", [(2, (2, 1, 1), ["--no-overlap"]), (4, (2, 2, 1), ["--no-overlap"]),
                                                   (2, (2, 1, 1), []), (3, (3, 1, 1), []),
                                                   (4, (2, 2, 1), [])])
def test_rccl_graph_bitwise(h3d, gpu, tmp_path, world, decomp, schedule):
    """RCCL send / recv groups and all-reduces recorded into hipGraphs
    (--rccl-graph, the default): the single-stream schedule, and the
    overlapped three-stream schedule (one linear graph per stream, device-side
    cross-stream waits; x slabs and 2D blocks).  The ranks
    replay graphs (graph_launches > 0), exit cleanly and give the field of
    the eager single-process solve bit for bit.  Reference per-iteration
    comm: heat3D.cu:619-641 (halo), 1062-1063 (reduction)."""
    n, eps = 33, 1e-4
    extra = schedule + ["--rccl-graph", "--watchdog", "60", "--stream-graphs", "on"]
    mp.start_processes(native_rccl_gpu_worker,
                       args=(world, free_port(), str(tmp_path), n, eps, decomp, "fp64", extra),
                       nprocs=world, join=True, start_method="spawn")
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="hip", device=0, graph=False)
    r1 = single.run()
    it, err, name, graphs = open(tmp_path / "result.txt").read().split()
    assert int(graphs) > 0, "no hipGraph was replayed"
    assert int(it) == r1["conv_iter"] and name == "rccl"
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


@pytest.mark.parametrize("decomp,dtype", [((2, 2, 2), "fp64"), ((2, 2, 2), "fp32"), ((4, 2, 1), "fp64"),
                                          ((4, 2, 1), "fp32")])
def test_rccl_8rank_blocks_bitwise(h3d, gpu, tmp_path, decomp, dtype):
    """BASELINE configs 4 and 5 decompose 2x2x2 (6 neighbours): z faces packed
    and sent through ncclSend / ncclRecv with real peers, axis-ordered 3-axis
    deep halos (edges and corners ride the later phases), the overlapped
    boundary onion and the lagged all-reduce — 8 processes on the one GPU,
    eager replay (--stream-graphs auto: the overlapped schedule's per-stream
    graphs are opt-in, and never with more than 4 ranks on a device).  Bitwise equal to the one-rank solve of
    the same dtype, same stopping iteration.  eps 1e-2 (188 iterations): 8
    ranks on one GPU over RCCL's loopback network transport take ~80 ms per
    step (profiles/r06/rccl8_2x2x2_rehearsal.json).  Reference: heat3D.cu:243-263
    (Cartesian topology), 619-641 / 724-755 (6-face exchange)."""
    n, eps = 35, 1e-2
    os.environ["LOCAL_WORLD_SIZE"] = "8"  # inherited by the spawned ranks: 8 processes share the GPU
    try:
        mp.start_processes(native_rccl_gpu_worker,
                           args=(8, free_port(), str(tmp_path), n, eps, decomp, dtype, ["--watchdog", "60"]),
                           nprocs=8, join=True, start_method="spawn")
    finally:
        del os.environ["LOCAL_WORLD_SIZE"]
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="hip", device=0, dtype=dtype)
    r1 = single.run()
    it, err, name, graphs = open(tmp_path / "result.txt").read().split()
    assert int(it) == r1["conv_iter"] and name == "rccl"
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())
    meta = json.loads((tmp_path / "meta.json").read_text())
    assert meta["dims"] == list(decomp) and meta["stream_graphs"] == "off", meta


def test_bench_decomp_auto_times_candidates(gpu, tmp_path):
    """``bench.py --gpus 4 --decomp auto``: every rank times each candidate
    process grid (4x1x1 slabs, 2x2x1 blocks) through real RCCL at start-up,
    the job keeps the fastest by its slowest rank, and the JSON lists every
    candidate's ms/step (4 processes share the one GPU here, so the pick
    itself says nothing about xGMI)."""
    out = tmp_path / "d.json"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--comm", "rccl",
                        "--rccl-host-split", "--grid", "96", "--steps", "6", "--warmup", "3",
                        "--converge-eps", "0", "--profile-sweeps", "0", "--decomp-trial-steps", "12",
                        "--timeout", "150", "--json-out", str(out)],
                       capture_output=True, text=True, timeout=170, cwd=ROOT,
                       env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(out.read_text())
    d = j["decomp_auto"]
    assert [t["dims"] for t in d["trials"]] == [[4, 1, 1], [2, 2, 1]], d
    assert all(t["ms_per_step"] > 0 for t in d["trials"])
    best = min(d["trials"], key=lambda t: t["ms_per_step"])
    assert d["dims"] in ([4, 1, 1], best["dims"])
    assert j["placement"][0]["dims"] == d["dims"] and j["halo_verified"]
    assert j["runtime"]["torch_loaded"] is False and "/opt/rocm" in j["runtime"]["hip_library"]
