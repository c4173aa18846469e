"""Worker functions for multi-process CPU tests (gloo, world_size > 1).

Each worker initialises torch.distributed (gloo, 127.0.0.1), runs a solver and
saves its results to ``outdir`` so the parent test can compare them.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _init(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    return dist


def native_socket_worker(rank, world, port, outdir, n, eps, decomp, dtype, extra_args=()):
    """Native engine, CPU backend, SocketComm bootstrapped through gloo."""
    dist = _init(rank, world, port)
    import heat3d_amd

    s = heat3d_amd.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", decomp=decomp, dtype=dtype,
                              threads=2, extra_args=list(extra_args))
    assert s.native.comm_name == "socket"
    if "--temporal" in extra_args:
        assert s.native.temporal_blocking == (int(extra_args[list(extra_args).index("--temporal") + 1]) >= 2)
    r = s.run()
    assert s.native.verify_halos() == 0  # checksums exchanged over the socket transport
    g = s.gather()
    ck = os.path.join(outdir, "ckpt")
    s.save_checkpoint(ck)
    s.write_tecplot(os.path.join(outdir, "out.dat"), "owned")
    if rank == 0:
        np.save(os.path.join(outdir, "field.npy"), g)
        with open(os.path.join(outdir, "result.txt"), "w") as f:
            f.write(f"{r['conv_iter']} {r['error_percent']!r} {r['norm']!r} {list(s.dims)}\n")
    else:
        assert g is None
    dist.barrier()
    dist.destroy_process_group()


def torch_reference_worker(rank, world, port, outdir, n, eps, decomp):
    """Pure-torch distributed oracle (gloo point-to-point halos)."""
    dist = _init(rank, world, port)
    import torch

    from heat3d_amd.parallel.torch_reference import TorchReferenceSolver

    s = TorchReferenceSolver((n, n, n), eps, 10 ** 6, dims=decomp)
    r = s.run()
    e, c = s.error_sum()
    t = torch.tensor([e, float(c)], dtype=torch.float64)
    dist.all_reduce(t)
    np.save(os.path.join(outdir, f"interior_{rank}.npy"), s.interior().numpy())
    with open(os.path.join(outdir, f"sub_{rank}.txt"), "w") as f:
        f.write(" ".join(str(v) for v in s.sub.gstart + s.sub.n) + "\n")
    if rank == 0:
        with open(os.path.join(outdir, "result.txt"), "w") as f:
            f.write(f"{r['conv_iter']} {100.0 * t[0].item() / t[1].item()!r}\n")
    dist.barrier()
    dist.destroy_process_group()


def native_staged_gpu_worker(rank, world, port, outdir, n, eps, decomp, dtype, extra_args=()):
    """Native engine, HIP backend on the one visible GPU, socket transport with
    host staging (RCCL refuses several ranks on one device): the multi-process
    GPU schedule — overlapped streams, deep halos, lagged all-reduce — across
    real processes."""
    dist = _init(rank, world, port)
    import heat3d_amd

    s = heat3d_amd.HeatSolver((n, n, n), 10 ** 6, eps, backend="hip", comm="socket", decomp=decomp,
                              dtype=dtype, device=0, extra_args=list(extra_args))
    assert s.native.comm_name == "staged-socket", s.native.comm_name
    r = s.run()
    assert s.native.verify_halos() == 0
    g = s.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "field.npy"), g)
        with open(os.path.join(outdir, "result.txt"), "w") as f:
            f.write(f"{r['conv_iter']} {r['error_percent']!r}\n")
    else:
        assert g is None
    dist.barrier()
    dist.destroy_process_group()


def native_staged_cpu_worker(rank, world, port, outdir, n, eps, decomp, extra_args=()):
    """CPU backend through the staging wrapper (comm="staged"): same schedule
    and transport as the GPU staged path, copies are host memcpy."""
    dist = _init(rank, world, port)
    import heat3d_amd

    s = heat3d_amd.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", comm="staged", decomp=decomp,
                              threads=2, extra_args=list(extra_args))
    assert s.native.comm_name == "staged-socket", s.native.comm_name
    r = s.run()
    assert s.native.verify_halos() == 0
    g = s.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "field.npy"), g)
        with open(os.path.join(outdir, "result.txt"), "w") as f:
            f.write(f"{r['conv_iter']}\n")
    dist.barrier()
    dist.destroy_process_group()


def native_rccl_gpu_worker(rank, world, port, outdir, n, eps, decomp, dtype, extra_args=()):
    """Native engine, HIP backend, a real multi-rank RCCL communicator with all
    ranks on the one visible GPU: every rank gets its own NCCL_HOSTID, so RCCL
    accepts the shared device (it refuses two ranks per GPU of one host) and
    carries the traffic over its network transport on loopback.  Exercises
    RcclComm::exchange (ncclSend / ncclRecv groups with real peers) and the
    all-reduce of the residual slots through the production schedule."""
    os.environ.update({"NCCL_HOSTID": f"heat3d-test-rank{rank}", "NCCL_SOCKET_IFNAME": "lo"})
    dist = _init(rank, world, port)
    import time

    import heat3d_amd

    t0 = time.perf_counter()

    def stage(what):  # progress on stderr (pytest -s shows it; a hang names its stage)
        print(f"[rccl worker {rank}/{world} {time.perf_counter() - t0:7.2f} s] {what}", file=sys.stderr, flush=True)

    s = heat3d_amd.HeatSolver((n, n, n), 10 ** 6, eps, backend="hip", comm="rccl", decomp=decomp,
                              dtype=dtype, device=0, extra_args=list(extra_args))
    stage("communicator up")
    assert s.native.comm_name.startswith("rccl"), s.native.comm_name
    assert s.native.comm_transport_ranks == world
    s.initialize()
    stage(f"initialized (stream graphs {s.native.stream_graphs_state})")
    r = s.run()
    stage(f"converged at {r['conv_iter']}")
    assert s.native.verify_halos() == 0  # checksums exchanged over RCCL
    g = s.gather()  # ncclSend / ncclRecv of every rank's block to rank 0
    stage("gathered")
    if rank == 0:
        np.save(os.path.join(outdir, "field.npy"), g)
        with open(os.path.join(outdir, "result.txt"), "w") as f:
            f.write(f"{r['conv_iter']} {r['error_percent']!r} {s.native.comm_name} {s.native.graph_launches}\n")
        with open(os.path.join(outdir, "meta.json"), "w") as f:
            json.dump({"dims": list(s.dims), "stream_graphs": s.native.stream_graphs_state,
                       "stream_graphs_canary": s.native.stream_graphs_note}, f)
    else:
        assert g is None
    dist.barrier()
    dist.destroy_process_group()


def native_socket_policy_worker(rank, world, port, outdir, n, eps, decomp, mode="measure"):
    """Remainder policy across real processes: every rank times its sweeps
    (--long-sweeps measure), the ranks vote over the socket transport, and
    run() (with a --time-limit iteration cap agreed by one more all-reduce)
    still reproduces the single-process field."""
    dist = _init(rank, world, port)
    import json

    import heat3d_amd

    s = heat3d_amd.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", decomp=decomp, threads=1,
                              extra_args=["--temporal", "3", "--long-sweeps", mode, "--time-limit", "60",
                                          "--check-every", "6"])
    s.initialize()
    with open(os.path.join(outdir, f"policy{rank}.json"), "w") as f:
        json.dump({"long": list(s.native.long_remainders), "costs": dict(s.native.sweep_costs),
                   "long_halo": s.native.long_halo_sweeps, "long_major": s.native.long_major}, f)
    # a step count with remainder 2 (long or partial per the vote), then run on
    s.step(20)
    r = s.run()
    g = s.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "field.npy"), g)
        with open(os.path.join(outdir, "result.txt"), "w") as f:
            f.write(f"{r['conv_iter']}\n")
    dist.barrier()
    dist.destroy_process_group()


def link_probe_worker(rank, world, port, outdir, nbytes):
    """Solver.link_probe over the socket transport: each rank exchanges
    `nbytes` with both ring neighbours; the job agrees on the slowest rate,
    and bench.py's decomposition vote (choose_dims) follows from it."""
    dist = _init(rank, world, port)
    import json

    import heat3d_amd
    from heat3d_amd.parallel import choose_dims

    s = heat3d_amd.HeatSolver((4 * world + 2, 8, 8), 1, 0.0, backend="cpu", decomp=(world, 1, 1), threads=1)
    gbps = s.native.link_probe(nbytes, 3)
    dims = choose_dims((1024, 1024, 1024), world, gbps)
    assert s.native.verify_halos() == 0
    with open(os.path.join(outdir, f"probe{rank}.json"), "w") as f:
        json.dump({"gbps": gbps, "dims": list(dims)}, f)
    dist.barrier()
    dist.destroy_process_group()
