"""Multi-process GPU runs on one MI355X: 2 or 4 processes share the device and
exchange halos over the host-staged socket transport (the reference's MPI
data path, heat3D.cu:610-755).  RCCL itself refuses two ranks on one device, so
this is how the non-local multi-process schedule (per-process streams,
overlapped x-slab / block sweeps with K-deep halos, lagged all-reduce of the
residual slots) runs on real GPU kernels here.  The gathered field must be
bitwise equal to the single-process GPU solve."""
import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import free_port
from _mp_workers import native_staged_gpu_worker

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,decomp,temporal", [(2, (2, 1, 1), "3"), (2, (2, 1, 1), "1"),
                                                    (4, (2, 2, 1), "3"), (4, (4, 1, 1), "2")])
def test_staged_multiprocess_gpu_bitwise(h3d, gpu, tmp_path, world, decomp, temporal):
    n, eps = 33, 1e-4
    mp.start_processes(native_staged_gpu_worker,
                       args=(world, free_port(), str(tmp_path), n, eps, decomp, "fp64", ["--temporal", temporal]),
                       nprocs=world, join=True, start_method="spawn")
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="hip", device=0)
    r1 = single.run()
    it, err = open(tmp_path / "result.txt").read().split()
    assert int(it) == r1["conv_iter"]
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


def test_cli_two_processes_one_gpu(heat3d_bin, gpu, tmp_path):
    """The heat3d CLI launched torchrun-style (RANK / WORLD_SIZE env) as two
    processes on the one GPU with --comm socket: HIP kernels, host-staged
    halos, the reference's golden iteration count (27^3, eps 1e-4)."""
    import os
    import subprocess

    port = free_port()
    procs = []
    for r in range(2):
        e = dict(os.environ)
        e.update({"WORLD_SIZE": "2", "RANK": str(r), "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(port), "HEAT3D_BOOTSTRAP_PORT": str(port)})
        procs.append(subprocess.Popen([heat3d_bin, "27", "27", "27", "100000", "1e-4", "--backend", "hip",
                                       "--comm", "socket", "--temporal", "3"], cwd=tmp_path, env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "converged in 1725 iterations" in outs[0][0]
    assert "comm=staged-socket ranks=2" in outs[0][0], outs[0][0]
    assert (tmp_path / "output" / "out.dat").read_text().count("ZONE") == 2


@pytest.mark.parametrize("rank,size,decomp,wire", [(1, 4, (4, 1, 1), "serial"), (5, 8, (2, 2, 2), "serial"),
                                                   (1, 4, (4, 1, 1), "overlap"), (1, 4, (4, 1, 1), "paced"),
                                                   (5, 8, (2, 2, 2), "paced")])
def test_phantom_rank_gpu(h3d, gpu, rank, size, decomp, wire):
    """PhantomComm on the GPU (tools/rank_proxy.py): one rank's full overlapped
    schedule with emulated halo delay kernels (after the stand-in copies, or
    ending a wire time after a device clock stamp taken before them);
    every issued iteration checked."""
    s = h3d.HeatSolver((97, 97, 97), 1 << 40, 0.0, backend="hip", device=0, decomp=decomp,
                       phantom=(rank, size), extra_args=["--temporal", "3", "--phantom-gbps", "50",
                                                         "--phantom-allreduce-us", "5", "--phantom-wire", wire])
    assert s.native.comm_name == "phantom"
    s.initialize()
    s.step(40)
    s.synchronize()
    st = s.state()
    assert st["iter"] == 40 and st["done"] == 0, st


def test_phantom_paced_wire_odd_fp32_faces(h3d, gpu):
    """--phantom-wire paced with fp32 faces that are not whole 16-byte words
    (2x2x2 blocks of a 91^3 grid): those exchanges take the serial wire."""
    s = h3d.HeatSolver((91, 91, 91), 1 << 40, 0.0, dtype="fp32", backend="hip", device=0, decomp=(2, 2, 2),
                       phantom=(5, 8), extra_args=["--temporal", "3", "--phantom-gbps", "50",
                                                   "--phantom-wire", "paced"])
    s.initialize()
    s.step(12)
    s.synchronize()
    assert s.state()["iter"] == 12


@pytest.mark.parametrize("n,rank,size,decomp,reserved", [(800, 0, 2, (2, 1, 1), 0), (800, 1, 8, (8, 1, 1), 8),
                                                          (400, 1, 2, (2, 1, 1), 8), (800, 7, 8, (2, 2, 2), 8)])
def test_comm_cu_reservation_rule(h3d, gpu, n, rank, size, decomp, reserved):
    """The overlapped multi-rank schedule keeps 8 CUs for the comm kernels,
    except under x-slab interiors of >= 2e8 points (394 x 798^2 here; the 2-
    and 4-GPU shares of 1024^3), which hide the halo chain even when RCCL's
    kernel waits for a CU (Solver::Solver, profiles/r05/proxy_runs.md)."""
    s = h3d.HeatSolver((n,) * 3, 1 << 40, 0.0, backend="hip", device=0, decomp=decomp, phantom=(rank, size),
                       extra_args=["--temporal", "3", "--phantom-gbps", "64"])
    assert s.native.reserved_cus == reserved, (n, decomp, s.native.reserved_cus)
    s.initialize()
    s.step(6)
    s.synchronize()
    assert s.state()["iter"] == 6


@pytest.mark.parametrize("rank,size,decomp", [(1, 8, (8, 1, 1)), (5, 8, (2, 2, 2))])
def test_phantom_paced_wire_moves_the_same_data(h3d, gpu, rank, size, decomp):
    """--phantom-wire paced (copies paced at the wire rate by a few workgroups
    per transfer) delivers the same bytes as the plain stand-in copies: the
    phantom rank's field after 30 steps is bitwise equal either way, and the
    paced exchanges last at least their wire time."""
    import time
    fields = {}
    for wire in ("serial", "paced"):
        s = h3d.HeatSolver((96, 96, 96), 1 << 40, 0.0, backend="hip", device=0, decomp=decomp,
                           phantom=(rank, size), graph=False,
                           extra_args=["--temporal", "3", "--phantom-gbps", "2", "--phantom-allreduce-us", "1",
                                       "--phantom-wire", wire])
        s.initialize()
        t0 = time.perf_counter()
        s.step(30)
        s.synchronize()
        el = time.perf_counter() - t0
        fields[wire] = s.local_field(0)
        face = 3 * 96 * 96 * 8 if decomp[0] == 8 else 3 * 48 * 48 * 8
        assert el >= 10 * face / 2e9 * 0.9, (wire, el)  # 10 exchanges of >= one face at 2 GB/s
    assert np.array_equal(fields["serial"].view(np.uint64), fields["paced"].view(np.uint64))
