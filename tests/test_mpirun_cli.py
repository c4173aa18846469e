"""The reference's launch contract under a real MPI launcher.

``mpirun -n P ./heat3D NX NY NZ ITER_MAX EPS`` (heat3D.cu:203-205 MPI_Init /
rank / size, 270-315 argument check and echo, 1078-1106 report).  MPICH's
hydra launcher (``mpirun``, present in this image) starts P processes of the
native CLI; each takes its rank from PMI_RANK / PMI_SIZE
(``make_solver_from_env``, csrc/runtime/solver.cpp), the ranks meet through
the TCP bootstrap and exchange halos over the socket transport (CPU backend:
no GPU here).  Rank 0 alone prints the banner and the report, the converged
iteration is the single-domain golden (decomposition-independent results),
and a wrong argument count prints the usage once and fails every rank.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import free_port

MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
pytestmark = pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun in this image")

_LAUNCHER_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                  "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "PMI_RANK", "PMI_SIZE")


def _mpirun(heat3d_bin, n, args, cwd, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCHER_VARS}
    env["HEAT3D_BOOTSTRAP_PORT"] = str(free_port())
    return subprocess.run([MPIRUN, "-n", str(n), heat3d_bin] + list(args), cwd=cwd, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n,decomp", [(4, None), (2, "1x2x1")])
def test_mpirun_reference_launch(heat3d_bin, tmp_path, n, decomp):
    args = ["33", "33", "33", "100000", "1e-5", "--backend", "cpu", "--comm", "socket", "--threads", "2"]
    if decomp:
        args += ["--decomp", decomp]
    r = _mpirun(heat3d_bin, n, args, tmp_path)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = r.stdout
    # one banner and one report for the whole job (rank 0), not one per process
    assert out.count("Runnung HeatEquation3D with the following arguments:") == 1, out
    assert out.count("Computational time (parallel): ") == 1
    assert out.count("L2-norm error:") == 1
    assert f"comm=socket ranks={n}" in out
    # App. B.3 golden of the single domain: the decomposition changes nothing
    assert "Simulation has converged in 3590 iterations with a convergence threshold of 1.000000e-05" in out
    assert "L2-norm error: 0.0287 %" in out
    # output/out.dat written once, one zone per rank with the rank column (heat3D.cu:1125-1162)
    lines = (tmp_path / "output" / "out.dat").read_text().split("\n")
    assert lines[0] == 'TITLE="out"' and lines[1] == 'VARIABLES = "X", "Y", "Z", "T", "rank"'
    assert sum(1 for l in lines if l.startswith("ZONE T = ")) == n


def test_mpirun_usage_error(heat3d_bin, tmp_path):
    """A wrong argument count: the usage text once (rank 0), every rank exits
    non-zero (the reference let ranks > 0 run on into stoi)."""
    r = _mpirun(heat3d_bin, 3, ["33", "33"], tmp_path, timeout=60)
    assert r.returncode != 0
    assert r.stdout.count("Incorrect number of command line arguments specified") == 1, r.stdout
    assert not (tmp_path / "output").exists()


@pytest.mark.gpu
def test_mpirun_hip_rccl(heat3d_bin, tmp_path):
    """The reference's exact GPU launch, ``mpirun -n P ./heat3D ...``
    (heat3D.cu:203-205 MPI_Init, 650-654 cudaSetDevice), through the native
    CLI with the HIP backend and RCCL: hydra's PMI_RANK / PMI_SIZE give the
    rank, MPI_LOCALRANKID the device (local rank mod visible GPUs), the ranks
    bootstrap the RCCL communicator over TCP.  One GPU here, so the launch is
    MPMD with a per-rank NCCL_HOSTID (RCCL refuses two ranks of one host on
    one device; as two "hosts" they talk over its socket transport on lo)."""
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCHER_VARS}
    env["HEAT3D_BOOTSTRAP_PORT"] = str(free_port())
    env["HEAT3D_SHOW_PLACEMENT"] = "1"
    args = ["33", "33", "33", "100000", "1e-5", "--backend", "hip", "--comm", "rccl", "--watchdog", "120"]
    cmd = [MPIRUN, "-genv", "NCCL_SOCKET_IFNAME", "lo"]
    for r in range(2):
        if r:
            cmd.append(":")
        cmd += ["-n", "1", "-env", "NCCL_HOSTID", f"heat3d-mpirun-rank{r}", heat3d_bin] + args
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = r.stdout
    assert out.count("Runnung HeatEquation3D with the following arguments:") == 1, out
    assert "Simulation has converged in 3590 iterations with a convergence threshold of 1.000000e-05" in out
    assert "L2-norm error: 0.0287 %" in out
    assert "backend=hip comm=rccl ranks=2" in out, out
    placed = sorted(l for l in r.stderr.splitlines() if l.startswith("heat3d: placement"))
    assert len(placed) == 2, r.stderr[-3000:]
    for rank, line in enumerate(placed):
        m = re.search(r"rank=(\d+) size=2 local_rank=(\d+) from=MPI_LOCALRANKID device=(\d+) of (\d+)", line)
        assert m, line
        assert int(m.group(1)) == int(m.group(2)) == rank and int(m.group(3)) == rank % int(m.group(4)), line
