"""Multi-process (gloo, world_size 2 and 4) CPU tests of the distributed path.

* native engine with the socket transport (the host-MPI analogue) across
  real processes must reproduce the single-process field bit for bit;
* an independent pure-torch distributed solver (gloo P2P halos) must agree
  with the native engine bit for bit.
"""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import free_port
from _mp_workers import link_probe_worker, native_socket_worker, torch_reference_worker


def _spawn(fn, world, *args):
    port = free_port()
    mp.start_processes(fn, args=(world, port) + args, nprocs=world, join=True, start_method="spawn")


@pytest.mark.parametrize("world,decomp", [(2, (2, 1, 1)), (2, (1, 1, 2)), (4, (2, 2, 1)), (4, (1, 2, 2))])
def test_native_socket_matches_single_process(h3d, tmp_path, world, decomp):
    n, eps = 23, 1e-4
    _spawn(native_socket_worker, world, str(tmp_path), n, eps, decomp, "fp64")
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu")
    r1 = single.run()
    it, err, norm, dims = open(tmp_path / "result.txt").read().split(" ", 3)
    assert int(it) == r1["conv_iter"]
    assert abs(float(err) - r1["error_percent"]) < 1e-12
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())
    # checkpoint written cooperatively by all ranks equals the single-process field
    import json

    meta = json.loads((tmp_path / "ckpt" / "meta.json").read_text())
    raw = np.fromfile(tmp_path / "ckpt" / meta["field"], dtype=np.float64).reshape(n, n, n)
    assert np.array_equal(raw, single.gather())
    # owned-layout Tecplot zones tile the grid: one zone per rank
    zones = h3d.utils.read_tecplot(str(tmp_path / "out.dat"))["zones"]
    assert len(zones) == world
    assert sum(np.prod(z["shape"]) for z in zones) == n ** 3


def test_native_socket_fp32(h3d, tmp_path):
    n, eps = 19, 1e-3
    _spawn(native_socket_worker, 2, str(tmp_path), n, eps, (2, 1, 1), "fp32")
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", dtype="fp32")
    r1 = single.run()
    assert int(open(tmp_path / "result.txt").read().split()[0]) == r1["conv_iter"]
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


@pytest.mark.parametrize("world,decomp", [(2, (2, 1, 1)), (4, (1, 2, 2))])
def test_torch_reference_matches_native(h3d, tmp_path, world, decomp):
    n, eps = 21, 1e-4
    _spawn(torch_reference_worker, world, str(tmp_path), n, eps, decomp)
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu")
    r1 = single.run()
    g = single.gather()
    it, err = open(tmp_path / "result.txt").read().split()
    assert int(it) == r1["conv_iter"]
    assert abs(float(err) - r1["error_percent"]) < 1e-9
    for r in range(world):
        gs = [int(v) for v in open(tmp_path / f"sub_{r}.txt").read().split()]
        st, cnt = gs[:3], gs[3:]
        part = np.load(tmp_path / f"interior_{r}.npy")
        sl = tuple(slice(st[a], st[a] + cnt[a]) for a in range(3))
        assert np.array_equal(part, g[sl]), f"rank {r} differs"


@pytest.mark.parametrize("world", [2, 3])
def test_native_socket_temporal_slabs(h3d, tmp_path, world):
    """2-step temporal blocking across processes: 2-plane x halos over the
    socket transport, bitwise equal to the single-process single-step solve."""
    n, eps = 23, 1e-4
    _spawn(native_socket_worker, world, str(tmp_path), n, eps, (world, 1, 1), "fp64", ["--temporal", "2"])
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", extra_args=["--temporal", "1"])
    r1 = single.run()
    assert int(open(tmp_path / "result.txt").read().split()[0]) == r1["conv_iter"]
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


@pytest.mark.parametrize("world,decomp", [(4, (2, 2, 1)), (4, (1, 2, 2)), (8, (2, 2, 2))])
def test_native_socket_temporal_blocks(h3d, tmp_path, world, decomp):
    """3-step temporal blocking across processes with y / z splits: the
    axis-ordered deep halo (pack -> exchange -> unpack per axis), overlapped
    boundary pieces, the lagged all-reduce of the residual slots — the
    non-local code path RCCL takes on a multi-GPU node — over the socket
    transport, bitwise equal to the single-process single-step solve."""
    n, eps = 27, 1e-4
    _spawn(native_socket_worker, world, str(tmp_path), n, eps, decomp, "fp64", ["--temporal", "3"])
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", extra_args=["--temporal", "1"])
    r1 = single.run()
    assert int(open(tmp_path / "result.txt").read().split()[0]) == r1["conv_iter"]
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


@pytest.mark.parametrize("world,decomp,temporal", [(2, (2, 1, 1), "3"), (4, (2, 2, 1), "3"), (2, (1, 2, 1), "1")])
def test_staged_comm_cpu(h3d, tmp_path, world, decomp, temporal):
    """StagedComm (the GPU ranks' host-staged socket transport) driven on the
    CPU backend: bitwise equal to the single-process solve."""
    from _mp_workers import native_staged_cpu_worker

    n, eps = 23, 1e-4
    _spawn(native_staged_cpu_worker, world, str(tmp_path), n, eps, decomp, ["--temporal", temporal])
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", extra_args=["--temporal", "1"])
    r1 = single.run()
    assert int(open(tmp_path / "result.txt").read().split()[0]) == r1["conv_iter"]
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


@pytest.mark.parametrize("world,decomp,mode", [(2, (2, 1, 1), "measure"), (3, (3, 1, 1), "measure"),
                                               (2, (2, 1, 1), "major"), (3, (3, 1, 1), "major")])
def test_remainder_policy_vote_across_processes(h3d, tmp_path, world, decomp, mode):
    """Solver::calibrate_remainders across real processes: each rank times
    its sweeps, the ranks agree by an all-reduce (their halo exchanges must
    pair up: a long sweep exchanges K+1 planes), and the solve stays bitwise
    equal to the single-process one."""
    import json

    from _mp_workers import native_socket_policy_worker

    n, eps = 31, 1e-4
    _spawn(native_socket_policy_worker, world, str(tmp_path), n, eps, decomp, mode)
    pol = [json.loads((tmp_path / f"policy{r}.json").read_text()) for r in range(world)]
    assert all(p["long_halo"] for p in pol)
    # major: long-major sweeps (every step count as many K+1-step sweeps as fit)
    assert all(p["long_major"] == (mode == "major") for p in pol), pol
    assert all(set(p["costs"]) == {"sweep3", "sweep4", "step", "sweep2"} for p in pol), pol
    assert all(p["long"] == pol[0]["long"] for p in pol), pol  # one decision for the job
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu")
    r1 = single.run()
    assert int(open(tmp_path / "result.txt").read().split()[0]) == r1["conv_iter"]
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


@pytest.mark.parametrize("world", [2, 3, 8])
def test_link_probe_vote(h3d, tmp_path, world):
    """The bench's --decomp auto: every rank times a face exchange with both
    ring neighbours (one peer for 2 ranks) over the job's transport and the
    ranks agree on the slowest rate, so they choose the same process grid."""
    import json

    _spawn(link_probe_worker, world, str(tmp_path), 1 << 20)
    res = [json.loads((tmp_path / f"probe{r}.json").read_text()) for r in range(world)]
    assert all(r == res[0] for r in res), res
    assert res[0]["gbps"] > 0
    assert res[0]["dims"][0] * res[0]["dims"][1] * res[0]["dims"][2] == world
