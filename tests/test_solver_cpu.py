"""Native engine on the CPU backend: goldens, decomposition
invariance (bitwise), schedules, checkpoint/restart, fault detection, ops."""
import numpy as np
import pytest
import torch


def _solve(h3d, n, eps, iters=10 ** 6, **kw):
    s = h3d.HeatSolver((n, n, n) if isinstance(n, int) else n, iters, eps, backend="cpu", **kw)
    return s, s.run()


@pytest.mark.parametrize("n,eps", [(27, 1e-3), (27, 1e-4), (27, 1e-5), (33, 1e-5), (64, 1e-3)])
def test_goldens_cpu(h3d, n, eps):
    it, err, norm = h3d.utils.golden(n, eps)
    s, r = _solve(h3d, n, eps)
    assert r["converged"] and r["conv_iter"] == it
    assert abs(r["error_percent"] - err) < 6e-5
    assert abs(r["norm"] - norm) < 1e-6


def test_itermax_not_converged(h3d):
    s, r = _solve(h3d, 27, 1e-5, iters=100)
    assert not r["converged"] and r["iterations"] == 100
    assert abs(r["error_percent"] - h3d.utils.goldens.ITERMAX_100_27) < 6e-5


@pytest.mark.parametrize("vr,decomp", [(2, None), (3, None), (4, (1, 2, 2)), (8, None), (8, (8, 1, 1)),
                                       (12, None)])
def test_virtual_ranks_bitwise(h3d, vr, decomp):
    s1, r1 = _solve(h3d, 29, 1e-4)
    s2, r2 = _solve(h3d, 29, 1e-4, virtual_ranks=vr, decomp=decomp)
    assert r1["conv_iter"] == r2["conv_iter"]
    assert np.array_equal(s1.gather(), s2.gather())
    assert r1["error_percent"] == pytest.approx(r2["error_percent"], rel=1e-12)


def test_anisotropic_grid_invariance(h3d):
    s1, r1 = _solve(h3d, (31, 17, 23), 1e-4)
    s2, r2 = _solve(h3d, (31, 17, 23), 1e-4, virtual_ranks=6, decomp=(3, 2, 1))
    assert r1["conv_iter"] == r2["conv_iter"]
    assert np.array_equal(s1.gather(), s2.gather())


@pytest.mark.parametrize("overlap", [True, False])
def test_overlap_schedule_same_result(h3d, overlap):
    s1, r1 = _solve(h3d, 25, 1e-4, virtual_ranks=4, overlap=True, check_every=1)
    s2, r2 = _solve(h3d, 25, 1e-4, virtual_ranks=4, overlap=overlap, check_every=13)
    assert r1["conv_iter"] == r2["conv_iter"]
    assert np.array_equal(s1.gather(), s2.gather())


def test_fp32_close_to_fp64(h3d):
    s64, r64 = _solve(h3d, 27, 1e-4)
    s32, r32 = _solve(h3d, 27, 1e-4, dtype="fp32")
    assert abs(r32["conv_iter"] - r64["conv_iter"]) <= 5
    assert np.max(np.abs(s32.gather() - s64.gather())) < 1e-4


def test_step_and_state(h3d):
    s = h3d.HeatSolver((21, 21, 21), 10 ** 6, 0.0, backend="cpu")
    s.initialize()
    s.step(37)
    s.synchronize()
    st = s.state()
    assert st["iter"] == 37 and st["done"] == 0 and st["conv_iter"] == -1


def test_gather_matches_model_initial_field(h3d):
    s = h3d.HeatSolver((13, 11, 9), 10, 1e-3, backend="cpu", virtual_ranks=4)
    s.initialize()
    g = s.gather()
    assert np.array_equal(g, s.model.initial_field())


@pytest.mark.parametrize("vr_restart", [1, 4])
def test_checkpoint_restart(h3d, tmp_path, vr_restart):
    full, rf = _solve(h3d, 23, 1e-4)
    a = h3d.HeatSolver((23, 23, 23), 300, 1e-4, backend="cpu", virtual_ranks=2)
    a.run()
    a.save_checkpoint(str(tmp_path / "ck"))
    b = h3d.HeatSolver((23, 23, 23), 10 ** 6, 1e-4, backend="cpu", virtual_ranks=vr_restart,
                       extra_args=["--restart", str(tmp_path / "ck")])
    rb = b.run()
    assert rb["conv_iter"] == rf["conv_iter"]
    assert np.array_equal(b.gather(), full.gather())


def test_periodic_checkpoint_flag(h3d, tmp_path):
    s = h3d.HeatSolver((17, 17, 17), 200, 1e-9, backend="cpu",
                       extra_args=["--checkpoint-every", "64", "--checkpoint-dir", str(tmp_path / "p")])
    s.run()
    import json

    meta = json.loads((tmp_path / "p" / "meta.json").read_text())
    assert meta["iteration"] == 192 and meta["N"] == [17, 17, 17]


def test_checkpoint_mismatch_rejected(h3d, tmp_path):
    a = h3d.HeatSolver((15, 15, 15), 10, 1e-4, backend="cpu")
    a.run()
    a.save_checkpoint(str(tmp_path / "ck"))
    with pytest.raises(Exception):
        h3d.HeatSolver((17, 17, 17), 10, 1e-4, backend="cpu", extra_args=["--restart", str(tmp_path / "ck")]).run()


def test_nan_fault_detected(h3d):
    s = h3d.HeatSolver((21, 21, 21), 1000, 1e-9, backend="cpu", virtual_ranks=2)
    s.initialize()
    s.native.inject(1, 2, 3, 4, float("nan"))
    r = s.run()
    assert r["fault"] and not r["converged"] and r["conv_iter"] == 0


def test_ops_cpu_bitwise(h3d):
    ops = h3d.ops
    for dt in (torch.float64, torch.float32):
        f = ops.PaddedField((7, 9, 11), dtype=dt)
        f.ghosted().copy_(torch.rand(9, 11, 13, dtype=torch.float64).to(dt))
        g = ops.PaddedField((7, 9, 11), dtype=dt)
        st = ops.new_state("cpu")
        ops.ftcs_step(f, g, (0.05, 0.06, 0.07), state=st)
        ref, res = ops.ftcs_reference(f.ghosted(), (0.05, 0.06, 0.07))
        assert torch.equal(g.owned(), ref)
        assert ops.residual_from_state(st) == res


def test_model_matches_native_init(h3d):
    m = h3d.HeatEquation3D((9, 10, 11))
    ext = h3d.native()
    f = h3d.ops.PaddedField((7, 8, 9))
    h3d.ops.init_field(f, (1, 1, 1), m.n, m.h)
    assert np.array_equal(f.ghosted().numpy(), m.initial_field())
    for p in [(0, 3, 4), (3, 9, 4), (8, 0, 10), (4, 4, 4)]:
        assert ext.boundary_value(*p, list(m.n), list(m.h)) == (m.boundary_value(*p) if
                                                               0 in p or p[0] == 8 or p[1] == 9 or p[2] == 10 else 0.0)


@pytest.mark.parametrize("vr,decomp", [(2, (2, 1, 1)), (8, (2, 2, 2))])
def test_verify_halos_detects_corruption(h3d, vr, decomp):
    s = h3d.HeatSolver((19, 19, 19), 10 ** 6, 0.0, backend="cpu", virtual_ranks=vr, decomp=decomp)
    s.initialize()
    s.step(7)
    assert s.native.verify_halos() == 0
    # corrupt one ghost value of subdomain 0 in the buffer the check inspects
    sub = s.native.local_subdomain(0)
    s.native.inject(0, sub["n"][0], 2, 3, 123.0, previous=True)
    assert s.native.verify_halos() >= 1


def test_phase_timers(h3d):
    s = h3d.HeatSolver((33, 33, 33), 100, 0.0, backend="cpu", virtual_ranks=4)
    s.initialize()
    s.native.set_phase_timing(True)
    s.step(5)
    t = dict(s.native.phase_times())
    assert set(t) == {"interior_ms", "halo_ms", "shell_ms", "reduce_check_ms", "iteration_ms"}
    assert t["iteration_ms"] >= t["interior_ms"] >= 0


@pytest.mark.parametrize("rank,size,decomp,temporal", [(1, 4, (4, 1, 1), "3"), (0, 2, (2, 1, 1), "1"),
                                                       (3, 8, (2, 2, 2), "3")])
def test_phantom_rank_proxy_runs(h3d, rank, size, decomp, temporal):
    """PhantomComm (tools/rank_proxy.py): one rank of a P-rank job alone in the
    process builds only its subdomain and runs its whole schedule, every
    issued iteration accounted for, nothing converges at eps 0."""
    s = h3d.HeatSolver((20, 20, 20), 1 << 40, 0.0, backend="cpu", decomp=decomp, phantom=(rank, size),
                       threads=2, extra_args=["--temporal", temporal, "--phantom-allreduce-us", "0",
                                              "--phantom-wire", ("serial", "overlap", "paced")[rank % 3]])
    assert s.native.comm_name == "phantom"
    s.initialize()
    s.step(13)
    s.synchronize()
    st = s.state()
    assert st["iter"] == 13 and st["done"] == 0, st


def test_checkpoint_crash_safety_and_checksum(h3d, tmp_path):
    """Checkpoints are crash-safe (field.<iter>.raw written to a temp file,
    fsync'd and renamed before meta.json is atomically switched to it; older
    fields removed) and verified on restart (size + checksum)."""
    import json

    ck = tmp_path / "ck"
    a = h3d.HeatSolver((19, 17, 21), 40, 0.0, backend="cpu", virtual_ranks=3)
    a.run()
    a.save_checkpoint(str(ck))
    a.step(7)
    a.save_checkpoint(str(ck))
    meta = json.loads((ck / "meta.json").read_text())
    assert meta["format"] == "heat3d-checkpoint-v2" and meta["iteration"] == 47
    assert meta["field"] == "field.47.raw" and meta["bytes"] == 19 * 17 * 21 * 8
    assert sorted(p.name for p in ck.iterdir()) == ["field.47.raw", "meta.json"]
    raw = np.fromfile(ck / meta["field"], dtype=np.uint64)
    assert f"{int(raw.sum(dtype=np.uint64)):016x}" == meta["checksum"]
    assert np.array_equal(raw.view(np.float64).reshape(19, 17, 21), a.gather())
    # a restart on another decomposition resumes the same trajectory
    b = h3d.HeatSolver((19, 17, 21), 60, 0.0, backend="cpu", virtual_ranks=2,
                       extra_args=["--restart", str(ck)])
    c = h3d.HeatSolver((19, 17, 21), 60, 0.0, backend="cpu")
    b.run(), c.run()
    assert np.array_equal(b.gather(), c.gather())
    # a corrupted (or half-written) field is refused, not silently loaded
    buf = bytearray((ck / meta["field"]).read_bytes())
    buf[8 * 2000] ^= 0x10
    (ck / meta["field"]).write_bytes(bytes(buf))
    with pytest.raises(Exception, match="checksum"):
        h3d.HeatSolver((19, 17, 21), 60, 0.0, backend="cpu", extra_args=["--restart", str(ck)]).run()
    (ck / meta["field"]).write_bytes(bytes(buf[:-8]))
    with pytest.raises(Exception, match="bytes"):
        h3d.HeatSolver((19, 17, 21), 60, 0.0, backend="cpu", extra_args=["--restart", str(ck)]).run()


def test_checkpoint_interrupted_save_cleaned(h3d, tmp_path):
    """A save that a crash interrupted leaves a full-grid field.<iter>.raw.tmp
    behind; the next successful save removes it, and meta.json
    never pointed at it, so a restart in between resumes the previous save."""
    import json

    ck = tmp_path / "ck"
    a = h3d.HeatSolver((19, 17, 21), 40, 0.0, backend="cpu", virtual_ranks=2)
    a.run()
    a.save_checkpoint(str(ck))
    (ck / "field.45.raw.tmp").write_bytes(b"\0" * 1000)  # the crash mid-save at iteration 45
    assert json.loads((ck / "meta.json").read_text())["field"] == "field.40.raw"
    b = h3d.HeatSolver((19, 17, 21), 40, 0.0, backend="cpu", extra_args=["--restart", str(ck)])
    b.initialize()
    assert b.state()["iter"] == 40
    a.step(9)
    a.save_checkpoint(str(ck))
    assert sorted(p.name for p in ck.iterdir()) == ["field.49.raw", "meta.json"]


def test_streamed_io_bounded_chunks(h3d, tmp_path):
    """With a 1 MiB staging chunk the checkpoint, the per-rank Tecplot zones
    and the root gather stream in many chunks and give the same bytes."""
    import filecmp

    s = h3d.HeatSolver((37, 29, 33), 30, 0.0, backend="cpu", virtual_ranks=4, decomp=(2, 2, 1))
    s.run()
    s.write_tecplot(str(tmp_path / "a.dat"), "owned")
    s.save_checkpoint(str(tmp_path / "ca"))
    g = s.gather()
    t = h3d.HeatSolver((37, 29, 33), 30, 0.0, backend="cpu", virtual_ranks=4, decomp=(2, 2, 1),
                       extra_args=["--io-stage-mb", "1"])
    t.run()
    t.write_tecplot(str(tmp_path / "b.dat"), "owned")
    t.save_checkpoint(str(tmp_path / "cb"))
    assert filecmp.cmp(tmp_path / "a.dat", tmp_path / "b.dat", shallow=False)
    assert filecmp.cmp(tmp_path / "ca" / "field.30.raw", tmp_path / "cb" / "field.30.raw", shallow=False)
    assert np.array_equal(t.gather(), g)
    zones = h3d.utils.read_tecplot(str(tmp_path / "b.dat"))["zones"]
    assert len(zones) == 4 and sum(np.prod(z["shape"]) for z in zones) == 37 * 29 * 33


def test_gather_refuses_oversized_grid(h3d):
    s = h3d.HeatSolver((40, 40, 40), 5, 0.0, backend="cpu", extra_args=["--host-mem-limit-gb", "0.0001"])
    s.run()
    with pytest.raises(Exception, match="host memory"):
        s.gather()


def test_memory_preflight(h3d):
    """Buffers are sized before any allocation: a configuration that does not
    fit the backend's free memory is refused with the numbers (here host RAM;
    HBM via hipMemGetInfo on the GPU backend, tests/test_gpu_solver.py)."""
    s = h3d.HeatSolver((40, 40, 40), 5, 0.0, backend="cpu")
    n = s.native
    assert n.planned_bytes >= 2 * 42 ** 3 * 8 and n.mem_total > 0 and 0 < n.mem_free_before <= n.mem_total
    free, total = n.mem_info()
    assert total == n.mem_total and free > 0
    # the phantom corner rank of 2x2x2 (K-deep y / z ghosts, packed face buffers)
    p = h3d.HeatSolver((48, 48, 48), 5, 0.0, backend="cpu", decomp=(2, 2, 2), phantom=(7, 8),
                       extra_args=["--temporal", "3"])
    assert p.native.planned_bytes > p.native.field_buffers * 24 ** 3 * 8
    with pytest.raises(Exception, match="memory preflight.*needs"):
        h3d.HeatSolver((6000, 6000, 6000), 5, 0.0, backend="cpu")
    # a reserve of all the memory there is (free memory moves while other
    # test processes run: the free figure of an earlier solver is not a bound)
    reserve = ["--mem-reserve-gb", str(n.mem_total / 1e9)]
    with pytest.raises(Exception, match="memory preflight"):
        h3d.HeatSolver((40, 40, 40), 5, 0.0, backend="cpu", extra_args=reserve)
    h3d.HeatSolver((40, 40, 40), 5, 0.0, backend="cpu", extra_args=reserve + ["--no-mem-preflight"])
