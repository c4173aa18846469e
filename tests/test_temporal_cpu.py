"""2-step temporal blocking with x-slab decompositions (2-plane halos), CPU
backend: the pair schedule (interior planes || deep halo -> boundary slabs,
convergence rollback) must reproduce the single-step solver bit for bit for
every slab count, overlap mode and iteration count.  The CPU backend's
stencil2 is the two-single-steps definition of the gfx950 kernel."""
import numpy as np
import pytest

T2 = ["--temporal", "2"]
T1 = ["--temporal", "1"]


def _pair(h3d, n, iters, eps, vr, overlap=True, extra=()):
    a = h3d.HeatSolver(n, iters, eps, backend="cpu", virtual_ranks=vr, decomp=(vr, 1, 1),
                       overlap=overlap, extra_args=T2 + list(extra))
    b = h3d.HeatSolver(n, iters, eps, backend="cpu", extra_args=T1)
    assert a.native.temporal_blocking and not b.native.temporal_blocking
    return a, b


@pytest.mark.parametrize("vr", [2, 3, 4])
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("iters", [1, 2, 5, 40])
def test_slab_pairs_match_single_step(h3d, vr, overlap, iters):
    a, b = _pair(h3d, (31, 17, 19), iters, 0.0, vr, overlap)
    ra, rb = a.run(), b.run()
    assert ra["iterations"] == rb["iterations"] == iters
    assert ra["last_residual"] == rb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("eps", [1e-3, 3e-4, 1e-4, 5e-5])
@pytest.mark.parametrize("vr", [2, 4])
def test_slab_pairs_convergence_rollback(h3d, eps, vr):
    # several eps so that convergence lands in both halves of a pair
    a, b = _pair(h3d, (27, 27, 27), 10 ** 6, eps, vr, extra=["--check-every", "6"])
    ra, rb = a.run(), b.run()
    assert ra["conv_iter"] == rb["conv_iter"] and ra["converged"]
    assert abs(ra["error_percent"] - rb["error_percent"]) < 1e-12  # summation order differs
    assert np.array_equal(a.gather(), b.gather())


def test_slab_pairs_thin_slabs(h3d):
    # 2..3 owned planes per slab: no interior between the boundary slabs, the
    # pair runs non-overlapped (halo, then one sweep)
    a, b = _pair(h3d, (12, 9, 10), 30, 0.0, 4)
    a.run(), b.run()
    assert np.array_equal(a.gather(), b.gather())


def test_single_plane_slabs_fall_back(h3d):
    # 1 owned plane per slab cannot feed a 2-plane halo: single-step schedule
    s = h3d.HeatSolver((7, 9, 9), 10, 0.0, backend="cpu", virtual_ranks=5, decomp=(5, 1, 1), extra_args=T2)
    assert not s.native.temporal_blocking


def test_block_decomposition_stays_single_step(h3d):
    s = h3d.HeatSolver((17, 17, 17), 10, 0.0, backend="cpu", virtual_ranks=4, decomp=(2, 2, 1), extra_args=T2)
    assert not s.native.temporal_blocking


def test_slab_pairs_verify_halos(h3d):
    a, _ = _pair(h3d, (25, 15, 15), 20, 0.0, 3)
    a.run()
    assert a.native.verify_halos() == 0
    # corrupt a sent face of the last input buffer: the deep-halo checksum sees it
    a.native.inject(1, 1, 3, 3, 123.0, True)
    assert a.native.verify_halos() >= 1


def test_slab_pairs_odd_steps_and_state(h3d):
    # step() with odd counts mixes single steps and pairs on the same fields
    a, b = _pair(h3d, (29, 13, 13), 10 ** 6, 0.0, 3)
    a.initialize(), b.initialize()
    for k in (3, 4, 1, 7, 2):
        a.step(k)
        b.step(k)
    a.synchronize(), b.synchronize()
    assert a.state()["iter"] == b.state()["iter"] == 17
    assert np.array_equal(a.gather(), b.gather())
