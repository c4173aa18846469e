"""2-step temporally blocked gfx950 kernel (stencil_tb2.hip) and the solver's
double-step schedule: bitwise identical to two single steps / to the
single-step solver, including convergence in the first half of a pair."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

VARIANTS_F64 = ["tb2", "tb2:2:2:1:8", "tb2:2:2:1:16", "tb2:2:3:1:4", "tb2:2:4:2:4", "tb2:2:4:4:2", "tb2:2:4:1:4", "tb2:2:4:2:2", "tb2:2:8:2:2",
                "tb2:2:4:2:4:5", "tb2:2:4:2:4:1", "tb2:2:2:2:8"]
VARIANTS_F32 = ["tb2", "tb2:4:2:1:8", "tb2:4:3:1:4", "tb2:4:4:2:4", "tb2:4:4:2:2", "tb2:2:4:2:4", "tb2:4:4:2:4:3"]


def _field(ops, n, dtype, gpu, seed):
    g = torch.Generator().manual_seed(seed)
    f = ops.PaddedField(n, dtype=dtype)
    f.ghosted().copy_(torch.rand(tuple(v + 2 for v in n), generator=g, dtype=torch.float64).to(dtype))
    d = ops.PaddedField(n, dtype=dtype, device=gpu)
    d.flat.copy_(f.flat)
    return f, d


@pytest.mark.parametrize("dtype,variants", [(torch.float64, VARIANTS_F64), (torch.float32, VARIANTS_F32)])
@pytest.mark.parametrize("n", [(9, 13, 130), (17, 21, 259), (5, 3, 64), (40, 33, 1022), (3, 30, 7), (33, 1, 513)])
def test_stencil2_bitwise(h3d, gpu, dtype, variants, n):
    ops = h3d.ops
    D = (0.06, 0.05, 0.04)
    host, dev = _field(ops, n, dtype, gpu, 11)
    # reference: two single steps, ghosts held fixed
    T = host.ghosted().clone()
    u, r1 = ops.ftcs_reference(T, D)
    T1 = T.clone()
    T1[1:-1, 1:-1, 1:-1] = u
    t2, r2 = ops.ftcs_reference(T1, D)
    for v in variants:
        out = ops.PaddedField(n, dtype=dtype, device=gpu)
        out.flat.fill_(-3.0)
        st = ops.new_state(gpu)
        ops.ftcs_step2(dev, out, D, kernel=v, state=st, slot=0)
        torch.cuda.synchronize()
        got = out.owned().cpu()
        assert torch.equal(got, t2), f"{v} {dtype} {n}: max diff {(got - t2).abs().max().item()}"
        assert ops.residual_from_state(st, 0) == r1, v
        assert ops.residual_from_state(st, 1) == r2, v


@pytest.mark.parametrize("n,eps", [(27, 1e-3), (27, 1e-4), (33, 1e-5), (64, 1e-3), (65, 1e-5)])
def test_temporal_solver_goldens(h3d, gpu, n, eps):
    it, err, _ = h3d.utils.golden(n, eps)
    s = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="hip")
    assert s.native.temporal_blocking
    r = s.run()
    assert r["conv_iter"] == it and abs(r["error_percent"] - err) < 6e-5, r
    c = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu")
    c.run()
    assert np.array_equal(s.gather(), c.gather())


@pytest.mark.parametrize("graph", [True, False])
@pytest.mark.parametrize("iters", [1, 2, 7, 64, 101])
def test_temporal_matches_single_step(h3d, gpu, graph, iters):
    a = h3d.HeatSolver((41, 37, 45), iters, 0.0, backend="hip", graph=graph, graph_chunk=8)
    b = h3d.HeatSolver((41, 37, 45), iters, 0.0, backend="hip", extra_args=["--temporal", "1"])
    ra, rb = a.run(), b.run()
    assert a.native.temporal_blocking and not b.native.temporal_blocking
    assert ra["iterations"] == rb["iterations"] == iters
    assert np.array_equal(a.gather(), b.gather())
    assert ra["last_residual"] == rb["last_residual"]


def test_temporal_fp32(h3d, gpu):
    a = h3d.HeatSolver((33, 33, 33), 10 ** 6, 1e-4, backend="hip", dtype="fp32")
    b = h3d.HeatSolver((33, 33, 33), 10 ** 6, 1e-4, backend="cpu", dtype="fp32")
    ra, rb = a.run(), b.run()
    assert ra["conv_iter"] == rb["conv_iter"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("vr", [2, 3, 4])
@pytest.mark.parametrize("overlap", [True, False])
def test_temporal_slabs_gpu(h3d, gpu, vr, overlap):
    # x slabs as virtual ranks on one GPU: interior planes on the compute
    # stream || 2-plane halo + boundary slabs on the comm stream
    n = (67, 45, 131)
    a = h3d.HeatSolver(n, 10 ** 6, 1e-4, backend="hip", virtual_ranks=vr, decomp=(vr, 1, 1), overlap=overlap)
    assert a.native.temporal_blocking
    b = h3d.HeatSolver(n, 10 ** 6, 1e-4, backend="cpu", extra_args=["--temporal", "1"])
    ra, rb = a.run(), b.run()
    assert ra["conv_iter"] == rb["conv_iter"]
    assert np.array_equal(a.gather(), b.gather())
    assert a.native.verify_halos() == 0


@pytest.mark.parametrize("iters", [3, 50])
def test_temporal_slabs_gpu_fixed_iters(h3d, gpu, iters):
    n = (70, 33, 64)
    a = h3d.HeatSolver(n, iters, 0.0, backend="hip", virtual_ranks=4, decomp=(4, 1, 1))
    b = h3d.HeatSolver(n, iters, 0.0, backend="hip", extra_args=["--temporal", "1"])
    ra, rb = a.run(), b.run()
    assert ra["iterations"] == rb["iterations"] == iters
    assert ra["last_residual"] == rb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())
