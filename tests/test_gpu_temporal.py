"""K-step temporally blocked gfx950 sweeps (the lean kernel stencil_tbl.hip and
its packed fp32 pair form stencil_tbp.hip) and the solver's sweep schedules:
bitwise identical to K single steps / to the single-step solver, all K
residuals included, convergence inside a sweep rolled back exactly."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

VARIANTS_F64 = ["auto", "tl2", "tl2:1:2:1:16:0:3", "tl2:1:3:1:16:0:3", "tl2:1:2:1:16:0:6", "tl2:1:2:1:16:5:3"]
VARIANTS_F32 = ["auto", "tl2", "tl2:2:2:1:16:0:3", "tl2:2:3:1:16:0:3", "tl2:1:3:1:16:0:3", "tl2:1:2:1:16:0:6"]


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


VARIANTS_K = {3: ["tl3", "tl3:1:3:1:16:0:4", "tl3:1:2:1:16:0:3", "tl3:1:3:1:16:5:3", "tl3:1:3:1:16:0:6",
                  "tl3:1:2:1:16:7:6", "tl3:1:6:1:8:0:3", "tl3:1:3:1:16:0:3:2", "tl3:1:3:1:16:0:3:19", "tl3:1:3:1:16:0:3:0",
                  "tl3:1:3:1:16:0:3:66"],
              4: ["tl4", "tl4:1:3:1:12:0:3:66", "tl4:1:2:1:16:0:4", "tl4:1:2:1:16:7:3", "tl4:1:2:1:16:0:6",
                  "tl4:1:2:1:16:5:6",
                  "tl4:1:6:1:8:0:3", "tl4:1:6:1:8:0:4", "tl4:1:5:1:8:0:3", "tl4:1:6:1:8:7:3",
                  "tl4:1:3:1:12:0:3:2", "tl4:1:3:1:12:0:3"],
              2: ["tl2", "tl2:1:2:1:16:0:3", "tl2:1:5:1:16:0:3:2", "tl2:1:5:1:16:0:3:66", "tl2:1:3:1:16:0:3:66"]}
# fp32: tlK:2:… is the packed-pair lean kernel (stencil_tbp.hip)
PAIR = {3: ["tl3:2:3:1:16:0:3", "tl3:2:3:1:16:0:3:2", "tl3:2:3:1:16:0:3:66", "tl3:2:3:1:16:0:4", "tl3:2:2:1:16:0:3", "tl3:2:3:1:16:5:3"],
        4: ["tl4:2:2:1:16:0:3", "tl4:2:2:1:16:0:4", "tl4:2:2:1:16:7:3", "tl4:2:2:1:16:0:3:64"],
        2: ["tl2:2:2:1:16:0:3", "tl2:2:3:1:16:0:3", "tl2:2:2:1:16:0:3:64"]}
VARIANTS_K_F32 = PAIR


def _last_only(kernel):
    """Spec store field bit 64: only the last step's residual is computed."""
    parts = kernel.split(":")
    return len(parts) > 7 and bool(int(parts[7]) & 64)


# fp64: the same kernel with 16-byte pairs (8 waves; round 5)
# (store field bit 64: the last step's residual only, the monotone check)
PAIR_F64 = {3: ["tl3:2", "tl3:2:4:1:8:0:3:0", "tl3:2:4:1:8:5:3:2", "tl3:2:4:1:8:0:3:66", "tl3:2:4:1:8:5:3:66"],
            4: ["tl4:2", "tl4:2:3:1:8:7:3:2", "tl4:2:3:1:8:0:3:66"],
            2: ["tl2:2", "tl2:2:6:1:8:0:3:2", "tl2:2:6:1:8:0:3:66"]}


@pytest.mark.parametrize("K", [2, 3, 4])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("n", [(9, 13, 130), (17, 21, 259), (5, 3, 64), (40, 33, 300), (3, 30, 7), (33, 1, 513)])
def test_stencil_k_bitwise(h3d, gpu, K, dtype, n):
    ops = h3d.ops
    D = (0.06, 0.05, 0.04)
    host, dev = _field(ops, n, dtype, gpu, 5)
    T = host.ghosted().clone()
    refs = []
    for _ in range(K):
        u, r = ops.ftcs_reference(T, D)
        T = T.clone()
        T[1:-1, 1:-1, 1:-1] = u
        refs.append(r)
    want = T[1:-1, 1:-1, 1:-1]
    for v in VARIANTS_K[K] + (VARIANTS_K_F32[K] if dtype == torch.float32 else PAIR_F64[K]):
        out = ops.PaddedField(n, dtype=dtype, device=gpu)
        out.flat.fill_(-3.0)
        st = ops.new_state(gpu)
        ops.ftcs_step2(dev, out, D, kernel=v, state=st, slot=0)
        torch.cuda.synchronize()
        got = out.owned().cpu()
        assert torch.equal(got, want), f"{v} {dtype} {n}: max diff {(got - want).abs().max().item()}"
        for s in range(K - 1 if _last_only(v) else 0, K):
            assert ops.residual_from_state(st, s) == refs[s], (v, s)


@pytest.mark.parametrize("K", [3, 4])
@pytest.mark.parametrize("vr,overlap", [(1, True), (3, True), (4, False)])
def test_temporal_depth_k_solver_gpu(h3d, gpu, K, vr, overlap):
    n = (67, 45, 131)
    a = h3d.HeatSolver(n, 10 ** 6, 1e-4, backend="hip", virtual_ranks=vr, decomp=(vr, 1, 1), overlap=overlap,
                       extra_args=["--temporal", str(K)])
    assert a.native.temporal_steps == K
    b = h3d.HeatSolver(n, 10 ** 6, 1e-4, backend="cpu", extra_args=["--temporal", "1"])
    ra, rb = a.run(), b.run()
    assert ra["conv_iter"] == rb["conv_iter"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("K", [3, 4])
def test_temporal_depth_k_goldens(h3d, gpu, K):
    for n, eps in ((27, 1e-3), (33, 1e-5), (64, 1e-3)):
        it, err, _ = h3d.utils.golden(n, eps)
        r = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="hip", extra_args=["--temporal", str(K)]).run()
        assert r["conv_iter"] == it and abs(r["error_percent"] - err) < 6e-5, (K, n, eps, r)


def _deep_random(ops, n, gx, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    f = ops.PaddedField(n, dtype=dtype, gx=gx)
    f.deep().copy_(torch.rand(f.deep().shape, generator=g, dtype=torch.float64).to(dtype))
    return f


@pytest.mark.parametrize("kernel", ["tl2", "tl3", "tl4", "tl4:1:2:1:16:0:4", "tl4:1:2:1:16:0:6",
                                    "tl4:1:6:1:8:0:3", "tl3:1:6:1:8:0:3"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("n0,box_x,side", [(4, (0, 4), "both"), (5, (0, 5), "lo"), (9, (0, 9), "hi"),
                                            (12, (4, 8), "both"), (12, (0, 4), "both"), (12, (8, 12), "both"),
                                            (30, (0, 30), "both")])
def test_sweep_deep_halo_matches_cpu(h3d, gpu, kernel, dtype, n0, box_x, side):
    """The slab path: K-plane ghost layers, u range widened into them, thin
    and partial x boxes.  gfx950 sweep == CPU K-single-steps definition."""
    _deep_halo_case(h3d, gpu, kernel, dtype, n0, box_x, side)


@pytest.mark.parametrize("kernel", PAIR[2] + PAIR[3] + PAIR[4])
@pytest.mark.parametrize("n0,box_x,side", [(4, (0, 4), "both"), (9, (0, 9), "hi"), (12, (4, 8), "both"),
                                            (30, (0, 30), "both")])
def test_sweep_pair_deep_halo_matches_cpu(h3d, gpu, kernel, n0, box_x, side):
    """The packed fp32 pair kernel on the slab path."""
    _deep_halo_case(h3d, gpu, kernel, torch.float32, n0, box_x, side)


@pytest.mark.parametrize("kernel", PAIR_F64[2] + PAIR_F64[3] + PAIR_F64[4])
@pytest.mark.parametrize("n0,box_x,side", [(4, (0, 4), "both"), (9, (0, 9), "hi"), (12, (4, 8), "both"),
                                            (30, (0, 30), "both"), (40, (3, 37), "both")])
def test_sweep_pair_f64_deep_halo_matches_cpu(h3d, gpu, kernel, n0, box_x, side):
    """The fp64 16-byte pair kernel on the slab path (the interior of a long
    x-slab share takes it when the start-up timing finds it faster)."""
    _deep_halo_case(h3d, gpu, kernel, torch.float64, n0, box_x, side)


@pytest.mark.parametrize("kernel", ["tl3", "tl3:1:3:1:16:0:3"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("n0,box_x,side,ny", [(12, (0, 3), "both", 64), (12, (9, 12), "both", 64),
                                               (6, (0, 3), "lo", 100), (9, (6, 9), "hi", 49),
                                               (20, (0, 4), "both", 70), (8, (0, 6), "both", 130)])
def test_sweep_thin_slab_y_marching(h3d, gpu, kernel, dtype, n0, box_x, side, ny):
    """Thin x slabs with a long y extent take the y-marching tiles (the
    default tl3 spec; an explicit shape stays x-marching): both equal the CPU
    K-single-steps definition."""
    _deep_halo_case(h3d, gpu, kernel, dtype, n0, box_x, side, ny)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("n0,box_x,side,ny", [(12, (0, 4), "both", 64), (12, (8, 12), "both", 64),
                                               (9, (0, 4), "lo", 100), (9, (5, 9), "hi", 70),
                                               (20, (0, 3), "both", 70), (20, (16, 20), "both", 63)])
def test_sweep_thin_slab_y_marching_k4(h3d, gpu, dtype, n0, box_x, side, ny):
    """The (K+1)-plane boundary slabs of long sweeps across x halos: K = 4
    y-marching tiles of 12 x-rows (ny < 16 x planes: the x-marching default)."""
    _deep_halo_case(h3d, gpu, "tl4", dtype, n0, box_x, side, ny)


def _deep_halo_case(h3d, gpu, kernel, dtype, n0, box_x, side, ny=37):
    ops = h3d.ops
    head = kernel.split(":")[0]
    K = int(head[2])
    n = (n0, ny, 133)
    ux = (-(K - 1) if side in ("lo", "both") else 0, n0 + (K - 1 if side in ("hi", "both") else 0))
    box = (box_x[0], box_x[1], 0, n[1], 0, n[2])
    D = (0.06, 0.05, 0.04)
    src = _deep_random(ops, n, K, dtype, 7)
    want = ops.PaddedField(n, dtype=dtype, gx=K)
    want.flat.fill_(-5.0)
    st_c = ops.new_state("cpu")
    ops.sweep(src, want, D, box, ux, kernel=kernel, state=st_c)
    dsrc = ops.PaddedField(n, dtype=dtype, device=gpu, gx=K)
    dsrc.flat.copy_(src.flat)
    got = ops.PaddedField(n, dtype=dtype, device=gpu, gx=K)
    got.flat.fill_(-5.0)
    st_g = ops.new_state(gpu)
    ops.sweep(dsrc, got, D, box, ux, kernel=kernel, state=st_g)
    torch.cuda.synchronize()
    x0, x1 = box_x
    a = got.owned().cpu()[x0:x1]
    b = want.owned()[x0:x1]
    assert torch.equal(a, b), f"{kernel} {n0} {box_x} {side}: max diff {(a - b).abs().max().item()}"
    for s in range(K - 1 if _last_only(kernel) else 0, K):
        assert ops.residual_from_state(st_g, s) == ops.residual_from_state(st_c, s), (kernel, s)


@pytest.mark.parametrize("K,vr", [(3, 8), (3, 1), (2, 4), (4, 3)])
def test_temporal_mixed_steps_gpu(h3d, gpu, K, vr):
    # single steps (3-stream overlapped schedule) interleaved with K-step
    # sweeps and their hipGraphs: every hand-over must be stream-ordered
    n = (37, 37, 70)
    a = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="hip", virtual_ranks=vr, decomp=(vr, 1, 1),
                       graph_chunk=12, extra_args=["--temporal", str(K)])
    b = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="cpu", extra_args=["--temporal", "1"])
    a.initialize(), b.initialize()
    for k in (1, 31, 2, 64, 5, 60, 7, 24):
        a.step(k)
        b.step(k)
    a.synchronize()
    assert a.state()["iter"] == b.state()["iter"] == 194
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("kernel2", ["tl3", "tl4", "tl2", "tl5", "tl3:1:3:1:16:0:4", "tl4:1:6:1:8:0:3"])
@pytest.mark.parametrize("vr", [1, 3])
def test_lean_kernel_solver_gpu(h3d, gpu, kernel2, vr):
    """Lean sweeps (stencil_tbl.hip) in the solver, single domain and x slabs:
    bitwise equal to the CPU single-step solver, same convergence."""
    n = (67, 45, 131)
    a = h3d.HeatSolver(n, 10 ** 6, 1e-4, backend="hip", virtual_ranks=vr, decomp=(vr, 1, 1),
                       extra_args=["--kernel2", kernel2])
    assert a.native.temporal_blocking and a.kernel.startswith(kernel2.split(":")[0]), a.kernel
    b = h3d.HeatSolver(n, 10 ** 6, 1e-4, backend="cpu", extra_args=["--temporal", "1"])
    ra, rb = a.run(), b.run()
    assert ra["conv_iter"] == rb["conv_iter"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("kernel2,dtype", [("tl3:2:3:1:16:0:3", "fp32"), ("tl4:2:2:1:16:0:3", "fp32"),
                                           ("tl2:2:2:1:16:0:3", "fp32")])
@pytest.mark.parametrize("vr", [1, 3])
def test_pair_kernel_solver_gpu(h3d, gpu, kernel2, dtype, vr):
    """The packed fp32 kernel in the solver (single domain, x slabs):
    bitwise equal to the CPU single-step solver, same convergence."""
    n = (67, 45, 131)
    a = h3d.HeatSolver(n, 10 ** 6, 1e-4, dtype=dtype, backend="hip", virtual_ranks=vr, decomp=(vr, 1, 1),
                       extra_args=["--kernel2", kernel2])
    assert a.native.temporal_blocking and a.kernel.startswith(kernel2), a.kernel
    b = h3d.HeatSolver(n, 10 ** 6, 1e-4, dtype=dtype, backend="cpu", extra_args=["--temporal", "1"])
    ra, rb = a.run(), b.run()
    assert ra["conv_iter"] == rb["conv_iter"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("kernel2", ["tl2", "tl3", "tl4", "tl5"])
def test_sweep_nan_faults(h3d, gpu, kernel2):
    """A NaN anywhere in the field reaches the convergence check as a fault
    (the kernel detects it on the stored T^{n+K} and poisons every slot)."""
    s = h3d.HeatSolver((41, 37, 45), 10 ** 6, 1e-5, backend="hip", extra_args=["--kernel2", kernel2])
    s.initialize()
    s.step(12)
    s.synchronize()
    s.native.inject(0, 20, 18, 22, float("nan"))
    r = s.run()
    assert r["fault"] and not r["converged"], r


@pytest.mark.parametrize("dims", [(2, 2, 2), (1, 2, 2), (2, 1, 3), (1, 3, 1), (1, 1, 2)])
@pytest.mark.parametrize("kernel2,dtype", [("tl2", "fp64"), ("tl3", "fp64"), ("tl4", "fp64"), ("tl4", "fp32"),
                                           ("tl3:1:6:1:8:0:3", "fp64"),
                                           ("tl3:2:3:1:16:0:3", "fp32"), ("tl4:2:2:1:16:0:3", "fp32")])
def test_block_decomposition_lean_kernel_gpu(h3d, gpu, dims, kernel2, dtype):
    """Deep y / z halos (axis-ordered exchange with edges and corners) and the
    lean kernel's y / z update ranges: virtual-rank block decompositions on
    the GPU equal the single-domain single-step run bit for bit."""
    n = (45, 61, 150)
    P = dims[0] * dims[1] * dims[2]
    a = h3d.HeatSolver(n, 29, 0.0, dtype=dtype, backend="hip", virtual_ranks=P, decomp=dims,
                       extra_args=["--kernel2", kernel2])
    b = h3d.HeatSolver(n, 29, 0.0, dtype=dtype, backend="hip", extra_args=["--temporal", "1"])
    assert a.native.temporal_blocking and a.native.kernel_name.startswith(kernel2.split(":")[0])
    ra, rb = a.run(), b.run()
    assert ra["iterations"] == rb["iterations"] == 29
    assert ra["last_residual"] == rb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("dims", [(2, 2, 2), (1, 2, 2)])
def test_block_decomposition_rollback_gpu(h3d, gpu, dims):
    P = dims[0] * dims[1] * dims[2]
    for eps in (1e-3, 9e-4, 8e-4):
        a = h3d.HeatSolver((33, 33, 33), 10 ** 6, eps, backend="hip", virtual_ranks=P, decomp=dims,
                           extra_args=["--check-every", "7"])
        b = h3d.HeatSolver((33, 33, 33), 10 ** 6, eps, backend="hip", extra_args=["--temporal", "1"])
        assert a.native.temporal_blocking
        ra, rb = a.run(), b.run()
        assert ra["conv_iter"] == rb["conv_iter"] and ra["converged"]
        assert np.array_equal(a.gather(), b.gather()), (dims, eps)


def _deep3_random(ops, n, g, dtype, seed):
    gen = torch.Generator().manual_seed(seed)
    f = ops.PaddedField(n, dtype=dtype, gx=g, gy=g, gz=g)
    f.deep3().copy_(torch.rand(f.deep3().shape, generator=gen, dtype=torch.float64).to(dtype))
    return f


@pytest.mark.parametrize("kernel", ["tl2", "tl3", "tl4", "tl3:1:3:1:16:0:4"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("box,sides", [((0, 12, 0, 50, 0, 140), "lo"), ((0, 12, 0, 50, 0, 140), "hi"),
                                       ((0, 12, 0, 50, 0, 140), "both"), ((0, 12, 4, 46, 0, 140), "both"),
                                       ((3, 9, 0, 4, 0, 140), "both"), ((0, 12, 46, 50, 5, 135), "both"),
                                       ((0, 12, 0, 50, 136, 140), "both"), ((2, 10, 3, 47, 0, 4), "both")])
def test_sweep_deep_yz_halo_matches_cpu(h3d, gpu, kernel, dtype, box, sides):
    """Deep ghosts on every axis (block decompositions): the lean kernel's
    y / z update ranges and its residual (only the box widened by K-1-s
    counts at stage s) equal the CPU K-single-steps definition on random
    fields, for thin / partial boxes such as the interior/boundary pieces."""
    _deep_yz_case(h3d, gpu, kernel, dtype, box, sides)


@pytest.mark.parametrize("kernel", ["tl3:2:3:1:16:0:3", "tl4:2:2:1:16:0:3", "tl2:2:2:1:16:0:3"])
@pytest.mark.parametrize("box,sides", [((0, 12, 0, 50, 0, 140), "lo"), ((0, 12, 0, 50, 0, 140), "both"),
                                       ((3, 9, 0, 4, 0, 140), "both"), ((0, 12, 46, 50, 5, 135), "both"),
                                       ((0, 12, 0, 50, 136, 140), "both"), ((2, 10, 3, 47, 0, 4), "both"),
                                       ((0, 12, 0, 50, 1, 139), "both"), ((0, 12, 0, 50, 3, 137), "hi")])
def test_sweep_pair_deep_yz_halo_matches_cpu(h3d, gpu, kernel, box, sides):
    """The packed fp32 pair kernel with y / z update ranges, odd and even box
    starts along z (its tiles start on an even column)."""
    _deep_yz_case(h3d, gpu, kernel, torch.float32, box, sides)


def _deep_yz_case(h3d, gpu, kernel, dtype, box, sides):
    ops = h3d.ops
    head = kernel.split(":")[0]
    K = int(head[2])
    n = (12, 50, 140)
    lo, hi = sides in ("lo", "both"), sides in ("hi", "both")
    u = []
    for a in range(3):
        u += [-(K - 1) if lo else 0, n[a] + (K - 1 if hi else 0)]
    D = (0.06, 0.05, 0.04)
    src = _deep3_random(ops, n, K, dtype, 11)
    want = ops.PaddedField(n, dtype=dtype, gx=K, gy=K, gz=K)
    want.flat.fill_(-5.0)
    st_c = ops.new_state("cpu")
    ops.sweep3(src, want, D, box, u, kernel=kernel, state=st_c)
    dsrc = ops.PaddedField(n, dtype=dtype, device=gpu, gx=K, gy=K, gz=K)
    dsrc.flat.copy_(src.flat)
    got = ops.PaddedField(n, dtype=dtype, device=gpu, gx=K, gy=K, gz=K)
    got.flat.fill_(-5.0)
    st_g = ops.new_state(gpu)
    ops.sweep3(dsrc, got, D, box, u, kernel=kernel, state=st_g)
    torch.cuda.synchronize()
    x0, x1, y0, y1, z0, z1 = box
    a = got.owned().cpu()[x0:x1, y0:y1, z0:z1]
    b = want.owned()[x0:x1, y0:y1, z0:z1]
    assert torch.equal(a, b), f"{kernel} {box} {sides}: max diff {(a - b).abs().max().item()}"
    s0 = K - 1 if _last_only(kernel) else 0
    res_c = [ops.residual_from_state(st_c, s) for s in range(s0, K)]
    res_g = [ops.residual_from_state(st_g, s) for s in range(s0, K)]
    assert res_c == res_g, (res_c, res_g)


@pytest.mark.parametrize("dims", [(2, 2, 2), (1, 2, 2), (2, 1, 3)])
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_block_overlap_gpu(h3d, gpu, dims, dtype):
    """Overlapped block sweeps on the GPU (three streams, lagged check) equal
    the exchange-first schedule and the single-domain run bit for bit."""
    P = dims[0] * dims[1] * dims[2]
    n = (61, 67, 150)
    a = h3d.HeatSolver(n, 31, 0.0, dtype=dtype, backend="hip", virtual_ranks=P, decomp=dims)
    b = h3d.HeatSolver(n, 31, 0.0, dtype=dtype, backend="hip", virtual_ranks=P, decomp=dims,
                       extra_args=["--no-block-overlap"])
    c = h3d.HeatSolver(n, 31, 0.0, dtype=dtype, backend="hip")
    assert a.native.field_buffers == 3 and b.native.field_buffers == 2
    ra, rb, rc = a.run(), b.run(), c.run()
    assert ra["last_residual"] == rb["last_residual"] == rc["last_residual"]
    ref = c.gather()
    assert np.array_equal(a.gather(), ref) and np.array_equal(b.gather(), ref)


def test_aligned_z_stride_solver_gpu(h3d, gpu):
    """A box thick enough for the 56-column (64-byte aligned) tile stride:
    bitwise equal to the CPU single-step solver."""
    n = (600, 40, 130)
    assert h3d.native().lean_z_stride(598, 38, 128, 3, 8, 48, 256, 6) == 56
    a = h3d.HeatSolver(n, 31, 0.0, backend="hip")
    b = h3d.HeatSolver(n, 31, 0.0, backend="cpu", extra_args=["--temporal", "1"])
    ra, rb = a.run(), b.run()
    assert ra["iterations"] == rb["iterations"] == 31 and ra["last_residual"] == rb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("iters", [7, 11, 12])
def test_temporal_k5_remainders(h3d, gpu, dtype, iters):
    """--temporal 5 with step counts that are not multiples of 5: the K+1 = 6
    long sweeps are taken only where that variant exists (fp32; fp64 has no
    K = 6 shape and falls back to partial sweeps) — bitwise equal to single
    steps either way (a K = 6 sweep used to be issued and throw)."""
    a = h3d.HeatSolver((41, 37, 45), iters, 0.0, dtype=dtype, backend="hip", extra_args=["--temporal", "5"])
    b = h3d.HeatSolver((41, 37, 45), iters, 0.0, dtype=dtype, backend="hip", extra_args=["--temporal", "1"])
    assert a.native.temporal_steps == 5
    ra, rb = a.run(), b.run()
    assert ra["iterations"] == rb["iterations"] == iters and ra["last_residual"] == rb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())


PREHEAT_GPU = [(1, (1, 1, 1)), (3, (3, 1, 1)), (8, (2, 2, 2))]


@pytest.mark.parametrize("vr,dims", PREHEAT_GPU)
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_preheat_state_neutral_gpu(h3d, gpu, vr, dims, dtype):
    """bench.py's preheat between the warm-up and the timed window:
    step(a); preheat(n); step(b) == step(a + b) bit for bit (field, residual,
    iteration count), graphs on, single domain / slabs (3 buffers) / 2x2x2."""
    n = (45, 61, 150)
    mk = lambda: h3d.HeatSolver(n, 10 ** 6, 0.0, dtype=dtype, backend="hip", virtual_ranks=vr, decomp=dims,
                                graph_chunk=12, extra_args=["--stream-graphs", "on"])
    for a_steps, b_steps in ((5, 20), (6, 12)):
        a, b = mk(), mk()
        a.initialize(), b.initialize()
        a.step(a_steps)
        a.prepare_steps(b_steps)
        assert a.native.preheat(5) == 5 * vr
        a.step(b_steps)
        b.step(a_steps + b_steps)
        a.synchronize(), b.synchronize()
        sa, sb = a.native.state(), b.native.state()
        assert sa["iter"] == sb["iter"] == a_steps + b_steps
        assert sa["last_residual"] == sb["last_residual"]
        assert np.array_equal(a.gather(), b.gather()), (vr, dtype, a_steps)


@pytest.mark.parametrize("vr,dims", PREHEAT_GPU)
def test_preheat_keeps_rollback_input_gpu(h3d, gpu, vr, dims):
    """Preheat after the converged sweep is a no-op (device done flag): the
    rollback input survives and run() ends on the same iteration and field."""
    n = (33, 33, 33)
    for eps in (1e-3, 9e-4, 8e-4):
        ref = h3d.HeatSolver(n, 10 ** 6, eps, backend="hip", virtual_ranks=vr, decomp=dims,
                             extra_args=["--check-every", "6"])
        rr = ref.run()
        c = rr["conv_iter"]
        end = (c // 3 + 1) * 3
        for extra_sweeps in (0, 1):
            s = h3d.HeatSolver(n, 10 ** 6, eps, backend="hip", virtual_ranks=vr, decomp=dims,
                               extra_args=["--check-every", "6"])
            s.initialize()
            s.step(end + 3 * extra_sweeps)
            s.native.preheat(4)
            r = s.run()
            assert r["converged"] and r["conv_iter"] == c, (eps, r, c)
            assert np.array_equal(s.gather(), ref.gather()), (vr, eps, extra_sweeps)


@pytest.mark.parametrize("vr,dims", [(3, (3, 1, 1)), (8, (8, 1, 1)), (8, (2, 2, 2)), (4, (1, 2, 2))])
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_long_sweeps_across_halos_gpu(h3d, gpu, vr, dims, dtype):
    """The driver's window at N > 1 (warm-up 5, then 20 steps = 4 x 3 + 2 x 4):
    long K+1 sweeps across the halos, including the (K+1)-plane boundary
    slabs (y-marching K = 4 thin-slab tiles), bitwise equal to single steps."""
    n = (82, 70, 150)
    a = h3d.HeatSolver(n, 10 ** 6, 0.0, dtype=dtype, backend="hip", virtual_ranks=vr, decomp=dims,
                       extra_args=["--long-sweeps", "on"])
    b = h3d.HeatSolver(n, 10 ** 6, 0.0, dtype=dtype, backend="hip", extra_args=["--temporal", "1"])
    assert a.native.long_halo_sweeps
    a.initialize(), b.initialize()
    for k in (5, 20, 11, 4):
        a.step(k)
        b.step(k)
        a.synchronize(), b.synchronize()
        sa, sb = a.native.state(), b.native.state()
        assert sa["iter"] == sb["iter"] and sa["last_residual"] == sb["last_residual"]
        assert np.array_equal(a.gather(), b.gather()), (vr, dims, dtype, k)
    assert a.native.verify_halos() == 0


@pytest.mark.parametrize("vr,dims", [(1, (1, 1, 1)), (3, (3, 1, 1)), (4, (4, 1, 1))])
def test_long_major_gpu(h3d, gpu, vr, dims):
    """--long-sweeps major: step counts run as many K+1-step (last-residual)
    sweeps as fit, across halos too; bitwise equal to single steps, and run()
    converges at the single steps' iteration (the replay of a long sweep).
    Block decompositions keep K-step sweeps (Solver::calibrate_remainders)."""
    n = (82, 70, 150)
    kw = dict(virtual_ranks=vr, decomp=dims) if vr > 1 else {}
    a = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="hip", extra_args=["--long-sweeps", "major"], **kw)
    b = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="hip", extra_args=["--temporal", "1"])
    a.initialize(), b.initialize()
    assert a.native.long_major
    for k in (5, 20, 11, 24):
        a.step(k)
        b.step(k)
        a.synchronize(), b.synchronize()
        sa, sb = a.native.state(), b.native.state()
        assert sa["iter"] == sb["iter"] and sa["last_residual"] == sb["last_residual"]
        assert np.array_equal(a.gather(), b.gather()), (vr, dims, k)
    if vr > 1:
        assert a.native.verify_halos() == 0
    for eps in (3e-4, 2.9e-4):
        c = h3d.HeatSolver(n, 10 ** 6, eps, backend="hip", extra_args=["--long-sweeps", "major"], **kw)
        d = h3d.HeatSolver(n, 10 ** 6, eps, backend="hip", extra_args=["--temporal", "1"])
        rc, rd = c.run(), d.run()
        assert rc["converged"] and rc["conv_iter"] == rd["conv_iter"], (eps, rc, rd)
        assert rc["last_residual"] == rd["last_residual"]
        assert np.array_equal(c.gather(), d.gather())


@pytest.mark.parametrize("vr,dims,n", [(8, (2, 2, 2), (82, 180, 260)), (4, (1, 2, 2), (40, 180, 380)),
                                        (4, (2, 2, 1), (90, 180, 100))])
@pytest.mark.parametrize("dtype,thin", [("fp64", False), ("fp32", False), ("fp64", True)])
def test_tile_thick_block_layers_gpu(h3d, gpu, vr, dims, n, dtype, thin):
    """Overlapped block sweeps with y / z boundary layers one tile stride
    thick (whole tiles; --thin-layers: K thick) on the device streams:
    regular, partial and long sweeps bitwise equal to single steps."""
    extra = ["--long-sweeps", "on"] + (["--thin-layers"] if thin else [])
    a = h3d.HeatSolver(n, 10 ** 6, 0.0, dtype=dtype, backend="hip", virtual_ranks=vr, decomp=dims, extra_args=extra)
    b = h3d.HeatSolver(n, 10 ** 6, 0.0, dtype=dtype, backend="hip", extra_args=["--temporal", "1"])
    a.initialize(), b.initialize()
    for k in (5, 20, 11, 4):
        a.step(k)
        b.step(k)
        a.synchronize(), b.synchronize()
        sa, sb = a.native.state(), b.native.state()
        assert sa["iter"] == sb["iter"] and sa["last_residual"] == sb["last_residual"]
        assert np.array_equal(a.gather(), b.gather()), (vr, dims, dtype, thin, k)
    assert a.native.verify_halos() == 0


@pytest.mark.parametrize("vr,dims", [(3, (3, 1, 1)), (8, (2, 2, 2))])
def test_long_sweep_across_halos_rollback_gpu(h3d, gpu, vr, dims):
    n = (33, 33, 33)
    for eps in (1e-3, 9e-4, 8e-4):
        ref = h3d.HeatSolver(n, 10 ** 6, eps, backend="hip", extra_args=["--temporal", "1"])
        rr = ref.run()
        c = rr["conv_iter"]
        for j in (c // 3, c // 3 - 1):
            s = h3d.HeatSolver(n, 10 ** 6, eps, backend="hip", virtual_ranks=vr, decomp=dims,
                               extra_args=["--long-sweeps", "on"])
            s.initialize()
            s.step(3 * j + 8)
            r = s.run()
            assert r["converged"] and r["conv_iter"] == c, (eps, j, r, c)
            assert np.array_equal(s.gather(), ref.gather()), (vr, eps, j)


@pytest.mark.parametrize("vr,dims", [(1, (1, 1, 1)), (3, (3, 1, 1))])
def test_remainder_policy_measured_gpu(h3d, gpu, vr, dims):
    """--long-sweeps auto (default): the start-up timing of the K, K+1 and
    partial sweeps picks, per remainder, long sweeps or a partial one; either
    way the result equals single steps bit for bit."""
    n = (82, 70, 150)
    a = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="hip", virtual_ranks=vr, decomp=dims)
    b = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="hip", extra_args=["--temporal", "1"])
    a.initialize(), b.initialize()
    costs = a.native.sweep_costs
    assert {"sweep3", "sweep4", "step", "sweep2"} <= set(costs) and all(v > 0 for v in costs.values()), costs
    # fp64 K = 2: three tile shapes timed (two lean, one pair), the partial
    # sweep costs the fastest
    shapes = [k for k in costs if k.startswith("sweep2[")]
    assert len(shapes) == 3 and costs["sweep2"] == min(costs[k] for k in shapes), costs
    # one subdomain: the pair form of the K and K+1 sweeps timed too, the
    # faster K form kept (Solver::pick_sweep_form); shares keep the lean form
    pair3 = [k for k in costs if k.startswith("sweep3[tl3:2")]
    assert len(pair3) == (1 if vr == 1 else 0), costs
    if pair3:
        assert pair3[0].startswith("sweep3[tl3:2") and any(k.startswith("sweep4[tl4:2") for k in costs), costs
        assert a.kernel.startswith("tl3:2" if costs[pair3[0]] < costs["sweep3"] else "tl3:1"), (a.kernel, costs)
    t3 = min(v for k, v in costs.items() if k.split("[")[0] == "sweep3")
    t4 = min(v for k, v in costs.items() if k.split("[")[0] == "sweep4")
    rem = a.native.long_remainders
    # with halos a long remainder must win by 15 % (Solver::calibrate_remainders)
    margin = 1.15 if vr > 1 else 1.0
    for r in (1, 2):
        assert (r in rem) == (r * (t4 - t3) * margin < costs["step" if r == 1 else "sweep2"]), (rem, costs)
    for k in (5, 20, 7):
        a.step(k)
        b.step(k)
    a.synchronize(), b.synchronize()
    assert a.native.state()["iter"] == b.native.state()["iter"] == 32
    assert np.array_equal(a.gather(), b.gather())
