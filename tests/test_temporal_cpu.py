"""K-step temporal blocking with x-slab decompositions (K-plane halos), CPU
backend: the sweep schedule (interior planes || deep halo -> boundary slabs,
convergence rollback) must reproduce the single-step solver bit for bit for
every depth K, slab count, overlap mode and iteration count.  The CPU
backend's multi-step sweep is the K-single-steps definition of the gfx950
kernel (stencil_tbl.hip / stencil_tbp.hip)."""
import numpy as np
import pytest

T2 = ["--temporal", "2"]
T1 = ["--temporal", "1"]
DEPTHS = [2, 3, 4]


def _pair(h3d, n, iters, eps, vr, overlap=True, extra=(), K=2):
    a = h3d.HeatSolver(n, iters, eps, backend="cpu", virtual_ranks=vr, decomp=(vr, 1, 1),
                       overlap=overlap, extra_args=["--temporal", str(K)] + list(extra))
    b = h3d.HeatSolver(n, iters, eps, backend="cpu", extra_args=T1)
    assert a.native.temporal_blocking and not b.native.temporal_blocking
    assert a.native.temporal_steps == K
    return a, b


@pytest.mark.parametrize("K", DEPTHS)
@pytest.mark.parametrize("vr", [1, 2, 3])
@pytest.mark.parametrize("iters", [1, 5, 17])
def test_depth_k_matches_single_step(h3d, K, vr, iters):
    a, b = _pair(h3d, (37, 17, 19), iters, 0.0, vr, K=K)
    ra, rb = a.run(), b.run()
    assert ra["iterations"] == rb["iterations"] == iters
    assert ra["last_residual"] == rb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("K", [3, 4])
@pytest.mark.parametrize("vr", [1, 3])
def test_depth_k_convergence_rollback(h3d, K, vr):
    # converged iteration lands at every offset inside a K-sweep
    for eps in (1e-3, 9e-4, 8e-4, 7e-4):
        a, b = _pair(h3d, (25, 25, 25), 10 ** 6, eps, vr, K=K, extra=["--check-every", "5"])
        ra, rb = a.run(), b.run()
        assert ra["conv_iter"] == rb["conv_iter"] and ra["converged"]
        assert np.array_equal(a.gather(), b.gather()), (K, vr, eps, rb["conv_iter"])


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


def test_block_decomposition_uses_lean_kernel(h3d):
    # y / z splits take temporal blocking too, with the lean kernel's y / z
    # update ranges; the retired round-1/2 kernel families are refused
    s = h3d.HeatSolver((17, 17, 17), 10, 0.0, backend="cpu", virtual_ranks=4, decomp=(2, 2, 1), extra_args=T2)
    assert s.native.temporal_blocking and s.native.temporal_steps == 2
    assert s.native.kernel_name.startswith("tl2"), s.native.kernel_name
    for old in ("tr2", "tb2", "tbk2", "tb3"):
        with pytest.raises(Exception, match="retired"):
            h3d.HeatSolver((17, 17, 17), 10, 0.0, backend="cpu", virtual_ranks=4, decomp=(2, 2, 1),
                           extra_args=T2 + ["--kernel2", old])


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


@pytest.mark.parametrize("K", [2, 3, 4])
@pytest.mark.parametrize("box_x,ux", [((0, 6), (-1, 7)), ((2, 4), (-3, 9)), ((0, 3), (0, 8)), ((3, 6), (-2, 6))])
def test_cpu_sweep_definition(h3d, K, box_x, ux):
    """ops.sweep on the CPU (the definition the gfx950 kernels are tested
    against) == K plain-torch steps on shrinking widened x ranges."""
    import torch
    ops = h3d.ops
    n = (6, 7, 9)
    ux = (max(ux[0], -(K - 1)), min(ux[1], n[0] + K - 1))
    g = torch.Generator().manual_seed(3)
    f = ops.PaddedField(n, gx=K)
    f.deep().copy_(torch.rand(f.deep().shape, generator=g, dtype=torch.float64))
    out = ops.PaddedField(n, gx=K)
    ops.sweep(f, out, (0.07, 0.05, 0.03), (box_x[0], box_x[1], 0, n[1], 0, n[2]), ux,
              kernel=f"tl{K}")
    T = f.deep().clone()  # plane index i <-> T[i + K]
    for s in range(K):
        w = K - 1 - s
        lo, hi = max(box_x[0] - w, ux[0]), min(box_x[1] + w, ux[1])
        new, _ = ops.ftcs_reference(T[lo + K - 1: hi + K + 1], (0.07, 0.05, 0.03))
        T = T.clone()
        T[lo + K: hi + K, 1:-1, 1:-1] = new
    assert torch.equal(out.owned()[box_x[0]:box_x[1]], T[box_x[0] + K: box_x[1] + K, 1:-1, 1:-1])


@pytest.mark.parametrize("K", [2, 3, 4])
def test_lagged_check_uses_three_buffers(h3d, K):
    """Overlapped x-slab sweeps lag the convergence check by one sweep (third
    field buffer, two residual-slot banks); --lag off restores the
    ping-pong schedule.  Both converge at the same iteration to the same field,
    with the converged iteration landing at every offset inside a sweep."""
    for eps in (1e-3, 9e-4, 8e-4, 7e-4):
        a, b = _pair(h3d, (37, 21, 19), 10 ** 6, eps, 3, K=K, extra=["--check-every", "5"])
        assert a.native.field_buffers == 3
        c = h3d.HeatSolver((37, 21, 19), 10 ** 6, eps, backend="cpu", virtual_ranks=3, decomp=(3, 1, 1),
                           extra_args=["--temporal", str(K), "--check-every", "5", "--lag", "off"])
        assert c.native.field_buffers == 2 and b.native.field_buffers == 2
        ra, rb, rc = a.run(), b.run(), c.run()
        assert ra["conv_iter"] == rb["conv_iter"] == rc["conv_iter"] and ra["converged"]
        ref = b.gather()
        assert np.array_equal(a.gather(), ref) and np.array_equal(c.gather(), ref), (K, eps)


BLOCKS = [(2, 2, 1), (1, 2, 2), (2, 2, 2), (1, 1, 3), (3, 2, 1), (1, 3, 1)]


@pytest.mark.parametrize("dims", BLOCKS)
@pytest.mark.parametrize("K", [2, 3, 4])
def test_block_decomposition_temporal_matches_single_step(h3d, dims, K):
    """K-step sweeps with deep y / z halos (axis-ordered exchange filling the
    edge and corner ghosts) reproduce the single-step solver bit for bit."""
    n = (27, 25, 29)
    P = dims[0] * dims[1] * dims[2]
    a = h3d.HeatSolver(n, 23, 0.0, backend="cpu", virtual_ranks=P, decomp=dims,
                       extra_args=["--temporal", str(K)])
    b = h3d.HeatSolver(n, 23, 0.0, backend="cpu", extra_args=T1)
    assert a.native.temporal_blocking and a.native.temporal_steps == K
    ra, rb = a.run(), b.run()
    assert ra["iterations"] == rb["iterations"] == 23
    assert ra["last_residual"] == rb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("dims", [(2, 2, 2), (1, 2, 2)])
@pytest.mark.parametrize("K", [3, 4])
def test_block_decomposition_temporal_rollback(h3d, dims, K):
    # converged iteration lands at every offset inside a K-sweep
    P = dims[0] * dims[1] * dims[2]
    for eps in (1e-3, 9e-4, 8e-4, 7e-4):
        a = h3d.HeatSolver((25, 25, 25), 10 ** 6, eps, backend="cpu", virtual_ranks=P, decomp=dims,
                           extra_args=["--temporal", str(K), "--check-every", "5"])
        b = h3d.HeatSolver((25, 25, 25), 10 ** 6, eps, backend="cpu", extra_args=T1)
        ra, rb = a.run(), b.run()
        assert ra["conv_iter"] == rb["conv_iter"] and ra["converged"]
        assert np.array_equal(a.gather(), b.gather()), (dims, K, eps)


def test_block_decomposition_verify_halos(h3d):
    s = h3d.HeatSolver((21, 23, 25), 12, 0.0, backend="cpu", virtual_ranks=8, decomp=(2, 2, 2),
                       extra_args=["--temporal", "3"])
    s.run()
    assert s.native.verify_halos() == 0


def test_block_decomposition_too_thin_falls_back(h3d):
    # 5 interior points over 3 ranks along y: some subdomain has < K = 3 rows
    s = h3d.HeatSolver((17, 7, 17), 10, 0.0, backend="cpu", virtual_ranks=3, decomp=(1, 3, 1),
                       extra_args=["--temporal", "3"])
    assert not s.native.temporal_blocking


@pytest.mark.parametrize("K", [3, 4])
@pytest.mark.parametrize("vr,dims", [(1, (1, 1, 1)), (3, (3, 1, 1)), (4, (2, 2, 1))])
@pytest.mark.parametrize("iters", [2, 5, 11])
def test_partial_sweep_remainders(h3d, K, vr, dims, iters):
    """Step counts that are not a multiple of K end with a partial sweep of
    2..K-1 steps (ring kernel of that depth) instead of single steps."""
    n = (31, 23, 27)
    a = h3d.HeatSolver(n, iters, 0.0, backend="cpu", virtual_ranks=vr, decomp=dims,
                       extra_args=["--temporal", str(K)])
    b = h3d.HeatSolver(n, iters, 0.0, backend="cpu", extra_args=T1)
    a.initialize()
    b.initialize()
    a.step(iters)
    b.step(iters)
    sa, sb = a.native.state(), b.native.state()
    assert sa["iter"] == sb["iter"] == iters and sa["last_residual"] == sb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("dims", [(2, 2, 2), (1, 2, 2), (2, 1, 3)])
def test_block_overlap_matches_exchange_first(h3d, dims):
    """Overlapped block sweeps (interior || axis-ordered halo -> onion of
    boundary pieces, lagged check on three buffers) equal the exchange-first
    schedule (--no-block-overlap) bit for bit, converged or not."""
    P = dims[0] * dims[1] * dims[2]
    n = (31, 29, 33)
    for eps in (0.0, 8e-4):
        a = h3d.HeatSolver(n, 10 ** 6 if eps else 25, eps, backend="cpu", virtual_ranks=P, decomp=dims,
                           extra_args=["--temporal", "3", "--check-every", "5"])
        b = h3d.HeatSolver(n, 10 ** 6 if eps else 25, eps, backend="cpu", virtual_ranks=P, decomp=dims,
                           extra_args=["--temporal", "3", "--check-every", "5", "--no-block-overlap"])
        assert a.native.field_buffers == 3 and b.native.field_buffers == 2
        ra, rb = a.run(), b.run()
        assert ra["conv_iter"] == rb["conv_iter"] and ra["last_residual"] == rb["last_residual"]
        assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("dims_a,dims_b", [((2, 2, 2), (1, 1, 1)), ((1, 1, 1), (2, 2, 1)), ((3, 1, 1), (1, 2, 2)),
                                           ((1, 3, 1), (2, 1, 1))])
def test_checkpoint_restart_across_temporal_decompositions(h3d, tmp_path, dims_a, dims_b):
    """A checkpoint written by a temporally blocked run (three buffers when
    overlapped) restarts on any other decomposition and finishes at the same
    iteration with the same field as an uninterrupted single-step solve."""
    n, eps = 25, 1e-4
    full = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", extra_args=T1)
    rf = full.run()
    Pa = dims_a[0] * dims_a[1] * dims_a[2]
    Pb = dims_b[0] * dims_b[1] * dims_b[2]
    a = h3d.HeatSolver((n, n, n), 301, eps, backend="cpu", virtual_ranks=Pa, decomp=dims_a,
                       extra_args=["--temporal", "3"])
    a.run()
    a.save_checkpoint(str(tmp_path / "ck"))
    b = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", virtual_ranks=Pb, decomp=dims_b,
                       extra_args=["--temporal", "3", "--restart", str(tmp_path / "ck")])
    rb = b.run()
    assert rb["conv_iter"] == rf["conv_iter"]
    assert np.array_equal(b.gather(), full.gather())


def test_lean_z_stride_model(h3d):
    """fp64 lean-kernel tiles store 56 columns (64-byte aligned strips) instead
    of 58 on thick boxes where the x-plan model predicts a shorter sweep, and
    keep 58 on thin slabs and where a tile column would cross a round."""
    n = h3d.native()
    zs = lambda *b: n.lean_z_stride(*b, 3, 8, 48, 256, 6)  # noqa: E731
    assert zs(1022, 1022, 1022) == 56 and zs(598, 38, 128) == 56
    assert zs(510, 510, 510) == 58                      # 9 -> 10 tile columns crosses a round
    assert zs(122, 1022, 1022) == 58 and zs(250, 1022, 1022) == 58  # 8- / 4-GPU slab shares
    assert n.lean_z_stride(1022, 1022, 1022, 3, 4, 48, 256, 6) == 58  # fp32: unchanged
    assert n.lean_z_stride(1022, 1022, 1022, 4, 8, 32, 256, 12) == 56  # 64 - 2K is aligned already


def test_lean_store_policy_defaults(h3d):
    """Lean sweeps of the default fp64 K = 3 / 4 shapes and of the fp32 K = 3
    pair shape store with the nt cache policy (profiles/nt_stores_r02.md);
    the fp64 K = 2 default is 16 waves x 5 rows with nt stores (80-row tiles,
    profiles/probes_r04.md); other shapes and explicit policies are left as
    given."""
    r = h3d.native().kernel_spec_resolved
    assert r("tl3", "fp64") == "tl3:1:3:1:16:0:3:2"
    assert r("tl4", "fp64") == "tl4:1:3:1:12:0:3:2"
    assert r("tl4:1:2:1:16", "fp64") == "tl4:1:2:1:16:0:3:2"
    assert r("tl2", "fp64") == "tl2:1:5:1:16:0:3:2"
    assert r("tl2:1:3:1:16", "fp64") == "tl2:1:3:1:16:0:3"
    assert r("tl3:1:3:1:16:0:3:0", "fp64") == "tl3:1:3:1:16:0:3"
    assert r("tl3:1:3:1:16:0:3:19", "fp64") == "tl3:1:3:1:16:0:3:19"
    assert r("tl3:1:2:1:16", "fp64") == "tl3:1:2:1:16:0:3"
    assert r("tl3", "fp32") == "tl3:2:3:1:16:0:3:2"
    assert r("tl4", "fp32") == "tl4:2:2:1:16:0:3"


def test_pair_z_stride_counts_bytes(h3d):
    """fp32 pair tiles: the aligned 112-column stride where it does not add a
    nearly empty tile column (2047^3: 1531 vs 1456 GLUPS), 120 where it would
    (1022^3: 9 columns of 120 vs 10 of 112, the last 14 wide: 1397 vs 1294) —
    tiling_cost charges the bytes of every tile, not only the makespan
    (profiles/xplan_calibration_r03.md)."""
    zs = lambda n: h3d.native().pair_z_stride(n, n, n, 3, 48, 256, 6)  # noqa: E731
    assert zs(1022) == 120 and zs(2047) == 112 and zs(4094) == 112


def test_x_plan_model(h3d):
    """The host x planner (binding x_plan): 1022^3 fp64 takes 7 segments of 146
    planes (3325 pieces = 12.99 rounds of 256, the best measured segment),
    thin slab shares whole-x pieces, the 4-GPU share a split tail; forced
    segments are honoured and the model never beats the ideal."""
    xp = h3d.native().x_plan
    p = xp(1022, 475, 256, 4, 6)
    assert p["seg"] == 146 and p["n1"] == 3325 and p["r"] == 0
    assert xp(122, 450, 256, 4, 6)["seg"] == 122
    t = xp(250, 450, 256, 4, 6)
    assert t["n1"] == 256 and t["r"] == 194 and t["nb2"] == 194 and 0 < t["split"] < 250
    assert xp(1022, 475, 256, 4, 6, 511)["seg"] == 511
    for nx, tiles in ((1022, 475), (122, 450), (2047, 931), (510, 117)):
        q = xp(nx, tiles, 256, 4, 6)
        assert q["makespan"] >= q["ideal"], q


def test_kernel_spec_z_stride_field(h3d):
    """Spec field 9 forces the z tile stride and survives resolution."""
    r = h3d.native().kernel_spec_resolved
    assert r("tl3:1:3:1:16:0:3:2:56", "fp64") == "tl3:1:3:1:16:0:3:2:56"
    assert r("tl3:2:3:1:16:0:3:2:112", "fp32") == "tl3:2:3:1:16:0:3:2:112"


PREHEAT_CASES = [(1, (1, 1, 1)), (3, (3, 1, 1)), (8, (2, 2, 2))]


@pytest.mark.parametrize("vr,dims", PREHEAT_CASES)
@pytest.mark.parametrize("a_steps,b_steps", [(6, 9), (5, 7), (9, 12)])
def test_preheat_is_state_neutral(h3d, vr, dims, a_steps, b_steps):
    """Solver::preheat (bench.py's untimed warm-up right before the timed
    window) rewrites nxt(cur()) with the next sweep's interior: step(a);
    preheat(n); step(b) equals step(a + b) bit for bit in field, residual
    and iteration count (single domain, x slabs on three buffers, 2x2x2)."""
    n = (29, 27, 31)
    mk = lambda: h3d.HeatSolver(n, 10 ** 6, 0.0, backend="cpu", virtual_ranks=vr, decomp=dims,
                                extra_args=["--temporal", "3"])
    a, b = mk(), mk()
    assert a.native.temporal_blocking
    if vr > 1:
        assert a.native.field_buffers == 3
    a.initialize(), b.initialize()
    a.step(a_steps)
    assert a.native.preheat(4) == 4 * vr
    a.step(b_steps)
    b.step(a_steps + b_steps)
    a.synchronize(), b.synchronize()
    sa, sb = a.native.state(), b.native.state()
    assert sa["iter"] == sb["iter"] == a_steps + b_steps
    assert sa["last_residual"] == sb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("vr,dims", PREHEAT_CASES)
def test_preheat_keeps_rollback_input(h3d, vr, dims):
    """A preheat issued after the converged sweep must not clobber that
    sweep's input buffer, which the rollback recomputes the final field from
    (with two buffers it is nxt(cur()) right after the sweep): the sweeps
    honour the device done flag.  Converged iterations land at every offset
    of a sweep; preheat right after the converged sweep and one sweep later."""
    n = (25, 25, 25)
    for eps in (1e-3, 9e-4, 8e-4):
        extra = ["--temporal", "3", "--check-every", "6"]
        ref = h3d.HeatSolver(n, 10 ** 6, eps, backend="cpu", virtual_ranks=vr, decomp=dims, extra_args=extra)
        rr = ref.run()
        assert rr["converged"]
        c = rr["conv_iter"]
        end = (c // 3 + 1) * 3  # first sweep boundary after the converged iteration
        for extra_sweeps in (0, 1):
            s = h3d.HeatSolver(n, 10 ** 6, eps, backend="cpu", virtual_ranks=vr, decomp=dims, extra_args=extra)
            s.initialize()
            s.step(end + 3 * extra_sweeps)
            s.native.preheat(3)
            r = s.run()
            assert r["converged"] and r["conv_iter"] == c, (eps, r, c)
            assert np.array_equal(s.gather(), ref.gather()), (vr, eps, extra_sweeps)


LONG_HALO = [(3, (3, 1, 1)), (2, (2, 1, 1)), (4, (2, 2, 1)), (8, (2, 2, 2)), (3, (1, 1, 3))]


@pytest.mark.parametrize("vr,dims", LONG_HALO)
@pytest.mark.parametrize("K", [2, 3])
def test_long_sweeps_across_halos(h3d, vr, dims, K):
    """Step counts that are not multiples of K end in sweeps of depth K+1
    across the halos (ghosts K+1 deep on split axes, exchanged K+1 deep
    before a long sweep only) — the driver's 20-step window at N > 1 runs
    4 x 3 + 2 x 4 instead of 6 x 3 + a partial 2 — bitwise equal to single
    steps for every count, mixed with regular sweeps on the same fields."""
    n = (33, 29, 31)
    a = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="cpu", virtual_ranks=vr, decomp=dims,
                       extra_args=["--temporal", str(K)])
    b = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="cpu", extra_args=T1)
    assert a.native.long_halo_sweeps
    assert list(a.native.ghost_depth) == [K + 1 if d > 1 else 1 for d in dims]
    a.initialize(), b.initialize()
    for k in (5, 20, 7, 11, 4):
        a.step(k)
        b.step(k)
        sa, sb = a.native.state(), b.native.state()
        assert sa["iter"] == sb["iter"] and sa["last_residual"] == sb["last_residual"]
        assert np.array_equal(a.gather(), b.gather()), (vr, dims, K, k)
    assert a.native.verify_halos() == 0


@pytest.mark.parametrize("thin", [False, True])
def test_tile_thick_block_layers(h3d, thin):
    """Overlapped block sweeps: y / z boundary layers one tile stride thick
    (42 rows, 58 columns at fp64 K = 3) where the subdomain has room, K thin
    with --thin-layers or without room; the pieces tile the owned box and the
    sweeps stay bitwise equal to single steps."""
    n = (14, 172, 236)   # 2x2 in y, z: owned 85 x 117 per rank
    extra = ["--temporal", "3"] + (["--thin-layers"] if thin else [])
    a = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="cpu", virtual_ranks=4, decomp=(1, 2, 2), extra_args=extra)
    b = h3d.HeatSolver(n, 10 ** 6, 0.0, backend="cpu", extra_args=T1)
    pieces = [list(p) for p in a.native.sweep_pieces(0)]   # rank 0: neighbours above in y and z
    ty, tz = (3, 3) if thin else (42, 58)
    assert pieces == [[0, 12, 0, 85 - ty, 0, 117 - tz],            # interior
                      [0, 12, 85 - ty, 85, 0, 117],                # y layer (full z)
                      [0, 12, 0, 85 - ty, 117 - tz, 117]], pieces  # z layer (interior y)
    a.initialize(), b.initialize()
    for k in (7, 6, 3):
        a.step(k)
        b.step(k)
        assert np.array_equal(a.gather(), b.gather()), (thin, k)


def test_retired_schedule_flags(h3d):
    """Round 4's opt-in schedule variants that lost on every configuration
    (core/rim interiors, chunked halos, boundary pieces after the interior on
    the compute stream) are refused with a clear message."""
    for flag in (["--core-rim"], ["--halo-chunks", "4"], ["--boundary-stream", "compute"]):
        with pytest.raises(Exception, match="retired"):
            h3d.HeatSolver((40, 37, 31), 10, 0.0, backend="cpu", virtual_ranks=2, decomp=(2, 1, 1),
                           extra_args=["--temporal", "3", *flag])


def test_long_sweeps_across_halos_off(h3d):
    """--no-long-sweeps keeps K-deep ghosts (remainders as partial sweeps)."""
    a = h3d.HeatSolver((33, 29, 31), 20, 0.0, backend="cpu", virtual_ranks=3, decomp=(3, 1, 1),
                       extra_args=["--temporal", "3", "--no-long-sweeps"])
    b = h3d.HeatSolver((33, 29, 31), 20, 0.0, backend="cpu", extra_args=T1)
    assert not a.native.long_halo_sweeps and list(a.native.ghost_depth) == [3, 1, 1]
    a.run(), b.run()
    assert np.array_equal(a.gather(), b.gather())


@pytest.mark.parametrize("vr,dims", [(3, (3, 1, 1)), (8, (2, 2, 2))])
def test_long_sweep_across_halos_rollback(h3d, vr, dims):
    """Convergence inside a long (K+1) sweep across halos: the rollback
    recomputes the final field from the sweep's input buffer, whose ghosts
    that sweep exchanged K+1 deep."""
    n = (25, 25, 25)
    for eps in (1e-3, 9e-4, 8e-4, 7e-4):
        ref = h3d.HeatSolver(n, 10 ** 6, eps, backend="cpu", extra_args=T1)
        rr = ref.run()
        c = rr["conv_iter"]
        for j in (c // 3, c // 3 - 1):
            s = h3d.HeatSolver(n, 10 ** 6, eps, backend="cpu", virtual_ranks=vr, decomp=dims,
                               extra_args=["--temporal", "3"])
            s.initialize()
            s.step(3 * j + 8)  # 3 j steps in K-sweeps, then 2 long sweeps over c
            r = s.run()
            assert r["converged"] and r["conv_iter"] == c, (eps, j, r, c)
            assert np.array_equal(s.gather(), ref.gather()), (vr, eps, j)


def test_best_fixed_segments_beat_the_plan_model():
    """The start-up tuner's extra x-schedule candidates (round 6): fixed
    segments of any length, whose last piece per tile is short.  In the
    dispatch model they beat the x plan where its equal pieces leave a round
    part-empty (1022^3 fp32 pairs: 225 tiles; 510^3 fp64: 117 tiles), and are
    never worse than the best equal split."""
    import heat3d_amd

    e = heat3d_amd.native()
    for nx, tiles, want in ((1022, 225, 0.92), (510, 117, 0.95), (1022, 475, 0.96), (2046, 882, 1.0)):
        segs = e.best_fixed_segments(nx, tiles, 256, 4, 6, 2)
        assert len(segs) == 2 and all(6 <= s <= nx for s in segs), segs
        best = e.x_plan(nx, tiles, 256, 4, 6, segs[0])["makespan"]
        plan = e.x_plan(nx, tiles, 256, 4, 6, 0)["makespan"]
        equal = min(e.x_plan(nx, tiles, 256, 4, 6, -(-nx // k))["makespan"] for k in range(1, 17))
        assert best <= want * plan and best <= equal, (nx, tiles, segs, best, plan, equal)
