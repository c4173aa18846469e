"""End-to-end native solver on the MI355X: goldens, decomposition invariance,
graph vs eager, overlap vs no overlap, RCCL (1 rank), checkpoint/restart."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(h3d, n, eps, iters=10 ** 6, **kw):
    s = h3d.HeatSolver((n, n, n), iters, eps, backend=kw.pop("backend", "hip"), **kw)
    r = s.run()
    return s, r


def test_native_extension_is_in_tree(h3d, gpu):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert os.path.abspath(h3d.native().__file__).startswith(root)


@pytest.mark.parametrize("n,eps", [(27, 1e-3), (27, 1e-5), (33, 1e-5), (64, 1e-3), (64, 1e-4), (65, 1e-5),
                                   (129, 1e-3)])
def test_goldens_gpu(h3d, gpu, n, eps):
    it, err, norm = h3d.utils.golden(n, eps)
    s, r = _solve(h3d, n, eps)
    assert s.backend == "hip"
    assert r["converged"] and r["conv_iter"] == it, r
    assert abs(r["error_percent"] - err) < 6e-5, r
    assert abs(r["norm"] - norm) < 1e-6


@pytest.mark.slow
def test_golden_129_1e5_gpu(h3d, gpu):
    it, err, _ = h3d.utils.golden(129, 1e-5)
    s, r = _solve(h3d, 129, 1e-5)
    assert r["conv_iter"] == it and abs(r["error_percent"] - err) < 6e-5, r


@pytest.mark.slow
@pytest.mark.parametrize("eps", [1e-3, 1e-4, 1e-5])
def test_goldens_257_gpu(h3d, gpu, eps):
    """Convergence parity at the largest size the survey modelled (App. B.3;
    91362 iterations at eps 1e-5)."""
    it, err, norm = h3d.utils.golden(257, eps)
    s, r = _solve(h3d, 257, eps)
    assert r["converged"] and r["conv_iter"] == it, r
    assert abs(r["error_percent"] - err) < 6e-5 and abs(r["norm"] - norm) < 1e-6, r


@pytest.mark.slow
def test_golden_257_slabs_gpu(h3d, gpu):
    """Same golden through the 8-slab overlapped schedule (K-deep halos,
    lagged check)."""
    it, err, _ = h3d.utils.golden(257, 1e-3)
    s, r = _solve(h3d, 257, 1e-3, virtual_ranks=8, decomp=(8, 1, 1))
    assert r["conv_iter"] == it and abs(r["error_percent"] - err) < 6e-5, r


@pytest.mark.slow
@pytest.mark.parametrize("vr", [1, 8])
def test_golden_513_gpu(h3d, gpu, vr):
    """Round-3 golden beyond the survey's sizes: 513^3 at eps 1e-3 converges
    at 2132 iterations, 42.7695 % (native CPU backend, 270 s on 6 threads;
    utils/goldens.py) — on the GPU as one domain and as 8 overlapped x slabs."""
    it, err, norm = h3d.utils.golden(513, 1e-3)
    kw = dict(virtual_ranks=vr, decomp=(vr, 1, 1)) if vr > 1 else {}
    s, r = _solve(h3d, 513, 1e-3, **kw)
    assert r["converged"] and r["conv_iter"] == it, r
    assert abs(r["error_percent"] - err) < 6e-5 and abs(r["norm"] - norm) < 1e-6, r


@pytest.mark.slow
@pytest.mark.parametrize("vr", [1, 8])
def test_golden_1024_gpu(h3d, gpu, vr):
    """Round-5 golden on the headline grid: 1024^3 at eps 1e-3 converges at
    2170 iterations, 46.2574 % (native CPU backend, 54 min on 6 threads;
    utils/goldens.py) — on the GPU as one domain (K = 3 / 4 sweeps, the
    bench's kernels) and as 8 overlapped x slabs (the 8-GPU decomposition)."""
    it, err, norm = h3d.utils.golden(1024, 1e-3)
    kw = dict(virtual_ranks=vr, decomp=(vr, 1, 1)) if vr > 1 else {}
    s, r = _solve(h3d, 1024, 1e-3, **kw)
    assert r["converged"] and r["conv_iter"] == it, r
    assert abs(r["error_percent"] - err) < 6e-5 and abs(r["norm"] - norm) < 1e-6, r


def test_hbm_preflight(h3d, gpu):
    """planned_bytes is what the solver takes from HBM (hipMemGetInfo before /
    after), and a configuration that cannot fit is refused before allocating:
    8192^3 fp32 on 2x2x2 GPUs needs 3 x 275 GB on each."""
    s = h3d.HeatSolver((320, 320, 320), 10, 0.0, backend="hip", virtual_ranks=4, decomp=(4, 1, 1))
    n = s.native
    free_after, total = n.mem_info()
    used = n.mem_free_before - free_after
    assert total == n.mem_total and total > 250e9
    assert n.planned_bytes <= used + (64 << 20) and used <= n.planned_bytes + (512 << 20), (used, n.planned_bytes)
    with pytest.raises(Exception, match="memory preflight"):
        h3d.HeatSolver((8192,) * 3, 10, 0.0, dtype="fp32", backend="hip", decomp=(2, 2, 2), phantom=(7, 8),
                       device=0)
    assert abs(n.mem_info()[0] - free_after) < (256 << 20)  # the refused solver allocated nothing


def test_gpu_equals_cpu_bitwise(h3d, gpu):
    sg, rg = _solve(h3d, 41, 1e-4)
    sc, rc = _solve(h3d, 41, 1e-4, backend="cpu")
    assert rg["conv_iter"] == rc["conv_iter"]
    assert np.array_equal(sg.gather(), sc.gather())


@pytest.mark.parametrize("vr,decomp", [(2, None), (4, None), (8, None), (8, (8, 1, 1)), (6, (1, 3, 2)),
                                       (8, (2, 2, 2))])
def test_virtual_ranks_bitwise(h3d, gpu, vr, decomp):
    s1, r1 = _solve(h3d, 37, 1e-4)
    sp, rp = _solve(h3d, 37, 1e-4, virtual_ranks=vr, decomp=decomp)
    assert rp["conv_iter"] == r1["conv_iter"]
    assert np.array_equal(s1.gather(), sp.gather())


@pytest.mark.parametrize("graph,overlap", [(False, False), (False, True), (True, False), (True, True)])
def test_schedules_bitwise(h3d, gpu, graph, overlap):
    base, rb = _solve(h3d, 45, 1e-4, virtual_ranks=4, graph=False, overlap=False, check_every=1)
    s, r = _solve(h3d, 45, 1e-4, virtual_ranks=4, graph=graph, overlap=overlap, check_every=7,
                  graph_chunk=6, extra_args=["--stream-graphs", "on"])
    assert r["conv_iter"] == rb["conv_iter"]
    assert np.array_equal(s.gather(), base.gather())


@pytest.mark.parametrize("kernel", ["naive", "tile", "tile:2:4:2:4"])
def test_kernel_variants_solver(h3d, gpu, kernel):
    s, r = _solve(h3d, 64, 1e-3, kernel=kernel)
    assert r["conv_iter"] == 1915


def test_rccl_single_rank(h3d, gpu):
    """RcclComm with nranks = 1 (the installed RCCL refuses two ranks per GPU)."""
    ext = h3d.native()
    uid = ext.rccl_unique_id()
    assert len(uid) == 128
    s = ext.Solver(["33", "33", "33", "10000", "1e-5", "--backend", "hip"], rank=0, size=1, comm="rccl",
                   unique_id=uid, device=0)
    s.initialize()
    r = s.run()
    assert r["converged"] and r["conv_iter"] == 3590
    assert s.comm_name == "rccl"


def test_fp32_solver(h3d, gpu):
    sg, rg = _solve(h3d, 33, 1e-4, dtype="fp32")
    sc, rc = _solve(h3d, 33, 1e-4, dtype="fp32", backend="cpu")
    assert rg["conv_iter"] == rc["conv_iter"]
    assert np.array_equal(sg.gather(), sc.gather())
    it64 = _solve(h3d, 33, 1e-4)[1]["conv_iter"]
    assert abs(rg["conv_iter"] - it64) <= 5


def test_checkpoint_restart_gpu(h3d, gpu, tmp_path):
    full, rf = _solve(h3d, 31, 1e-4)
    a = h3d.HeatSolver((31, 31, 31), 500, 1e-4, backend="hip")
    a.run()
    a.save_checkpoint(str(tmp_path / "ck"))
    b = h3d.HeatSolver((31, 31, 31), 10 ** 6, 1e-4, backend="hip", virtual_ranks=4,
                       extra_args=["--restart", str(tmp_path / "ck")])
    rb = b.run()
    assert rb["conv_iter"] == rf["conv_iter"]
    assert np.array_equal(b.gather(), full.gather())


def test_nan_fault_detected(h3d, gpu):
    s = h3d.HeatSolver((21, 21, 21), 1000, 1e-9, backend="hip")
    s.initialize()
    s.native.inject(0, 5, 5, 5, float("nan"))
    r = s.run()
    assert r["fault"] and not r["converged"]


@pytest.mark.parametrize("n,eps,kernel2,dtype", [((33, 33, 33), 1e-5, "auto", "fp64"),
                                                 ((33, 33, 33), 3e-4, "auto", "fp64"),
                                                 ((33, 33, 33), 2.9e-4, "auto", "fp64"),
                                                 ((33, 33, 33), 2.8e-4, "auto", "fp64"),
                                                 ((65, 47, 130), 1e-4, "tl3:1:3:1:16:0:3:2", "fp64"),
                                                 ((65, 47, 130), 1e-4, "tl3:2:4:1:8:0:3:2", "fp64"),
                                                 ((64, 64, 64), 1e-4, "auto", "fp32"),
                                                 ((67, 45, 131), 1e-4, "vr3", "fp64"),
                                                 ((40, 44, 48), 3e-4, "vr2x2", "fp64"),
                                                 ((67, 45, 131), 1e-4, "vr3-nolag", "fp32")])
def test_monotone_check_bitwise(h3d, gpu, n, eps, kernel2, dtype):
    """Full sweeps after iteration 0 compute only their last step's residual
    (kResidualLastOnly; the FTCS residual max-norm never grows) and the sweep
    that converges is replayed with all of them (Solver::resolve_coarse): the
    same stopping iteration, last residual, norm and field, bit for bit, as
    every step's residual (--no-monotone-check), wherever in its sweep the
    converged step falls."""
    # vr*: virtual ranks (overlapped slabs / blocks: the check kernel after the
    # all-reduce, interior last-residual-only, boundary slabs every residual)
    if kernel2.startswith("vr"):
        decomp = {"vr3": (3, 1, 1), "vr2x2": (1, 2, 2), "vr3-nolag": (3, 1, 1)}[kernel2]
        extra = ["--lag", "off"] if kernel2.endswith("nolag") else []
        kw = dict(backend="hip", dtype=dtype, virtual_ranks=decomp[0] * decomp[1] * decomp[2], decomp=decomp,
                  extra_args=extra)
    else:
        kw = dict(backend="hip", dtype=dtype, extra_args=["--kernel2", kernel2])
    a = h3d.HeatSolver(n, 10 ** 6, eps, **kw)
    b = h3d.HeatSolver(n, 10 ** 6, eps, **dict(kw, extra_args=kw["extra_args"] + ["--no-monotone-check"]))
    a.initialize()
    b.initialize()
    assert a.native.monotone_check and not b.native.monotone_check
    ra, rb = a.run(), b.run()
    assert ra["converged"] and ra["conv_iter"] == rb["conv_iter"], (ra, rb)
    assert ra["last_residual"] == rb["last_residual"] and ra["norm"] == rb["norm"]
    assert np.array_equal(a.gather(), b.gather())
    # step() callers read the resolved iteration through state() too.  (Their
    # field is T at the end of the converging sweep, which depends on how the
    # steps were cut into sweeps: the start-up timing of the two solvers may
    # choose different remainder sweeps, so it is not compared here.)
    for s in (a, b):
        s.initialize()
        s.step(ra["conv_iter"] + 7)
        s.synchronize()
    sa, sb = a.state(), b.state()
    assert sa["conv_iter"] == sb["conv_iter"] == ra["conv_iter"] and sa["done"] == sb["done"] == 1, (sa, sb)
    assert sa["last_residual"] == sb["last_residual"] and sa["iter"] == sb["iter"]


@pytest.mark.parametrize("chunk", [5, 4, 7])
@pytest.mark.parametrize("vr", [1, 3])
def test_monotone_check_partial_and_long_sweeps(h3d, gpu, chunk, vr):
    """step() in chunks that are not multiples of K = 3 ends every chunk in a
    partial sweep or runs long (K+1) ones (the remainder policy): those run
    their last-residual variants too, and a convergence inside one resolves to
    the every-step iteration.  Several thresholds move the converged step
    through the sweeps of the chunks."""
    kw = dict(backend="hip", virtual_ranks=vr, decomp=(vr, 1, 1))
    for eps in (3e-4, 2.9e-4, 2.8e-4, 2.7e-4, 2.6e-4):
        out = []
        for extra in ([], ["--no-monotone-check"]):
            s = h3d.HeatSolver((33, 33, 33), 10 ** 6, eps, extra_args=extra, **kw)
            s.initialize()
            while True:
                s.step(chunk)
                s.synchronize()
                st = s.state()
                if st["done"]:
                    break
            out.append(st)
        a, b = out
        assert a["conv_iter"] == b["conv_iter"] and a["last_residual"] == b["last_residual"], (eps, a, b)
        assert a["fault"] == b["fault"] == 0


def test_monotone_check_nan_fault_iteration(h3d, gpu):
    """A NaN that appears inside a last-residual-only sweep is attributed to
    the iteration the every-step check names (the replay finds it)."""
    res = []
    for extra in ([], ["--no-monotone-check"]):
        s = h3d.HeatSolver((21, 21, 21), 1000, 1e-9, backend="hip", extra_args=extra)
        s.initialize()
        s.step(12)
        s.synchronize()
        s.native.inject(0, 5, 5, 5, float("nan"))
        res.append(s.run())
    assert res[0]["fault"] and res[1]["fault"] and res[0]["conv_iter"] == res[1]["conv_iter"], res


@pytest.mark.parametrize("vr", [1, 2])
def test_schedule_autotune_bitwise(h3d, gpu, vr):
    """Start-up timing of the interior sweeps' x schedules (Solver::tune_schedules,
    hip::tune_x_schedule): the candidates write the next buffer without residual
    state, the chosen schedule is kept per kernel and box, and the run is bitwise
    the run with the dispatch model's schedule (--no-autotune)."""
    n, iters = (200, 67, 131), 61
    kw = dict(virtual_ranks=vr, decomp=(vr, 1, 1)) if vr > 1 else {}
    # auto tunes single-subdomain runs only; "on" forces it for the slabs too
    a = h3d.HeatSolver(n, iters, 0.0, backend="hip", extra_args=["--autotune", "on" if vr > 1 else "auto"], **kw)
    b = h3d.HeatSolver(n, iters, 0.0, backend="hip", extra_args=["--no-autotune"], **kw)
    ra, rb = a.run(), b.run()
    assert ra["iterations"] == rb["iterations"] == iters and ra["last_residual"] == rb["last_residual"]
    assert np.array_equal(a.gather(), b.gather())
    tuned = h3d.native().tuned_schedules()
    # one domain: the 198 interior planes of the 200-point grid; slabs: the
    # interior of a 99-plane share (the K = 3 planes at the neighbour face are
    # boundary slabs)
    mine = [t for t in tuned if t["kernel"] == "tl-fp64" and (t["nx"] == 198 if vr == 1 else 90 <= t["nx"] <= 99)]
    assert mine, tuned
    for t in mine:
        assert t["candidates"] >= 2 and t["ms"] > 0 and t["ms"] <= t["ms_model"] + 1e-9, t
        assert t["L"] == -3 or t["L"] > 0, t


@pytest.mark.parametrize("n,eps,kernel2,dtype", [((33, 33, 33), 1e-5, "auto", "fp64"),
                                                 ((65, 47, 130), 1e-4, "tl3:2", "fp64"),
                                                 ((64, 64, 64), 1e-4, "auto", "fp32"),
                                                 ((40, 40, 40), 1e-3, "tl4", "fp64")])
def test_fused_check_bitwise(h3d, gpu, n, eps, kernel2, dtype):
    """Single-subdomain sweeps check convergence in their last workgroup
    (StencilParams::fuse_check) instead of a check kernel after them: the same
    stopping iteration, residual history and field, bit for bit, as the
    separate check (--no-fused-check); also a converged run's remaining
    sweeps (no-ops whose workgroups still take their tickets) keep counting."""
    kw = dict(backend="hip", dtype=dtype, extra_args=["--kernel2", kernel2])
    a = h3d.HeatSolver(n, 10 ** 6, eps, **kw)
    b = h3d.HeatSolver(n, 10 ** 6, eps, **dict(kw, extra_args=kw["extra_args"] + ["--no-fused-check"]))
    ra, rb = a.run(), b.run()
    assert ra["converged"] and ra["conv_iter"] == rb["conv_iter"], (ra, rb)
    assert ra["last_residual"] == rb["last_residual"] and ra["norm"] == rb["norm"]
    assert np.array_equal(a.gather(), b.gather())
    # past convergence: more (no-op) sweeps still advance the check count alike
    i0 = a.state()["iter"]
    for s in (a, b):
        s.step(30)
        s.synchronize()
    sa, sb = a.state(), b.state()
    assert sa["iter"] == sb["iter"] >= i0 + 30 and sa["conv_iter"] == sb["conv_iter"] == ra["conv_iter"], (sa, sb)
    assert sa["done"] == sb["done"] == 1 and sa["fault"] == sb["fault"] == 0
