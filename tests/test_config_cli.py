"""CLI contract (reference heat3D.cu:270-315, 1078-1106)."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT, free_port, run_cli

REF_OUT = "/root/reference/HeatEquation3D/output/out.dat"


def test_config_parse(ext):
    c = ext.config_parse(["27", "28", "29", "100", "1e-5", "--dtype", "fp32", "--decomp", "2x1x1"])
    assert tuple(c["n"]) == (27, 28, 29) and c["iter_max"] == 100 and c["eps"] == 1e-5
    assert c["dtype"] == "fp32" and tuple(c["decomp"]) == (2, 1, 1)
    for bad in (["27", "27", "27", "100"], ["a", "1", "1", "1", "1"], ["27"] * 3 + ["1", "x"],
                ["2", "27", "27", "1", "1"], ["27"] * 3 + ["1", "1", "--bogus"], ["27"] * 3 + ["1", "1", "--decomp", "2x2"]):
        with pytest.raises(ext.UsageError):
            ext.config_parse(bad)


def test_physics_constants(ext):
    p = ext.physics(27, 27, 27)
    assert p["h"][0] == 1.0 / 26.0
    # D = dt / h^2 = CFL / 6 = 1/15 on a cube
    assert all(abs(d - 1 / 15) < 1e-15 for d in p["D"])
    q = ext.physics(11, 21, 41)
    hmin = min(q["h"])
    assert abs(q["dt"] - 0.4 / 6 * hmin ** 2) < 1e-18


def test_banner_exact_bytes(heat3d_bin, tmp_path):
    r = run_cli(["27", "27", "27", "100", "1e-05", "--backend", "cpu", "--output", "none"], tmp_path)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")
    assert lines[0] == "Runnung HeatEquation3D with the following arguments: "
    assert lines[1] == f"executable:               {heat3d_bin}"
    assert lines[2:7] == ["number of cells in x:     27", "number of cells in y:     27",
                          "number of cells in z:     27", "max number of iterations: 100",
                          "convergence threshold:    1e-05"]
    assert lines[7] == ""
    assert lines[8].startswith("Computational time (parallel): ")
    assert len(lines[8].split(": ")[1].split(".")[1]) == 6
    assert lines[9] == ""
    assert lines[10] == "Simulation did not converge within 100 iterations."
    assert lines[11] == "L2-norm error: 26.0129 %"


def test_converged_report_and_output(heat3d_bin, tmp_path):
    r = run_cli(["27", "27", "27", "100000", "1e-5", "--backend", "cpu", "--json-out", "run.json"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "Simulation has converged in 2513 iterations with a convergence threshold of 1.000000e-05" in r.stdout
    assert "L2-norm error: 0.0192 %" in r.stdout
    out = (tmp_path / "output" / "out.dat").read_text().split("\n")
    ref = open(REF_OUT).read().split("\n")
    assert out[:3] == ref[:3]  # header byte-compatible with the shipped artifact
    assert len(out) == len(ref)
    # coordinate columns identical to the reference artifact (T differs: its run was broken)
    for a, b in zip(out[3:200], ref[3:200]):
        assert a[:45] == b[:45]
    j = json.loads((tmp_path / "run.json").read_text())
    assert j["conv_iter"] == 2513 and j["converged"] and j["backend"] == "cpu"


def test_usage_error_exit_code(heat3d_bin, tmp_path):
    r = run_cli(["27", "27"], tmp_path)
    assert r.returncode != 0
    assert "bin/HeatEquation3D NUM_CELLS_X NUM_CELLS_Y NUM_CELLS_Z ITER_MAX EPS" in r.stdout


def test_virtual_ranks_cli_ref_layout(heat3d_bin, tmp_path):
    # 27^3 on 8 virtual ranks: reference-legal -> 8 zones of 14^3 with a rank column
    r = run_cli(["27", "27", "27", "100000", "1e-4", "--backend", "cpu", "--virtual-ranks", "8"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "converged in 1725 iterations" in r.stdout
    lines = (tmp_path / "output" / "out.dat").read_text().split("\n")
    assert lines[1] == 'VARIABLES = "X", "Y", "Z", "T", "rank"'
    assert lines[2] == 'ZONE T = "0", I=14, J=14, K=14, F=POINT'
    assert lines[3 + 14 ** 3] == 'ZONE T = "1", I=14, J=14, K=14, F=POINT'
    assert lines[4].endswith("    0") and len(lines[4]) == 65


def test_compat_zone_titles(heat3d_bin, tmp_path):
    r = run_cli(["27", "27", "27", "10", "1e-4", "--backend", "cpu", "--virtual-ranks", "2", "--compat"], tmp_path)
    assert r.returncode == 0
    txt = (tmp_path / "output" / "out.dat").read_text()
    assert txt.count('ZONE T = "0"') == 2  # reference bug A14 reproduced under --compat


def test_cli_multiprocess_socket(heat3d_bin, tmp_path):
    """Two CLI processes (torchrun-style env) over the socket transport."""
    import subprocess

    port = free_port()
    env = {"WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
           "HEAT3D_BOOTSTRAP_PORT": str(port)}
    procs = []
    for r in range(2):
        e = dict(os.environ)
        e.update(env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r)})
        procs.append(subprocess.Popen([heat3d_bin, "27", "27", "27", "100000", "1e-4", "--backend", "cpu",
                                       "--threads", "2"], cwd=tmp_path, env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "converged in 1725 iterations" in outs[0][0]
    assert "comm=socket ranks=2" in outs[0][0]
    assert outs[1][0] == ""  # only rank 0 reports
    zones = (tmp_path / "output" / "out.dat").read_text().count("ZONE")
    assert zones == 2


@pytest.mark.parametrize("gpus,decomp,temporal", [(2, None, "0"), (4, "1x2x2", "0"), (3, None, "0"),
                                                   (2, None, "3"), (4, "2x2x1", "3")])
def test_threads_per_rank_cli(heat3d_bin, tmp_path, gpus, decomp, temporal):
    """--gpus N: N ranks in one process, one host thread each (the
    ncclCommInitAll-style runtime; TCP sockets between the threads on the CPU
    backend).  Same report and checkpoint as the single-rank run, also with
    K-step temporal blocking (x slabs and y/z blocks across threads)."""
    base = ["23", "23", "23", "100000", "1e-4", "--backend", "cpu", "--output", "none"]
    one = run_cli(base + ["--checkpoint-every", "64", "--checkpoint-dir", "c1", "--json-out", "a.json"], tmp_path)
    assert one.returncode == 0, one.stderr
    args = base + ["--gpus", str(gpus), "--checkpoint-every", "64", "--checkpoint-dir", "cn", "--json-out", "b.json",
                   "--temporal", temporal]
    if decomp:
        args += ["--decomp", decomp]
    many = run_cli(args, tmp_path, env={"HEAT3D_BOOTSTRAP_PORT": str(free_port())})
    assert many.returncode == 0, many.stderr
    a = json.loads((tmp_path / "a.json").read_text())
    b = json.loads((tmp_path / "b.json").read_text())
    assert b["ranks"] == gpus and b["comm"] == "socket"
    assert a["conv_iter"] == b["conv_iter"] and abs(a["error_percent"] - b["error_percent"]) < 1e-12
    assert many.stdout.count("Runnung HeatEquation3D") == 1  # one report per job, not per thread
    fa = json.loads((tmp_path / "c1" / "meta.json").read_text())["field"]
    fb = json.loads((tmp_path / "cn" / "meta.json").read_text())["field"]
    ra = np.fromfile(tmp_path / "c1" / fa, dtype=np.float64)
    rb = np.fromfile(tmp_path / "cn" / fb, dtype=np.float64)
    assert np.array_equal(ra, rb)


def test_threads_per_rank_needs_devices(heat3d_bin, tmp_path):
    r = run_cli(["23", "23", "23", "10", "1e-4", "--backend", "hip", "--gpus", "64"], tmp_path)
    assert r.returncode != 0


def test_schedule_flags(heat3d_bin, tmp_path):
    """--autotune auto|on|off and --no-autotune parse (round 3); a bad value
    is a usage error with a non-zero exit; --help lists the flag."""
    ok = run_cli(["27", "27", "27", "50", "0", "--backend", "cpu", "--autotune", "on", "--output", "none"], tmp_path)
    assert ok.returncode == 0, ok.stdout + ok.stderr
    ok = run_cli(["27", "27", "27", "50", "0", "--backend", "cpu", "--no-autotune", "--output", "none"], tmp_path)
    assert ok.returncode == 0, ok.stdout + ok.stderr
    bad = run_cli(["27", "27", "27", "50", "0", "--backend", "cpu", "--autotune", "sometimes"], tmp_path)
    assert bad.returncode != 0 and "--autotune auto|on|off" in (bad.stdout + bad.stderr)
    h = run_cli(["--help"], tmp_path)
    assert "--autotune auto|on|off" in h.stdout + h.stderr


def test_progress_heartbeat(heat3d_bin, tmp_path):
    """--progress S: run() prints a heartbeat to stderr (iteration, relative
    residual, eps, elapsed, GLUPS) at most every S seconds, so that long
    convergence runs stay visibly alive; stdout keeps the reference report."""
    r = run_cli(["33", "33", "33", "100000", "1e-5", "--backend", "cpu", "--output", "none",
                 "--progress", "0.001", "--check-every", "64"], tmp_path)
    assert r.returncode == 0, r.stderr
    beats = [l for l in r.stderr.splitlines() if l.startswith("heat3d: progress iteration")]
    assert beats, r.stderr[-2000:]
    its = [int(l.split()[3]) for l in beats]
    assert its == sorted(its) and its[-1] <= 3591
    assert "relative" in beats[0] and "(eps 1.000e-05)" in beats[0]
    assert "heat3d: progress" not in r.stdout
    assert "Simulation has converged in 3590 iterations" in r.stdout
    bad = run_cli(["33", "33", "33", "10", "1e-5", "--backend", "cpu", "--progress", "-1"], tmp_path)
    assert bad.returncode != 0


@pytest.mark.parametrize("gpus", [1, 3])
def test_time_limit(heat3d_bin, tmp_path, gpus):
    """--time-limit S: run() stops unconverged after about S seconds; the
    wall budget becomes one iteration cap agreed by every rank (min over the
    ranks' projections, one all-reduce), so the ranks stop at the same
    iteration and the job exits cleanly (3 ranks: socket transport)."""
    args = ["65", "65", "65", "100000000", "1e-12", "--backend", "cpu", "--output", "none", "--threads", "2",
            "--time-limit", "2", "--check-every", "16", "--json-out", "t.json"]
    if gpus > 1:
        args += ["--gpus", str(gpus)]
    r = run_cli(args, tmp_path, env={"HEAT3D_BOOTSTRAP_PORT": str(free_port())})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Simulation did not converge" in r.stdout
    j = json.loads((tmp_path / "t.json").read_text())
    assert not j["converged"] and 0 < j["seconds"] < 6, j
