"""hipGraphs of every schedule (BASELINE config 5: "hipGraph-captured iteration").

Stream capture of the overlapped three-stream schedule overflowed the host
stack inside hipStreamEndCapture; the backend now builds graphs explicitly
(csrc/runtime/hip_backend.cpp).  Each case runs the same solve eagerly and as
graph replays in a subprocess (a runtime crash must surface as a failed exit
code, not take the test runner down) and requires bitwise-equal fields,
the same iteration count and graph launches actually made.
``tools/graph_capture_repro.hip`` holds the minimal capture patterns (side
streams waiting on each other, the origin waiting mid-capture) that the HIP
runtime handles; they run here too and must exit cleanly.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

PROBE = os.path.join(ROOT, "tools", "graph_multistream_probe.py")


@pytest.mark.parametrize("args", [
    ["--n", "96", "--ranks", "8", "--decomp", "8x1x1"],             # overlapped x slabs, lagged check
    ["--n", "96", "--ranks", "8", "--decomp", "2x2x2"],             # blocks: 3 halo phases
    ["--n", "80", "--ranks", "4", "--decomp", "4x1x1", "--dtype", "fp32"],
    ["--n", "256", "--decomp", "8x1x1", "--phantom", "1/8"],         # one rank of 8, emulated RCCL
    ["--n", "200", "--decomp", "2x2x2", "--phantom", "5/8"],
    ["--n", "128", "--ranks", "1", "--decomp", "1x1x1"],             # single stream
], ids=["slab8", "block8", "slab4-fp32", "phantom-slab", "phantom-block", "single"])
def test_graph_bitwise_vs_eager(gpu, args):
    p = subprocess.run([sys.executable, PROBE, "--steps", "72"] + args, capture_output=True, text=True,
                       timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert "bitwise_equal: True graph_used: True" in p.stdout


def test_capture_patterns_exit_cleanly(gpu):
    exe = os.path.join(ROOT, "build", "graph_capture_repro")  # built by __graft_entry__.build()
    assert os.path.exists(exe), exe
    p = subprocess.run([exe, "4"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count(" ok") == 4 and "done, 0 wrong" in p.stdout


def test_short_bench_replays_graph(h3d, gpu):
    """The driver's short run (20 steps after 5 warm-up) replays a graph sized
    to the step count, captured before the timed region (prepare_steps)."""
    s = h3d.HeatSolver((130, 130, 130), 1 << 40, 0.0, backend="hip", device=0)
    s.initialize()
    s.step(5)
    s.prepare_steps(20)
    g0 = s.native.graph_launches
    s.step(20)
    s.synchronize()
    assert s.native.graph_launches - g0 == 1
    assert s.state()["iter"] == 25


def test_stream_graph_wait_timeout_flags_fault(h3d, gpu):
    """The safety net of the per-stream graphs: a device-side cross-stream
    wait that outlasts --watchdog gives up, sets fault = 2 and the done flag
    (later sweeps are no-ops) instead of holding the GPU.  A phantom rank
    whose emulated halo takes ~3 s (a link of 4e-5 GB/s) makes the compute
    stream's wait for the boundary slabs exceed a 0.5 s watchdog."""
    import time

    s = h3d.HeatSolver((64, 64, 64), 1 << 40, 0.0, backend="hip", device=0, decomp=(8, 1, 1), phantom=(1, 8),
                       graph_chunk=6,
                       extra_args=["--phantom-gbps", "4e-5", "--phantom-allreduce-us", "1", "--watchdog", "0.5",
                                   "--long-sweeps", "off"])
    s.initialize()
    g0 = s.native.graph_launches
    t0 = time.perf_counter()
    s.step(6)   # one graph of two sweeps: the second interior waits for the first boundary slabs
    s.synchronize()
    el = time.perf_counter() - t0
    assert s.native.graph_launches - g0 == 1
    st = s.state()
    assert st["fault"] == 2 and st["done"] == 1, st
    assert el < 60, el   # the two emulated halos (~3 s each) end, nothing waits for ever
