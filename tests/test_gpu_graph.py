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
    """The safety net of the per-stream graphs in steady state: a device-side
    cross-stream wait that outlasts --watchdog gives up, sets fault = 2 and
    the done flag (later sweeps are no-ops) instead of holding the GPU, and
    synchronize() raises.  A phantom rank whose emulated halo takes ~3 s (a
    link of 4e-5 GB/s) makes the compute stream's wait for the boundary slabs
    exceed a 0.5 s watchdog.  (--graph-canary 0: no start-up canary, which
    would have turned the graphs off.)"""
    import time

    s = h3d.HeatSolver((64, 64, 64), 1 << 40, 0.0, backend="hip", device=0, decomp=(8, 1, 1), phantom=(1, 8),
                       graph_chunk=6,
                       extra_args=["--phantom-gbps", "4e-5", "--phantom-allreduce-us", "1", "--watchdog", "0.5",
                                   "--long-sweeps", "off", "--lag", "off", "--graph-canary", "0", "--stream-graphs", "on"])
    s.initialize()
    assert s.native.stream_graphs_state == "unverified"
    g0 = s.native.graph_launches
    t0 = time.perf_counter()
    s.step(6)   # one graph of two sweeps: the second interior waits for the first boundary slabs
    with pytest.raises(RuntimeError, match="timed out"):
        s.synchronize()
    el = time.perf_counter() - t0
    assert s.native.graph_launches - g0 == 1
    st = s.state()
    assert st["fault"] == 2 and st["done"] == 1, st
    assert el < 60, el   # the two emulated halos (~3 s each) end, nothing waits for ever


def test_stream_graph_canary_falls_back_to_eager(h3d, gpu):
    """The start-up canary: a per-stream graph replay whose device-side wait
    outlasts --graph-canary (an emulated halo of ~0.6 s against 0.2 s) turns
    the graphs off in the same process; the solver re-initialises and the run
    continues eagerly and correctly — no hang, no fault, no graph launch."""
    import time

    args = ["--phantom-gbps", "2e-4", "--phantom-allreduce-us", "1", "--long-sweeps", "off", "--lag", "off"]
    t0 = time.perf_counter()
    s = h3d.HeatSolver((64, 64, 64), 1 << 40, 0.0, backend="hip", device=0, decomp=(8, 1, 1), phantom=(1, 8),
                       graph_chunk=6, extra_args=args + ["--graph-canary", "0.2", "--stream-graphs", "on"])
    s.initialize()
    el = time.perf_counter() - t0
    assert s.native.stream_graphs_state == "fallback", s.native.stream_graphs_note
    assert "timed out" in s.native.stream_graphs_note
    assert el < 60, el
    st = s.state()
    assert st["iter"] == 0 and st["fault"] == 0 and st["done"] == 0, st
    g0 = s.native.graph_launches
    s.step(6)
    s.synchronize()
    assert s.native.graph_launches == g0
    st = s.state()
    assert st["iter"] == 6 and st["fault"] == 0 and st["done"] == 0, st
    # the same steps with graphs off from the start: the same field
    e = h3d.HeatSolver((64, 64, 64), 1 << 40, 0.0, backend="hip", device=0, decomp=(8, 1, 1), phantom=(1, 8),
                       graph_chunk=6, extra_args=args + ["--no-stream-graphs"])
    e.initialize()
    assert e.native.stream_graphs_state == "off"
    e.step(6)
    e.synchronize()
    import numpy as np

    assert np.array_equal(s.local_field(0, True), e.local_field(0, True))


def test_stream_graph_canary_passes(h3d, gpu):
    """A healthy phantom rank: the canary replays, keeps the graphs, and the
    timed steps replay them; the field after the canary is the initial one."""
    import numpy as np

    args = ["--phantom-gbps", "50", "--long-sweeps", "off"]
    s = h3d.HeatSolver((96, 96, 96), 1 << 40, 0.0, backend="hip", device=0, decomp=(8, 1, 1), phantom=(2, 8),
                       extra_args=args + ["--stream-graphs", "on"])
    s.initialize()
    assert s.native.stream_graphs_state == "on", s.native.stream_graphs_note
    assert "graphs" in s.native.stream_graphs_note and "eager" in s.native.stream_graphs_note
    st = s.state()
    assert st["iter"] == 0 and st["fault"] == 0, st
    g0 = s.native.graph_launches
    s.step(36)
    s.synchronize()
    assert s.native.graph_launches > g0
    e = h3d.HeatSolver((96, 96, 96), 1 << 40, 0.0, backend="hip", device=0, decomp=(8, 1, 1), phantom=(2, 8),
                       extra_args=args + ["--no-graph"])
    e.initialize()
    e.step(36)
    e.synchronize()
    assert np.array_equal(s.local_field(0, True), e.local_field(0, True))


def test_stream_graphs_auto_is_eager(h3d, gpu):
    """--stream-graphs auto replays the overlapped multi-rank schedule eagerly
    (measured faster on the 8-GPU share: Solver::stream_graphs_enabled); the
    single-stream schedule keeps its graph."""
    s = h3d.HeatSolver((96, 96, 96), 1 << 40, 0.0, backend="hip", device=0, decomp=(8, 1, 1), phantom=(2, 8),
                       extra_args=["--phantom-gbps", "50"])
    s.initialize()
    assert s.native.stream_graphs_state == "off", s.native.stream_graphs_note
    g0 = s.native.graph_launches
    s.step(36)
    s.synchronize()
    assert s.native.graph_launches == g0
    one = h3d.HeatSolver((96, 96, 96), 1 << 40, 0.0, backend="hip", device=0)
    one.initialize()
    assert one.native.stream_graphs_state == "n/a"
    one.step(36)
    one.synchronize()
    assert one.native.graph_launches > 0
