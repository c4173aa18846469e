"""Torch-free multi-process bootstrap (bench.py's ranks): the native HostGroup
carries the socket transport's address table, barriers, object all-gathers and
the max over ranks; the ranks never import torch, and the solve is bitwise
equal to the single-process one."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import free_port

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world,decomp", [(2, "2x1x1"), (4, "2x2x1")])
def test_hostgroup_socket_job_is_torch_free(h3d, tmp_path, world, decomp):
    n, eps = 23, 1e-4
    port, hport = free_port(), free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HEAT3D_HOSTGROUP_PORT=str(hport), HEAT3D_RUNTIME="rocm")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_hostgroup_worker.py"), str(tmp_path),
                                       str(n), str(eps), decomp], env=env))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0] * world, rcs
    res = json.loads((tmp_path / "result.json").read_text())
    assert res["objs"] == [{"rank": r, "iter": res["iter"]} for r in range(world)]
    assert res["max"] == world - 1
    single = h3d.HeatSolver((n, n, n), 10 ** 6, eps, backend="cpu", extra_args=["--temporal", "1"])
    r1 = single.run()
    assert res["iter"] == r1["conv_iter"]
    assert np.array_equal(np.load(tmp_path / "field.npy"), single.gather())


def test_runtime_policy_refuses_torch_first(tmp_path):
    """HEAT3D_RUNTIME=rocm after torch was imported must fail loudly (the
    extension would bind torch's bundled HIP runtime)."""
    code = ("import sys; sys.path.insert(0, %r); import torch, os; os.environ['HEAT3D_RUNTIME'] = 'rocm'\n"
            "try:\n    import heat3d_amd\nexcept RuntimeError as e:\n    print('refused:', e); sys.exit(0)\n"
            "sys.exit(1)") % os.path.dirname(HERE)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "refused" in r.stdout, (r.stdout, r.stderr)


def test_single_process_collectives_do_not_import_torch():
    """bench.py at N = 1 calls the host collectives with no group: they must
    not import torch (round 6: a barrier that did cost ~1.4 s right before the
    timed window and loaded torch's second HIP runtime into the process)."""
    code = ("import sys, os; sys.path.insert(0, %r); os.environ['HEAT3D_RUNTIME'] = 'rocm'\n"
            "import heat3d_amd\n"
            "from heat3d_amd.parallel.distributed import barrier, all_gather_objects, max_over_ranks\n"
            "barrier(None); assert all_gather_objects({'a': 1}, None) == [{'a': 1}]; assert max_over_ranks(2.0) == 2.0\n"
            "assert 'torch' not in sys.modules, sorted(m for m in sys.modules if m.startswith('torch'))[:5]\n"
            "print('ok')") % os.path.dirname(HERE)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout, r.stderr)
