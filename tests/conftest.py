import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BIN = os.path.join(ROOT, "build", "heat3d")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built():
    import heat3d_amd

    if not heat3d_amd.native_available() or not os.path.exists(BIN):
        import __graft_entry__

        __graft_entry__.build()


@pytest.fixture(scope="session")
def h3d():
    _ensure_built()
    import heat3d_amd

    return heat3d_amd


@pytest.fixture(scope="session")
def ext(h3d):
    return h3d.native()


@pytest.fixture(scope="session")
def heat3d_bin(h3d):
    assert os.path.exists(BIN), "CLI binary not built"
    return BIN


@pytest.fixture(scope="session")
def gpu(ext):
    if ext.device_count() < 1:
        pytest.fail("GPU test requested but no HIP device is visible")
    import torch

    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def run_cli(args, cwd, env=None, timeout=600):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    if env:
        e.update(env)
    return subprocess.run([BIN] + [str(a) for a in args], cwd=cwd, env=e, capture_output=True,
                          text=True, timeout=timeout)


def free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
