"""Loader for the native extension ``_heat3d`` (built in-tree by CMake).

The extension links ``libamdhip64.so.7`` / ``librccl.so.1`` / ``libgomp.so.1``
by soname.  PyTorch-ROCm bundles its own copies of those libraries, so torch is
imported *first*: the extension then binds to the already-loaded runtime and
the process has exactly one HIP runtime and one RCCL.

On a machine with a GPU the extension must be present: every op fails loudly
instead of silently falling back to a slower path.
"""
from __future__ import annotations

import importlib
import os

_ext = None
_err: Exception | None = None

try:  # one HIP runtime per process: torch's, loaded before the extension
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None


def _load():
    global _ext, _err
    if _ext is not None or _err is not None:
        return
    try:
        _ext = importlib.import_module(__package__ + "._heat3d")
    except Exception as e:  # pragma: no cover - exercised when unbuilt
        _err = e


def available() -> bool:
    _load()
    return _ext is not None


def native():
    """Return the extension module or raise with build instructions."""
    _load()
    if _ext is None:
        raise RuntimeError(
            "heat3d native extension is not built (%s). Run `python -c 'import __graft_entry__ as g; "
            "g.build()'` or `cmake -S . -B build -G Ninja && ninja -C build` at the repo root." % _err
        )
    return _ext


def extension_path() -> str:
    return os.path.abspath(native().__file__)


def gpu_available() -> bool:
    """True when a HIP device is visible (does not initialise torch.cuda)."""
    return available() and native().device_count() > 0
