"""Loader for the native extension ``_heat3d`` (built in-tree by CMake).

The extension links ``libamdhip64.so.7`` / ``librccl.so.1`` / ``libgomp.so.1``
by soname (RUNPATH /opt/rocm/lib).  PyTorch-ROCm bundles its own copies of the
HIP runtime (7.0) and RCCL (2.26) under the same sonames, and the dynamic
linker reuses whichever copy is loaded first.  Which runtime a process runs on
is chosen here, once, before anything touches the GPU:

* ``HEAT3D_RUNTIME=rocm`` (bench.py's ranks, ``__graft_entry__.smoke()``):
  torch is never imported; the extension binds /opt/rocm's HIP 7.2 / RCCL
  2.27, the runtime of the native CLI ``build/heat3d``.  Importing torch
  before the package in such a process is an error (it would have bound
  torch's copies); importing it afterwards would load a second runtime, so
  these processes use :class:`heat3d_amd.parallel.distributed.HostGroup`
  instead of torch.distributed.
* default (the test suite, which uses torch as its numerics oracle): torch
  is imported *first*, the extension binds torch's already-loaded runtime,
  and the process still has exactly one HIP runtime and one RCCL.

``runtime()`` reports the versions and files actually bound.

On a machine with a GPU the extension must be present: every op fails loudly
instead of silently falling back to a slower path.
"""
from __future__ import annotations

import importlib
import os

_ext = None
_err: Exception | None = None

import sys

RUNTIME = os.environ.get("HEAT3D_RUNTIME", "auto").lower()
if RUNTIME not in ("auto", "torch", "rocm"):
    raise RuntimeError(f"HEAT3D_RUNTIME={RUNTIME!r}: expected rocm, torch or auto")
if RUNTIME == "rocm":
    if "torch" in sys.modules:
        raise RuntimeError("HEAT3D_RUNTIME=rocm but torch is already imported: the extension would bind torch's "
                           "bundled HIP runtime / RCCL; import heat3d_amd before torch, or not torch at all")
else:
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


def runtime() -> dict:
    """The HIP runtime / RCCL this process is bound to (versions, library files),
    the runtime policy and whether torch is loaded."""
    d = dict(native().runtime_info())
    d["policy"] = RUNTIME
    d["torch_loaded"] = "torch" in sys.modules
    return d


def gpu_available() -> bool:
    """True when a HIP device is visible (does not initialise torch.cuda)."""
    return available() and native().device_count() > 0
