"""Loaders for the native core.

* ``require_core()`` -> ``channel_gpu_amd._core``: Solver, config, plan, I/O, bootstrap (no torch).
* ``require_native()`` -> ``channel_gpu_amd._C``: everything in _core plus the torch-tensor entry
  points of every kernel (tests, experiments).

One HIP runtime per process.  By default torch is imported before the native core, so the core
binds to torch's bundled HIP runtime and RCCL (same SONAMEs: libamdhip64.so.7, librccl.so.1) and
torch tensors can share the device with the solver.  With ``CHANNEL_TORCH_FREE=1`` (bench.py, the
Python driver) torch is never imported: the core runs on /opt/rocm's HIP runtime and RCCL, exactly
like the C++ driver binary, and ``require_native()`` refuses.  On a machine with a GPU a missing
extension is an error, never a silent fallback: every GPU path runs the hand-written HIP kernels.
"""
from __future__ import annotations

import importlib
import os

_core = None
_C = None
_ERR: Exception | None = None


def torch_free() -> bool:
    return os.environ.get("CHANNEL_TORCH_FREE", "0") == "1"


def _load(name: str):
    global _ERR
    try:
        return importlib.import_module(f"channel_gpu_amd.{name}")
    except Exception as e:  # pragma: no cover - exercised only when the build is missing
        _ERR = e
        return None


def require_core():
    """The torch-free native module (imports torch first unless CHANNEL_TORCH_FREE=1)."""
    global _core
    if _core is None:
        if not torch_free():
            import torch  # noqa: F401  (bind the core to torch's HIP runtime)
        _core = _load("_core")
        if _core is None:
            raise RuntimeError(
                "channel_gpu_amd native core is not built or failed to load "
                f"({_ERR!r}); run `python tools/build.py` (gfx950, in-tree)")
    return _core


def require_native():
    """The torch extension (every kernel with tensor entry points + all of _core)."""
    global _C
    if _C is None:
        if torch_free():
            raise RuntimeError("CHANNEL_TORCH_FREE=1: this process runs without torch; use require_core()")
        import torch  # noqa: F401  (must precede the native import)

        _C = _load("_C")
        if _C is None:
            raise RuntimeError(
                "channel_gpu_amd native core is not built or failed to load "
                f"({_ERR!r}); run `python tools/build.py` (gfx950, in-tree)")
    return _C


def native_available() -> bool:
    try:
        require_core()
        return True
    except RuntimeError:
        return False


def native_path() -> str | None:
    try:
        return os.path.abspath(require_core().__file__)
    except RuntimeError:
        return None
