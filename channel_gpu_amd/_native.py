"""Loader for the native core (``channel_gpu_amd._C``).

``torch`` is imported first so that its bundled HIP runtime (libamdhip64.so.7) and RCCL are the
ones the native core binds to (same SONAMEs).  On a machine with a GPU a missing extension is an
error, never a silent fallback: every GPU path in this package runs the hand-written HIP kernels.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the native import)

_ERR: Exception | None = None
try:
    C = importlib.import_module("channel_gpu_amd._C")
except Exception as e:  # pragma: no cover - exercised only when the build is missing
    C = None
    _ERR = e


def native_available() -> bool:
    return C is not None


def require_native():
    """Return the native module or raise with build instructions."""
    if C is None:
        raise RuntimeError(
            "channel_gpu_amd native core is not built or failed to load "
            f"({_ERR!r}); run `python tools/build.py` (gfx950, in-tree)"
        )
    return C


def native_path() -> str | None:
    return None if C is None else os.path.abspath(C.__file__)
