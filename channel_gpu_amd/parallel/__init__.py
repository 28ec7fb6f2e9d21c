"""Decomposition math, the native (torch-free) rank bootstrap and the torch.distributed -> RCCL
bootstrap.

The torch.distributed helpers (``dist_info``, ``nccl_unique_id``: ``parallel/bootstrap.py``) load on
first use: importing this package must not import torch, or a torch-free process (bench.py, the
drivers) would bind torch's bundled HIP runtime and RCCL (same sonames as /opt/rocm's) before the
native core loads.
"""
from .decomposition import SlabDecomposition, balanced_split  # noqa: F401


def __getattr__(name: str):
    if name in ("dist_info", "nccl_unique_id"):
        from . import bootstrap

        return getattr(bootstrap, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
