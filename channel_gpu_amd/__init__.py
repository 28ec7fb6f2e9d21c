"""channel_gpu_amd — MI355X-native spectral DNS of incompressible turbulent channel flow.

Kim-Moin-Moser phi/omega_y formulation, Fourier (x, z) x compact finite differences (y), SMR RK3
with implicit viscous terms and constant flow rate: the capabilities of Nasrollah/CHANNEL_GPU,
re-designed for gfx950 (hand-written HIP kernels, RCCL all-to-all over xGMI, hipGraph per step).

Layout of the package
  models/     flow set-ups (turbulent channel, laminar Poiseuille, Orr-Sommerfeld mode)
  ops/        thin wrappers over every HIP kernel (tests, experiments)
  parallel/   decomposition math and the torch.distributed -> RCCL bootstrap
  utils/      config, restart/statistics file I/O, timing
  reference/  NumPy fp64 oracle solver (the CPU reference path)
"""
from __future__ import annotations

import torch  # noqa: F401  (load torch's HIP runtime before the native core)

from ._native import native_available, native_path, require_native
from .utils.config import default_config, load_config

__all__ = ["native_available", "native_path", "require_native", "load_config", "default_config", "ChannelFlow"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "ChannelFlow":
        from .models.channel import ChannelFlow

        return ChannelFlow
    raise AttributeError(name)
