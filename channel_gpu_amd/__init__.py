"""channel_gpu_amd — MI355X-native spectral DNS of incompressible turbulent channel flow.

Kim-Moin-Moser phi/omega_y formulation, Fourier (x, z) x compact finite differences (y), SMR RK3
with implicit viscous terms and constant flow rate: the capabilities of Nasrollah/CHANNEL_GPU,
re-designed for gfx950 (hand-written HIP kernels, RCCL all-to-all over xGMI, hipGraph per step).

Layout of the package
  _core       torch-free native bindings (Solver, config, plan, HDF5 I/O, bootstrap, communicators)
  _C          torch extension: _core plus tensor entry points of every HIP kernel (tests)
  models/     ChannelFlow (high-level run object), Orr-Sommerfeld eigen-solver and TS modes
  parallel/   decomposition math; native (TCP) and torch.distributed bootstraps of RCCL
  utils/      run.conf loading and BASELINE presets
  reference/  NumPy fp64 oracle solver (the CPU reference path)
  driver.py   python -m channel_gpu_amd.driver run.conf (torchrun-launchable, torch-free ranks)
"""
from __future__ import annotations

from ._native import native_available, native_path, require_core, require_native, torch_free
from .utils.config import default_config, load_config

__all__ = ["native_available", "native_path", "require_core", "require_native", "torch_free", "load_config",
           "default_config", "ChannelFlow"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "ChannelFlow":
        from .models.channel import ChannelFlow

        return ChannelFlow
    raise AttributeError(name)
