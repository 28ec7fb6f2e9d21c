"""High-level channel-flow DNS object (one per rank / GPU).

Wraps the C++ ``Solver`` (csrc/core/solver.cpp): state, RK3 stepping (one hipGraph per step),
reference-compatible logging/statistics files and HDF5 restarts, plus the time-averaged
turbulence statistics in wall units (``TurbulenceStatistics``).  Mirrors the reference driver
(main.c:10-150): config -> device -> setUp -> IC (random / file) -> RKstep -> writeData.

Bootstrap: inside an initialised torch.distributed job the torch control plane hands out the
RCCL id (``parallel.bootstrap``); otherwise the torch-free native TCP rendezvous does
(``parallel.native_bootstrap``), which is what the driver and bench.py use.
"""
from __future__ import annotations

import sys

import numpy as np

from .._native import require_core
from ..utils.config import default_config, load_config
from .statistics import TurbulenceStatistics


def _torch_dist_initialized() -> bool:
    d = sys.modules.get("torch.distributed")
    return bool(d is not None and d.is_available() and d.is_initialized())


class ChannelFlow:
    def __init__(self, config=None, *, device: int | None = None, **overrides):
        C = require_core()
        if config is None:
            cfg = default_config(**overrides)
        elif isinstance(config, str):
            cfg = load_config(config, [f"{k}={v}" for k, v in overrides.items()])
        else:
            cfg = config
            for k, v in overrides.items():
                setattr(cfg, k, v)
            cfg.validate()
        if _torch_dist_initialized():
            import torch

            from ..parallel.bootstrap import dist_info, nccl_unique_id

            rank, world, local = dist_info()
            if device is None:
                device = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(device)
            uid = nccl_unique_id()
        else:
            from ..parallel.native_bootstrap import init_native

            ri = init_native()
            rank, world, uid = ri.rank, ri.world, ri.uid
            device = ri.device if device is None else device
        if C.device_count() < 1:
            raise RuntimeError("ChannelFlow needs an MI355X GPU; use channel_gpu_amd.reference for the CPU path")
        self.rank, self.world, self.device = rank, world, device
        self.solver = C.Solver(cfg, rank, world, device, uid)
        self.cfg = cfg
        self.statistics = TurbulenceStatistics(np.asarray(self.solver.grid.y), 1.0 / cfg.Re)

    # ---- setup -----------------------------------------------------------------------------
    @property
    def plan(self):
        return self.solver.plan

    @property
    def y(self) -> np.ndarray:
        return np.asarray(self.solver.grid.y)

    def initialize(self):
        c = self.cfg
        if c.ic == "file":
            self.solver.read_restart(c.in_G, c.in_DDV, c.in_UMEAN)
        else:
            self.solver.init_ic()
        self.solver.prepare()
        return self

    def set_state(self, phi, omega, U):
        self.solver.set_state(np.asarray(phi, complex), np.asarray(omega, complex), np.asarray(U, float))
        self.solver.prepare()

    def get_state(self):
        return self.solver.get_state()

    # ---- stepping ---------------------------------------------------------------------------
    def step(self, n: int = 1):
        for _ in range(n):
            self.solver.step(False)

    def run(self, nsteps: int | None = None, verbose: bool = True):
        self.solver.run(self.cfg.nsteps if nsteps is None else nsteps, verbose)

    def synchronize(self):
        self.solver.synchronize()

    def log(self):
        return self.solver.log()

    # ---- output ------------------------------------------------------------------------------
    def save(self, g: str, ddv: str, umean: str = "-"):
        self.solver.write_restart(g, ddv, umean)

    def load(self, g: str, ddv: str, umean: str = "-"):
        self.solver.read_restart(g, ddv, umean)
        self.solver.prepare()

    def mean_profile(self) -> np.ndarray:
        return np.asarray(self.solver.mean_profile())

    # ---- time-averaged statistics -------------------------------------------------------------
    def sample_statistics(self, nsteps: int, every: int = 10):
        """Advance ``nsteps`` steps, sampling U(y), the plane r.m.s. and <u'v'> (the reference's
        calcSt cadence, statistics.cu:161-243) every ``every`` steps into ``self.statistics``."""
        done = 0
        while done < nsteps:
            k = min(every, nsteps - done)
            for i in range(k):
                self.solver.step(i == k - 1)
            done += k
            if k == every:
                L = self.solver.log()
                self.statistics.add(np.asarray(self.solver.mean_profile()), np.asarray(self.solver.stats()), L.utau_lo,
                                    L.utau_hi, L.time)
        return self.statistics

    def grid_points(self) -> int:
        c = self.cfg
        return c.NX * c.NY * (2 * c.NZ - 2)
