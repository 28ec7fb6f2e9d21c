"""Run configuration (``run.conf``, libconfig syntax) — thin layer over the C++ parser.

Same keys as the reference run.conf (run.conf:1-23: application.NX/NY/NZ, input.{G,DDV,UMEAN},
output.{G,DDV,UMEAN}, path) plus the optional keys of SURVEY §5.6 (Re, Q, LX, LZ, nsteps, cfl,
stats_every, symmetry_every, checkpoint_every, precision, decomposition, seed, ic, ...).
"""
from __future__ import annotations

from typing import Iterable

from .._native import require_core


def load_config(path: str, overrides: Iterable[str] = ()):
    """Parse a run.conf file; ``overrides`` are ``key=value`` strings (CLI ``--set``)."""
    return require_core().Config.from_file(path, list(overrides))


def config_from_string(text: str, overrides: Iterable[str] = ()):
    return require_core().Config.from_string(text, list(overrides))


def default_config(**kw):
    """A Config with the reference defaults, updated from keyword arguments."""
    c = require_core().Config()
    for k, v in kw.items():
        if not hasattr(c, k):
            raise KeyError(f"unknown config key {k!r}")
        setattr(c, k, v)
    c.validate()
    return c


def reference_preset(name: str, **kw):
    """Named BASELINE configurations (BASELINE.json "configs")."""
    presets = {
        # laminar Poiseuille plumbing check, CPU reference path
        "poiseuille": dict(NX=32, NY=33, NZ=17, Re=100.0, ic="laminar", precision="fp64"),
        # reference run.conf grid (128 x 128 x 128 physical, Re=3250)
        "ref128": dict(NX=128, NY=129, NZ=65, Re=3250.0, precision="fp32"),
        # Re = 3130 gives Re_tau ~ 180 at Q = 1.8 (configs/retau180_128x129x128.conf, the validation run)
        "retau180": dict(NX=128, NY=129, NZ=65, Re=3130.0, precision="fp64"),
        "retau550": dict(NX=512, NY=257, NZ=257, Re=11150.0, precision="fp32"),
        "retau950": dict(NX=1024, NY=385, NZ=513, Re=20700.0, precision="fp32"),
        "retau2000": dict(NX=2048, NY=633, NZ=1025, Re=48300.0, precision="fp32"),
    }
    if name not in presets:
        raise KeyError(f"unknown preset {name!r}; have {sorted(presets)}")
    d = dict(presets[name])
    d.update(kw)
    return default_config(**d)
