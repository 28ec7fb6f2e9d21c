"""Compact state snapshots (NumPy .npz, plain arrays only: loaded with allow_pickle=False).

* ``save_snapshot`` / ``load_snapshot``: the full retained-mode state (phi, omega_y, U) in
  float32, with step/time and the grid; used to resume long validation runs between jobs.
* ``export_seed`` / ``load_seed``: a ~1 MB seed of a developed turbulent state — only
  |kx| <= kx_max, kz <= kz_max, float16 — committed under tests/data for the turbulence
  regression test (the truncated modes regrow within a few hundred steps).

These complement, not replace, the reference-format HDF5 restart files (Solver.write_restart).
"""
from __future__ import annotations

import numpy as np


def save_snapshot(path: str, phi, om, U, *, step: int, time: float, cfg=None):
    extra = {}
    if cfg is not None:
        extra = dict(NX=cfg.NX, NY=cfg.NY, NZ=cfg.NZ, Re=cfg.Re)
    np.savez_compressed(path, phi=np.asarray(phi).astype(np.complex64), om=np.asarray(om).astype(np.complex64),
                        U=np.asarray(U, float), step=step, time=time, **extra)


def load_snapshot(path: str):
    """(phi, om, U, step, time) with complex128 fields."""
    d = np.load(path)
    return (d["phi"].astype(np.complex128), d["om"].astype(np.complex128), d["U"].astype(float), int(d["step"]),
            float(d["time"]))


def export_seed(state: str, out: str, kx_max: int = 32, kz_max: int = 21):
    """Compact seed of a save_snapshot file: |kx| <= kx_max, kz <= kz_max, float16 re/im."""
    d = np.load(state)
    nkx = d["phi"].shape[1]
    Kx = (nkx - 1) // 2
    ix = np.r_[0:kx_max + 1, nkx - kx_max:nkx]
    arrs = {}
    for k in ("phi", "om"):
        q = d[k][:, ix, :kz_max + 1]
        arrs[k + "_re"] = q.real.astype(np.float16)
        arrs[k + "_im"] = q.imag.astype(np.float16)
    np.savez_compressed(out, U=d["U"], kx_max=kx_max, kz_max=kz_max, Kx=Kx, nkz=d["phi"].shape[2], time=d["time"],
                        **{k: d[k] for k in ("Re", "NX", "NY", "NZ") if k in d}, **arrs)


def load_seed(path: str):
    """(phi, om, U) full retained-mode arrays [NY, nkx, nkz] (complex128) from an export_seed file."""
    d = np.load(path)
    kx_max, kz_max, Kx, nkz = (int(d[k]) for k in ("kx_max", "kz_max", "Kx", "nkz"))
    nkx = 2 * Kx + 1
    ix = np.r_[0:kx_max + 1, nkx - kx_max:nkx]
    out = []
    for k in ("phi", "om"):
        q = np.zeros((d["U"].size, nkx, nkz), complex)
        q[:, ix, :kz_max + 1] = d[k + "_re"].astype(float) + 1j * d[k + "_im"].astype(float)
        out.append(q)
    return out[0], out[1], d["U"].astype(float)
