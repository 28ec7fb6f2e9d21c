#!/usr/bin/env python3
"""High-wavenumber energy of fp32-storage vs fp64-storage runs from the same band-limited IC.

The random IC fills |kx| <~ 40, kz <~ 20 only (envelope exp(-k^2/32), solver.cpp init_ic), so the
upper kz and kx bands start empty (exactly zero in fp32).  Two things can fill them: the physical
cascade (identical in both precisions) and storage round-off amplified by the wall influence
correction at wavenumbers the y grid cannot resolve (README, "fp32 storage and the high
wavenumbers").  Every --every steps this logs, per precision, the kinetic energy (u, v, w at the
spectra planes) in the bands kz >= nkz/4, nkz/2, 3 nkz/4 and |kx| >= Kx/2, as fractions of the
total, so the two trajectories can be compared: where fp32 tracks fp64 the high-band content is
physics; where fp32 sits orders of magnitude above, it is round-off.

  python tools/highband.py --grid 1024x385x1024 --re 20700 --steps 2000 --every 100 --out f.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def band_fractions(sp: dict) -> dict:
    ekz = np.asarray(sp["ekz"]).sum(axis=(0, 1))  # over u, v, w and planes -> [nkz]
    ekx = np.asarray(sp["ekx"]).sum(axis=(0, 1))  # -> [Kx + 1]
    tot = float(ekz.sum())
    nkz, nkx = ekz.size, ekx.size
    out = {"E": tot}
    for q in (4, 2):
        out[f"kz>={nkz // q}"] = float(ekz[nkz // q:].sum()) / tot if tot > 0 else 0.0
    out[f"kz>={3 * nkz // 4}"] = float(ekz[3 * nkz // 4:].sum()) / tot if tot > 0 else 0.0
    out[f"kx>={nkx // 2}"] = float(ekx[nkx // 2:].sum()) / tot if tot > 0 else 0.0
    return out


def run(args, precision: str, log) -> list:
    os.environ["CHANNEL_TORCH_FREE"] = "1"
    from channel_gpu_amd import require_core
    from channel_gpu_amd.utils.config import default_config

    C = require_core()
    NX, NY, NZP = (int(v) for v in args.grid.lower().split("x"))
    planes = args.planes or f"{max(1, NY // 40)},{NY // 8},{NY // 2}"
    cfg = default_config(NX=NX, NY=NY, NZ=NZP // 2 + 1, Re=args.re, precision=precision, ic="random",
                         ic_amplitude=args.amp, stats_every=0, log_every=0, symmetry_every=0,
                         spectra_planes=planes, **({"dt_fixed": args.dt} if args.dt > 0 else {}))
    s = C.Solver(cfg, 0, 1, 0, b"")
    s.init_ic()
    s.prepare()
    rows = []
    t0 = time.perf_counter()
    for n in range(args.steps + 1):
        if n % args.every == 0 or n == args.steps:
            sp = s.spectra()
            rec = {"precision": precision, "step": n, "time": s.time(), "health": int(s.health())}
            rec.update(band_fractions(sp))
            rec["wall_s"] = round(time.perf_counter() - t0, 2)
            rows.append(rec)
            print(json.dumps(rec), file=log, flush=True)
            print(json.dumps(rec), flush=True)
            if rec["health"]:
                break
        if n < args.steps:
            s.step(False)
    del s
    return rows


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="1024x385x1024")
    ap.add_argument("--re", type=float, default=20700.0)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--amp", type=float, default=0.05)
    ap.add_argument("--dt", type=float, default=0.0, help="fixed dt (0: CFL-controlled)")
    ap.add_argument("--planes", default="")
    ap.add_argument("--precisions", default="fp32,fp64")
    ap.add_argument("--out", default="gpurun_out/highband.jsonl")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    res = {}
    with open(args.out, "w") as log:
        for prec in args.precisions.split(","):
            res[prec] = run(args, prec, log)
    if "fp32" in res and "fp64" in res:
        print("step  " + "  ".join(f"{k:>22s}" for k in res["fp32"][0] if k.startswith("k")))
        for a, b in zip(res["fp32"], res["fp64"]):
            cells = [f"{a[k]:.3e}/{b[k]:.3e}" for k in a if k.startswith("k")]
            print(f"{a['step']:5d} " + "  ".join(f"{c:>22s}" for c in cells))


if __name__ == "__main__":
    main()
