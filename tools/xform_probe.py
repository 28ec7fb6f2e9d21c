#!/usr/bin/env python3
"""Time the x -> z -> x transform stage of one RK3 substep on its own (no K-SPEC), for A/B runs of
the pipeline switches (CHANNEL_YCHUNK, CHANNEL_YSTREAMS, CHANNEL_FFT_DIAG, ...), which are read once
per process: run one process per setting.

  python tools/xform_probe.py --grid 1024x385x1024 --reps 20      -> one JSON line
  --force-comm: the P > 1 pipeline on a 1-rank RCCL communicator (exchange segments, kx sub-blocks)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="1024x385x1024")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--force-comm", action="store_true")
    args = ap.parse_args()
    os.environ["CHANNEL_TORCH_FREE"] = "1"
    from channel_gpu_amd import require_core
    from channel_gpu_amd.utils.config import default_config

    C = require_core()
    NX, NY, NZP = (int(v) for v in args.grid.lower().split("x"))
    cfg = default_config(NX=NX, NY=NY, NZ=NZP // 2 + 1, Re=20700.0, precision=args.precision, ic="random",
                         ic_amplitude=0.05, stats_every=0, log_every=0, symmetry_every=0)
    s = C.Solver(cfg, 0, 1, 0, C.new_unique_id() if args.force_comm else b"")
    s.init_ic()
    s.prepare()
    for _ in range(args.warmup):
        s.transforms_debug(False)
    s.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        s.transforms_debug(False)
    s.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / args.reps
    env = {k: v for k, v in os.environ.items() if k.startswith("CHANNEL_") and k != "CHANNEL_TORCH_FREE"}
    print(json.dumps({"grid": args.grid, "precision": args.precision, "ms_per_substep_transforms": round(ms, 4),
                      "ms_per_step_transforms": round(3 * ms, 3), "comm": s.comm_kind(), "env": env}), flush=True)


if __name__ == "__main__":
    main()
