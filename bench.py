#!/usr/bin/env python3
"""Headline benchmark: wall-seconds per RK3 step and grid-points/second of the channel DNS at
Re_tau ~ 950 on the 1024 x 385 x 1024 grid (BASELINE.json), fp32 storage (fp64 y-solves), on N
GPUs of one node with the slab decomposition (one rank per GPU, RCCL all-to-all over xGMI).

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

Synthetic data: a seeded random divergence-free velocity field on a laminar mean profile
(no checkpoint is available offline).  W untimed warm-up steps (graph capture happens there), then
exactly K RK3 steps timed between barrier + device synchronisation on every rank; the MAX over
ranks is reported.  Total work is fixed as N grows ("strong" scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# analytic K20X-class model floor of the reference at this grid, s per RK3 step
REF_MODEL_FLOOR_S = {1: 23.5, 2: 11.8, 4: 6.0, 8: 3.0}
# BASELINE.json configs by grid (NX, NY, Nz_physical)
RE_TAU_LABEL = {(32, 33, 32): "laminar Poiseuille", (128, 129, 128): "Re_tau~180", (512, 257, 512): "Re_tau~550",
                (1024, 385, 1024): "Re_tau~950", (2048, 633, 2048): "Re_tau~2000"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grid", default="1024x385x1024", help="NX x NY x Nz_physical")
    ap.add_argument("--re", type=float, default=20700.0, help="1/nu (Re_tau~950 at Q=1.8, SURVEY App. C)")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--decomposition", default="slab", choices=["slab", "pencil"])
    ap.add_argument("--pr", type=int, default=0, help="pencil rows (0 = automatic, most square)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--phases", action="store_true", help="per-phase timing (eager, synchronising)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from channel_gpu_amd.parallel.bootstrap import init_distributed, nccl_unique_id
    from channel_gpu_amd import require_native
    from channel_gpu_amd.utils.config import default_config

    rank, world, local = init_distributed()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    C = require_native()
    NX, NY, NZP = (int(v) for v in args.grid.lower().split("x"))
    cfg = default_config(NX=NX, NY=NY, NZ=NZP // 2 + 1, Re=args.re, precision=args.precision, ic="random",
                         ic_amplitude=0.05, stats_every=0, log_every=0, symmetry_every=0, checkpoint_every=0,
                         health_check=True, decomposition=args.decomposition, pr=args.pr)
    uid = nccl_unique_id()
    solver = C.Solver(cfg, rank, world, torch.cuda.current_device(), uid)
    if args.no_graph:
        solver.set_use_graph(False)
    solver.init_ic()
    solver.prepare()

    def barrier():
        solver.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        solver.step(False)
    barrier()
    if args.phases:
        solver.set_phase_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        solver.step(False)
    barrier()
    dt_wall = time.perf_counter() - t0
    if world > 1:
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([dt_wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_wall = float(t.item())
    L = solver.log()
    s_per_step = dt_wall / max(1, args.steps)
    pts = NX * NY * NZP
    value = pts / s_per_step
    floor = REF_MODEL_FLOOR_S.get(world) if (NX, NY, NZP) == (1024, 385, 1024) else None
    out = {
        "metric": "wall-sec/RK3-step + grid-pts/sec at Re_tau=950, 1024x385x1024, 1/2/4/8 GPU",
        "value": value,
        "unit": "grid-pts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * s_per_step,
        "wall_sec_per_step": s_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "reference_model_floor_s_per_step": floor,
        "speedup_vs_reference_model_floor": (floor / s_per_step) if floor else None,
        "dtype": "fp32 storage, fp64 y-solves" if args.precision == "fp32" else args.precision,
        "data": "synthetic (seeded random divergence-free IC on the laminar profile)",
        "config": {
            "model": f"channel DNS {RE_TAU_LABEL.get((NX, NY, NZP), 'custom grid')} (Re={args.re:g}, Q=1.8, LX=2pi, LZ=pi)",
            "grid": f"{NX}x{NY}x{NZP}",
            "global_batch": 1,
            "seq_len": pts,
            "parallelism": (f"slab{world}" if solver.plan.Pr == 1
                            else f"pencil{solver.plan.Pr}x{solver.plan.Pc}"),
            "hipgraph": not args.no_graph,
        },
        "health": int(L.health),
        "dt": L.dt,
    }
    if args.phases:
        out["phase_ms_per_step"] = [x / max(1, args.steps) for x in solver.phase_times_ms()]
    if os.environ.get("CHANNEL_KSPEC_PROF"):
        # shader-clock cycles per K-SPEC phase, summed over all waves (warmup + timed steps)
        cyc = solver.kspec_profile()
        tot = sum(cyc) or 1.0
        out["kspec_phase_fraction"] = [round(c / tot, 4) for c in cyc]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
