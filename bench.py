#!/usr/bin/env python3
"""Headline benchmark: wall-seconds per RK3 step and grid-points/second of the channel DNS at
Re_tau ~ 950 on the 1024 x 385 x 1024 grid (BASELINE.json), fp32 storage (fp64 y-solves), on N
GPUs of one node with the slab decomposition (one rank per GPU, RCCL all-to-all over xGMI).

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N > 1`` without a torchrun environment launches itself under torch.distributed.run as a
child process (before anything touches the GPU) and exits with its return code.

Ranks never import torch: the solver runs on /opt/rocm's HIP runtime and RCCL, bootstrapped by a
native TCP rendezvous (channel_gpu_amd.parallel.native_bootstrap); torch.distributed.run is only
the launcher.

Synthetic data: a seeded random divergence-free velocity field on a laminar mean profile
(no checkpoint is available offline).  W untimed warm-up steps (the first one eager, then graph
capture), then exactly K RK3 steps timed between barrier + device synchronisation on every rank;
the MAX over ranks is reported.  Total work is fixed as N grows ("strong" scaling).  Per-step
device times (hipEvents between graph launches) give the median and p90.  For P > 1 a few extra,
untimed, eagerly-run steps with per-phase events give the exchange time and per-peer bandwidth.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# analytic K20X-class model floor of the reference at this grid (a model, not a
# measurement: the reference publishes no numbers and cannot run this grid), s per RK3 step
REF_MODEL_FLOOR_S = {1: 23.5, 2: 11.8, 4: 6.0, 8: 3.0}
# BASELINE.json configs by grid (NX, NY, Nz_physical)
RE_TAU_LABEL = {(32, 33, 32): "laminar Poiseuille", (128, 129, 128): "Re_tau~180", (512, 257, 512): "Re_tau~550",
                (1024, 385, 1024): "Re_tau~950", (2048, 633, 2048): "Re_tau~2000"}
# environment switches that skip work inside the timed region (diagnosis only)
WORK_SKIPPING_ENV = ("CHANNEL_FFT_DIAG",)
HEADLINE_METRIC = "wall-sec/RK3-step + grid-pts/sec at Re_tau=950, 1024x385x1024, 1/2/4/8 GPU"
# statistics cadence of the reference (FREC_STATS = 10, channel.h:82; computed in nonLinear.c:11-12):
# every 10th timed step also accumulates the plane statistics in its last substep
STATS_EVERY = 10
# xGMI model: one link per peer pair, ~153 GB/s per link (point-to-point, no switch)
XGMI_LINK_GBPS = 153.0
# slot 7: milliseconds in which a K-SPEC interval and an exchange interval ran at once (P > 1)
PHASES = ["kspec", "x_backward", "z_physical", "x_forward", "a2a", "reduce", "io", "kspec_a2a_overlap"]


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n: int) -> int:
    """Run this script under torch.distributed.run with n ranks (child process, no exec)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def _pct(v: list[float], q: float) -> float:
    s = sorted(v)
    if not s:
        return float("nan")
    i = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
    return s[i]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grid", default="1024x385x1024", help="NX x NY x Nz_physical")
    ap.add_argument("--re", type=float, default=20700.0, help="1/nu (Re_tau~950 at Q=1.8, SURVEY App. C)")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--decomposition", default="slab", choices=["slab", "pencil"])
    ap.add_argument("--pr", type=int, default=0, help="pencil rows (0 = automatic: the fewest bytes on the busiest link, 4x2 at 8 ranks)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--phases", action="store_true",
                    help="after the timed steps, time a few more eagerly with per-phase hipEvents")
    ap.add_argument("--phase-steps", type=int, default=3)
    ap.add_argument("--stats-every", type=int, default=STATS_EVERY,
                    help="plane statistics every k-th step inside the timed region (0 = never)")
    args = ap.parse_args()

    bad = [e for e in WORK_SKIPPING_ENV if os.environ.get(e, "0") not in ("", "0")]
    if bad:
        raise SystemExit(f"refusing to benchmark with work-skipping diagnostics enabled: {bad}")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(_self_launch(args.gpus))

    # torch-free ranks: the solver runs on /opt/rocm's HIP runtime and RCCL (like the C++ driver);
    # the native TCP rendezvous hands out the communicator id
    os.environ["CHANNEL_TORCH_FREE"] = "1"
    from channel_gpu_amd import require_core
    from channel_gpu_amd.parallel.decomposition import PencilDecomposition, SlabDecomposition
    from channel_gpu_amd.parallel.native_bootstrap import init_native
    from channel_gpu_amd.utils.config import default_config

    # (a torch import here would bind torch's bundled HIP runtime and RCCL before the native core)
    assert "torch" not in sys.modules, "bench.py ranks must not import torch"
    if args.gpus > 1:
        # a first multi-GPU run must fail diagnosably, well inside the driver's time limit: the
        # communication watchdog raises on every rank after 120 s without progress (instead of a
        # kill with no diagnosis), and each rank prints a stderr line after the eager warm-up step,
        # the graph capture and the first replay
        os.environ.setdefault("CHANNEL_COMM_TIMEOUT_S", "120")
        os.environ.setdefault("CHANNEL_MARKERS", "1")
    ri = init_native()
    rank, world = ri.rank, ri.world
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    C = require_core()
    NX, NY, NZP = (int(v) for v in args.grid.lower().split("x"))
    cfg = default_config(NX=NX, NY=NY, NZ=NZP // 2 + 1, Re=args.re, precision=args.precision, ic="random",
                         ic_amplitude=0.05, stats_every=0, log_every=0, symmetry_every=0, checkpoint_every=0,
                         health_check=True, decomposition=args.decomposition, pr=args.pr)
    solver = C.Solver(cfg, rank, world, ri.device, ri.uid)
    if args.no_graph:
        solver.set_use_graph(False)
    solver.init_ic()
    solver.prepare()

    def barrier():
        solver.barrier()  # device allreduce over the solver's communicator + stream sync

    def max_over_ranks(x: float) -> float:
        return float(solver.max_over_ranks(float(x)))

    se = max(0, args.stats_every)
    # the warm-up captures both step graphs (with and without the statistics pass) when it has at
    # least two steps, so no capture falls inside the timed region
    for i in range(args.warmup):
        solver.step(se > 0 and args.warmup >= 2 and i == args.warmup - 1)
    barrier()
    solver.set_step_timing(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        solver.step(se > 0 and (i + 1) % se == 0)
    barrier()
    dt_wall = max_over_ranks(time.perf_counter() - t0)
    step_ms = solver.step_times_ms()
    solver.set_step_timing(False)
    med = max_over_ranks(_pct(step_ms, 0.5))
    p90 = max_over_ranks(_pct(step_ms, 0.9))
    graph = bool(solver.graph_active())
    L = solver.log()

    phase = None
    if args.phases or solver.comm_kind() != "none":
        # untimed for the headline: eager steps with per-phase events (serialised at P = 1)
        solver.reset_phase_times()
        solver.set_phase_timing(True)
        ps = max(1, args.phase_steps)
        for _ in range(ps):
            solver.step(False)
        solver.set_phase_timing(False)
        barrier()
        phase = [max_over_ranks(x / ps) for x in solver.phase_times_ms()]

    s_per_step = dt_wall / max(1, args.steps)
    pts = NX * NY * NZP
    value = pts / s_per_step
    floor = REF_MODEL_FLOOR_S.get(world) if (NX, NY, NZP) == (1024, 385, 1024) else None
    parallelism = f"slab{world}" if solver.plan.Pr == 1 else f"pencil{solver.plan.Pr}x{solver.plan.Pc}"
    headline = (NX, NY, NZP) == (1024, 385, 1024) and args.precision == "fp32" and solver.plan.Pr == 1
    if headline:
        metric = HEADLINE_METRIC
    else:
        why = []
        if (NX, NY, NZP) != (1024, 385, 1024):
            why.append("not the headline grid")
        if args.precision != "fp32":
            why.append(f"{args.precision} storage")
        if solver.plan.Pr != 1:
            why.append(f"{parallelism} decomposition")
        metric = f"wall-sec/RK3-step + grid-pts/sec at {NX}x{NY}x{NZP} ({', '.join(why)})"
    out = {
        "metric": metric,
        "value": value,
        "unit": "grid-pts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * s_per_step,
        "ms_per_step_median": med,
        "ms_per_step_p90": p90,
        "wall_sec_per_step": s_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "reference_model_floor_s_per_step_analytic": floor,
        "dtype": "fp32 storage, fp64 y-solves" if args.precision == "fp32" else args.precision,
        "data": "synthetic (seeded random divergence-free IC on the laminar profile)",
        "config": {
            "model": f"channel DNS {RE_TAU_LABEL.get((NX, NY, NZP), 'custom grid')} (Re={args.re:g}, Q=1.8, LX=2pi, LZ=pi)",
            "grid": f"{NX}x{NY}x{NZP}",
            "global_batch": 1,
            "seq_len": pts,
            "parallelism": parallelism,
            "stats_every": se,
            "hipgraph": graph,
            "comm": solver.comm_kind(),
        },
        "health": int(L.health),
        "dt": L.dt,
    }
    esz = 16 if args.precision == "fp64" else 8
    if world > 1:
        # exchange model: the busiest peer pair's bytes per step over one xGMI link
        if solver.plan.Pr == 1:
            dec = SlabDecomposition(NX, NY, NZP // 2 + 1, world)
            peer = max(max(b for q, b in enumerate(dec.a2a_bytes_per_peer_per_step(r, esz)) if q != r)
                       for r in range(world))
        else:
            pd = PencilDecomposition(NX, NY, NZP // 2 + 1, solver.plan.Pr, solver.plan.Pc)
            peer = 0
            for r in range(world):
                eb = pd.exchange_bytes_per_substep(r, esz)
                peer = max(peer, 3 * max(eb["A"] // max(1, pd.Pc - 1), eb["B"] // max(1, pd.Pr - 1) if pd.Pr > 1 else 0))
        out["a2a_model_bytes_per_peer_per_step"] = int(peer)
        out["a2a_model_ms_per_step"] = round(peer / (XGMI_LINK_GBPS * 1e9) * 1e3, 4)
    if phase is not None:
        out["phase_ms_per_step"] = {k: round(v, 4) for k, v in zip(PHASES, phase) if v > 0}
        out["phase_sum_ms_compute"] = round(sum(phase[i] for i in (0, 1, 2, 3)), 4)
        if solver.comm_kind() != "none" and solver.plan.Pr == 1:
            dec = SlabDecomposition(NX, NY, NZP // 2 + 1, world)
            per_peer = [b for q, b in enumerate(dec.a2a_bytes_per_peer_per_step(rank, esz)) if q != rank or world == 1]
            a2a_ms = phase[4]
            out["a2a_ms_per_step"] = round(a2a_ms, 4)
            out["a2a_bytes_per_peer_per_step"] = int(max(per_peer))
            out["a2a_GBps_per_peer"] = (round(max(per_peer) / (a2a_ms * 1e-3) / 1e9, 2) if a2a_ms > 0 else None)
    if os.environ.get("CHANNEL_KSPEC_PROF"):
        # shader-clock cycles per K-SPEC phase, summed over all waves (warmup + timed steps)
        cyc = solver.kspec_profile()
        tot = sum(cyc) or 1.0
        out["kspec_phase_fraction"] = [round(c / tot, 4) for c in cyc]
    if ri.uid and world == 1:
        out["forced_comm"] = True
    if rank == 0:
        print(json.dumps(out), flush=True)
    barrier()
    del solver


if __name__ == "__main__":
    main()
