#!/usr/bin/env python3
"""Turbulent channel validation run (BASELINE config 2: Re_tau~180, 128x129x128, fp64).

From the seeded random divergence-free IC through transition to a statistically steady state,
then time-averaged statistics in wall units (SURVEY §4.2 "Physics: turbulent"; the reference ran
this case for 30,000 steps and compared its stdout blocks with known values by eye,
RK3.c:124-185, meanUevol.c:489-560, statistics.cu:161-243).

  python tools/turbulence.py --out gpurun_out/turb --transition 60000 --average 120000

Writes into --out: timeseries.txt (step, t, dt, Re_tau, U_c+, flux error every --log-every
steps), profiles.txt (U+, u'+, v'+, w'+, -u'v'+ vs y+), summary.json, the reference .dat files
(stats cadence 10) and a float32 retained-mode snapshot of the final state (state_fp32.npz) that
seeds the slow regression test.  Optionally --resume from such a snapshot.
Torch-free process (ROCm HIP runtime + RCCL, like bench.py and the drivers).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("CHANNEL_TORCH_FREE", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from channel_gpu_amd.models.channel import ChannelFlow  # noqa: E402
from channel_gpu_amd.utils.config import load_config  # noqa: E402
from channel_gpu_amd.utils.snapshots import export_seed, load_snapshot, save_snapshot  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="configs/retau180_128x129x128.conf")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--out", default="gpurun_out/turb")
    ap.add_argument("--transition", type=int, default=60000, help="steps before averaging starts")
    ap.add_argument("--average", type=int, default=120000, help="averaging steps")
    ap.add_argument("--sample-every", type=int, default=10)
    ap.add_argument("--log-every", type=int, default=1000)
    ap.add_argument("--amplitude", type=float, default=0.05, help="random IC amplitude (per mode)")
    ap.add_argument("--resume", default="", help="state_fp32.npz to start from instead of the random IC")
    ap.add_argument("--export-seed", nargs=2, metavar=("STATE_NPZ", "OUT_NPZ"),
                    help="write the compact regression-test seed of a state file and exit")
    a = ap.parse_args()
    if a.export_seed:
        export_seed(*a.export_seed)
        return 0

    os.makedirs(a.out, exist_ok=True)
    path = os.path.abspath(a.out) + "/"
    cfg = load_config(a.config, [f"path={path}", "log_every=0", "stats_every=0", "checkpoint_every=0",
                                 f"ic_amplitude={a.amplitude}"] + a.set)
    flow = ChannelFlow(cfg)
    s = flow.solver
    step0, t0 = 0, 0.0
    if a.resume:
        phi, om, U, step0, t0 = load_snapshot(a.resume)
        flow.set_state(phi, om, U)
        s.set_time(t0, 0.0)
    else:
        flow.initialize()
    y = np.asarray(s.grid.y)
    trap = np.asarray(s.grid.trap)
    nu = 1.0 / cfg.Re
    ts = open(path + "timeseries.txt", "a")
    ts.write("# step time dt Re_tau Uc_plus flux_err umax vmax wmax ms_per_step\n")
    wall0 = time.perf_counter()
    tlog = wall0

    def log_line(step: int):
        nonlocal tlog
        L = s.log()
        if L.health:
            raise SystemExit(f"non-finite state at step {step}")
        U = np.asarray(s.mean_profile())
        flux_err = abs(float(trap @ U) - cfg.Q)
        ut = L.utau
        now = time.perf_counter()
        ms = 1e3 * (now - tlog) / a.log_every
        tlog = now
        ts.write(f"{step} {L.time:.6f} {L.dt:.6e} {ut / nu:.4f} {U[len(U) // 2] / ut:.4f} {flux_err:.3e} "
                 f"{L.umax:.4f} {L.vmax:.4f} {L.wmax:.4f} {ms:.4f}\n")
        ts.flush()
        print(f"step {step} t={L.time:.2f} dt={L.dt:.3e} Re_tau={ut / nu:.2f} Uc+={U[len(U) // 2] / ut:.2f} "
              f"flux_err={flux_err:.1e} {ms:.3f} ms/step", flush=True)

    # transition
    n = 0
    while n < a.transition:
        k = min(a.log_every, a.transition - n)
        for _ in range(k):
            s.step(False)
        n += k
        log_line(step0 + n)
    # averaging
    st = flow.statistics
    st.reset()
    m = 0
    while m < a.average:
        k = min(a.log_every, a.average - m)
        flow.sample_statistics(k, a.sample_every)
        m += k
        log_line(step0 + n + m)
    summary = st.summary()
    summary.update({"NX": cfg.NX, "NY": cfg.NY, "NZ": cfg.NZ, "Re": cfg.Re, "precision": cfg.precision,
                    "steps_transition": a.transition, "steps_average": a.average, "sample_every": a.sample_every,
                    "wall_s": time.perf_counter() - wall0, "resume": a.resume or None,
                    "lx": cfg.LX, "lz": cfg.LZ, "y_wall_first": float(y[1] - y[0])})
    st.write(path + "profiles.txt")
    with open(path + "summary.json", "w") as f:
        json.dump(summary, f, indent=1)
    L = s.log()
    save_snapshot(path + "state_fp32.npz", *flow.get_state(), step=step0 + n + m, time=L.time, cfg=cfg)
    print(json.dumps(summary), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
