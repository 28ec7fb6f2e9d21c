"""Python driver: ``python -m channel_gpu_amd.driver run.conf [--set key=value] [--steps N]``.

Same behaviour as the C++ binary ``bin/channel_mi355x`` (and the reference's channelMPI.bin,
main.c:10-150), for launches through ``torchrun`` / ``torch.distributed.run`` (one rank per GPU):
config -> device = LOCAL_RANK -> RCCL communicator -> IC (files or generated) -> RK3 loop with
the reference stdout blocks and .dat statistics -> G/DDV/UMEAN restart files.  The ranks are
torch-free (native TCP rendezvous of the RCCL id; /opt/rocm HIP runtime and RCCL).
"""
from __future__ import annotations

import argparse
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="channel_gpu_amd.driver")
    ap.add_argument("config", nargs="?", default="run.conf")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)

    import os

    os.environ.setdefault("CHANNEL_TORCH_FREE", "1")
    from .models.channel import ChannelFlow
    from .utils.config import load_config

    cfg = load_config(a.config, a.set)
    flow = ChannelFlow(cfg)
    rank, world = flow.rank, flow.world
    flow.initialize()
    n = cfg.nsteps if a.steps is None else a.steps
    t0 = time.perf_counter()
    flow.run(n, verbose=not a.quiet)
    sec = time.perf_counter() - t0
    if rank == 0:
        pts = cfg.NX * cfg.NY * (2 * cfg.NZ - 2)
        print(f"\nchannel_gpu_amd: {n} RK3 steps on {world} rank(s) in {sec:.3f} s "
              f"({1e3 * sec / max(n, 1):.3f} ms/step, {pts * n / max(sec, 1e-30):.3e} grid-pts/s)")
    if cfg.out_G != "-" and cfg.out_DDV != "-":
        flow.save(cfg.out_G, cfg.out_DDV, cfg.out_UMEAN)
    return 0


if __name__ == "__main__":
    sys.exit(main())
