#!/usr/bin/env python3
"""Diagnosis of the CHANNEL_PSTREAMS=2 capture crash: a process that imports torch
first binds torch's bundled HIP runtime and RCCL (same sonames as /opt/rocm's), then captures the
P > 1 step graph with the second compute stream forked next to the RCCL exchanges on a 1-rank
RCCL communicator.  Prints which HIP runtime the process bound and, on a crash, the native
backtrace (install_crash_handler).

  CHANNEL_PSTREAMS=2 CHANNEL_PSTREAMS_CAPTURE=1 CHANNEL_MARKERS=1 python tools/pstreams_capture_probe.py [--torch-free]
(CHANNEL_MARKERS=1: the solver's stderr markers around the capture, instantiation and first replay;
CHANNEL_GRAPH_DOT=<prefix>: the captured step graph's topology, where the capture completes)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--torch-free" in sys.argv:
    os.environ["CHANNEL_TORCH_FREE"] = "1"
from channel_gpu_amd._native import require_core  # noqa: E402
from channel_gpu_amd.utils.config import default_config  # noqa: E402

C = require_core()  # (imports torch first unless CHANNEL_TORCH_FREE=1)
C.install_crash_handler()
hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
v = ctypes.c_int(0)
hip.hipRuntimeGetVersion(ctypes.byref(v))
maps = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln or "librccl" in ln]
print("hip runtime", v.value, sorted(set(maps)), flush=True)
os.environ.setdefault("CHANNEL_YCHUNK", "8")
cfg = default_config(NX=64, NY=65, NZ=33, Re=1000.0, precision="fp64", ic="random", ic_amplitude=0.2, stats_every=0,
                     log_every=0, symmetry_every=0)
s = C.Solver(cfg, 0, 1, 0, C.new_unique_id())
C.install_crash_handler()  # again: RCCL's communicator setup may install its own SIGSEGV handler
s.init_ic()
s.prepare()
for i in range(4):
    s.step(False)
    s.synchronize()
    print("step", i, "graph", s.graph_active(), flush=True)
print("PSTREAMS_PROBE_OK", flush=True)
