#!/usr/bin/env python3
"""Build and run the host-code sanitizer self-test.

Compiles the CPU components of the native core (csrc/core/{config,grid,plan,io}.cpp) together with
tests/native/host_selftest.cpp using AddressSanitizer + UndefinedBehaviorSanitizer
(`-fsanitize=address,undefined`, host only: GPU ASan / xnack are not available on the MI355X
pool) and runs the binary.  Any sanitizer report aborts the run with a non-zero exit status.

    python tools/host_sanitize.py [--out build/asan]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["csrc/core/config.cpp", "csrc/core/grid.cpp", "csrc/core/plan.cpp", "csrc/core/io.cpp",
           "tests/native/host_selftest.cpp"]
FLAGS = ["-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
         "-fno-sanitize-recover=undefined", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
         "-Icsrc/include"]


def compiler() -> str | None:
    for c in ("g++", "clang++"):
        if shutil.which(c):
            return c
    return None


def build(out_dir: str) -> str:
    cxx = compiler()
    if cxx is None:
        raise RuntimeError("no host C++ compiler")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "host_selftest")
    cmd = [cxx, *FLAGS, *[os.path.join(ROOT, s) for s in SOURCES], "-o", exe, "-ldl"]
    subprocess.run(cmd, cwd=ROOT, check=True)
    return exe


def run(exe: str) -> subprocess.CompletedProcess:
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:halt_on_error=1:exitcode=23"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1:exitcode=24"
    with tempfile.TemporaryDirectory() as d:
        return subprocess.run([exe, d], cwd=ROOT, env=env, capture_output=True, text=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "build", "asan"))
    a = ap.parse_args()
    r = run(build(a.out))
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
