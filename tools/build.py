#!/usr/bin/env python3
"""Build the native core of channel_gpu_amd in-tree (gfx950 only).

Products
  channel_gpu_amd/lib/libchannel_core.so   HIP kernels + C++ core (solver, RCCL comm, HDF5 I/O, config)
  channel_gpu_amd/_core<EXT_SUFFIX>        torch-free pybind11 bindings (Solver, config, I/O, bootstrap)
  channel_gpu_amd/_C<EXT_SUFFIX>           PyTorch tensor entry points of every kernel (+ re-exports _core)
  bin/channel_mi355x                       C++ driver binary (run.conf, MPI bootstrap of RCCL)

Incremental: an object is rebuilt when its source or any header under csrc/include is newer.
The reference built one binary with mpic++/nvcc for sm_35 (Makefile:1-28) and baked the grid
size in with -D macros; everything here is runtime-sized.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shlex
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CHANNEL_ARCH", "gfx950")
OBJ = os.path.join(ROOT, "build", "obj")
LIBDIR = os.path.join(ROOT, "channel_gpu_amd", "lib")
CORE_SO = os.path.join(LIBDIR, "libchannel_core.so")
EXT_SO = os.path.join(ROOT, "channel_gpu_amd", "_C" + sysconfig.get_config_var("EXT_SUFFIX"))
CORE_EXT_SO = os.path.join(ROOT, "channel_gpu_amd", "_core" + sysconfig.get_config_var("EXT_SUFFIX"))
DRIVER = os.path.join(ROOT, "bin", "channel_mi355x")
INC = os.path.join(ROOT, "csrc", "include")
CONDA = "/opt/conda"

COMMON = ["-O3", "-std=c++17", "-fPIC", f"-I{INC}", "-Wno-unused-result"]
DEVICE = [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-mcode-object-version=5"]


def _newest_header() -> float:
    hs = glob.glob(os.path.join(INC, "**", "*.hpp"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd[:3])} ... {cmd[-1]}")
    elif verbose and r.stdout.strip():
        print(r.stdout)


def _stale(out: str, deps: list[str], hdr_time: float) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps) or hdr_time > t


def _depfile_deps(obj: str) -> list[str] | None:
    """Headers an object was compiled against (from the compiler's -MMD file), or None."""
    d = obj + ".d"
    if not os.path.exists(d):
        return None
    text = open(d).read().replace("\\\n", " ")
    deps = []
    for line in text.splitlines():
        if ":" not in line:
            continue
        for tok in line.split(":", 1)[1].split():
            if tok.endswith((".hpp", ".h")) and tok.startswith(ROOT):
                deps.append(tok)
    return deps


def _obj_stale(obj: str, src: str, hdr_time: float) -> bool:
    deps = _depfile_deps(obj)
    if deps is None:  # no dependency file yet: any newer header rebuilds
        return _stale(obj, [src], hdr_time)
    return _stale(obj, [src] + [h for h in deps if os.path.exists(h)], 0.0) or any(not os.path.exists(h) for h in deps)


def _torch_flags() -> tuple[list[str], list[str]]:
    import torch.utils.cpp_extension as ce  # noqa: F401  (paths only; no JIT build)
    import torch

    inc = []
    for p in ce.include_paths():
        inc.append(f"-I{p}")
    inc.append(f"-I{sysconfig.get_paths()['include']}")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = inc + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                    "-DUSE_ROCM", "-D__HIP_PLATFORM_AMD__"]
    libdir = ce.library_paths()[0]
    ldflags = [f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
               f"-Wl,-rpath,{libdir}"]
    return cflags, ldflags


def build(verbose: bool = False, jobs: int = 8, driver: bool = True) -> None:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    hdr = _newest_header()
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "core", "*.cpp")) +
                  glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    # longest compiles first (the 1024/2048-point transform units and K-SPEC take minutes each)
    heavy = ("fft_pow2_1024", "fft_pow2_2048", "kspec", "fft_pow2.", "fft_r")
    srcs.sort(key=lambda s: next((i for i, h in enumerate(heavy) if h in os.path.basename(s)), len(heavy)))
    objs, jobs_list = [], []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        objs.append(o)
        if _obj_stale(o, s, hdr):
            flags = COMMON + DEVICE  # host .cpp too: hipcc compiles it as HIP; gfx950 code objects only
            extra = ["-x", "hip"] if s.endswith(".hip") else []
            jobs_list.append([HIPCC] + flags + extra + ["-MMD", "-MF", o + ".d", "-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, c, verbose) for c in jobs_list]:
            f.result()
    if _stale(CORE_SO, objs, 0.0):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", CORE_SO, "-L/opt/rocm/lib", "-lrccl",
              "-lrocprofiler-sdk-roctx", "-ldl", "-Wl,-rpath,/opt/rocm/lib", "-Wl,-soname,libchannel_core.so"], verbose)
    # torch-free bindings: pybind11 headers of the torch wheel (one pybind11 type registry shared
    # with _C), no libtorch
    import torch

    tinc = os.path.join(os.path.dirname(torch.__file__), "include")
    csrc_ = os.path.join(ROOT, "csrc", "bindings", "core_module.cpp")
    cobj = os.path.join(OBJ, "core_module.o")
    if _obj_stale(cobj, csrc_, hdr) or _stale(CORE_EXT_SO, [cobj, CORE_SO], 0.0):
        if _obj_stale(cobj, csrc_, hdr):
            _run([HIPCC, "-O2", "-std=c++17", "-fPIC", *DEVICE, f"-I{INC}", f"-I{tinc}", f"-I{sysconfig.get_paths()['include']}",
                  "-MMD", "-MF", cobj + ".d", "-c", csrc_, "-o", cobj], verbose)
        _run([HIPCC, "-shared", "-fPIC", cobj, "-o", CORE_EXT_SO, f"-L{LIBDIR}", "-lchannel_core",
              "-Wl,-rpath,$ORIGIN/lib"], verbose)
    # torch bindings
    bsrc = os.path.join(ROOT, "csrc", "bindings", "bindings.cpp")
    bobj = os.path.join(OBJ, "bindings.o")
    if _obj_stale(bobj, bsrc, hdr) or _stale(EXT_SO, [bobj, CORE_SO], 0.0):
        tcf, tld = _torch_flags()
        if _obj_stale(bobj, bsrc, hdr):
            _run([HIPCC, "-O2", "-std=c++17", "-fPIC", *DEVICE, f"-I{INC}", *tcf, "-MMD", "-MF", bobj + ".d", "-c", bsrc, "-o",
                  bobj], verbose)
        _run([HIPCC, "-shared", "-fPIC", bobj, "-o", EXT_SO, f"-L{LIBDIR}", "-lchannel_core", *tld,
              "-Wl,-rpath,$ORIGIN/lib"], verbose)
    if driver:
        # the driver bootstraps RCCL over TCP (csrc/core/bootstrap.cpp): no MPI link dependency
        dsrc = os.path.join(ROOT, "csrc", "driver", "main.cpp")
        os.makedirs(os.path.dirname(DRIVER), exist_ok=True)
        if _stale(DRIVER, [dsrc, CORE_SO], hdr):
            _run([HIPCC, "-O2", "-std=c++17", *DEVICE, f"-I{INC}", dsrc, "-o", DRIVER, f"-L{LIBDIR}", "-lchannel_core",
                  "-Wl,-rpath,$ORIGIN/../channel_gpu_amd/lib", "-Wl,-rpath,/opt/rocm/lib"], verbose)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--no-driver", action="store_true")
    a = ap.parse_args()
    build(a.verbose, a.jobs, driver=not a.no_driver)
    print("built:", os.path.relpath(CORE_SO, ROOT), os.path.relpath(CORE_EXT_SO, ROOT), os.path.relpath(EXT_SO, ROOT))


if __name__ == "__main__":
    main()
