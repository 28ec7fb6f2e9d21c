#!/usr/bin/env python3
"""Register / occupancy table of the kernels in one HIP translation unit (device-only compile with
-Rpass-analysis=kernel-resource-usage), filtered by a substring of the mangled name.

  python tools/regs.py csrc/kernels/fft_pow2.hip zphys_kernelILi1024
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    src, pat = os.path.abspath(sys.argv[1]), (sys.argv[2] if len(sys.argv) > 2 else "")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", f"-I{ROOT}/csrc/include", "-Wno-unused-result",
           "--offload-arch=gfx950", "-munsafe-fp-atomics", "-mcode-object-version=5", "--cuda-device-only", "-c", src,
           "-o", "/tmp/regs_probe.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp")
    if r.returncode:
        sys.exit(r.stderr[-4000:])
    cur, rows = None, []
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for d in rows:
        if pat in d["name"]:
            print(f"{d['name'][:90]:90s} vgpr={d.get('VGPRs', '?'):>4} agpr={d.get('AGPRs', '?'):>4} "
                  f"vspill={d.get('VGPRs Spill', '?'):>4} sspill={d.get('SGPRs Spill', '?'):>4} "
                  f"occ={d.get('Occupancy [waves/SIMD]', '?')} lds={d.get('LDS Size [bytes/block]', '?')}")


if __name__ == "__main__":
    main()
