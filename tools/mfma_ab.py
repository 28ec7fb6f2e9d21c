#!/usr/bin/env python3
"""A/B of the wall-normal D1 operator: partitioned Thomas + PCR solve (VALU, one wave per line)
against the dense D1 on the matrix cores (v_mfma_f64_16x16x4_f64, 8 lines per block).

  python tools/mfma_ab.py [--lines 65536] [--reps 20]

Prints one JSON line per NY with the per-call times (hipEvents) and the max relative difference
between the two.  Run it under `rocprofv3 --kernel-trace --stats` for kernel times and under
`rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 ...` for the MFMA counters.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from channel_gpu_amd._native import require_native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ny", default="33,65,129,192")
    args = ap.parse_args()
    nat = require_native()
    for NY in (int(v) for v in args.ny.split(",")):
        Y = nat.YLineOps(NY)
        g = torch.Generator(device="cuda").manual_seed(NY)
        x = torch.randn(NY, args.lines, dtype=torch.complex128, device="cuda", generator=g)
        res = {}
        for name, fn in (("pcr", lambda: Y.apply(0, x)), ("mfma", lambda: Y.d1_mfma(x))):
            out = fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                out = fn()
            b.record()
            torch.cuda.synchronize()
            res[name] = (a.elapsed_time(b) * 1e3 / args.reps, out)
        diff = ((res["pcr"][1] - res["mfma"][1]).abs().max() / res["pcr"][1].abs().max()).item()
        print(json.dumps({"NY": NY, "lines": args.lines, "pcr_us": round(res["pcr"][0], 1),
                          "mfma_us": round(res["mfma"][0], 1),
                          "mfma_over_pcr": round(res["mfma"][0] / res["pcr"][0], 2), "max_rel_diff": diff}),
              flush=True)


if __name__ == "__main__":
    main()
