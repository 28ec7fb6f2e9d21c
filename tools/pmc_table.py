#!/usr/bin/env python3
"""Per-kernel roofline table from rocprofv3 PMC passes (counter_collection.csv files).

  python tools/pmc_table.py DIR [DIR ...] > profiles/<name>.md

Each DIR is one `rocprofv3 --kernel-trace --pmc ...` output directory (one counter group per run,
see tools/gpu.sh pmc).  Values are averaged per kernel over its dispatches; the duration is the
counter-collection dispatch time of the pass that carried FETCH_SIZE (counter passes serialise
kernels, so durations are indicative).  HBM bytes follow the gfx950 calibration of
MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a wide streaming read, so bytes = 2*FETCH_SIZE*1024 +
WRITE_SIZE*1024 (an upper bound for narrower access patterns).  Wave-cycle shares use
SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY = SQ_WAVE_CYCLES.
"""
from __future__ import annotations

import collections
import csv
import glob
import sys


def load(dirs):
    val = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for d in dirs:
        for f in glob.glob(f"{d}/*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                val[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[k][(d, r["Dispatch_Id"])] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    return val, dur


def main():
    val, dur = load(sys.argv[1:])
    rows = []
    for k, c in val.items():
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        ds = list(dur[k].values())
        t = sum(ds) / len(ds) if ds else 0.0
        fetch = avg.get("FETCH_SIZE")
        write = avg.get("WRITE_SIZE")
        byts = (2 * fetch * 1024 if fetch is not None else 0) + (write * 1024 if write is not None else 0)
        wc = avg.get("SQ_WAVE_CYCLES", 0)
        shares = {n: (100.0 * avg[n] / wc) if wc and n in avg else float("nan")
                  for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")}
        rows.append((k, len(ds) // max(1, len(sys.argv) - 1), t, byts, avg, shares))
    rows.sort(key=lambda r: -r[2] * max(1, r[1]))
    print("| kernel | us/dispatch | HBM GB/dispatch | TB/s | VALU insts/wave | LDS insts/wave | LDS bank-conflict % | "
          "active % | wait-mem % | wait-issue % |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for k, n, t, byts, avg, share in rows:
        share = share.get
        if t < 2e-6:
            continue
        waves = avg.get("SQ_WAVES", 0) or float("nan")
        conf = 100.0 * avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"] if avg.get("SQ_LDS_IDX_ACTIVE") else float("nan")
        name = k.split("(")[0].replace("void ", "").replace("channel::", "")
        print(f"| `{name}` | {1e6 * t:.1f} | {byts / 1e9:.3f} | {byts / t / 1e12 if t else 0:.2f} | "
              f"{avg.get('SQ_INSTS_VALU', float('nan')) / waves:.0f} | {avg.get('SQ_INSTS_LDS', float('nan')) / waves:.0f} | "
              f"{conf:.1f} | {share('SQ_ACTIVE_INST_ANY'):.0f} | {share('SQ_WAIT_ANY'):.0f} | {share('SQ_WAIT_INST_ANY'):.0f} |")


if __name__ == "__main__":
    main()
