#!/usr/bin/env python3
"""Aggregate rocprofv3 counter_collection.csv files per kernel (sum over dispatches)."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r.get("Dispatch_Id", ""))
for k, c in agg.items():
    n = max(1, len(calls[k]))
    print(f"== {k}  dispatches={n}")
    for name, v in sorted(c.items()):
        print(f"   {name:24s} {v / n:16.4g}")
