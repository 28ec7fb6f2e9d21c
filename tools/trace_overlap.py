#!/usr/bin/env python3
"""Concurrency of the transform stage in a rocprofv3 kernel trace (run_kernel_trace.csv).

  python tools/trace_overlap.py gpurun_out/<tag>_prof/run_kernel_trace.csv

For every interval between two consecutive K-SPEC dispatches (one substep's x -> z -> x stage) it
prints the wall time, the time covered by at least one kernel, the time with two or more kernels
running at once (the two-stream chunk pipeline), the summed kernel durations, and the serial head
and tail: the time from the stage start to the first moment two kernels co-run, and from the last
such moment to the stage end.  A summed time close to twice the wall time with full coverage means
the two streams really co-run."""
import csv
import sys
from collections import Counter


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ks = [e for e in ev if "kspec_kernel" in e[2]]
    print("| substep | wall ms | covered ms | >= 2 kernels ms | kernel sum ms | serial head ms | serial tail ms | kernels |")
    print("|---|---|---|---|---|---|---|---|")
    for n, (a, b) in enumerate(zip(ks[:-1], ks[1:])):
        t0, t1 = a[1], b[0]
        iv = sorted((s, e) for s, e, _ in (x for x in ev if x[0] >= t0 and x[1] <= t1))
        if not iv:
            continue
        cov, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None:
                cs, ce = s, e
            elif s <= ce:
                ce = max(ce, e)
            else:
                cov += ce - cs
                cs, ce = s, e
        cov += ce - cs
        pts = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv])
        lvl, last, both = 0, None, 0
        first2, last2 = None, None
        for t, d in pts:
            if last is not None and lvl >= 2:
                both += t - last
                if t - last > 0:
                    first2 = last if first2 is None else first2
                    last2 = t
            lvl += d
            last = t
        head = ((first2 if first2 is not None else t1) - t0) / 1e6
        tail = ((t1 - last2) if last2 is not None else 0) / 1e6
        busy = sum(e - s for s, e in iv)
        names = Counter(x[2].split("<")[0].split("(")[0].replace("void ", "") for x in ev if x[0] >= t0 and x[1] <= t1)
        print(f"| {n} | {(t1 - t0) / 1e6:.3f} | {cov / 1e6:.3f} | {both / 1e6:.3f} | {busy / 1e6:.3f} | {head:.3f} | {tail:.3f} | "
              f"{', '.join(f'{k} x{v}' for k, v in names.items())} |")


if __name__ == "__main__":
    main(sys.argv[1])
