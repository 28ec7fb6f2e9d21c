#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of the transform stage in a rocprofv3 kernel trace.

  python tools/trace_gaps.py gpurun_out/<tag>_prof/run_kernel_trace.csv [skip_substeps]

Between two consecutive K-SPEC dispatches (one substep's x -> z -> x stage) the kernels are merged
into busy intervals over ALL queues; a gap is time inside the stage with no kernel running.  Per
hardware queue it also prints the gaps between a kernel's end and the next kernel on the same
queue (a chunk's xb -> zphys -> xf chain on one stream).  Prints median / p90 / total gap per
substep and the stage's wall and kernel-covered time.  The first `skip_substeps` stages (warm-up,
graph capture) are dropped (default 3).

  --segments name:n,name:n,...  label consecutive stages (after the skipped ones) and print one
                                summary line per label: e.g. bench.py --steps 3 --warmup 1 at P > 1
                                is "eager:3,graph:9,phase:9" (the eager warm-up step, three replayed
                                step graphs, then bench's eager per-phase-event steps)."""
import csv
import statistics
import sys
from collections import defaultdict


def pct(v, q):
    s = sorted(v)
    return s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))] if s else float("nan")


def main(path: str, skip: int = 3, segments=None) -> None:
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    ks = [e for e in ev if "kspec_kernel" in e[2]]
    print("| substep | wall ms | covered ms | idle ms | all-queue gaps: n / median / p90 us | same-queue gaps: n / median / p90 us |")
    print("|---|---|---|---|---|---|")
    tot_wall = tot_idle = 0.0
    stages = []  # (wall, covered, all-queue gaps, same-queue gaps) per stage
    for n, (a, b) in enumerate(zip(ks[:-1], ks[1:])):
        if n < skip:
            continue
        t0, t1 = a[1], b[0]
        iv = [x for x in ev if x[0] >= t0 and x[1] <= t1]
        if not iv:
            continue
        gaps, cov = [], 0
        cs, ce = iv[0][0], iv[0][1]
        if cs > t0:
            gaps.append(cs - t0)
        for s, e, _, _ in iv[1:]:
            if s <= ce:
                ce = max(ce, e)
            else:
                cov += ce - cs
                gaps.append(s - ce)
                cs, ce = s, e
        cov += ce - cs
        if t1 > ce:
            gaps.append(t1 - ce)
        perq = defaultdict(list)
        for s, e, _, q in iv:
            perq[q].append((s, e))
        qg = []
        for q, l in perq.items():
            l.sort()
            qg += [max(0, l[i + 1][0] - l[i][1]) for i in range(len(l) - 1)]
        wall = (t1 - t0) / 1e6
        idle = wall - cov / 1e6
        tot_wall += wall
        tot_idle += idle
        stages.append((wall, cov / 1e6, gaps, qg))
        print(f"| {n} | {wall:.3f} | {cov / 1e6:.3f} | {idle:.3f} | {len(gaps)} / {pct(gaps, 0.5) / 1e3:.1f} / "
              f"{pct(gaps, 0.9) / 1e3:.1f} | {len(qg)} / {pct(qg, 0.5) / 1e3:.1f} / {pct(qg, 0.9) / 1e3:.1f} |")
    if segments:
        print("\n| stages | n | wall ms / stage | covered ms / stage | all-queue gaps: n / median / p90 us | same-queue gaps: median / p90 us |")
        print("|---|---|---|---|---|---|")
        i = 0
        for name, cnt in segments:
            sel = stages[i:i + cnt]
            i += cnt
            if not sel:
                continue
            g = [x for s in sel for x in s[2]]
            q = [x for s in sel for x in s[3]]
            print(f"| {name} | {len(sel)} | {statistics.mean(s[0] for s in sel):.3f} | {statistics.mean(s[1] for s in sel):.3f} | "
                  f"{len(g)} / {pct(g, 0.5) / 1e3:.1f} / {pct(g, 0.9) / 1e3:.1f} | {pct(q, 0.5) / 1e3:.1f} / {pct(q, 0.9) / 1e3:.1f} |")
    if tot_wall:
        print(f"\ntotal: stage wall {tot_wall:.3f} ms, idle {tot_idle:.3f} ms ({100 * tot_idle / tot_wall:.1f} %)")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--segments")]
    segs = None
    for a in sys.argv[1:]:
        if a.startswith("--segments="):
            segs = [(x.split(":")[0], int(x.split(":")[1])) for x in a.split("=", 1)[1].split(",")]
    main(args[0], int(args[1]) if len(args) > 1 else 3, segs)
