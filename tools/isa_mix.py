#!/usr/bin/env python3
"""Static instruction mix of the kernels in a gfx950 assembly file (hipcc -S --cuda-device-only),
per kernel and per basic block, to see where a kernel's VALU / LDS / VMEM instructions are.

  python tools/isa_mix.py kernels.s [name-substring] [--blocks]
"""
import collections
import re
import sys


def classify(op: str) -> str:
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main() -> None:
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    blocks = "--blocks" in sys.argv
    funcs, cur, blk = {}, None, None
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            funcs[cur] = collections.OrderedDict()
            blk = "entry"
            funcs[cur][blk] = []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        m = re.match(r"^(\.LBB\w+):", line)
        if m:
            blk = m.group(1)
            funcs[cur][blk] = []
            continue
        s = line.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        funcs[cur][blk].append(s.split()[0])
    for f, bbs in funcs.items():
        if pat not in f:
            continue
        tot = collections.Counter()
        for ops in bbs.values():
            for op in ops:
                tot[classify(op)] += 1
                tot[op] += 1
        print(f[:110])
        print("  total:", {k: tot[k] for k in ("valu", "lds", "vmem", "salu", "wait")})
        top = [(k, v) for k, v in tot.most_common(60) if k not in ("valu", "lds", "vmem", "salu", "wait", "other")]
        print("  top ops:", top[:40])
        if blocks:
            for b, ops in bbs.items():
                c = collections.Counter(classify(o) for o in ops)
                if len(ops) > 20:
                    print(f"   {b:24s} n={len(ops):5d} valu={c['valu']:5d} lds={c['lds']:4d} vmem={c['vmem']:4d} "
                          f"salu={c['salu']:4d} wait={c['wait']:4d}")


if __name__ == "__main__":
    main()
