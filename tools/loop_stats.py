#!/usr/bin/env python3
"""Per-loop instruction counts of a gfx950 .s file (innermost loops).

Blocks carry the compiler's comment "in Loop: Header=BBk_n Depth=d" (or
"Loop Header: Depth=d" on the header itself) naming their innermost loop; the
instructions of every block of a loop are counted: VALU, SALU, vector memory,
LDS, waitcnt, and the IEEE-division / packed / mov subsets.

    python tools/loop_stats.py file.s [kernel-substring] [--min-loads N]
"""
import re
import sys
from collections import Counter


def parse(path, kpat=""):
    kernel = None
    loops = {}          # (kernel, header) -> Counter
    depth = {}
    cur = None
    with open(path) as f:
        lines = f.readlines()
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            kernel = m.group(1)
            cur = None
            continue
        if kernel is None or kpat not in kernel:
            continue
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", ln)
        if m:
            cur = None
            lab = m.group(1)
            mm = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", ln)
            if mm:
                cur = (kernel, "BB" + mm.group(1))
                depth[cur] = int(mm.group(2))
            else:
                # header: the marker is on a following comment line
                for j in range(i + 1, min(i + 4, len(lines))):
                    mm = re.search(r"Loop Header: Depth=(\d+)", lines[j])
                    if mm:
                        cur = (kernel, lab.lstrip(".").lstrip("L"))
                        depth[cur] = int(mm.group(1))
                        break
                    if not lines[j].lstrip().startswith(";"):
                        break
            continue
        if cur is None:
            continue
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        c = loops.setdefault(cur, Counter())
        c["total"] += 1
        if op.startswith("v_"):
            c["valu"] += 1
            if op.startswith("v_pk_"):
                c["pk"] += 1
            if op.startswith("v_mov"):
                c["mov"] += 1
            if op.startswith("v_div_") or op.startswith("v_rcp"):
                c["div/rcp"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("s_nop"):
            c["nop"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith(("global_load", "buffer_load")):
            c["vmem_ld"] += 1
        elif op.startswith(("global_store", "buffer_store")):
            c["vmem_st"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("scratch_"):
            c["scratch"] += 1
    return loops, depth


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    min_loads = 0
    if "--min-loads" in sys.argv:
        min_loads = int(sys.argv[sys.argv.index("--min-loads") + 1])
        args = [a for a in args if a != str(min_loads)]
    path = args[0]
    kpat = args[1] if len(args) > 1 else ""
    loops, depth = parse(path, kpat)
    keys = ("total", "valu", "pk", "mov", "div/rcp", "salu", "nop", "waitcnt", "vmem_ld", "lds", "scratch")
    for (k, h), c in loops.items():
        if c["vmem_ld"] < min_loads:
            continue
        print(f"{k[:60]:60s} {h:9s} d{depth[(k, h)]} " + " ".join(f"{x}={c[x]}" for x in keys))


if __name__ == "__main__":
    main()
