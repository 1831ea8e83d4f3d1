#!/usr/bin/env python3
"""Print the basic blocks of one kernel in a hipcc --save-temps .s file: label, number of
VALU / SALU / LDS / VMEM instructions, and branch targets (loops show as back edges)."""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\d+_\d+|" + re.escape(name) + "):", l)
    if m:
        cur = {"label": m.group(1)[:20], "v": 0, "s": 0, "ds": 0, "vm": 0, "f64": 0, "br": [], "wait": 0}
        blocks.append(cur)
        continue
    t = l.strip().split()
    if not t or t[0].startswith((";", ".")) or cur is None:
        continue
    op = t[0]
    if op.startswith("v_"):
        cur["v"] += 1
        cur["f64"] += "_f64" in op
    elif op.startswith("s_waitcnt"):
        cur["wait"] += 1
    elif op.startswith("s_cbranch") or op == "s_branch":
        cur["br"].append(t[1][:14])
        cur["s"] += 1
    elif op.startswith("s_"):
        cur["s"] += 1
    elif op.startswith("ds_"):
        cur["ds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cur["vm"] += 1
for b in blocks:
    print(f"{b['label']:20s} v={b['v']:4d} f64={b['f64']:3d} s={b['s']:4d} ds={b['ds']:3d} vm={b['vm']:2d} "
          f"w={b['wait']:2d} -> {' '.join(b['br'])}")
