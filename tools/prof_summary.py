#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory: per-kernel average time (kernel trace)
and per-launch counter means (FETCH_SIZE/WRITE_SIZE in KB as rocprofv3 reports them)."""
import collections
import csv
import json
import sys

base = sys.argv[1].rstrip("/") + "/"
out = {"kernels": {}, "counters": {}}
for r in csv.DictReader(open(base + "trace/trace_kernel_stats.csv")):
    out["kernels"][r["Name"]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                 "min_us": float(r["MinNs"]) / 1e3}
for f in ("fetch", "write", "tcc", "sq"):
    try:
        rows = list(csv.DictReader(open(f"{base}{f}/{f}_counter_collection.csv")))
    except FileNotFoundError:
        continue
    d = collections.defaultdict(list)
    for r in rows:
        d[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in d.items():
        out["counters"].setdefault(k, {})[c] = sum(v) / len(v)
if len(sys.argv) > 2 and sys.argv[2] == "--json":
    print(json.dumps(out, indent=1))
else:
    for k, v in sorted(out["kernels"].items(), key=lambda x: -x[1]["avg_us"]):
        if "rocclr" in k:
            continue
        c = out["counters"].get(k, {})
        extra = " ".join(f"{n}={c[n]:.3g}" for n in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum",
                         "TCC_MISS_sum", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                         "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAVES") if n in c)
        print(f"{k[:48]:48s} {v['avg_us']:9.1f}us  {extra}")
