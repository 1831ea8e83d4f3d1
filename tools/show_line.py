#!/usr/bin/env python3
"""Print the headline and each extra config of a bench.py JSON line compactly."""
import json
import sys

d = json.load(open(sys.argv[1]))


def show(name, x):
    r = x["roofline"]
    print(f"{name:14s} {x['value']:.4g}/s {x['ms_per_step']:.3f} ms  frac {r['frac']:.4f}  "
          f"{x.get('parity', '')[:60]}  status {x.get('status')}")
    print("   stages", {k: round(v, 3) for k, v in x.get("stage_ms", {}).items()})
    print("   io_frac", {k: v["io_frac"] for k, v in r["kernels"].items()})


show("default", d)
for k in ("tb_uniform", "zipf_1b", "mixed_tenants"):
    if k in d:
        show(k, d[k])
if "config1" in d:
    c = d["config1"]
    print("config1", c["engine_value"], c["cpu_port_value"], c["parity"])
print("footprint", d.get("hbm_footprint_gb"))
