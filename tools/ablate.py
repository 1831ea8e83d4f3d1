#!/usr/bin/env python3
"""Interleaved A/B timing of measurement-only kernel variants (rl_tune "ablate") in ONE
process on the bench workload. Prints per-stage median ms for each variant."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))
import torch  # noqa: E402

import rl_amd  # noqa: E402
from bench import CONFIGS, NS, T0_NS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="tb_uniform")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--variants", default="ablate=0/ablate=256/ablate=512/ablate=1024",
                help="'/'-separated variants, each a ','-separated list of rl_tune key=value")
args = ap.parse_args()
cfg = CONFIGS[args.config]
n = cfg["batch"]
torch.cuda.set_device(0)
eng = rl_amd.Engine(device=0, max_batch=n, capacity=cfg["capacity"], stage_timing=True)
for l in cfg["limiters"]:
    eng.add_limiter(*l)
dev = torch.device("cuda", 0)
keys = torch.empty(n, dtype=torch.int64, device=dev)
permits = torch.empty(n, dtype=torch.int32, device=dev)
now = torch.empty(n, dtype=torch.int64, device=dev)
eng.synth_trace(n, keys, permits, now, None, seed=cfg["seed"], n_keys=cfg["n_keys"],
                dist=cfg["dist"], zipf_s=cfg.get("zipf_s", 1.1), permits_max=cfg["permits_max"],
                t0_ns=T0_NS, span_ns=cfg["span_ns"], n_total=n)
allowed = torch.empty(n, dtype=torch.uint8, device=dev)
remaining = torch.empty(n, dtype=torch.int64, device=dev)
variants = args.variants.split("/")


DEFAULTS = {"ablate": 0, "upsweep_per_cu": 0, "scatter_per_cu": 0,
            "unpermute_per_cu": 0, "hot_threshold": 16384}


def apply(v):
    for k, x in DEFAULTS.items():          # every variant starts from the defaults
        eng.tune(k, x)
    for kv in v.split(","):
        k, x = kv.split("=")
        eng.tune(k, int(x))



res = {v: {} for v in variants}
for v in variants:                                  # warm every variant once
    apply(v)
    eng.execute_device(n, keys, permits, now, None, None, allowed, remaining)
eng.stage_times()
for r in range(args.rounds):
    for v in variants:
        apply(v)
        eng.execute_device(n, keys, permits, now, None, None, allowed, remaining)
        st = eng.stage_times()
        for k, ms in st.items():
            res[v].setdefault(k, []).append(ms)
eng.tune("ablate", 0)
out = {}
for v in variants:
    out[v] = {k: round(statistics.median(x), 4) for k, x in res[v].items()
              if k in ("upsweep0", "scan0", "scatter0", "region", "unpermute", "total")}
    print(v, json.dumps(out[v]))
