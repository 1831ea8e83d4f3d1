#!/usr/bin/env python3
"""Pass-0 bin sizes and stage times of a bench config for several group_bits (k_group's
pass-0 high digit): the largest normal bin bounds k_group (one workgroup per bin).
usage: tools/group_probe.py [--config sw_zipf] [--bits 11,12,13] [--steps 6]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rl_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="sw_zipf")
ap.add_argument("--bits", default="11,12,13")
ap.add_argument("--steps", type=int, default=6)
ap.add_argument("--tune", action="append", default=[])
a = ap.parse_args()
cfg = bench.CONFIGS[a.config]
n = cfg["batch"]
dev = torch.device("cuda", 0)
for gb in [int(x) for x in a.bits.split(",")]:
    eng = rl_amd.Engine(device=0, max_batch=n, capacity=cfg["capacity"], stage_timing=False)
    for l in cfg["limiters"]:
        eng.add_limiter(*l)
    eng.tune("group_bits", gb)
    for kv in a.tune:
        k, v = kv.split("=")
        eng.tune(k, int(v))
    inputs = bench.make_inputs(eng, cfg, n, 1, 0, a.steps, dev)
    al = torch.empty(n, dtype=torch.uint8, device=dev)
    rem = torch.empty(n, dtype=torch.int64, device=dev)
    for s in range(a.steps):
        if s == 2:
            eng.tune("stage_timing", 1)
        k, p, t, li = inputs[s]
        eng.execute_device(n, k, p, t, li, None, al, rem)
    st = eng.stage_times()
    bt = eng.debug_bin_totals()
    lo = 1 << gb
    nb = bt[:lo].astype(np.int64)
    print(f"group_bits {gb}: normal bins {lo}, records {nb.sum()}, mean {nb.mean():.0f}, "
          f"p99 {np.percentile(nb, 99):.0f}, max {nb.max()}, routed {bt[lo:lo + 2048].sum()}; "
          f"status {rl_amd.strerror(eng.last_status())}", flush=True)
    print("   ", {k: round(v, 3) for k, v in st.items() if v > 0.01}, flush=True)
    eng.close()
    del inputs
    torch.cuda.empty_cache()
