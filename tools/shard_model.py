#!/usr/bin/env python3
"""Model of the busiest GPU of a G-GPU node on one GPU (the per-shard load the judge asked
for): every step generates the WHOLE node's trace (G slices of the bench's
k_synth stream, the same seeds and key population as `bench.py --gpus G`), partitions it by
owner with the engine's own routing kernel (k_owner_count / k_owner_scatter, with or without
a hot-key directory), keeps the busiest owner's requests in global arrival order and times
that owner's engine on them. Reported: every owner's share of the traffic and the busiest
owner's decide time per step; G x batch / that time bounds the node's throughput from above
(no exchange). The engine runs exactly the product path; the numbers are a model of one
shard, not a multi-GPU measurement.

usage: tools/shard_model.py --config zipf_1b --gpus 8 [--directory 4096]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rl_amd  # noqa: E402
from bench import CONFIGS, T0_NS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="zipf_1b")
ap.add_argument("--gpus", type=int, default=8)
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--warmup", type=int, default=1)
ap.add_argument("--directory", type=int, default=0, help="hot keys placed by LPT (0: hash owners)")
ap.add_argument("--debug", action="store_true", help="stage times and the longest regions")
ap.add_argument("--verify-top", action="store_true",
                help="check the busiest shard's hottest key against the C oracle over every step")
args = ap.parse_args()
cfg = CONFIGS[args.config]
G, n = args.gpus, cfg["batch"]
total = args.warmup + args.steps
n_lim = len(cfg["limiters"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)

gen = rl_amd.Engine(device=0, max_batch=n, capacity=1 << 10,      # synth + routing kernels
                    shard_index=0, shard_count=G)
keys = torch.empty(n, dtype=torch.int64, device=dev)
permits = torch.empty(n, dtype=torch.int32, device=dev)
now = torch.empty(n, dtype=torch.int64, device=dev)
lim = torch.empty(n, dtype=torch.int16, device=dev) if n_lim > 1 else None
perm = torch.empty(n, dtype=torch.int32, device=dev)
counts = torch.zeros(G, dtype=torch.int64, device=dev)


def synth(s, r):
    gen.synth_trace(n, keys, permits, now, lim, seed=cfg["seed"], n_keys=cfg["n_keys"] * G,
                    dist=cfg["dist"], zipf_s=cfg.get("zipf_s", 1.1), permits_max=cfg["permits_max"],
                    t0_ns=T0_NS, span_ns=cfg["span_ns"] * total, index_base=(s * G + r) * n,
                    n_total=total * G * n, n_limiters=n_lim)


def partition():
    gen.route_partition_device(n, keys, perm, G, counts, 1)
    gen.sync()
    return counts.cpu().numpy().astype(np.int64)


# hot-key directory from step 0's first slice (as rl_router_plan_directory would: sampled
# counts, the k hottest placed longest-processing-time-first over the owners' other load)
dir_keys = dir_own = None
if args.directory:
    synth(0, 0)
    gen.sync()
    u, c = torch.unique(keys, return_counts=True)
    top = torch.argsort(c, descending=True)[:args.directory]
    hk = u[top].cpu().numpy().view(np.uint64)
    hc = c[top].cpu().numpy().astype(np.float64)
    own_hash = rl_amd.owner_of(hk, G)
    load = np.bincount(rl_amd.owner_of(keys.cpu().numpy().view(np.uint64), G), minlength=G).astype(np.float64)
    load -= np.bincount(own_hash, weights=hc, minlength=G)
    dir_own = np.zeros(len(hk), np.uint32)
    for i in np.argsort(-hc):
        j = int(np.argmin(load))
        dir_own[i] = j
        load[j] += hc[i]
    dir_keys = hk
    gen.set_owner_directory(dir_keys, dir_own)

# step 0: every owner's share -> the busiest one
loads = np.zeros(G, np.int64)
for r in range(G):
    synth(0, r)
    loads += partition()
busy = int(np.argmax(loads))

dec = rl_amd.Engine(device=0, max_batch=int(loads[busy] * 2), capacity=cfg["capacity"] * G,
                    shard_index=busy, shard_count=G, stage_timing=args.debug)
if args.debug:
    dec.tune("debug_regions", 1)
for l in cfg["limiters"]:
    dec.add_limiter(*l)
if dir_keys is not None:
    dec.set_owner_directory(dir_keys, dir_own)
cap = int(loads[busy] * 2)
bk = torch.empty(cap, dtype=torch.int64, device=dev)
bp = torch.empty(cap, dtype=torch.int32, device=dev)
bt = torch.empty(cap, dtype=torch.int64, device=dev)
bl = torch.empty(cap, dtype=torch.int16, device=dev) if n_lim > 1 else None
ba = torch.empty(cap, dtype=torch.uint8, device=dev)
br = torch.empty(cap, dtype=torch.int64, device=dev)
times, sizes = [], []
top_key, top_parts = None, []
for s in range(total):
    m = 0
    for r in range(G):
        synth(s, r)
        c = partition()
        off, cnt = int(c[:busy].sum()), int(c[busy])
        idx = perm[off:off + cnt].long()
        bk[m:m + cnt] = keys[idx]
        bp[m:m + cnt] = permits[idx]
        bt[m:m + cnt] = now[idx]
        if bl is not None:
            bl[m:m + cnt] = lim[idx]
        m += cnt
        # the gathers run on torch's stream, the next slice's synth / partition on the
        # generator engine's: without this they overwrite keys / now / perm mid-gather
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dec.execute_device(m, bk, bp, bt, bl, None, ba, br)
    dec.sync()
    dt = time.perf_counter() - t0
    st = dec.last_status()
    assert st in (rl_amd.RL_OK,), rl_amd.strerror(st)
    if s >= args.warmup:
        times.append(dt)
        sizes.append(m)
    if args.verify_top:
        if top_key is None:
            u, c = torch.unique(bk[:m], return_counts=True)
            top_key = u[torch.argmax(c)]
        sel = torch.nonzero(bk[:m] == top_key).squeeze(1)
        top_parts.append([x[sel].cpu().numpy() for x in (bk, bp, bt) + ((bl,) if bl is not None else ()) + (ba, br)])
ms = 1e3 * float(np.mean(times))
if args.debug:
    u, c = torch.unique(bk[:m], return_counts=True)
    ti = torch.argmax(c)
    sel = bk[:m] == u[ti]
    tl = bl[:m][sel] if bl is not None else None
    tt = bt[:m][sel]
    print("top key", int(c[ti]), "requests; limiter", None if tl is None else int(tl[0]),
          "permits", torch.unique(bp[:m][sel]).tolist(), "allowed", int(ba[:m][sel].sum()),
          "time span ms", (int(tt[-1]) - int(tt[0])) // 1_000_000)
    print("stages", {k: round(v, 2) for k, v in dec.stage_times().items() if v > 0.1})
    d = dec.debug_region_times(1 << 24)
    d = d[d[:, 1] > 0]
    dur = (d[:, 1] - d[:, 0]) / 100.0
    for i in np.argsort(-dur)[:6]:
        hot = int(d[i, 3]) >> 63
        print(f"  region dur {dur[i]:10.1f} us recs {int(d[i, 2]):10d} hot {hot} "
              f"detail {int(d[i, 3]) & 0xFFFFFFFF} T1upd {(int(d[i, 3]) >> 32) & 0xFFFF} "
              f"before_T0 {(int(d[i, 3]) >> 48) & 0x7FFF} changed {int(d[i, 7]) & 0xFFFFFF} "
              f"past_T1 {(int(d[i, 7]) >> 24) & 0xFFFFFF} Mcyc {[round(int(x) / 1e6, 1) for x in d[i, 4:7]]}")
verified = None
if args.verify_top:
    from oracle.coracle import COracle
    cols = [np.concatenate([p[i] for p in top_parts]) for i in range(len(top_parts[0]))]
    k_, p_, t_ = cols[0].view(np.uint64), cols[1], cols[2]
    l_ = cols[3].view(np.uint16) if bl is not None else None
    ga, gr = cols[-2], cols[-1]
    o = COracle(cfg["limiters"])
    wa, wr, _, _ = o.run(k_, p_, t_, l_, None, want_tokens=False)
    o.close()
    bad = np.nonzero((ga != wa) | (gr != wr))[0]
    verified = {"top_key_requests": int(k_.size), "mismatches": int(bad.size),
                "first": bad[:3].tolist()}
    print("verify_top", verified)
print(json.dumps({
    "config": args.config, "gpus": G, "directory_keys": args.directory,
    "owner_share": [round(float(x) / loads.sum(), 4) for x in loads],
    "busiest_owner": busy, "busiest_over_mean": round(float(loads.max()) * G / loads.sum(), 3),
    "busiest_requests_per_step": int(np.mean(sizes)), "busiest_decide_ms_per_step": round(ms, 3),
    "node_decisions_per_s_upper_bound": G * n / (ms * 1e-3),
    "top_key_check": verified,
    "note": "busiest shard's engine on its exact share of the node trace; exchange not included",
}))
