#!/usr/bin/env python3
"""Per-region timeline of the region stage for one bench config (GPU box): which regions
take longest, how many records/rounds they had, and when they started."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rl_amd  # noqa: E402
from bench import CONFIGS, T0_NS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="sw_zipf")
ap.add_argument("--batches", type=int, default=3)
ap.add_argument("--tune", action="append", default=[])
args = ap.parse_args()
cfg = CONFIGS[args.config]
n = cfg["batch"]
torch.cuda.set_device(0)
eng = rl_amd.Engine(device=0, max_batch=n, capacity=cfg["capacity"], stage_timing=True)
for l in cfg["limiters"]:
    eng.add_limiter(*l)
eng.tune("debug_regions", 1)
for kv in args.tune:
    k, v = kv.split("=")
    eng.tune(k, int(v))
dev = torch.device("cuda", 0)
keys = torch.empty(n, dtype=torch.int64, device=dev)
permits = torch.empty(n, dtype=torch.int32, device=dev)
now = torch.empty(n, dtype=torch.int64, device=dev)
allowed = torch.empty(n, dtype=torch.uint8, device=dev)
remaining = torch.empty(n, dtype=torch.int64, device=dev)
n_lim = len(cfg["limiters"])
lim = torch.empty(n, dtype=torch.int16, device=dev) if n_lim > 1 else None
nb = 1 << 24
for b in range(args.batches):
    eng.synth_trace(n, keys, permits, now, lim, seed=cfg["seed"], n_keys=cfg["n_keys"],
                    dist=cfg["dist"], zipf_s=cfg.get("zipf_s", 1.1), permits_max=cfg["permits_max"],
                    t0_ns=T0_NS, span_ns=cfg["span_ns"] * args.batches, index_base=b * n,
                    n_total=n * args.batches, n_limiters=n_lim)
    eng.execute_device(n, keys, permits, now, lim, None, allowed, remaining)
    eng.sync()
    st = eng.stage_times()
    d = eng.debug_region_times(nb)
    idx = np.nonzero(d[:, 1] > 0)[0]
    d = d[idx]
    # limiter of each region: limiters own consecutive power-of-two region ranges
    bases, acc = [], 0
    for _ in cfg["limiters"]:
        regions = -(-max(cfg["capacity"] * 2, rl_amd.REGION_SLOTS) // rl_amd.REGION_SLOTS)
        k = max((regions - 1).bit_length(), 3)
        bases.append(acc)
        acc += 1 << k
    lim_of = np.searchsorted(np.array(bases), idx, side="right") - 1
    t0 = d[:, 0].min()
    dur = (d[:, 1] - d[:, 0]) / 100.0          # us
    hot = (d[:, 3] >> np.uint64(63)) == 1
    rounds = d[:, 3] & np.uint64((1 << 63) - 1)
    print(f"batch {b}: region stage {st['region']:.2f} ms hot {st['hot_fill']:.2f} ms; "
          f"{len(d)} regions, {hot.sum()} hot; span {(d[:, 1].max() - t0) / 100:.0f} us")
    order = np.argsort(-dur)[:12]
    for i in order:
        rr = int(rounds[i])
        cyc = " ".join(f"{x / 1e6:6.2f}" for x in d[i, 4:7])
        w7 = int(d[i, 7])
        cyc2 = " ".join(f"{x / 1e6:6.2f}" for x in d[i, 8:11])
        what = (f"detail {rr & 0xFFFFFFFF:7d} changed {w7 & 0xFFFFFF:6d} "
                f"T1 updates {(rr >> 32) & 0xFFFF:6d} HOT Mcyc det/run/T1 {cyc} pre/pass1/pass2 {cyc2} "
                f"other-key recs {int(d[i, 11])} prefetched {int(d[i, 12])} build Mcyc {d[i, 13] / 1e6:.2f} "
                f"bisect lanes {int(d[i, 14])} SW run Mcyc setup/greedy/rem/commit "
                f"{' '.join(f'{x / 1e6:.2f}' for x in d[i, 15:19])} greedy steps {int(d[i, 19])} "
                f"WALK allows {int(d[i, 20])} finds {int(d[i, 21])} Mcyc find/walk "
                f"{d[i, 22] / 1e6:.2f} {d[i, 23] / 1e6:.2f} close/allow {d[i, 24] / 1e6:.2f} "
                f"{d[i, 25] / 1e6:.2f} block loads {int(d[i, 26])}"
                if hot[i] else f"rounds {rr:8d}")
        print(f"   dur {dur[i]:9.1f} us start {(d[i, 0] - t0) / 100:9.1f} us  lim {lim_of[i]} "
              f"recs {int(d[i, 2]):9d} {what}")
    late = np.argsort(-(d[:, 1].astype(np.int64)))[:6]
    print("   latest ends: " + "; ".join(
        f"{'hot' if hot[i] else 'normal'} recs {int(d[i, 2])} start {(d[i, 0] - t0) / 100:.0f} "
        f"end {(d[i, 1] - t0) / 100:.0f} us" for i in late))
    nh = ~hot
    ends = (d[nh, 1] - t0) / 100
    for q in ((0.5, 0.9, 0.99, 0.999, 1.0) if nh.any() else ()):
        print(f"   normal regions end quantile {q}: {np.quantile(ends, q):9.1f} us")
    print(f"   hot: details {int((rounds[hot] & np.uint64(0xFFFFFFFF)).sum())}, changes "
          f"{int((d[hot, 7] & np.uint64(0xFFFFFF)).sum())}, detail Mcyc {d[hot, 4].sum() / 1e6:.1f}, "
          f"pass1 Mcyc {d[hot, 9].sum() / 1e6:.1f}")
    print(f"   normal: sum dur {dur[nh].sum() / 1e3:.1f} ms, recs {int(d[nh, 2].sum())}, "
          f"rounds {int(rounds[nh].sum())}")
    if nh.any():
        dn = d[nh].astype(np.int64)
        load = (dn[:, 0] - dn[:, 4]) / 100.0
        strm = (dn[:, 5] - dn[:, 0]) / 100.0
        wb = (dn[:, 1] - dn[:, 5]) / 100.0
        for name, m in (("image", dn[:, 6] == 0), ("sparse", dn[:, 6] == 1)):
            if m.any():
                sl = np.maximum(1, (dn[m, 2] + 63) // 64).sum()
                print(f"   {name} regions {int(m.sum())}: mean us load {load[m].mean():.2f} stream "
                      f"{strm[m].mean():.2f} write-back {wb[m].mean():.2f}; recs/region "
                      f"{dn[m, 2].mean():.0f}; total wave-ms {(load[m] + strm[m] + wb[m]).sum() / 1e3:.0f}; "
                      f"per 64-record slice: rounds {(dn[m, 3] & ((1 << 62) - 1)).sum() / sl:.2f} "
                      f"greedy steps {dn[m, 7].sum() / sl:.2f} probe passes {dn[m, 8].sum() / sl:.2f}")
