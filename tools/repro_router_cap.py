#!/usr/bin/env python3
"""Repro (GPU box): the owner-1 engine of the 2-shard mixed_tenants router test, fed the
owner's merged batches directly (no exchange), routing on / off; status, stats and parity."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rl_amd  # noqa: E402
from oracle.coracle import COracle  # noqa: E402
from test_gpu_router import _bench_slice  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "mixed_tenants"
cfg = bench.CONFIGS[cfg_name]
world, steps, n = 2, 2, 1 << 21
torch.cuda.set_device(0)
gen = rl_amd.Engine(device=0, max_batch=n, capacity=1 << 10)
batches = []
for st in range(steps):
    parts = []
    for rank in range(world):
        xs = _bench_slice(gen, cfg, st, rank, world, steps, n)
        gen.sync()
        parts.append([x.cpu().numpy() for x in xs])
    batches.append([np.concatenate([p[i] for p in parts]) for i in range(4)])
gen.close()
owners = [int(sys.argv[2])] if len(sys.argv) > 2 else range(world)
for owner in owners:
    sel = [rl_amd.owner_of(b[0].view(np.uint64), world) == owner for b in batches]
    obs = [[x[m] for x in b] for b, m in zip(batches, sel)]
    for tune in ([], [("route", 0)]):
        e = rl_amd.Engine(device=0, max_batch=world * n, capacity=1 << 22, shard_index=owner,
                          shard_count=world)
        for l in cfg["limiters"]:
            e.add_limiter(*l)
        for k, v in tune:
            e.tune(k, v)
        got = [[], []]
        for st, b in enumerate(obs):
            a, r, t, s = e.execute(b[0].view(np.uint64), b[1], b[2], b[3].view(np.uint16), None)
            stt = e.stats()
            print(f"owner {owner} {tune} step {st}: n {len(a)} status {rl_amd.strerror(s)} "
                  f"cap_err {stt['capacity_errors']} distinct {stt['distinct_keys']}", flush=True)
            got[0].append(a); got[1].append(r)
        e.close()
        keys = np.concatenate([b[0] for b in obs]).view(np.uint64)
        o = COracle(cfg["limiters"], nthreads=16)
        wa, wr, _, _ = o.run(keys, np.concatenate([b[1] for b in obs]), np.concatenate([b[2] for b in obs]),
                             np.concatenate([b[3] for b in obs]).view(np.uint16), want_tokens=False)
        o.close()
        ga, gr = np.concatenate(got[0]), np.concatenate(got[1])
        bad = np.nonzero((ga != wa) | (gr != wr))[0]
        print(f"owner {owner} {tune}: {len(bad)} mismatches (first {bad[:5]})", flush=True)
