#!/usr/bin/env python3
"""Repro (GPU box): bench.py's 2-rank python-router path on one GPU (as the router test),
with each owner engine's received batches dumped and replayed in a fresh engine."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, world, port, cfg_name, steps, n, out):
    import bench
    import rl_amd
    from rl_amd.router import DeviceOps, Router
    from test_gpu_router import _bench_slice
    cfg = bench.CONFIGS[cfg_name]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = rl_amd.Engine(device=0, max_batch=world * n, capacity=1 << 22, shard_index=rank,
                        shard_count=world)
    for l in cfg["limiters"]:
        eng.add_limiter(*l)
    slices = [_bench_slice(eng, cfg, s, rank, world, steps, n) for s in range(steps)]
    eng.sync()
    ops = DeviceOps(eng, world, dev, n)
    dumps = []
    orig = ops.decide_return

    def spy(m, k, p, t, lim, width, src_counts, wide=False):
        dumps.append([x[:m].cpu().numpy() for x in (k, p, t)] + [None if lim is None else lim[:m].cpu().numpy()])
        r = orig(m, k, p, t, lim, width, src_counts, wide)
        st = eng.last_status()
        s = eng.stats()
        print(f"rank {rank} batch {len(dumps) - 1}: m {m} wide {wide} status {rl_amd.strerror(st)} "
              f"cap_err {s['capacity_errors']}", flush=True)
        return r
    ops.decide_return = spy
    router = Router(ops, world, rank, exchange_device="cpu")
    for s in range(steps):
        k, p, t, li = slices[s]
        a = torch.empty(n, dtype=torch.uint8, device=dev)
        r = torch.empty(n, dtype=torch.int64, device=dev)
        router.step(k, p, t, a, r, li)
        eng.sync()
    try:
        router.finish()
    except Exception as ex:  # noqa: BLE001
        print(f"rank {rank} finish: {ex}", flush=True)
    np.savez(f"{out}.{rank}.npz", **{f"b{i}_{j}": x for i, d in enumerate(dumps) for j, x in enumerate(d)
                                       if x is not None})
    dist.destroy_process_group()


if __name__ == "__main__":
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "mixed_tenants"
    world, steps, n = 2, 2, 1 << 21
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = "gpurun_out/flow"
    mp.spawn(worker, args=(world, port, cfg_name, steps, n, out), nprocs=world, join=True)
    import bench
    import rl_amd
    from oracle.coracle import COracle
    cfg = bench.CONFIGS[cfg_name]
    torch.cuda.set_device(0)
    for rank in range(world):
        z = np.load(f"{out}.{rank}.npz")
        for tune in ([], [("route", 0)]):
            e = rl_amd.Engine(device=0, max_batch=world * n, capacity=1 << 22, shard_index=rank,
                              shard_count=world)
            for l in cfg["limiters"]:
                e.add_limiter(*l)
            for k, v in tune:
                e.tune(k, v)
            for b in range(steps):
                k, p, t = z[f"b{b}_0"], z[f"b{b}_1"], z[f"b{b}_2"]
                li = z[f"b{b}_3"] if f"b{b}_3" in z else None
                a, r, _, st = e.execute(k.view(np.uint64), p, t, None if li is None else li.view(np.uint16), None)
                print(f"replay rank {rank} {tune} batch {b}: m {len(k)} status {rl_amd.strerror(st)} "
                      f"cap_err {e.stats()['capacity_errors']} min now {t.min()} max now {t.max()}", flush=True)
            e.close()
