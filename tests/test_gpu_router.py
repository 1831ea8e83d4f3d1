"""Sharded engines + routing kernels on the GPU: two ranks share the box's one GPU
(two engines, shard 0/2 and 1/2), exchanging requests through gloo on the host. The
decisions must equal the single-process oracle on the global stream."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NS = 1_000_000
T0 = 1_700_000_000_000


def _trace(steps, world, n):
    import rl_amd
    rng = np.random.default_rng(7)
    total = steps * world * n
    ranks = np.minimum(rng.zipf(1.2, total), 100_000) - 1
    keys = rl_amd.mix64(ranks.astype(np.uint64))
    permits = rng.integers(1, 5, total).astype(np.int32)
    now = (T0 * NS + np.sort(rng.integers(0, 30_000 * NS, total))).astype(np.int64)
    lim = (ranks % 2).astype(np.uint16)                  # each key belongs to one limiter
    return keys, permits, now, lim


def _worker(rank, world, port, steps, n, out):
    import rl_amd
    from rl_amd.router import DeviceOps, Router
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = rl_amd.Engine(device=0, max_batch=4 * n, capacity=1 << 16, shard_index=rank,
                        shard_count=world)
    eng.add_limiter(rl_amd.TB, 50, 60000, 10.0)
    eng.add_limiter(rl_amd.SW, 30, 5000, 0.0)
    router = Router(DeviceOps(eng, world, dev, n), world, rank, exchange_device="cpu")
    keys, permits, now, lim = _trace(steps, world, n)
    res_a, res_r = [], []
    for s in range(steps):
        sl = slice((s * world + rank) * n, (s * world + rank + 1) * n)
        k = torch.from_numpy(keys[sl].view(np.int64).copy()).to(dev)
        p = torch.from_numpy(permits[sl].copy()).to(dev)
        t = torch.from_numpy(now[sl].copy()).to(dev)
        li = torch.from_numpy(lim[sl].view(np.int16).copy()).to(dev)
        a = torch.empty(n, dtype=torch.uint8, device=dev)
        r = torch.empty(n, dtype=torch.int64, device=dev)
        router.step(k, p, t, a, r, li)
        eng.sync()
        res_a.append(a.cpu().numpy())
        res_r.append(r.cpu().numpy())
    assert eng.last_status() == rl_amd.RL_OK
    np.savez(f"{out}.{rank}.npz", a=np.concatenate(res_a), r=np.concatenate(res_r))
    dist.destroy_process_group()


def test_two_shards_one_gpu(tmp_path):
    from oracle.coracle import COracle
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world, steps, n = 2, 3, 100_000
    out = str(tmp_path / "r")
    mp.spawn(_worker, args=(world, port, steps, n, out), nprocs=world, join=True)
    keys, permits, now, lim = _trace(steps, world, n)
    wa, wr, _, _ = COracle([[1, 50, 60000, 10.0], [0, 30, 5000, 0.0]]).run(
        keys, permits, now, lim, want_tokens=False)
    for rank in range(world):
        d = np.load(f"{out}.{rank}.npz")
        for st in range(steps):
            sl = slice((st * world + rank) * n, (st * world + rank + 1) * n)
            assert np.array_equal(d["a"][st * n:(st + 1) * n], wa[sl])
            assert np.array_equal(d["r"][st * n:(st + 1) * n], wr[sl])
