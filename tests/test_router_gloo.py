"""The multi-GPU routing protocol (rl_amd.router.Router) under gloo, world_size 2, on
CPU: owner partition -> all-to-all -> per-shard decisions -> reverse all-to-all ->
unpermute must reproduce the single-process oracle on the global stream exactly.
Per-shard decisions use the CPU oracle here (test stand-in for the HIP engine)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rl_amd
from rl_amd.router import Router
from oracle.coracle import COracle

NS = 1_000_000
T0 = 1_700_000_000_000
LIMS = [[rl_amd.TB, 50, 60000, 10.0], [rl_amd.SW, 30, 5000, 0.0]]


class HostOps:
    def __init__(self, world):
        self.world = world
        self.o = COracle(LIMS)

    def partition(self, n, keys):
        own = rl_amd.owner_of(keys.numpy().view(np.uint64), self.world)
        self.perm = np.argsort(own, kind="stable")
        return np.bincount(own, minlength=self.world).tolist()

    def pack(self, n, keys, permits, now, limiter=None):
        return (keys[self.perm].clone(), permits[self.perm].clone(), now[self.perm].clone(),
                None if limiter is None else limiter[self.perm].clone())

    def recv_buffers(self, m, with_limiter=False):
        return (torch.empty(m, dtype=torch.int64), torch.empty(m, dtype=torch.int32),
                torch.empty(m, dtype=torch.int64),
                torch.empty(m, dtype=torch.int16) if with_limiter else None)

    def decide(self, m, k, p, t, lim=None):
        kk = k.numpy().view(np.uint64)
        lm = None if lim is None else lim.numpy().view(np.uint16)
        a, r, _, _ = self.o.run(kk, p.numpy(), t.numpy(), lm, None, want_tokens=False)
        return torch.from_numpy(r * 2 + a.astype(np.int64))

    def back_buffer(self, n):
        return torch.empty(n, dtype=torch.int64)

    def unpack(self, n, back, allowed, remaining):
        b = back.numpy()
        allowed.numpy()[self.perm] = (b & 1).astype(np.uint8)
        remaining.numpy()[self.perm] = b >> 1

    def sync(self):
        pass


def global_trace(steps, world, n):
    rng = np.random.default_rng(42)
    total = steps * world * n
    ranks = np.minimum(rng.zipf(1.3, total), 5000) - 1
    keys = rl_amd.mix64(ranks.astype(np.uint64))
    permits = rng.integers(1, 5, total).astype(np.int32)
    now = (T0 * NS + np.sort(rng.integers(0, 20_000 * NS, total))).astype(np.int64)
    lim = (ranks % len(LIMS)).astype(np.uint16)          # each key belongs to one limiter
    return keys, permits, now, lim


def _worker(rank, world, port, steps, n, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    keys, permits, now, lim = global_trace(steps, world, n)
    router = Router(HostOps(world), world, rank)
    got_a, got_r = [], []
    for s in range(steps):
        sl = slice((s * world + rank) * n, (s * world + rank + 1) * n)
        k = torch.from_numpy(keys[sl].view(np.int64).copy())
        p = torch.from_numpy(permits[sl].copy())
        t = torch.from_numpy(now[sl].copy())
        li = torch.from_numpy(lim[sl].view(np.int16).copy())
        a = torch.empty(n, dtype=torch.uint8)
        r = torch.empty(n, dtype=torch.int64)
        router.step(k, p, t, a, r, li)
        got_a.append(a.numpy().copy())
        got_r.append(r.numpy().copy())
    np.savez(f"{out_path}.{rank}.npz", a=np.concatenate(got_a), r=np.concatenate(got_r))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_router_matches_single_process_oracle(tmp_path, world):
    steps, n = 3, 3000
    out = str(tmp_path / "res")
    mp.spawn(_worker, args=(world, _free_port(), steps, n, out), nprocs=world, join=True)
    keys, permits, now, lim = global_trace(steps, world, n)
    wa, wr, _, _ = COracle(LIMS).run(keys, permits, now, lim, None, want_tokens=False)
    for rank in range(world):
        d = np.load(f"{out}.{rank}.npz")
        for s in range(steps):
            sl = slice((s * world + rank) * n, (s * world + rank + 1) * n)
            assert np.array_equal(d["a"][s * n:(s + 1) * n], wa[sl]), (rank, s)
            assert np.array_equal(d["r"][s * n:(s + 1) * n], wr[sl]), (rank, s)
