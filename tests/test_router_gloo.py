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


_NP_W = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}
_NP_U = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


class HostOps:
    def __init__(self, world):
        self.world = world
        self.o = COracle(LIMS)

    def partition(self, n, keys):
        own = rl_amd.owner_of(keys.numpy().view(np.uint64), self.world)
        self.perm = np.argsort(own, kind="stable")
        return np.bincount(own, minlength=self.world).tolist()

    def pack(self, n, keys, permits, now, limiter=None):
        self.packs_wide = getattr(self, "packs_wide", 0) + 1
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

    # compact wire layout: the same encoding as k_route_pack_wire / k_route_unwire
    def result_width(self):
        top = (max(l[1] for l in LIMS) + 3) * 2 + 1
        return 1 if top < 256 else 2 if top < 65536 else 4 if top < 2**32 else 8

    def pack_wire(self, n, keys, permits, now, limiter=None):
        t = now.numpy()
        base = int(np.floor_divide(t[0], NS)) - 2**31 if n else 0
        rel = np.floor_divide(t[self.perm], NS) - base
        ovf = int(((rel < 0) | (rel > 0xFFFFFFFF)).any())
        w1 = (permits.numpy()[self.perm].view(np.uint32).astype(np.uint64) << np.uint64(32)) | \
            (rel.astype(np.uint64) & np.uint64(0xFFFFFFFF))
        wire = np.stack([keys.numpy()[self.perm], w1.view(np.int64)], 1)
        self.packs_wire = getattr(self, "packs_wire", 0) + 1
        return (torch.from_numpy(wire.copy()),
                None if limiter is None else limiter[self.perm].clone(),
                torch.tensor([base, ovf], dtype=torch.int64))

    def wire_recv_buffers(self, m, with_limiter=False):
        return (torch.empty((m, 2), dtype=torch.int64),
                torch.empty(m, dtype=torch.int16) if with_limiter else None)

    def unwire(self, m, wire, bases, counts):
        w = wire.numpy()
        w1 = w[:, 1].view(np.uint64)
        p = (w1 >> np.uint64(32)).astype(np.uint32).view(np.int32)
        rel = (w1 & np.uint64(0xFFFFFFFF)).astype(np.int64)
        t = (np.repeat(np.asarray(bases, np.int64), counts) + rel) * NS
        return torch.from_numpy(w[:, 0].copy()), torch.from_numpy(p.copy()), torch.from_numpy(t)

    def decide_packed(self, m, k, p, t, lim, width):
        kk = k.numpy().view(np.uint64)
        lm = None if lim is None else lim.numpy().view(np.uint16)
        a, r, _, _ = self.o.run(kk, p.numpy(), t.numpy(), lm, None, want_tokens=False)
        v = ((r + 3) << 1) | a.astype(np.int64)
        return torch.from_numpy(v.astype(_NP_W[width]))

    def back_buffer_packed(self, n, width):
        return torch.from_numpy(np.empty(n, _NP_W[width]))

    def unpack_packed(self, n, back, width, allowed, remaining):
        v = back.numpy().view(_NP_U[width]).astype(np.int64)
        allowed.numpy()[self.perm] = (v & 1).astype(np.uint8)
        remaining.numpy()[self.perm] = (v >> 1) - 3


    def unpack(self, n, back, allowed, remaining):
        b = back.numpy()
        allowed.numpy()[self.perm] = (b & 1).astype(np.uint8)
        remaining.numpy()[self.perm] = b >> 1

    def sync(self):
        pass


def global_trace(steps, world, n, span_ms=20_000):
    rng = np.random.default_rng(42)
    total = steps * world * n
    ranks = np.minimum(rng.zipf(1.3, total), 5000) - 1
    keys = rl_amd.mix64(ranks.astype(np.uint64))
    permits = rng.integers(1, 5, total).astype(np.int32)
    now = (T0 * NS + np.sort(rng.integers(0, span_ms * NS, total))).astype(np.int64)
    lim = (ranks % len(LIMS)).astype(np.uint16)          # each key belongs to one limiter
    return keys, permits, now, lim


def _worker(rank, world, port, steps, n, out_path, span_ms=20_000):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    keys, permits, now, lim = global_trace(steps, world, n, span_ms)
    ops = HostOps(world)
    router = Router(ops, world, rank)
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
    np.savez(f"{out_path}.{rank}.npz", a=np.concatenate(got_a), r=np.concatenate(got_r),
             wide_steps=getattr(ops, "packs_wide", 0))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,span_ms", [(2, 20_000), (4, 20_000), (2, 1 << 36)])
def test_router_matches_single_process_oracle(tmp_path, world, span_ms):
    """span 2^36 ms: every rank's slice spans more than the 32-bit wire time, so the router falls
    back to the wide layout (all ranks agree through the header's overflow flags)."""
    steps, n = 3, 3000
    out = str(tmp_path / "res")
    mp.spawn(_worker, args=(world, _free_port(), steps, n, out, span_ms), nprocs=world, join=True)
    keys, permits, now, lim = global_trace(steps, world, n, span_ms)
    wa, wr, _, _ = COracle(LIMS).run(keys, permits, now, lim, None, want_tokens=False)
    for rank in range(world):
        d = np.load(f"{out}.{rank}.npz")
        for s in range(steps):
            sl = slice((s * world + rank) * n, (s * world + rank + 1) * n)
            assert np.array_equal(d["a"][s * n:(s + 1) * n], wa[sl]), (rank, s)
            assert np.array_equal(d["r"][s * n:(s + 1) * n], wr[sl]), (rank, s)
        assert int(d["wide_steps"]) == (steps if span_ms > 1 << 35 else 0)
