"""Multi-GPU request routing.

Every rank is a front-end holding a contiguous slice of the global arrival stream
(rank-major: rank r's slice precedes rank r+1's). Keys are sharded by owner =
top log2(G) bits of mix64(key_hash); each shard's engine owns its keys' state, so no
state is ever shared between GPUs. One step:

  1. stable partition of the local slice by owner (HIP kernel)       -> perm, counts
  2. all_to_all_single(counts)                                        (G x int64)
  3. all_to_all_single(key / permits / now) with those splits         (RCCL over xGMI)
     The owner receives its requests grouped by source rank in rank order, so within a
     key they are in global arrival order.
  4. the owner's engine decides them                                   (HIP pipeline)
  5. all_to_all_single(decisions) back, reversed splits
  6. scatter decisions back to the caller's order through perm        (HIP kernel)

The protocol is written once against a small `ops` interface: DeviceOps drives the HIP
library on torch device tensors (the product path); tests/ supply a host
implementation to check the protocol under gloo on CPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

import rl_amd


class DeviceOps:
    """Routing primitives on one GPU (librl_engine.so kernels)."""

    def __init__(self, eng: "rl_amd.Engine", world: int, device, capacity: int,
                 want_limiter: bool = False):
        self.eng, self.world, self.dev = eng, world, device
        self.cap = capacity
        i64, i32 = torch.int64, torch.int32
        self.perm = torch.empty(capacity, dtype=i32, device=device)
        self.k_s = torch.empty(capacity, dtype=i64, device=device)
        self.p_s = torch.empty(capacity, dtype=i32, device=device)
        self.t_s = torch.empty(capacity, dtype=i64, device=device)
        self.k_r = torch.empty(capacity * 2, dtype=i64, device=device)
        self.p_r = torch.empty(capacity * 2, dtype=i32, device=device)
        self.t_r = torch.empty(capacity * 2, dtype=i64, device=device)
        self.allowed_r = torch.empty(capacity * 2, dtype=torch.uint8, device=device)
        self.remaining_r = torch.empty(capacity * 2, dtype=i64, device=device)
        self.packed_r = torch.empty(capacity * 2, dtype=i64, device=device)
        self.packed_b = torch.empty(capacity, dtype=i64, device=device)

    def partition(self, n, keys):
        counts = self.eng.route_partition(n, keys, self.perm, self.world)
        return [int(c) for c in counts]

    def pack(self, n, keys, permits, now):
        self.eng.route_pack(n, self.perm, keys, permits, now, None, self.k_s, self.p_s,
                            self.t_s, None)
        return self.k_s[:n], self.p_s[:n], self.t_s[:n]

    def recv_buffers(self, m):
        if m > self.k_r.numel():
            raise RuntimeError(f"router: {m} requests routed to this shard exceed its buffers")
        return self.k_r[:m], self.p_r[:m], self.t_r[:m]

    def decide(self, m, k, p, t):
        self.eng.execute_device(m, k, p, t, None, None, self.allowed_r, self.remaining_r)
        self.eng.route_fold(m, self.allowed_r, self.remaining_r, self.packed_r)
        return self.packed_r[:m]

    def back_buffer(self, n):
        return self.packed_b[:n]

    def unpack(self, n, packed_back, allowed, remaining):
        self.eng.route_unpack(n, self.perm, packed_back, allowed, remaining)

    def sync(self):
        self.eng.sync()


class Router:
    def __init__(self, ops, world: int, rank: int, exchange_device=None, group=None):
        self.ops, self.world, self.rank, self.group = ops, world, rank, group
        self.xdev = exchange_device        # None: exchange the tensors where they live

    def _x(self, t):
        return t if self.xdev is None else t.to(self.xdev)

    def step(self, keys, permits, now, allowed, remaining):
        n = keys.shape[0]
        counts = self.ops.partition(n, keys)
        k_s, p_s, t_s = self.ops.pack(n, keys, permits, now)
        self.ops.sync()                     # HIP work is on the engine stream
        dev = k_s.device if self.xdev is None else self.xdev
        send_c = torch.tensor(counts, dtype=torch.int64, device=dev)
        recv_c = torch.empty(self.world, dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv_c, send_c, group=self.group)
        rc = [int(x) for x in recv_c.tolist()]
        m = sum(rc)
        k_r, p_r, t_r = self.ops.recv_buffers(m)
        for dst, src in ((k_r, k_s), (p_r, p_s), (t_r, t_s)):
            if self.xdev is None:
                dist.all_to_all_single(dst, src, rc, counts, group=self.group)
            else:
                tmp = torch.empty(m, dtype=dst.dtype, device=self.xdev)
                dist.all_to_all_single(tmp, self._x(src), rc, counts, group=self.group)
                dst.copy_(tmp)
        packed = self.ops.decide(m, k_r, p_r, t_r)
        self.ops.sync()
        back = self.ops.back_buffer(n)
        if self.xdev is None:
            dist.all_to_all_single(back, packed, counts, rc, group=self.group)
        else:
            tmp = torch.empty(n, dtype=back.dtype, device=self.xdev)
            dist.all_to_all_single(tmp, self._x(packed), counts, rc, group=self.group)
            back.copy_(tmp)
        self.ops.unpack(n, back, allowed, remaining)
        return m
