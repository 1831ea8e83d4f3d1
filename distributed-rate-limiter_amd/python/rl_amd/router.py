"""Multi-GPU request routing.

Every rank is a front-end holding a contiguous slice of the global arrival stream
(rank-major: rank r's slice precedes rank r+1's). Keys are sharded by owner =
top log2(G) bits of mix64(key_hash); each shard's engine owns its keys' state, so no
state is ever shared between GPUs. One step:

  1. stable partition of the local slice by owner (HIP kernel)       -> perm, counts
  2. all_to_all_single(counts)                                        (G x int64)
  3. all_to_all_single(key / permits / now [/ limiter]) with those splits (RCCL over xGMI;
     the u16 limiter ids travel as bytes)
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

    def __init__(self, eng: "rl_amd.Engine", world: int, device, capacity: int):
        self.eng, self.world, self.dev = eng, world, device
        self.cap = capacity
        i64, i32, i16 = torch.int64, torch.int32, torch.int16
        self.perm = torch.empty(capacity, dtype=i32, device=device)
        self.k_s = torch.empty(capacity, dtype=i64, device=device)
        self.p_s = torch.empty(capacity, dtype=i32, device=device)
        self.t_s = torch.empty(capacity, dtype=i64, device=device)
        self.l_s = torch.empty(capacity, dtype=i16, device=device)
        self.k_r = torch.empty(capacity * 2, dtype=i64, device=device)
        self.p_r = torch.empty(capacity * 2, dtype=i32, device=device)
        self.t_r = torch.empty(capacity * 2, dtype=i64, device=device)
        self.l_r = torch.empty(capacity * 2, dtype=i16, device=device)
        self.allowed_r = torch.empty(capacity * 2, dtype=torch.uint8, device=device)
        self.remaining_r = torch.empty(capacity * 2, dtype=i64, device=device)
        self.packed_r = torch.empty(capacity * 2, dtype=i64, device=device)
        self.packed_b = torch.empty(capacity, dtype=i64, device=device)

    # A router step runs on one dedicated torch stream (stream_ctx): every engine call is
    # ordered on it, and so are the collectives of torch.distributed, so no host
    # synchronisation is needed between a kernel and the all-to-all that consumes its
    # output (or the reverse). (torch's default stream has handle 0, which the C-ABI reads
    # as "the engine's own stream": hence a stream of our own.)
    def stream_ctx(self):
        if not hasattr(self, "_torch_stream"):
            self._torch_stream = torch.cuda.Stream(self.dev)
        self._torch_stream.wait_stream(torch.cuda.current_stream(self.dev))
        return torch.cuda.stream(self._torch_stream)

    def _stream(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def partition(self, n, keys):
        counts = self.eng.route_partition(n, keys, self.perm, self.world, stream=self._stream())
        return [int(c) for c in counts]

    def pack(self, n, keys, permits, now, limiter=None):
        self.eng.route_pack(n, self.perm, keys, permits, now, limiter, self.k_s, self.p_s,
                            self.t_s, None if limiter is None else self.l_s,
                            stream=self._stream())
        return (self.k_s[:n], self.p_s[:n], self.t_s[:n],
                None if limiter is None else self.l_s[:n])

    def recv_buffers(self, m, with_limiter=False):
        if m > self.k_r.numel():
            raise RuntimeError(f"router: {m} requests routed to this shard exceed its buffers")
        return self.k_r[:m], self.p_r[:m], self.t_r[:m], (self.l_r[:m] if with_limiter else None)

    def decide(self, m, k, p, t, lim=None):
        s = self._stream()
        self.eng.execute_device(m, k, p, t, lim, None, self.allowed_r, self.remaining_r, stream=s)
        self.eng.route_fold(m, self.allowed_r, self.remaining_r, self.packed_r, stream=s)
        return self.packed_r[:m]

    def back_buffer(self, n):
        return self.packed_b[:n]

    def unpack(self, n, packed_back, allowed, remaining):
        self.eng.route_unpack(n, self.perm, packed_back, allowed, remaining, stream=self._stream())

    def sync(self):
        torch.cuda.current_stream(self.dev).synchronize()
        self.eng.sync()


class Router:
    def __init__(self, ops, world: int, rank: int, exchange_device=None, group=None):
        self.ops, self.world, self.rank, self.group = ops, world, rank, group
        self.xdev = exchange_device        # None: exchange the tensors where they live

    def _a2a(self, dst, src, recv_splits, send_splits):
        """all_to_all_single; int16 tensors travel as bytes (no 16-bit NCCL type)."""
        if src.dtype == torch.int16:
            dst, src = dst.view(torch.uint8), src.view(torch.uint8)
            recv_splits = [2 * x for x in recv_splits]
            send_splits = [2 * x for x in send_splits]
        if self.xdev is None:
            dist.all_to_all_single(dst, src, recv_splits, send_splits, group=self.group)
        else:
            tmp = torch.empty(dst.numel(), dtype=dst.dtype, device=self.xdev)
            dist.all_to_all_single(tmp, src.to(self.xdev), recv_splits, send_splits,
                                   group=self.group)
            dst.copy_(tmp)

    def step(self, keys, permits, now, allowed, remaining, limiter=None):
        ctx = getattr(self.ops, "stream_ctx", None)
        if ctx is None:
            return self._step(keys, permits, now, allowed, remaining, limiter)
        with ctx():
            m = self._step(keys, permits, now, allowed, remaining, limiter)
        # later work on the caller's stream sees the decisions
        torch.cuda.current_stream(keys.device).wait_stream(self.ops._torch_stream)
        return m

    def _step(self, keys, permits, now, allowed, remaining, limiter=None):
        n = keys.shape[0]
        counts = self.ops.partition(n, keys)
        k_s, p_s, t_s, l_s = self.ops.pack(n, keys, permits, now, limiter)
        # (ops run on torch's current stream: the collectives below are ordered after them)
        dev = k_s.device if self.xdev is None else self.xdev
        send_c = torch.tensor(counts, dtype=torch.int64, device=dev)
        recv_c = torch.empty(self.world, dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv_c, send_c, group=self.group)
        rc = [int(x) for x in recv_c.tolist()]
        m = sum(rc)
        k_r, p_r, t_r, l_r = self.ops.recv_buffers(m, limiter is not None)
        for dst, src in ((k_r, k_s), (p_r, p_s), (t_r, t_s), (l_r, l_s)):
            if src is not None:
                self._a2a(dst, src, rc, counts)
        packed = self.ops.decide(m, k_r, p_r, t_r, l_r)
        back = self.ops.back_buffer(n)
        self._a2a(back, packed, counts, rc)
        self.ops.unpack(n, back, allowed, remaining)
        return m
