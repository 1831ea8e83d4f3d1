"""Multi-GPU request routing.

Every rank is a front-end holding a contiguous slice of the global arrival stream
(rank-major: rank r's slice precedes rank r+1's). Keys are sharded by owner =
top log2(G) bits of mix64(key_hash); each shard's engine owns its keys' state, so no
state is ever shared between GPUs. One step:

  1. stable partition of the local slice by owner, packed into the 16-B wire layout
     {key_hash, permits << 32 | now_ms - base_ms} (HIP kernels)      -> perm, counts, base
  2. all_to_all_single of a G x 3 header: (count for you, my base_ms, my overflow flag)
  3. ONE all_to_all_single of the wire records with those splits (RCCL over xGMI), plus
     the u16 limiter ids (as bytes) when there are several limiters. The owner receives
     its requests grouped by source rank in rank order, so within a key they are in
     global arrival order.
  4. the owner unpacks them (per-source base) and its engine decides  (HIP pipeline)
  5. all_to_all_single of the decisions back, reversed splits, in the engine's packed
     width: ((remaining + 3) << 1 | allowed), 1 B per decision for every maxPermits <= 124
  6. scatter decisions back to the caller's order through perm        (HIP kernel)

Per request that is 16 B out and 1 B back over xGMI (the SoA layout would be 20 B + 8 B).
A source whose batch spans more than 2^31 ms either side of its first request cannot use
the 32-bit relative time: every rank sees that source's flag in the header, and the
whole step then travels in the wide SoA layout (key / permits / now_ns, int64 decisions).

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
        self.wire_s = torch.empty((capacity, 2), dtype=i64, device=device)
        self.wire_r = torch.empty((capacity * 2, 2), dtype=i64, device=device)
        self.hdr = torch.zeros(2, dtype=i64, device=device)

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

    # ---- compact wire layout (default)
    def result_width(self):
        return self.eng.result_width()

    def pack_wire(self, n, keys, permits, now, limiter=None):
        self.eng.route_pack_wire(n, self.perm, keys, permits, now, limiter, self.wire_s,
                                 None if limiter is None else self.l_s, self.hdr,
                                 stream=self._stream())
        return self.wire_s[:n], (None if limiter is None else self.l_s[:n]), self.hdr

    def wire_recv_buffers(self, m, with_limiter=False):
        if m > self.wire_r.shape[0]:
            raise RuntimeError(f"router: {m} requests routed to this shard exceed its buffers")
        return self.wire_r[:m], (self.l_r[:m] if with_limiter else None)

    def unwire(self, m, wire, bases, counts):
        self.eng.route_unwire(m, wire, bases, counts, self.k_r, self.p_r, self.t_r,
                              stream=self._stream())
        return self.k_r[:m], self.p_r[:m], self.t_r[:m]

    def decide_packed(self, m, k, p, t, lim, width):
        s = self._stream()
        self.eng.execute_device(m, k, p, t, lim, None, self.allowed_r, self.remaining_r, stream=s)
        out = self.packed_r.view(torch.uint8)[:m * width].view(_WIDTH_DTYPE[width])
        self.eng.route_fold_packed(m, self.allowed_r, self.remaining_r, out, width, stream=s)
        return out

    def back_buffer_packed(self, n, width):
        return self.packed_b.view(torch.uint8)[:n * width].view(_WIDTH_DTYPE[width])

    def unpack_packed(self, n, back, width, allowed, remaining):
        self.eng.route_unpack_packed(n, self.perm, back, width, allowed, remaining,
                                     stream=self._stream())

    def unpack(self, n, packed_back, allowed, remaining):
        self.eng.route_unpack(n, self.perm, packed_back, allowed, remaining, stream=self._stream())

    def sync(self):
        torch.cuda.current_stream(self.dev).synchronize()
        self.eng.sync()


_WIDTH_DTYPE = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


class Router:
    def __init__(self, ops, world: int, rank: int, exchange_device=None, group=None):
        self.ops, self.world, self.rank, self.group = ops, world, rank, group
        self.xdev = exchange_device        # None: exchange the tensors where they live

    def _a2a(self, dst, src, recv_splits, send_splits):
        """all_to_all_single; int16 tensors travel as bytes (no 16-bit NCCL type)."""
        if src.dtype == torch.int16:
            dst, src = dst.view(torch.uint8), src.view(torch.uint8)
            if recv_splits is not None:
                recv_splits = [2 * x for x in recv_splits]
                send_splits = [2 * x for x in send_splits]
        if self.xdev is None:
            dist.all_to_all_single(dst, src, recv_splits, send_splits, group=self.group)
        else:
            tmp = torch.empty(dst.shape, dtype=dst.dtype, device=self.xdev)
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
        wire, l_s, hdr = self.ops.pack_wire(n, keys, permits, now, limiter)
        # (ops run on torch's current stream: the collectives below are ordered after them)
        dev = wire.device if self.xdev is None else self.xdev
        send_h = torch.empty((self.world, 3), dtype=torch.int64, device=dev)
        send_h[:, 0] = torch.tensor(counts, dtype=torch.int64, device=dev)
        send_h[:, 1:] = hdr.to(dev).view(1, 2)
        recv_h = torch.empty((self.world, 3), dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv_h, send_h, group=self.group)
        rows = recv_h.tolist()
        rc = [int(r[0]) for r in rows]
        if any(int(r[2]) for r in rows):      # some source cannot use the compact layout
            return self._step_wide(n, counts, rc, keys, permits, now, allowed, remaining,
                                   limiter)
        m = sum(rc)
        wire_r, l_r = self.ops.wire_recv_buffers(m, limiter is not None)
        self._a2a(wire_r, wire, rc, counts)
        if l_s is not None:
            self._a2a(l_r, l_s, rc, counts)
        k_r, p_r, t_r = self.ops.unwire(m, wire_r, [int(r[1]) for r in rows], rc)
        width = self.ops.result_width()
        packed = self.ops.decide_packed(m, k_r, p_r, t_r, l_r, width)
        back = self.ops.back_buffer_packed(n, width)
        self._a2a(back, packed, counts, rc)
        self.ops.unpack_packed(n, back, width, allowed, remaining)
        return m

    def _step_wide(self, n, counts, rc, keys, permits, now, allowed, remaining, limiter):
        k_s, p_s, t_s, l_s = self.ops.pack(n, keys, permits, now, limiter)
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
