"""Multi-GPU request routing.

Every rank is a front-end holding a contiguous slice of the global arrival stream
(rank-major: rank r's slice precedes rank r+1's). Keys are sharded by owner =
top log2(G) bits of mix64(key_hash); each shard's engine owns its keys' state, so no
state is ever shared between GPUs. One step:

  1. stable partition of the local slice by owner (HIP), the per-owner counts written on
     the device straight into column 0 of a G x 4 header; the requests packed into the
     16-B wire layout {key_hash, permits << 32 | now_ms - base_ms}
  2. all_to_all_single of the header: (count for you, my base_ms, my overflow flag, my
     engine's status two steps back) — then ONE host read of the sent and received
     headers (the only host synchronisation of a step: the payload splits live there)
  3. ONE all_to_all_single of the wire records with those splits (RCCL over xGMI), plus
     the u16 limiter ids (as bytes) when there are several limiters. The owner receives
     its requests grouped by source rank in rank order, so within a key they are in
     global arrival order.
  4. the owner unpacks them (per-source base) and its engine decides  (HIP pipeline)
  5. all_to_all_single of the decisions back in the engine's packed width
     ((remaining + 3) << 1 | allowed, 1 B per decision for every maxPermits <= 124), one
     segment per source followed by a small exception block that carries, exactly, the
     rare remainders outside that width (token-bucket balances below -3 after time
     regression); the byte splits follow from the header
  6. scatter decisions back to the caller's order through perm        (HIP kernel)

Per request that is 16 B out and 1 B back over xGMI (the SoA layout would be 20 B + 8 B).
A source whose batch spans more than 2^31 ms either side of its first request cannot use
the 32-bit relative time: every rank sees that source's flag in the header, and the
whole step then travels in the wide SoA layout (key / permits / now_ns, int64 decisions).

Failure behaviour is collective: every rank publishes its engine's batch status in the
header, so an engine error (e.g. RL_E_CAPACITY) raises RouterError on EVERY rank at the
same step (two steps after the batch it concerns); `finish()` collects the last ones.
Receive buffers grow with the received count (up to G x the per-rank batch the engine
was sized for), so a skewed step never fails on one rank alone.

The protocol is written once against a small `ops` interface: DeviceOps drives the HIP
library on torch device tensors (the product path); tests/ supply a host
implementation to check the protocol under gloo on CPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

import rl_amd

# Exception entries per (owner, source) pair per step (16 B each). Beyond that, the
# decisions stay exact but the extra out-of-range remainders read RL_REMAINING_ERROR and
# finish() reports RL_E_CAPACITY on every rank.
EXC_CAP = 4096


class RouterError(RuntimeError):
    def __init__(self, statuses):
        self.statuses = statuses
        super().__init__("router: engine status " + ", ".join(
            f"rank {r}: {rl_amd.strerror(s)}" for r, s in enumerate(statuses) if s < 0))


def _fatal(st):
    """Statuses that fail a step (invalid requests are per-request results, not failures)."""
    return st < 0 and st != rl_amd.RL_E_INVALID_REQUEST


class DeviceOps:
    """Routing primitives on one GPU (librl_engine.so kernels)."""

    def __init__(self, eng: "rl_amd.Engine", world: int, device, capacity: int):
        self.eng, self.world, self.dev = eng, world, device
        self.cap = capacity                    # largest per-rank batch (n) of this router
        i64, i32, i16 = torch.int64, torch.int32, torch.int16
        self.perm = torch.empty(capacity, dtype=i32, device=device)
        self.k_s = torch.empty(capacity, dtype=i64, device=device)
        self.p_s = torch.empty(capacity, dtype=i32, device=device)
        self.t_s = torch.empty(capacity, dtype=i64, device=device)
        self.l_s = torch.empty(capacity, dtype=i16, device=device)
        self.packed_b = torch.empty(capacity, dtype=i64, device=device)
        self.wire_s = torch.empty((capacity, 2), dtype=i64, device=device)
        self.hdr = torch.zeros(2, dtype=i64, device=device)
        self.lost_dev = torch.zeros(1, dtype=torch.int32, device=device)
        self._recv_cap = 0
        self._grow_recv(capacity * 2)
        self._ret_in = torch.empty(0, dtype=torch.uint8, device=device)
        self._ret_out = torch.empty(0, dtype=torch.uint8, device=device)

    def _grow_recv(self, m):
        """Receive-side buffers for m requests (grown, never shrunk)."""
        if m <= self._recv_cap:
            return
        m = max(m, self._recv_cap * 3 // 2)
        i64, i32, i16 = torch.int64, torch.int32, torch.int16
        d = self.dev
        self.k_r = torch.empty(m, dtype=i64, device=d)
        self.p_r = torch.empty(m, dtype=i32, device=d)
        self.t_r = torch.empty(m, dtype=i64, device=d)
        self.l_r = torch.empty(m, dtype=i16, device=d)
        self.allowed_r = torch.empty(m, dtype=torch.uint8, device=d)
        self.remaining_r = torch.empty(m, dtype=i64, device=d)
        self.packed_r = torch.empty(m, dtype=i64, device=d)
        self.wire_r = torch.empty((m, 2), dtype=i64, device=d)
        self._recv_cap = m

    @staticmethod
    def _bytes(buf, nbytes, dev):
        return buf if buf.numel() >= nbytes else torch.empty(max(nbytes, buf.numel() * 3 // 2),
                                                             dtype=torch.uint8, device=dev)

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

    def header(self):
        return torch.zeros((self.world, 4), dtype=torch.int64, device=self.dev)

    def partition(self, n, keys, hdr):
        """perm + per-owner counts into hdr[:, 0] on the device (no host round-trip)."""
        if n > self.cap:
            raise ValueError(f"router: batch {n} exceeds the router capacity {self.cap}")
        self.eng.route_partition_device(n, keys, self.perm, self.world, hdr, hdr.shape[1],
                                        stream=self._stream())

    def engine_status(self):
        """Status of the last batch this engine decided (complete by the time it is asked:
        the header exchange that precedes the call is ordered after it)."""
        return self.eng.last_status()

    def pack(self, n, keys, permits, now, limiter=None):
        self.eng.route_pack(n, self.perm, keys, permits, now, limiter, self.k_s, self.p_s,
                            self.t_s, None if limiter is None else self.l_s,
                            stream=self._stream())
        return (self.k_s[:n], self.p_s[:n], self.t_s[:n],
                None if limiter is None else self.l_s[:n])

    def recv_buffers(self, m, with_limiter=False):
        self._grow_recv(m)
        return self.k_r[:m], self.p_r[:m], self.t_r[:m], (self.l_r[:m] if with_limiter else None)

    def decide(self, m, k, p, t, lim=None):
        s = self._stream()
        self.eng.tune("wide_records", 1)         # the merged batch may span > 2^32 ms
        try:
            self.eng.execute_device(m, k, p, t, lim, None, self.allowed_r, self.remaining_r, stream=s)
        finally:
            self.eng.tune("wide_records", 0)
        self.eng.route_fold(m, self.allowed_r, self.remaining_r, self.packed_r, stream=s)
        return self.packed_r[:m]

    def back_buffer(self, n):
        return self.packed_b[:n]

    def unpack(self, n, packed_back, allowed, remaining):
        self.eng.route_unpack(n, self.perm, packed_back, allowed, remaining, stream=self._stream())

    # ---- compact wire layout (default)
    def result_width(self):
        return self.eng.result_width()

    def pack_wire(self, n, keys, permits, now, limiter=None):
        self.eng.route_pack_wire(n, self.perm, keys, permits, now, limiter, self.wire_s,
                                 None if limiter is None else self.l_s, self.hdr,
                                 stream=self._stream())
        return self.wire_s[:n], (None if limiter is None else self.l_s[:n]), self.hdr

    def wire_recv_buffers(self, m, with_limiter=False):
        self._grow_recv(m)
        return self.wire_r[:m], (self.l_r[:m] if with_limiter else None)

    def unwire(self, m, wire, bases, counts):
        self.eng.route_unwire(m, wire, bases, counts, self.k_r, self.p_r, self.t_r,
                              stream=self._stream())
        return self.k_r[:m], self.p_r[:m], self.t_r[:m]

    def return_bytes(self, counts, width):
        return self.eng.route_return_bytes(counts, width, EXC_CAP)

    def decide_return(self, m, k, p, t, lim, width, src_counts, wide=False):
        """Decide the received requests; decisions in the segmented return layout (one
        segment + exception block per source)."""
        s = self._stream()
        if wide:
            self.eng.tune("wide_records", 1)
        try:
            self.eng.execute_device(m, k, p, t, lim, None, self.allowed_r, self.remaining_r,
                                    stream=s)
        finally:
            if wide:
                self.eng.tune("wide_records", 0)
        nb = self.return_bytes(src_counts, width)
        self._ret_out = self._bytes(self._ret_out, nb, self.dev)
        out = self._ret_out[:nb]
        self.eng.route_fold_return(m, self.allowed_r, self.remaining_r, out, width, src_counts,
                                   EXC_CAP, stream=s)
        return out

    def return_buffer(self, counts, width):
        nb = self.return_bytes(counts, width)
        self._ret_in = self._bytes(self._ret_in, nb, self.dev)
        return self._ret_in[:nb]

    def unpack_return(self, n, back, width, counts, allowed, remaining):
        self.eng.route_unpack_return(n, self.perm, back, width, counts, EXC_CAP, allowed,
                                     remaining, self.lost_dev, stream=self._stream())

    def lost(self):
        return int(self.lost_dev.item())

    def sync(self):
        torch.cuda.current_stream(self.dev).synchronize()
        self.eng.sync()


_WIDTH_DTYPE = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


class Router:
    def __init__(self, ops, world: int, rank: int, exchange_device=None, group=None):
        self.ops, self.world, self.rank, self.group = ops, world, rank, group
        self.xdev = exchange_device        # None: exchange the tensors where they live
        self._pub = rl_amd.RL_OK           # status this rank publishes in the next header
        self._pending = False              # a decided batch whose status is not read yet

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

    def _check(self, statuses):
        if any(_fatal(int(x)) for x in statuses):
            raise RouterError([int(x) for x in statuses])

    def _step(self, keys, permits, now, allowed, remaining, limiter=None):
        n = keys.shape[0]
        send_h = self.ops.header()
        self.ops.partition(n, keys, send_h)                    # column 0, on the device
        wire, l_s, hdr = self.ops.pack_wire(n, keys, permits, now, limiter)
        send_h[:, 1:3] = hdr.view(1, 2)
        send_h[:, 3] = self._pub
        # (ops run on torch's current stream: the collectives below are ordered after them)
        if self.xdev is not None:
            send_h = send_h.to(self.xdev)
        recv_h = torch.empty_like(send_h)
        dist.all_to_all_single(recv_h, send_h, group=self.group)
        both = torch.cat([send_h, recv_h]).tolist()             # the step's one host sync
        counts = [int(r[0]) for r in both[:self.world]]
        rows = both[self.world:]
        rc = [int(r[0]) for r in rows]
        # the previous batch is complete (ordered before the header exchange): its status is
        # published in the next header; the statuses received now are every rank's view of
        # its batch two steps back — identical on all ranks, so all raise together
        if self._pending:
            self._pub = int(self.ops.engine_status())
            self._pending = False
        self._check([r[3] for r in rows])
        if any(int(r[2]) for r in rows):      # some source cannot use the compact layout
            m = self._step_wide(n, counts, rc, keys, permits, now, allowed, remaining, limiter)
        else:
            m = sum(rc)
            wire_r, l_r = self.ops.wire_recv_buffers(m, limiter is not None)
            self._a2a(wire_r, wire, rc, counts)
            if l_s is not None:
                self._a2a(l_r, l_s, rc, counts)
            bases = [int(r[1]) for r in rows]
            k_r, p_r, t_r = self.ops.unwire(m, wire_r, bases, rc)
            width = self.ops.result_width()
            # sources with far-apart time bases (skewed clocks): the merged batch may span
            # more than the engine's compact 2^32 ms, so it runs in full-width records
            live = [b for b, c in zip(bases, rc) if c]
            far = bool(live) and max(live) - min(live) > (1 << 30)
            out = self.ops.decide_return(m, k_r, p_r, t_r, l_r, width, rc, wide=far)
            back = self.ops.return_buffer(counts, width)
            seg = lambda c: self.ops.return_bytes([c], width)   # noqa: E731
            self._a2a(back, out, [seg(c) for c in counts], [seg(c) for c in rc])
            self.ops.unpack_return(n, back, width, counts, allowed, remaining)
        self._pending = True
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

    def finish(self):
        """Collect every rank's last batch status (collective; call on every rank after the
        last step). Raises RouterError on every rank if any engine failed or an exact
        remainder was lost; returns the worst status otherwise."""
        if self._pending:
            self._pub = int(self.ops.engine_status())
            self._pending = False
        lost = self.ops.lost()
        mine = torch.tensor([self._pub if lost == 0 else rl_amd.RL_E_CAPACITY], dtype=torch.int64)
        dev = self.xdev or (self.ops.dev if hasattr(self.ops, "dev") else "cpu")
        mine = mine.to(dev)
        allst = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(allst, mine, group=self.group)
        sts = [int(x.item()) for x in allst]
        self._check(sts)
        return min(sts)
