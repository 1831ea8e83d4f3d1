"""ctypes driver of the C-ABI multi-GPU router (rl_router_*, include/rl_engine.h) — the
product path a JNI / FFM caller uses, driven here by bench.py --gpus N.

Transports (include/rl_engine.h `rl_transport`):
  * "rccl": librl_rccl.so (include/rl_rccl.h) — one RCCL communicator over xGMI, its
    unique id handed from rank 0 to the others through torch.distributed;
  * "host": every all-to-all goes through the host over torch.distributed (gloo) — a
    functional rehearsal of the N > 1 path when several ranks share one GPU (RCCL refuses
    two ranks on one device). Its numbers mean nothing.

The router runs every step on its own stream; rl_router_step makes one host
synchronisation per step (the header exchange: RCCL takes per-peer counts on the host).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch
import torch.distributed as dist

import rl_amd

_rccl = None
_hip = None

_A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                        ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                        ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p)


class Transport(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("all_to_all_v", ctypes.c_void_p)]


def rccl_lib():
    global _rccl
    if _rccl is None:
        rl_amd.lib()                                   # one HIP runtime (torch's) first
        path = os.path.join(rl_amd.PKG_DIR, "librl_rccl.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: run `make -C {rl_amd.PKG_DIR}`")
        L = ctypes.CDLL(path)
        L.rl_rccl_unique_id.argtypes = [ctypes.c_void_p]
        L.rl_transport_rccl_create.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_int, ctypes.POINTER(Transport)]
        L.rl_transport_rccl_destroy.argtypes = [ctypes.POINTER(Transport)]
        L.rl_transport_rccl_destroy.restype = None
        _rccl = L
    return _rccl


def hip_lib():
    """The HIP runtime already loaded by torch (same soname as librl_engine.so links)."""
    global _hip
    if _hip is None:
        rl_amd.lib()
        H = ctypes.CDLL("libamdhip64.so.7")
        H.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        H.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        _hip = H
    return _hip


_D2H, _H2D = 2, 1


class HostTransport:
    """all_to_all_v through the host (torch.distributed, gloo): rehearsal only."""

    def __init__(self, world, group=None):
        self.world, self.group = world, group
        self.fn = _A2A(self._a2a)                      # keep the callback alive

    def _a2a(self, ctx, send, so, sb, recv, ro, rb, stream):
        try:
            H = hip_lib()
            send, recv = send or 0, recv or 0
            if H.hipStreamSynchronize(stream) != 0:
                return -1
            G = self.world
            sbs = [int(sb[p]) for p in range(G)]
            rbs = [int(rb[p]) for p in range(G)]
            inp = torch.empty(sum(sbs), dtype=torch.uint8)
            o = 0
            for p in range(G):
                if sbs[p]:
                    if H.hipMemcpy(inp.data_ptr() + o, send + int(so[p]), sbs[p], _D2H) != 0:
                        return -1
                o += sbs[p]
            out = torch.empty(sum(rbs), dtype=torch.uint8)
            dist.all_to_all_single(out, inp, rbs, sbs, group=self.group)
            o = 0
            for p in range(G):
                if rbs[p]:
                    if H.hipMemcpy(recv + int(ro[p]), out.data_ptr() + o, rbs[p], _H2D) != 0:
                        return -1
                o += rbs[p]
            return 0
        except Exception:                              # never unwind into C
            return -1


class RouterOpts(ctypes.Structure):
    _fields_ = [("max_batch", ctypes.c_size_t), ("recv_cap", ctypes.c_size_t)]


class RouterStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in ("steps", "rounds", "split_steps", "max_recv",
                                               "header_sync_ns", "recv_cap", "reserved_bytes")]


class CRouter:
    """rl_router_create_ex / step / finish / plan_directory / stats / destroy over one engine.
    recv_cap: requests the owner's engine decides per exchange round (0: min(world, 2) x
    max_batch, clamped to the engine's max_batch); a step in which an owner receives more
    is split into rounds by every rank alike."""

    def __init__(self, eng: "rl_amd.Engine", world: int, rank: int, max_batch: int,
                 transport: str = "rccl", device: int = 0, group=None, recv_cap: int = 0):
        self._L = rl_amd.lib()
        self.world, self.rank = world, rank
        self.t = Transport()
        self._kind = transport
        if transport == "rccl":
            R = rccl_lib()
            uid = (ctypes.c_uint8 * 128)()
            if rank == 0:
                st = R.rl_rccl_unique_id(uid)
                if st != rl_amd.RL_OK:
                    raise rl_amd.RlError(st, "rl_rccl_unique_id")
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=0, group=group)
            uid = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
            st = R.rl_transport_rccl_create(uid, world, rank, device, ctypes.byref(self.t))
            if st != rl_amd.RL_OK:
                raise rl_amd.RlError(st, "rl_transport_rccl_create")
        elif transport == "host":
            self._host = HostTransport(world, group)
            self.t.ctx = None
            self.t.all_to_all_v = ctypes.cast(self._host.fn, ctypes.c_void_p)
        else:
            raise ValueError(transport)
        vp = ctypes.c_void_p
        L = self._L
        L.rl_router_create_ex.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.POINTER(Transport), ctypes.POINTER(RouterOpts),
                                          ctypes.POINTER(vp)]
        L.rl_router_stats_get.argtypes = [vp, ctypes.POINTER(RouterStats)]
        L.rl_router_step.argtypes = [vp, ctypes.c_size_t] + [vp] * 7
        L.rl_router_finish.argtypes = [vp]
        L.rl_router_plan_directory.argtypes = [vp, ctypes.c_size_t, vp, vp, ctypes.c_uint64,
                                               ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), vp]
        L.rl_router_destroy.argtypes = [vp]
        L.rl_router_destroy.restype = None
        h = vp()
        o = RouterOpts(max_batch, recv_cap)
        st = L.rl_router_create_ex(eng.handle, world, rank, ctypes.byref(self.t), ctypes.byref(o),
                                   ctypes.byref(h))
        if st != rl_amd.RL_OK:
            raise rl_amd.RlError(st, "rl_router_create_ex")
        self._h = h

    def step(self, n, keys, permits, now_ns, limiter, allowed, remaining, stream=None):
        p = rl_amd._p
        st = self._L.rl_router_step(self._h, n, p(keys), p(permits), p(now_ns), p(limiter),
                                    p(allowed), p(remaining), p(stream))
        if st < 0 and st != rl_amd.RL_E_INVALID_REQUEST:
            raise rl_amd.RlError(st, "rl_router_step")
        return st

    def finish(self) -> int:
        st = self._L.rl_router_finish(self._h)
        if st < 0 and st != rl_amd.RL_E_INVALID_REQUEST:
            raise rl_amd.RlError(st, "rl_router_finish")
        return st

    def plan_directory(self, keys, counts, sampled: int, k: int) -> int:
        """Hot-key directory from this rank's candidates (collective)."""
        keys = np.ascontiguousarray(keys, np.uint64)
        counts = np.ascontiguousarray(counts, np.uint64)
        placed = ctypes.c_uint32(0)
        st = self._L.rl_router_plan_directory(self._h, len(keys),
                                              keys.ctypes.data if len(keys) else None,
                                              counts.ctypes.data if len(counts) else None,
                                              int(sampled), int(k), ctypes.byref(placed), None)
        if st != rl_amd.RL_OK:
            raise rl_amd.RlError(st, "rl_router_plan_directory")
        return placed.value

    def stats(self) -> dict:
        st = RouterStats()
        self._L.rl_router_stats_get(self._h, ctypes.byref(st))
        return {f: getattr(st, f) for f, _ in RouterStats._fields_}

    def close(self):
        if getattr(self, "_h", None):
            self._L.rl_router_destroy(self._h)
            self._h = None
        if self._kind == "rccl" and self.t.ctx:
            rccl_lib().rl_transport_rccl_destroy(ctypes.byref(self.t))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
