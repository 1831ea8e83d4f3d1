"""ctypes binding of librl_engine.so (include/rl_engine.h) for tests and bench.py.

This is plumbing around the C-ABI: every decision is made by the HIP kernels in
librl_engine.so. There is no CPU fallback — if the library is missing or no GPU is
present, constructing an Engine raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REPO = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("RL_ENGINE_LIB") or os.path.join(PKG_DIR, "librl_engine.so")  # A/B builds only
HEADER = os.path.join(REPO, "include", "rl_engine.h")

RL_OK = 0
RL_E_INVALID_ARG = -1
RL_E_INVALID_REQUEST = -2
RL_E_CAPACITY = -3
RL_E_DEVICE = -4
RL_E_NOMEM = -5
RL_E_TOO_LARGE = -6
RL_E_LIMITERS = -7
RL_E_INTERNAL = -8      # engine logic error (include/rl_engine.h)

SW, TB = 0, 1
OP_ACQUIRE, OP_PEEK, OP_RESET = 0, 1, 2
REM_UNKNOWN, REM_INVALID, REM_ERROR = -1, -2, -3
OPT_STAGE_TIMING = 1
OPT_PIPELINE = 2       # RL_OPT_PIPELINE: partition of batch k+1 overlaps batch k's decisions
OPT_FIXED_CAPACITY = 4  # RL_OPT_FIXED_CAPACITY: no on-demand table growth
REGION_SLOTS = 256          # kRegionSlots in csrc/rl_device.hpp (state slots per region)
MIN_REGIONS = 8             # kRegionsPerBin: every limiter has at least one bin of regions
DIST_UNIFORM, DIST_ZIPF = 0, 1

EXPORTS = [
    "rl_create", "rl_destroy", "rl_add_limiter", "rl_add_limiter_ex", "rl_try_acquire_batch",
    "rl_execute_batch", "rl_execute_batch_device", "rl_last_status", "rl_available", "rl_reset",
    "rl_batch_stats_get", "rl_stage_times", "rl_sync", "rl_strerror", "rl_abi_version",
    "rl_owner_of", "rl_route_partition", "rl_synth_trace_device", "rl_tune",
    "rl_route_pack", "rl_route_fold", "rl_route_unpack", "rl_debug_fetch",
    "rl_route_pack_wire", "rl_route_unwire", "rl_result_width", "rl_route_fold_packed",
    "rl_route_unpack_packed", "rl_export_state", "rl_import_state",
    "rl_sweep_expired", "rl_route_return_bytes", "rl_route_fold_return",
    "rl_route_unpack_return", "rl_route_partition_device", "rl_set_owner_directory",
    "rl_owner_of_engine", "rl_router_create", "rl_router_step", "rl_router_finish",
    "rl_router_plan_directory", "rl_router_destroy", "rl_pin_host", "rl_unpin_host",
    "rl_grow_limiter", "rl_limiter_slots", "rl_router_create_ex", "rl_router_stats_get",
]
RCCL_EXPORTS = ["rl_rccl_unique_id", "rl_transport_rccl_create", "rl_transport_rccl_destroy"]
STATE_SW_BUCKET, STATE_TB_BUCKET = 0, 1
# rl_state_entry (include/rl_engine.h): one live Redis key ("rl:<key>:<W>" / "tb:<key>")
STATE_DTYPE = np.dtype([("key_hash", "<u8"), ("limiter", "<u2"), ("kind", "u1"),
                        ("reserved", "u1", (5,)), ("window_start_ms", "<i8"), ("count", "<i8"),
                        ("tokens", "<f8"), ("last_refill_ms", "<i8"), ("expire_at_ms", "<i8")])
assert STATE_DTYPE.itemsize == 56


class RlError(RuntimeError):
    def __init__(self, status, where=""):
        self.status = status
        super().__init__(f"{where}: {strerror(status)} ({status})")


class Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("max_batch", ctypes.c_uint64), ("default_capacity", ctypes.c_uint64),
                ("shard_index", ctypes.c_uint32), ("shard_count", ctypes.c_uint32),
                ("max_skew_ms", ctypes.c_int64)]


LIM_LOCAL_CACHE = 1


class LimiterConfig(ctypes.Structure):
    _fields_ = [("algo", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("max_permits", ctypes.c_int64), ("window_ms", ctypes.c_int64),
                ("refill_per_s", ctypes.c_double), ("capacity", ctypes.c_uint64),
                ("local_cache_ttl_ms", ctypes.c_int64)]


class BatchStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("n", "allowed", "distinct_keys", "invalid",
                                                 "capacity_errors", "regions_touched",
                                                 "table_bytes", "cache_hits", "table_grows",
                                                 "hot_regions", "routed")]


class TraceSpec(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("n_keys", ctypes.c_uint64), ("dist", ctypes.c_int32),
                ("permits_max", ctypes.c_int32), ("zipf_s", ctypes.c_double),
                ("t0_ns", ctypes.c_int64), ("span_ns", ctypes.c_int64),
                ("index_base", ctypes.c_uint64), ("n_total", ctypes.c_uint64),
                ("n_limiters", ctypes.c_uint16), ("reserved", ctypes.c_uint16 * 3)]


_lib = None


def build(force: bool = False) -> str:
    """Compile librl_engine.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    if force:
        subprocess.check_call(["make", "-s", "-C", PKG_DIR, "clean"])
    subprocess.check_call(["make", "-s", "-j8", "-C", PKG_DIR])    # make skips up-to-date targets
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    # torch (ROCm) ships its own libamdhip64.so.7; the engine links the same soname. Load
    # torch first so both share ONE HIP runtime in this process (device pointers from torch
    # tensors are then valid for the engine and torch can still initialise afterwards).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run `make -C {PKG_DIR}` (no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u16, u32, i32, i64, dbl = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint16,
                                       ctypes.c_uint32, ctypes.c_int32, ctypes.c_int64,
                                       ctypes.c_double)
    L.rl_create.argtypes = [ctypes.POINTER(Opts), ctypes.POINTER(vp)]
    L.rl_destroy.argtypes = [vp]
    L.rl_destroy.restype = None
    L.rl_add_limiter.argtypes = [vp, ctypes.c_int, i64, i64, dbl, ctypes.POINTER(u16)]
    L.rl_add_limiter_ex.argtypes = [vp, ctypes.POINTER(LimiterConfig), ctypes.POINTER(u16)]
    L.rl_try_acquire_batch.argtypes = [vp, sz] + [vp] * 7
    L.rl_execute_batch.argtypes = [vp, sz] + [vp] * 8
    L.rl_execute_batch_device.argtypes = [vp, sz] + [vp] * 9
    L.rl_last_status.argtypes = [vp]
    L.rl_available.argtypes = [vp, u16, sz, vp, vp, vp]
    L.rl_reset.argtypes = [vp, u16, sz, vp, vp]
    L.rl_batch_stats_get.argtypes = [vp, ctypes.POINTER(BatchStats)]
    L.rl_stage_times.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p),
                                 ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    L.rl_sync.argtypes = [vp]
    L.rl_tune.argtypes = [vp, ctypes.c_char_p, i64]
    L.rl_strerror.argtypes = [ctypes.c_int]
    L.rl_strerror.restype = ctypes.c_char_p
    L.rl_owner_of.argtypes = [ctypes.c_uint64, u16, u32]
    L.rl_owner_of.restype = u32
    L.rl_route_partition.argtypes = [vp, sz, vp, vp, u32, vp, vp, vp]
    L.rl_route_pack.argtypes = [vp, sz] + [vp] * 10
    L.rl_route_fold.argtypes = [vp, sz] + [vp] * 4
    L.rl_route_unpack.argtypes = [vp, sz] + [vp] * 5
    L.rl_route_pack_wire.argtypes = [vp, sz] + [vp] * 9
    L.rl_route_unwire.argtypes = [vp, sz, vp, u32, vp, vp, vp, vp, vp, vp]
    L.rl_result_width.argtypes = [vp]
    L.rl_route_fold_packed.argtypes = [vp, sz, vp, vp, vp, ctypes.c_int, vp]
    L.rl_route_unpack_packed.argtypes = [vp, sz, vp, vp, ctypes.c_int, vp, vp, vp]
    L.rl_debug_fetch.argtypes = [vp, ctypes.c_char_p, vp, sz]
    L.rl_synth_trace_device.argtypes = [vp, ctypes.POINTER(TraceSpec), sz, vp, vp, vp, vp, vp]
    L.rl_export_state.argtypes = [vp, i64, vp, sz, ctypes.POINTER(sz)]
    L.rl_import_state.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.rl_sweep_expired.argtypes = [vp, i64, ctypes.POINTER(ctypes.c_uint64)]
    L.rl_route_return_bytes.argtypes = [u32, vp, ctypes.c_int, u32]
    L.rl_route_return_bytes.restype = ctypes.c_uint64
    L.rl_route_fold_return.argtypes = [vp, sz, vp, vp, vp, ctypes.c_int, u32, vp, u32, vp]
    L.rl_route_unpack_return.argtypes = [vp, sz, vp, vp, ctypes.c_int, u32, vp, u32, vp, vp, vp, vp]
    L.rl_route_partition_device.argtypes = [vp, sz, vp, u32, vp, vp, sz, vp]
    L.rl_set_owner_directory.argtypes = [vp, sz, vp, vp]
    L.rl_owner_of_engine.argtypes = [vp, ctypes.c_uint64]
    L.rl_pin_host.argtypes = [vp, vp, sz]
    L.rl_grow_limiter.argtypes = [vp, u16, ctypes.c_uint64]
    L.rl_limiter_slots.argtypes = [vp, u16, ctypes.POINTER(ctypes.c_uint64)]
    L.rl_unpin_host.argtypes = [vp, vp]
    L.rl_owner_of_engine.restype = u32
    _lib = L
    return L


def strerror(status: int) -> str:
    return lib().rl_strerror(int(status)).decode()


def _p(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data_as(ctypes.c_void_p)
    if hasattr(a, "data_ptr"):          # torch tensor (device memory)
        assert a.is_contiguous()
        return ctypes.c_void_p(a.data_ptr())
    return ctypes.c_void_p(int(a))


def mix64(x):
    """splitmix64 finaliser (the engine's key mixer), numpy uint64 vectorised."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(30))
        x = x * np.uint64(0xBF58476D1CE4E5B9)
        x = x ^ (x >> np.uint64(27))
        x = x * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x


def key_hash(key: str) -> int:
    """String -> 64-bit key hash as the C++ host API computes it (host/ratelimiter.cpp
    keyHash: FNV-1a 64 over the UTF-8 bytes, then the splitmix64 finaliser)."""
    h = 0xCBF29CE484222325
    for c in key.encode("utf-8"):
        h = ((h ^ c) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return int(mix64(np.uint64(h)))


def owner_of(keys, shard_count: int):
    if shard_count <= 1:
        return np.zeros(np.shape(keys), np.uint32)
    s = int(shard_count).bit_length() - 1
    return (mix64(keys) >> np.uint64(64 - s)).astype(np.uint32)


class Engine:
    """One engine = one GPU's state table + stream (rl_create)."""

    def __init__(self, device: int = 0, max_batch: int = 1 << 22, capacity: int = 1 << 20,
                 stage_timing: bool = False, shard_index: int = 0, shard_count: int = 1,
                 max_skew_ms: int = 0, pipeline: bool = False, fixed_capacity: bool = False):
        self._L = lib()
        o = Opts(device=device, flags=(OPT_STAGE_TIMING if stage_timing else 0) |
                 (OPT_PIPELINE if pipeline else 0) | (OPT_FIXED_CAPACITY if fixed_capacity else 0),
                 max_batch=max_batch, default_capacity=capacity, shard_index=shard_index,
                 shard_count=shard_count, max_skew_ms=max_skew_ms)
        h = ctypes.c_void_p()
        st = self._L.rl_create(ctypes.byref(o), ctypes.byref(h))
        if st != RL_OK:
            raise RlError(st, "rl_create")
        self._h = h
        self.limiters = []
        # RL_TUNE="key=value,...": engine knobs for every engine of the process (A/B and
        # diagnostics runs of the test suite; every setting gives the same decisions)
        for kv in filter(None, os.environ.get("RL_TUNE", "").split(",")):
            k, v = kv.split("=")
            self.tune(k.strip(), int(v))

    def close(self):
        if getattr(self, "_h", None):
            self._L.rl_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def add_limiter(self, algo, max_permits, window_ms, refill_per_s=0.0, capacity=0,
                    local_cache_ttl_ms=0) -> int:
        """local_cache_ttl_ms > 0: the sliding window's Caffeine local cache (parity mode,
        the default, has it off as the reference's own test does)."""
        c = LimiterConfig(algo=int(algo), flags=LIM_LOCAL_CACHE if local_cache_ttl_ms else 0,
                          max_permits=int(max_permits), window_ms=int(window_ms),
                          refill_per_s=float(refill_per_s), capacity=int(capacity),
                          local_cache_ttl_ms=int(local_cache_ttl_ms))
        lid = ctypes.c_uint16()
        st = self._L.rl_add_limiter_ex(self._h, ctypes.byref(c), ctypes.byref(lid))
        if st != RL_OK:
            raise RlError(st, "rl_add_limiter")
        self.limiters.append((algo, max_permits, window_ms, refill_per_s))
        return lid.value

    def execute(self, keys, permits, now_ns, limiter=None, ops=None, want_tokens=True):
        """Host-buffer batch. Returns (allowed u8, remaining i64, tokens f64|None, status)."""
        keys = np.ascontiguousarray(keys, np.uint64)
        permits = np.ascontiguousarray(permits, np.int32)
        now_ns = np.ascontiguousarray(now_ns, np.int64)
        limiter = None if limiter is None else np.ascontiguousarray(limiter, np.uint16)
        ops = None if ops is None else np.ascontiguousarray(ops, np.uint8)
        n = keys.shape[0]
        allowed = np.zeros(n, np.uint8)
        remaining = np.zeros(n, np.int64)
        tokens = np.zeros(n, np.float64) if want_tokens else None
        st = self._L.rl_execute_batch(self._h, n, _p(keys), _p(permits), _p(now_ns), _p(limiter),
                                      _p(ops), _p(allowed), _p(remaining), _p(tokens))
        if st in (RL_E_DEVICE, RL_E_NOMEM, RL_E_TOO_LARGE):
            raise RlError(st, "rl_execute_batch")
        return allowed, remaining, tokens, st

    def grow_limiter(self, limiter: int, min_keys: int) -> None:
        st = self._L.rl_grow_limiter(self._h, limiter, min_keys)
        if st != RL_OK:
            raise RlError(st, "rl_grow_limiter")

    def limiter_slots(self, limiter: int) -> int:
        v = ctypes.c_uint64()
        st = self._L.rl_limiter_slots(self._h, limiter, ctypes.byref(v))
        if st != RL_OK:
            raise RlError(st, "rl_limiter_slots")
        return v.value

    def pin_host(self, arr) -> int:
        """rl_pin_host on a numpy array reused across host batches (status code)."""
        return self._L.rl_pin_host(self._h, _p(arr), arr.nbytes)

    def unpin_host(self, arr) -> int:
        return self._L.rl_unpin_host(self._h, _p(arr))

    def try_acquire_batch(self, keys, permits, now_ns, limiter=None):
        a, r, _, st = self.execute(keys, permits, now_ns, limiter, None, want_tokens=False)
        return a, r, st

    def execute_device(self, n, keys, permits, now_ns, limiter, ops, allowed, remaining,
                       tokens=None, stream=None):
        """Device-resident batch (torch tensors or raw device pointers); asynchronous."""
        st = self._L.rl_execute_batch_device(self._h, n, _p(keys), _p(permits), _p(now_ns),
                                             _p(limiter), _p(ops), _p(allowed), _p(remaining),
                                             _p(tokens), _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_execute_batch_device")

    def last_status(self) -> int:
        return self._L.rl_last_status(self._h)

    def available(self, limiter, keys, now_ns):
        keys = np.ascontiguousarray(keys, np.uint64)
        now_ns = np.ascontiguousarray(now_ns, np.int64)
        out = np.zeros(keys.shape[0], np.int64)
        st = self._L.rl_available(self._h, int(limiter), keys.shape[0], _p(keys), _p(now_ns),
                                  _p(out))
        return out, st

    def reset(self, limiter, keys, now_ns):
        keys = np.ascontiguousarray(keys, np.uint64)
        now_ns = np.ascontiguousarray(now_ns, np.int64)
        return self._L.rl_reset(self._h, int(limiter), keys.shape[0], _p(keys), _p(now_ns))

    def export_state(self, now_ns):
        """Live state at now_ns in the Redis layout: a STATE_DTYPE array (rl_export_state)."""
        n = ctypes.c_size_t(0)
        st = self._L.rl_export_state(self._h, int(now_ns), None, 0, ctypes.byref(n))
        while True:
            if st == RL_OK and n.value == 0:
                return np.zeros(0, STATE_DTYPE)
            if st not in (RL_OK, RL_E_TOO_LARGE):
                raise RlError(st, "rl_export_state")
            out = np.zeros(n.value + 1024, STATE_DTYPE)   # state may grow between calls
            st = self._L.rl_export_state(self._h, int(now_ns), _p(out), out.shape[0], ctypes.byref(n))
            if st == RL_OK:
                return out[:n.value]

    def import_state(self, entries):
        """Load STATE_DTYPE entries (rl_import_state). Returns (status, entries taken)."""
        entries = np.ascontiguousarray(entries, STATE_DTYPE)
        n = ctypes.c_size_t(0)
        st = self._L.rl_import_state(self._h, _p(entries) if entries.shape[0] else None,
                                     entries.shape[0], ctypes.byref(n))
        return st, n.value

    def sweep_expired(self, now_ns) -> int:
        """Free every slot with no bucket live at now_ns (rl_sweep_expired); returns the count."""
        n = ctypes.c_uint64(0)
        st = self._L.rl_sweep_expired(self._h, int(now_ns), ctypes.byref(n))
        if st != RL_OK:
            raise RlError(st, "rl_sweep_expired")
        return n.value

    def stats(self) -> dict:
        s = BatchStats()
        self._L.rl_batch_stats_get(self._h, ctypes.byref(s))
        return {f: getattr(s, f) for f, _ in BatchStats._fields_}

    def stage_times(self) -> dict:
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        k = self._L.rl_stage_times(self._h, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(k)}

    def tune(self, key: str, value: int):
        st = self._L.rl_tune(self._h, key.encode(), int(value))
        if st != RL_OK:
            raise RlError(st, "rl_tune")

    def debug_region_times(self, n_bins):
        """Per-bin {t_start, t_end, records, rounds} of the last batch (rl_tune debug_regions)."""
        out = np.zeros((n_bins, 28), np.uint64)     # kDbgWords
        k = self._L.rl_debug_fetch(self._h, b"region_times", _p(out), out.nbytes)
        if k < 0:
            raise RlError(k, "rl_debug_fetch")
        return out[:k]

    def debug_bin_totals(self):
        """The last batch's pass-0 bin sizes (2^kMaxDigitBits entries; the unused ones stale)."""
        out = np.zeros(1 << 13, np.uint32)
        k = self._L.rl_debug_fetch(self._h, b"bin_totals", _p(out), out.nbytes)
        if k < 0:
            raise RlError(k, "rl_debug_fetch")
        return out[:k]

    def sync(self):
        st = self._L.rl_sync(self._h)
        if st != RL_OK:
            raise RlError(st, "rl_sync")

    def route_partition(self, n, keys_dev, perm_dev, shard_count, stream=None):
        counts = np.zeros(shard_count, np.uint64)
        st = self._L.rl_route_partition(self._h, n, _p(keys_dev), None, shard_count,
                                        _p(perm_dev), _p(counts), _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_partition")
        return counts

    def route_pack(self, n, perm, key, permits, now, limiter, key_o, permits_o, now_o, limiter_o,
                   stream=None):
        st = self._L.rl_route_pack(self._h, n, _p(perm), _p(key), _p(permits), _p(now),
                                   _p(limiter), _p(key_o), _p(permits_o), _p(now_o),
                                   _p(limiter_o), _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_pack")

    def route_fold(self, n, allowed, remaining, packed, stream=None):
        st = self._L.rl_route_fold(self._h, n, _p(allowed), _p(remaining), _p(packed), _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_fold")

    def route_unpack(self, n, perm, packed, allowed, remaining, stream=None):
        st = self._L.rl_route_unpack(self._h, n, _p(perm), _p(packed), _p(allowed), _p(remaining),
                                     _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_unpack")

    def route_pack_wire(self, n, perm, key, permits, now, limiter, wire_o, limiter_o, hdr,
                        stream=None):
        st = self._L.rl_route_pack_wire(self._h, n, _p(perm), _p(key), _p(permits), _p(now),
                                        _p(limiter), _p(wire_o), _p(limiter_o), _p(hdr),
                                        _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_pack_wire")

    def route_unwire(self, m, wire, src_base, src_count, key_o, permits_o, now_o, stream=None):
        base = np.ascontiguousarray(src_base, dtype=np.int64)
        cnt = np.ascontiguousarray(src_count, dtype=np.uint64)
        st = self._L.rl_route_unwire(self._h, m, _p(wire), len(base), base.ctypes.data,
                                     cnt.ctypes.data, _p(key_o), _p(permits_o), _p(now_o),
                                     _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_unwire")

    def result_width(self):
        w = self._L.rl_result_width(self._h)
        if w < 0:
            raise RlError(w, "rl_result_width")
        return w

    def route_fold_packed(self, n, allowed, remaining, packed, width, stream=None):
        st = self._L.rl_route_fold_packed(self._h, n, _p(allowed), _p(remaining), _p(packed),
                                          width, _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_fold_packed")

    def route_unpack_packed(self, n, perm, packed, width, allowed, remaining, stream=None):
        st = self._L.rl_route_unpack_packed(self._h, n, _p(perm), _p(packed), width, _p(allowed),
                                            _p(remaining), _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_unpack_packed")

    def route_return_bytes(self, seg_counts, width, exc_cap):
        c = np.ascontiguousarray(seg_counts, dtype=np.uint64)
        return int(self._L.rl_route_return_bytes(len(c), c.ctypes.data, width, exc_cap))

    def route_fold_return(self, m, allowed, remaining, out, width, seg_counts, exc_cap,
                          stream=None):
        c = np.ascontiguousarray(seg_counts, dtype=np.uint64)
        st = self._L.rl_route_fold_return(self._h, m, _p(allowed), _p(remaining), _p(out), width,
                                          len(c), c.ctypes.data, exc_cap, _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_fold_return")

    def route_unpack_return(self, n, perm, inp, width, seg_counts, exc_cap, allowed, remaining,
                            lost, stream=None):
        c = np.ascontiguousarray(seg_counts, dtype=np.uint64)
        st = self._L.rl_route_unpack_return(self._h, n, _p(perm), _p(inp), width, len(c),
                                            c.ctypes.data, exc_cap, _p(allowed), _p(remaining),
                                            _p(lost), _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_unpack_return")

    def set_owner_directory(self, keys, owners):
        k = np.ascontiguousarray(keys, np.uint64)
        o = np.ascontiguousarray(owners, np.uint32)
        st = self._L.rl_set_owner_directory(self._h, len(k), _p(k) if len(k) else None,
                                            _p(o) if len(o) else None)
        if st != RL_OK:
            raise RlError(st, "rl_set_owner_directory")

    def owner_of(self, key_hash) -> int:
        return int(self._L.rl_owner_of_engine(self._h, int(key_hash)))

    def route_partition_device(self, n, keys_dev, perm_dev, shard_count, counts_dev, stride,
                               stream=None):
        st = self._L.rl_route_partition_device(self._h, n, _p(keys_dev), shard_count, _p(perm_dev),
                                               _p(counts_dev), stride, _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_route_partition_device")

    def synth_trace(self, n, keys, permits, now_ns, limiter, *, seed, n_keys, dist=DIST_UNIFORM,
                    zipf_s=1.1, permits_max=4, t0_ns=1_700_000_000_000 * 1_000_000,
                    span_ns=2_000_000_000, index_base=0, n_total=None, n_limiters=1,
                    stream=None):
        spec = TraceSpec(seed=seed, n_keys=n_keys, dist=dist, permits_max=permits_max,
                         zipf_s=zipf_s, t0_ns=t0_ns, span_ns=span_ns, index_base=index_base,
                         n_total=n_total or n, n_limiters=n_limiters)
        st = self._L.rl_synth_trace_device(self._h, ctypes.byref(spec), n, _p(keys), _p(permits),
                                           _p(now_ns), _p(limiter), _p(stream))
        if st != RL_OK:
            raise RlError(st, "rl_synth_trace_device")
