"""TEST INFRASTRUCTURE ONLY — ctypes loader for the C oracle (oracle/rl_oracle.c).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
parity checker; never by the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "librl_oracle.so")
_lib = None

SW, TB = 0, 1


def build() -> str:
    src = os.path.join(_HERE, "rl_oracle.c")
    if (not os.path.exists(_LIB_PATH)
            or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_create.restype = ctypes.c_void_p
        L.orc_destroy.argtypes = [ctypes.c_void_p]
        L.orc_add_limiter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                      ctypes.c_int64, ctypes.c_double]
        L.orc_add_limiter.restype = ctypes.c_int
        vp = ctypes.c_void_p
        L.orc_run.argtypes = [vp, ctypes.c_size_t] + [vp] * 8
        L.orc_run.restype = ctypes.c_size_t
        L.orc_run_sharded.argtypes = [vp, ctypes.c_int, ctypes.c_size_t] + [vp] * 8
        L.orc_run_sharded.restype = ctypes.c_size_t
        L.orc_live_keys.argtypes = [vp]
        L.orc_live_keys.restype = ctypes.c_size_t
        L.orc_set_local_cache.argtypes = [vp, ctypes.c_int, ctypes.c_int64]
        L.orc_cache_hits.argtypes = [vp]
        L.orc_cache_hits.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class COracle:
    """Sequential (or key-sharded multi-threaded) replay of the reference semantics."""

    def __init__(self, limiters=(), nthreads: int = 1):
        self._L = lib()
        self.nthreads = max(1, int(nthreads))
        self._states = [self._L.orc_create() for _ in range(self.nthreads)]
        self.n_limiters = 0
        for spec in limiters:
            self.add_limiter(*spec)

    def add_limiter(self, algo, max_permits, window_ms, refill_per_s=0.0, capacity=0,
                    local_cache_ttl_ms=0) -> int:
        ids = {self._L.orc_add_limiter(s, int(algo), int(max_permits), int(window_ms),
                                       float(refill_per_s)) for s in self._states}
        (lid,) = ids
        if lid < 0:
            raise ValueError("invalid limiter config (RateLimitConfig.validate)")
        if local_cache_ttl_ms:
            for s in self._states:
                self._L.orc_set_local_cache(s, lid, int(local_cache_ttl_ms))
        self.n_limiters += 1
        return lid

    def cache_hits(self) -> int:
        return sum(self._L.orc_cache_hits(s) for s in self._states)

    def run(self, keys, permits, now_ns, limiter=None, ops=None, want_tokens=True):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        now_ns = np.ascontiguousarray(now_ns, dtype=np.int64)
        limiter = None if limiter is None else np.ascontiguousarray(limiter, dtype=np.uint16)
        ops = None if ops is None else np.ascontiguousarray(ops, dtype=np.uint8)
        n = keys.shape[0]
        allowed = np.zeros(n, np.uint8)
        remaining = np.zeros(n, np.int64)
        tokens = np.full(n, np.nan, np.float64) if want_tokens else None
        if self.nthreads == 1:
            bad = self._L.orc_run(self._states[0], n, _p(keys), _p(permits), _p(now_ns),
                                  _p(limiter), _p(ops), _p(allowed), _p(remaining), _p(tokens))
        else:
            arr = (ctypes.c_void_p * self.nthreads)(*self._states)
            bad = self._L.orc_run_sharded(ctypes.cast(arr, ctypes.c_void_p), self.nthreads, n,
                                          _p(keys), _p(permits), _p(now_ns), _p(limiter),
                                          _p(ops), _p(allowed), _p(remaining), _p(tokens))
        return allowed, remaining, tokens, int(bad)

    def live_keys(self) -> int:
        return sum(self._L.orc_live_keys(s) for s in self._states)

    def close(self):
        for s in self._states:
            self._L.orc_destroy(s)
        self._states = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
