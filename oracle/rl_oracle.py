"""TEST INFRASTRUCTURE ONLY — pure-Python twin of oracle/rl_oracle.c.

Second, independently written restatement of the reference semantics, used to
cross-check the C oracle on small traces and to generate the golden fixtures in
tests/golden/. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may use anything under oracle/; the product never does.

It models Redis literally: a dict from the reference's own key strings
("rl:<key>:<windowStart>", "tb:<key>", prefixed with the limiter id — SURVEY.md
§8(a) A12) to a value and a PEXPIRE deadline, with lazy expiry (expired iff
now > expireAt).

Reference lines restated:
  SlidingWindowRateLimiter.java:85-188  (tryAcquire, getAvailablePermits, reset,
                                         getCurrentCount, getWindowKey)
  TokenBucketRateLimiter.java:38-68     (Lua), :85 (ratePerMs), :105-158
  RedisRateLimitStorage.java:38-59      (incrementAndExpire, get), :133-139 (eval)
  RateLimitConfig.java:46-56            (validate)
  SlidingWindowRateLimiter.java:57-64,93-100,106-108,119-121,148-150
                                        (the Caffeine local cache, when enabled)

The Caffeine 3.1.8 cache (pom.xml:23; not vendored) is restated from its published
behaviour: `expireAfterWrite(ttl)` — an entry written at time w is returned by
getIfPresent at time t iff t - w < ttl — and `put` overwrites value and write time. The
trace clock is the request's now at ms resolution. `maximumSize(10000)` eviction
(W-TinyLFU, non-deterministic) is not modelled: exact while at most 10k keys are cached.
"""
from __future__ import annotations

import math
import struct

SW, TB = 0, 1
OP_ACQUIRE, OP_PEEK, OP_RESET = 0, 1, 2
REM_UNKNOWN, REM_INVALID = -1, -2
INT64_MAX = (1 << 63) - 1
INT64_MIN = -(1 << 63)


def jdiv(a: int, b: int) -> int:
    """Java long division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def jrem(a: int, b: int) -> int:
    """Java long remainder (sign of the dividend)."""
    return a - jdiv(a, b) * b


def java_d2l(d: float) -> int:
    """JLS 5.1.3 narrowing of double to long."""
    if d != d:
        return 0
    if d >= 9.223372036854775807e18:
        return INT64_MAX
    if d <= -9.223372036854775808e18:
        return INT64_MIN
    return int(d)


def floor_div_ms(now_ns: int) -> int:
    return now_ns // 1_000_000  # Python // is floorDiv


def f64(x: float) -> float:
    """Round-trip through IEEE binary64 (documentation: Python floats already are)."""
    return struct.unpack("<d", struct.pack("<d", x))[0]


class Redis:
    """Minimal Redis keyspace with lazy PEXPIRE semantics."""

    def __init__(self):
        self.kv: dict[str, object] = {}
        self.exp: dict[str, int] = {}

    def _alive(self, k: str, now: int) -> bool:
        # A pure function of (deadline, now): expired iff now > expireAt. The entry is not
        # deleted when a read finds it expired, so a later-arriving request with an EARLIER
        # now (time regression) still sees it; under per-key non-decreasing time this is
        # the same as Redis deleting it (the single logical clock of SURVEY §8(c)).
        if k not in self.kv:
            return False
        return not (k in self.exp and now > self.exp[k])

    def get(self, k: str, now: int) -> int:  # RedisRateLimitStorage.get
        return int(self.kv[k]) if self._alive(k, now) else 0

    def incr_pexpire(self, k: str, ttl: int, now: int) -> int:  # incrementAndExpire
        v = (int(self.kv[k]) if self._alive(k, now) else 0) + 1
        self.kv[k] = v
        self.exp[k] = now + ttl
        return v

    def hmget(self, k: str, now: int):
        if not self._alive(k, now):
            return None, None
        h = self.kv[k]
        return h["tokens"], h["last_refill"]

    def hmset_pexpire(self, k: str, tokens: float, last: float, ttl: int, now: int):
        # HMSET stores the Lua numbers as strings; %.17g / shortest round-trip is exact.
        self.kv[k] = {"tokens": float(repr(tokens)), "last_refill": float(repr(last))}
        self.exp[k] = now + ttl

    def delete(self, k: str):
        self.kv.pop(k, None)
        self.exp.pop(k, None)


class Limiter:
    def __init__(self, lid: int, algo: int, max_permits: int, window_ms: int,
                 refill_per_s: float, local_cache_ttl_ms: int = 0):
        # RateLimitConfig.validate (RateLimitConfig.java:46-56)
        if max_permits <= 0:
            raise ValueError("maxPermits must be positive")
        if window_ms <= 0:
            raise ValueError("window must be a positive duration")
        if refill_per_s < 0:
            raise ValueError("refillRate cannot be negative")
        if algo == TB and refill_per_s <= 0:  # TokenBucketRateLimiter.java:77-79
            raise ValueError("Token bucket requires positive refillRate")
        self.lid, self.algo = lid, algo
        self.max_permits, self.window_ms = max_permits, window_ms
        self.refill_rate = refill_per_s
        self.rate_per_ms = refill_per_s / 1000.0  # TokenBucketRateLimiter.java:85
        # SW local cache (SlidingWindowRateLimiter.java:57-64); TB has none
        self.cache_ttl = int(local_cache_ttl_ms) if algo == SW else 0


class PyOracle:
    def __init__(self):
        self.redis = Redis()
        self.limiters: list[Limiter] = []
        self.cache: dict[tuple, tuple] = {}     # (lid, key) -> (value, write_ms)
        self.cache_hits = 0                     # ratelimiter.cache.hits (:75-77)

    def add_limiter(self, algo, max_permits, window_ms, refill_per_s=0.0, capacity=0,
                    local_cache_ttl_ms=0) -> int:
        self.limiters.append(Limiter(len(self.limiters), algo, max_permits, window_ms,
                                     refill_per_s, local_cache_ttl_ms))
        return len(self.limiters) - 1

    # ---- Caffeine local cache (expireAfterWrite) ----
    def _cache_get(self, L: Limiter, key, now):
        e = self.cache.get((L.lid, key))
        if e is None or not (now - e[1] < L.cache_ttl):
            return None
        return e[0]

    def _cache_put(self, L: Limiter, key, value, now):
        self.cache[(L.lid, key)] = (value, now)

    # ---- sliding window ----
    @staticmethod
    def _window_key(lid, key, ts, w):  # getWindowKey :185-188
        window_start = jdiv(ts, w) * w
        return f"{lid}|rl:{key}:{window_start}"

    def _current_count(self, L: Limiter, key, now) -> int:  # :158-180
        w = L.window_ms
        curr = self.redis.get(self._window_key(L.lid, key, now, w), now)
        prev = self.redis.get(self._window_key(L.lid, key, now - w, w), now)
        pct = float(jrem(now, w)) / float(w)
        prev_weight = 1.0 - pct
        return java_d2l(float(prev) * prev_weight + float(curr))

    def _sw_acquire(self, L: Limiter, key, permits, now):
        if L.cache_ttl:                                   # :93-100
            cached = self._cache_get(L, key, now)
            if cached is not None and cached >= L.max_permits:
                self.cache_hits += 1
                return 0, max(0, L.max_permits - self._current_count(L, key, now))
        cc = self._current_count(L, key, now)
        if cc + permits > L.max_permits:
            allowed = 0
            if L.cache_ttl:                               # :106-108
                self._cache_put(L, key, cc, now)
        else:
            nc = self.redis.incr_pexpire(self._window_key(L.lid, key, now, L.window_ms),
                                         L.window_ms, now)
            if L.cache_ttl:                               # :119-121
                self._cache_put(L, key, nc, now)
            allowed = int(nc <= L.max_permits)
        return allowed, max(0, L.max_permits - self._current_count(L, key, now))

    # ---- token bucket (Lua) ----
    def _tb_acquire(self, L: Limiter, key, permits, now):
        if permits > L.max_permits:  # :110-116
            return 0, REM_UNKNOWN, math.nan
        capacity = float(L.max_permits)
        rate = L.rate_per_ms
        requested = float(permits)
        nowf = float(now)
        k = f"{L.lid}|tb:{key}"
        tokens, last = self.redis.hmget(k, now)
        if tokens is None:
            tokens, last = capacity, nowf
        elapsed = nowf - last
        add = elapsed * rate
        x = tokens + add
        tokens = x if x < capacity else capacity  # Lua 5.1 math.min(capacity, x)
        if tokens >= requested:
            tokens = tokens - requested
            self.redis.hmset_pexpire(k, tokens, nowf, L.window_ms * 2, now)
            allowed = 1
        else:
            allowed = 0
        return allowed, java_d2l(tokens), tokens

    def _tb_peek(self, L: Limiter, key, now):
        capacity = float(L.max_permits)
        tokens, last = self.redis.hmget(f"{L.lid}|tb:{key}", now)
        if tokens is None:
            t = capacity
        else:
            x = tokens + (float(now) - last) * L.rate_per_ms
            t = x if x < capacity else capacity
        return java_d2l(t), t

    # ---- state export / import in the Redis layout (rl_export_state / rl_import_state) ----
    def keyspace(self, now_ms):
        """Every key live at now_ms (RedisRateLimitStorage.java:52-59 expiry) as tuples
        (limiter, key_hash, kind, window_start, count, tokens, last_refill, expire_at), sorted
        like rl_export_state. SW keys "rl:<key>:<W>" (SlidingWindowRateLimiter.java:185-188),
        TB hashes "tb:<key>" (TokenBucketRateLimiter.java:46-48,63-64)."""
        out = []
        for k in list(self.redis.kv):
            if not self.redis._alive(k, now_ms):
                continue
            lid, rest = k.split("|", 1)
            if rest.startswith("rl:"):
                _, key, w0 = rest.split(":")
                out.append((int(lid), int(key), 0, int(w0), int(self.redis.kv[k]), 0.0, 0,
                            self.redis.exp[k]))
            else:
                h = self.redis.kv[k]
                out.append((int(lid), int(rest[3:]), 1, 0, 0, h["tokens"], int(h["last_refill"]),
                            self.redis.exp[k]))
        out.sort(key=lambda x: (x[0], x[1], x[3]))
        return out

    def load_keyspace(self, entries):
        """Inverse of keyspace(): SET/HMSET each entry with its PEXPIRE deadline."""
        for lid, key, kind, w0, count, tokens, last, exp in entries:
            k = f"{lid}|rl:{key}:{w0}" if kind == 0 else f"{lid}|tb:{key}"
            self.redis.kv[k] = int(count) if kind == 0 else {"tokens": float(tokens),
                                                              "last_refill": float(last)}
            self.redis.exp[k] = int(exp)

    def run(self, keys, permits, now_ns, limiter=None, ops=None):
        """Replay requests in arrival order; returns (allowed, remaining, tokens_after)."""
        n = len(keys)
        allowed, remaining, tokens = [0] * n, [0] * n, [math.nan] * n
        for i in range(n):
            lid = int(limiter[i]) if limiter is not None else 0
            op = int(ops[i]) if ops is not None else OP_ACQUIRE
            p = int(permits[i])
            key = int(keys[i])
            if lid >= len(self.limiters) or op > OP_RESET or (op == OP_ACQUIRE and p <= 0):
                allowed[i], remaining[i] = 0, REM_INVALID
                continue
            L = self.limiters[lid]
            now = floor_div_ms(int(now_ns[i]))
            if op == OP_ACQUIRE:
                if L.algo == SW:
                    allowed[i], remaining[i] = self._sw_acquire(L, key, p, now)
                else:
                    allowed[i], remaining[i], tokens[i] = self._tb_acquire(L, key, p, now)
            elif op == OP_PEEK:
                if L.algo == SW:
                    remaining[i] = max(0, L.max_permits - self._current_count(L, key, now))
                else:
                    remaining[i], tokens[i] = self._tb_peek(L, key, now)
            else:
                if L.algo == SW:  # SlidingWindowRateLimiter.reset :139-153
                    w = L.window_ms
                    self.redis.delete(self._window_key(L.lid, key, now, w))
                    self.redis.delete(self._window_key(L.lid, key, now - w, w))
                    self.cache.pop((L.lid, key), None)    # :148-150 invalidate
                else:  # TokenBucketRateLimiter.reset :153-158
                    self.redis.delete(f"{L.lid}|tb:{key}")
        return allowed, remaining, tokens
