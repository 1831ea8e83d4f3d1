#!/usr/bin/env python3
"""Generates tests/golden/kats.json and tests/golden/traces.npz.

Run from the repo root:  python tests/golden/make_golden.py

kats.json — known-answer tests. Every case lists limiters, requests and the
EXPECTED outputs written out by hand below (derivation in each case's "why"),
never computed by an oracle. Provenance:
  * "ref:*"  restate the reference's own unit tests
             (/root/reference/src/test/java/com/ratelimiter/algorithms/
              SlidingWindowRateLimiterTest.java, @Disabled upstream) as traces
             through a real keyspace with a pinned clock.
  * "doc:*"  the only outputs the reference itself publishes for this path:
             README.md:83-95 and API_EXAMPLES.md:39-101 (api 100/min -> remaining
             97 after three requests, 0 once exceeded; login 10/min -> 7 after three;
             burst token bucket cap 50 at 10/s, batch of 20 -> tokens_remaining 30).
             These pin SW and TB against reference-held artefacts.
  * "hand:*" hand-derived edge cases from SURVEY.md §8(c): window boundaries,
             Redis TTL lapse, TB expiry, early reject, negative elapsed, and
             traces where an FMA-contracted implementation would differ from
             the reference's separately rounded Java/Lua arithmetic.
At generation time both oracles (oracle/rl_oracle.py and the C oracle) must
reproduce every expected value; the tests re-check this on every run.

traces.npz — small seeded random traces (a few thousand requests) whose
expected outputs come from the Python twin oracle, cross-checked against the
C oracle when generated. These are regression vectors for the GPU path (they
are not independent pins; the KATs are).
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.rl_oracle import PyOracle, SW, TB  # noqa: E402

NS = 1_000_000
T0 = 1_700_000_000_000          # ms; 1.7e12 % 60000 == 20000, % 1000 == 0
W60 = (T0 // 60000) * 60000     # a 60 s window start
INV = -2
UNK = -1


def req(key, permits, now_ms, lim=0, op=0, now_ns_extra=0):
    return [int(key), int(permits), int(now_ms) * NS + now_ns_extra, int(lim), int(op)]


def case(name, why, limiters, requests, expected):
    """expected: list of [allowed, remaining, tokens_after | None]."""
    assert len(requests) == len(expected), name
    return {"name": name, "why": why, "limiters": limiters, "requests": requests,
            "expected": expected}


def kats():
    out = []
    LIM10 = [[SW, 10, 1000, 0.0]]  # SlidingWindowRateLimiterTest.java:41-45
    W = (T0 // 1000) * 1000

    out.append(case(
        "ref:shouldAllowRequestsUnderLimit",
        "SlidingWindowRateLimiterTest.java:50-64 — fresh key, 3 acquires, counter goes 1,2,3;"
        " prev bucket empty so estimate = curr and remaining = 10 - curr.",
        LIM10, [req(7, 1, W + 10) for _ in range(3)],
        [[1, 9, None], [1, 8, None], [1, 7, None]]))

    reqs = [req(7, 1, W + 10) for _ in range(11)]
    exp = [[1, 9 - i, None] for i in range(10)] + [[0, 0, None]]
    out.append(case(
        "ref:shouldRejectWhenLimitExceeded",
        "SlidingWindowRateLimiterTest.java:66-78 — at count 10 the 11th request is denied"
        " and not counted (the following peek still reads 0 available).",
        LIM10, reqs + [req(7, 0, W + 10, op=1)], exp + [[0, 0, None]]))

    # prev window: 10 requests at W-50 (alive until W+950); current window at W+950:
    # pw = 1 - 0.95 = 0.050000000000000044, 10*pw = 0.5000000000000004
    reqs = [req(8, 1, W - 50) for _ in range(10)] + [req(8, 1, W + 950) for _ in range(11)]
    exp = [[1, 9 - i, None] for i in range(10)]
    # in window W: est before c-th = trunc(0.5000000000000004 + c) = c, allowed while c+1<=10
    # remaining after = 10 - trunc(0.5.. + c+1) = 9 - c
    exp += [[1, 9 - c, None] for c in range(10)] + [[0, 0, None]]
    out.append(case(
        "ref:shouldRejectWhenLimitExceeded/bothBuckets",
        "Mock returned 10 for both buckets; reached here with prev=10, curr=10 at pct 0.95:"
        " est = trunc(10*0.050000000000000044 + 10) = 10 -> 10+1 > 10 deny, no INCR.",
        LIM10, reqs, exp))

    # shouldHandleMultiplePermits: prev 5 @W-100 (alive to W+900), curr 5 @W+10,
    # then at W+850 (pw = 0.15000000000000002): acquire(5), acquire(1), acquire(4)
    reqs = [req(9, 1, W - 100) for _ in range(5)] + [req(9, 1, W + 10) for _ in range(5)]
    reqs += [req(9, 5, W + 850), req(9, 1, W + 850), req(9, 4, W + 850)]
    exp = [[1, 9 - i, None] for i in range(5)]
    # at W+10: pw = 0.99, 5*0.99 = 4.95; est_c = trunc(4.95 + c); after c+1: trunc(4.95+c+1)
    exp += [[1, 10 - (4 + c + 1), None] for c in range(5)]
    # W+850: 5*0.15000000000000002 = 0.7500000000000001; est = trunc(0.75.. + 5) = 5;
    # 5+5 <= 10 -> allowed, INCR by ONE (not 5): curr 6 -> remaining 10 - 6 = 4
    # acquire(1): est 6, 7 <= 10 allowed -> curr 7 -> remaining 3
    # acquire(4): est 7, 11 > 10 -> denied, remaining 3
    exp += [[1, 4, None], [1, 3, None], [0, 3, None]]
    out.append(case(
        "ref:shouldHandleMultiplePermits",
        "SlidingWindowRateLimiterTest.java:80-100 restated with a real keyspace at pw=0.15"
        " (the mock needed pw<0.2). Pins SURVEY §0.7: tryAcquire(key,5) checks +5 but INCRs"
        " by 1 (SlidingWindowRateLimiter.java:104 vs :116).",
        LIM10, reqs, exp))

    # shouldReportAvailablePermits: prev 7 @W-50, curr 7 @W+900 (pw = 0.09999999999999998)
    reqs = [req(10, 1, W - 50) for _ in range(7)] + [req(10, 1, W + 900) for _ in range(7)]
    reqs += [req(10, 0, W + 900, op=1)]
    exp = [[1, 9 - i, None] for i in range(7)]
    # at W+900: 7*pw = 0.6999999999999998; est = trunc(0.69.. + c) = c
    exp += [[1, 9 - c, None] for c in range(7)]
    exp += [[0, 3, None]]  # trunc(0.6999999999999998 + 7) = 7 -> 10 - 7 = 3
    out.append(case(
        "ref:shouldReportAvailablePermits",
        "SlidingWindowRateLimiterTest.java:102-111 — get=7 for both buckets; available = 3"
        " holds because 7*pw < 1 at pct 0.9.",
        LIM10, reqs, exp))

    reqs = [req(11, 1, W - 50) for _ in range(4)] + [req(11, 1, W + 100) for _ in range(3)]
    reqs += [req(11, 0, W + 200, op=2), req(11, 0, W + 200, op=1), req(11, 1, W + 200)]
    exp = [[1, 9 - i, None] for i in range(4)]
    # W+100: pw=0.9, 4*0.9=3.6; est_c = trunc(3.6+c); remaining after = 10 - trunc(3.6+c+1)
    exp += [[1, 10 - (3 + c + 1), None] for c in range(3)]
    exp += [[0, 0, None], [0, 10, None], [1, 9, None]]
    out.append(case(
        "ref:shouldResetLimits",
        "SlidingWindowRateLimiterTest.java:113-122 — reset deletes the current and previous"
        " window buckets (SlidingWindowRateLimiter.java:139-153): afterwards 10 available.",
        LIM10, reqs, exp))

    out.append(case(
        "ref:shouldRejectInvalidPermits",
        "SlidingWindowRateLimiterTest.java:124-132 — permits 0 and -1 throw"
        " IllegalArgumentException (engine: RL_REMAINING_INVALID, state untouched).",
        LIM10, [req(12, 0, W), req(12, -1, W), req(12, 1, W)],
        [[0, INV, None], [0, INV, None], [1, 9, None]]))

    reqs = [req(13, 1, W + 5) for _ in range(200)]
    exp = [[1, 9 - i, None] for i in range(10)] + [[0, 0, None]] * 190
    out.append(case(
        "ref:shouldHandleConcurrentRequests",
        "SlidingWindowRateLimiterTest.java:134-176 asserts success > 0 for 200 requests;"
        " replayed in arrival order exactly 10 succeed (max 10 per window).",
        LIM10, reqs, exp))

    # ---------- hand-derived SW ----------
    L = [[SW, 100, 60000, 0.0]]
    # boundary: 30 requests at W60-1 (pct=(w-1)/w), then at W60 (pct 0, pw 1.0)
    reqs = [req(20, 1, W60 - 1) for _ in range(30)] + [req(20, 1, W60) for _ in range(3)]
    reqs += [req(20, 0, W60, op=1), req(20, 0, W60 + 59999, op=1), req(20, 0, W60 + 60000, op=1)]
    exp = []
    # before: prev window (W60-60000) empty; est = c
    exp += [[1, 99 - c, None] for c in range(30)]
    # at W60: prev = 30 with pw = 1.0 -> est = 30 + c
    exp += [[1, 100 - (30 + c + 1), None] for c in range(3)]
    exp += [[0, 67, None]]
    # W60+59999: pct = 59999/60000 = 0.9999833333333333, pw = 1.6666666666720342e-05;
    # prev bucket last INCR at W60-1 -> expireAt W60+59999 -> still alive (now == expireAt);
    # 30*pw = 0.0005000000000016103 -> est = trunc(0.0005.. + 3) = 3 -> 97
    exp += [[0, 97, None]]
    # W60+60000: new window; prev = bucket W60 (3, alive: last W60 + 60000), curr 0, pw = 1
    exp += [[0, 97, None]]
    out.append(case(
        "hand:sw:windowBoundary",
        "now%w == w-1 and now%w == 0: pct = 0 gives prevWeight = 1.0 exactly; bucket alive"
        " at now == lastIncr + w (Redis expires only when now > expireAt).",
        L, reqs, exp))

    # TTL lapse: prev bucket last INCR at W60+100; at W60+60000+100 alive, +101 expired.
    reqs = [req(21, 1, W60 + 100) for _ in range(50)]
    reqs += [req(21, 0, W60 + 60100, op=1), req(21, 0, W60 + 60101, op=1)]
    exp = [[1, 99 - c, None] for c in range(50)]
    # at W60+60100: pct = 100/60000 = 0.0016666666666666668, pw = 0.9983333333333333;
    # 50*pw = 49.916666666666664 -> est 49 -> 51 available
    exp += [[0, 51, None]]
    # at +60101: prev expired (now > W60+100+60000) -> reads 0 although weight is ~1
    exp += [[0, 100, None]]
    out.append(case(
        "hand:sw:prevBucketTtlLapse",
        "SURVEY §0.3: PEXPIRE w on every INCR makes the previous bucket vanish once"
        " now > lastIncr(prev) + w, even though its weight is still non-zero.",
        L, reqs, exp))

    # permits > max: deny, no INCR, remaining reflects state
    reqs = [req(22, 1, W60 + 5), req(22, 101, W60 + 5), req(22, 100, W60 + 5),
            req(22, 99, W60 + 5)]
    exp = [[1, 99, None], [0, 99, None], [0, 99, None], [1, 98, None]]
    out.append(case(
        "hand:sw:permitsAboveMax",
        "est + permits > max denies without INCR; an allowed request INCRs by 1 only.",
        L, reqs, exp))

    # FMA discriminator (search in SURVEY §0.5): w=60000, prev 864, curr 398 at r=57500:
    # separately rounded est = 434; an FMA would give trunc(433.99999999999994) = 433.
    L2 = [[SW, 1000, 60000, 0.0]]
    Wb = W60 + 60000
    reqs = [req(23, 1, Wb - 100) for _ in range(864)]
    reqs += [req(23, 1, Wb + 57500) for _ in range(398)]
    reqs += [req(23, 0, Wb + 57500, op=1)]
    exp = [[1, 999 - c, None] for c in range(864)]
    # at Wb+57500: pct = 0.9583333333333334, pw = 0.04166666666666663,
    # 864*pw = 35.99999999999997 = 36 - 2^-45 exactly. c + 36 - 2^-45 is representable
    # while c + 36 <= 256 (ulp <= 2^-45) -> trunc = 35 + c; from c + 36 = 257 on the ulp is
    # 2^-44, the value is a tie and rounds to even = c + 36 -> trunc = 36 + c.
    exp2 = []
    for c in range(398):
        after = c + 1
        est_after = 35 + after if after + 36 <= 256 else 36 + after
        exp2.append([1, 1000 - est_after, None])
    exp += exp2 + [[0, 566, None]]
    out.append(case(
        "hand:sw:fmaDiscriminator",
        "(long)(prevCount*prevWeight + currCount) with two roundings (Java :174): at prev=864,"
        " curr=398, pw=0.04166666666666663 the sum rounds to 434.0; a fused multiply-add gives"
        " 433.99999999999994 -> 433. Also pins the rounding of 35.99999999999997 + c.",
        L2, reqs, exp))

    # Java truncating division for now < w: windowStart(now - w) = 0 = windowStart(now)
    L3 = [[SW, 10, 1000, 0.0]]
    reqs = [req(24, 1, 500) for _ in range(3)] + [req(24, 0, 500, op=1)]
    # at now=500: curr = prev = bucket 0; pw = 0.5; est = trunc(c*0.5 + c)
    # c=0 -> 0; after 1: trunc(1.5)=1 -> 9; c=1: est=1, after 2: trunc(3.0)=3 -> 7;
    # c=2: est=3, after 3: trunc(4.5)=4 -> 6; peek: 6
    exp = [[1, 9, None], [1, 7, None], [1, 6, None], [0, 6, None]]
    out.append(case(
        "hand:sw:javaTruncDivNearEpoch",
        "getWindowKey(key, now - w, w) with Java's truncating division maps now - w < 0 to"
        " window 0 for 0 <= now < w, so the current bucket is read twice.",
        L3, reqs, exp))

    # ---------- hand-derived TB ----------
    TBL = [[TB, 50, 1000, 10.0]]  # rate 0.01/ms, TTL 2000 ms, 2w*rate = 20 < cap
    reqs = [req(30, 40, T0), req(30, 1, T0 + 2000),
            req(31, 40, T0), req(31, 1, T0 + 2001)]
    exp = [[1, 10, 10.0],
           [1, 29, 29.0],   # alive at last+2w: 10 + 2000*0.01 = 30.0 -> 29.0
           [1, 10, 10.0],
           [1, 49, 49.0]]   # expired (now > last+2w): restarts full 50 -> 49
    out.append(case(
        "hand:tb:expiryBoundary",
        "PEXPIRE 2*window refreshed only on allow (TokenBucketRateLimiter.java:64,127); an"
        " expired bucket restarts full (:50-53) — matters because 2w*rate = 20 < cap 50.",
        TBL, reqs, exp))

    reqs = [req(32, 51, T0), req(32, 50, T0), req(32, 1, T0 + 100)]
    exp = [[0, UNK, None], [1, 0, 0.0], [1, 0, 0.0]]  # 0 + 100*0.01 = 1.0 -> 0.0
    out.append(case(
        "hand:tb:earlyReject",
        "permits > maxPermits is rejected before any storage access (:110-116) and leaves"
        " the bucket untouched (next request still sees a fresh full bucket).",
        TBL, reqs, exp))

    reqs = [req(33, 10, T0), req(33, 1, T0 - 100), req(33, 45, T0 - 100)]
    # x = 40 + (-100)*0.01 = 40 - 1.0 = 39.0 -> 38.0; then 38 < 45 deny (returns 38.0)
    exp = [[1, 40, 40.0], [1, 38, 38.0], [0, 38, 38.0]]
    out.append(case(
        "hand:tb:negativeElapsed",
        "elapsed = now - last_refill is not clamped (Lua :56-57); time regression removes"
        " tokens.",
        TBL, reqs, exp))

    reqs = [req(34, 3, T0), req(34, 0, T0 + 50, op=1), req(34, 0, T0 + 60, op=2),
            req(34, 0, T0 + 70, op=1), req(34, 50, T0 + 70)]
    exp = [[1, 47, 47.0],
           [0, 47, 47.5],   # peek: 47 + 50*0.01 = 47.5
           [0, 0, None],    # reset
           [0, 50, 50.0],   # absent -> capacity
           [1, 0, 0.0]]
    out.append(case(
        "hand:tb:peekReset",
        "build-defined peek (reference TB getAvailablePermits is broken: GET on a hash) and"
        " reset = DEL tb:key (:153-158).",
        TBL, reqs, exp))

    # FMA flips found by search (drain with 12x4 permits, then refills); separate rounding
    # (Lua) vs a single fused rounding differ at the decision threshold.
    d = [(T0, 4)] * 12
    flips = [
        (d + [(T0 + 72, 1), (T0 + 266, 4), (T0 + 268, 1), (T0 + 400, 4)],
         "tokens 2.6799999999999997 + 132*0.01: Lua 4.0 (allow), fused 3.9999999999999996"),
        (d + [(T0 + 27, 1), (T0 + 109, 1), (T0 + 200, 2)],
         "tokens 1.0899999999999999 + 91*0.01: Lua 2.0 (allow), fused 1.9999999999999998"),
        (d[:10] + [(T0 + 28, 1), (T0 + 85, 4), (T0 + 206, 2), (T0 + 289, 3), (T0 + 312, 2),
                   (T0 + 500, 3)],
         "tokens 1.1199999999999997 + 188*0.01: Lua 3.0 (allow), fused 2.9999999999999996"),
        (d + [(T0 + 30, 3), (T0 + 30, 2), (T0 + 42, 2), (T0 + 108, 1), (T0 + 242, 2),
              (T0 + 300, 2)],
         "tokens 0.07999999999999985 + 192*0.01: Lua 1.9999999999999998 (deny), fused 2.0"),
    ]
    for i, (seq, why) in enumerate(flips):
        reqs = [req(40 + i, p, t) for (t, p) in seq]
        out.append(case(f"hand:tb:fmaFlip{i}", why, TBL, reqs, lua_expect(seq)))

    # time regression (front-ends with skewed clocks): Redis keys every window separately
    reqs = [req(60, 1, W + 990) for _ in range(3)] + [req(60, 1, W + 1005), req(60, 1, W + 995),
                                                      req(60, 1, W + 1010)]
    # W+990 x3: fresh key -> 9, 8, 7. W+1005: prev = bucket W = 3 (alive to W+1990),
    # pw = 0.995, 3*0.995 = 2.985 -> est 2, allow, after trunc(3.985) = 3 -> 7.
    # W+995 (back into window W): curr = bucket W = 3, prev = bucket W-1000 absent -> est 3,
    # allow, INCR bucket W -> 4 (bucket W+1000 untouched) -> 6.
    # W+1010: curr = 1, prev = bucket W = 4 (alive to W+1995), pw = 0.99, 3.96 + 1 -> 4,
    # allow -> curr 2, trunc(5.96) = 5 -> 5.
    exp = [[1, 9, None], [1, 8, None], [1, 7, None], [1, 7, None], [1, 6, None], [1, 5, None]]
    out.append(case(
        "hand:sw:regressionPrevWindow",
        "a request whose now falls back into the previous window INCRs that window's bucket"
        " (RedisRateLimitStorage.java:38-49 keys by window start, :185-188) and leaves the"
        " newer bucket intact; the next request in the newer window weights the grown bucket.",
        [[SW, 10, 1000, 0.0]], reqs, exp))

    # a drained bucket read 1000 ms, 500 ms and 100 s before its last refill: the Lua reply
    # integer of a negative balance (tokens - 10, -5, -1000) — below the packed result range
    reqs = [req(35, 50, T0), req(35, 1, T0 - 1000), req(35, 1, T0 - 500),
            req(35, 1, T0 - 100_000), req(35, 0, T0 - 300, op=1), req(35, 1, T0 + 100)]
    exp = [[1, 0, 0.0], [0, -10, -10.0], [0, -5, -5.0], [0, -1000, -1000.0], [0, -3, -3.0],
           [1, 0, 0.0]]
    out.append(case(
        "hand:tb:deepNegative",
        "elapsed < 0 is not clamped (Lua :56-58): the balance and its reply integer go far"
        " below zero; nothing is persisted on deny (:66-67), so T0+100 refills from 0.",
        TBL, reqs, exp))

    # ---------- the SW local cache (Caffeine, expireAfterWrite 100 ms) ----------
    LC = [[SW, 10, 1000, 0.0, 0, 100]]   # [algo, max, w, refill, capacity, localCacheTtl ms]
    reqs = [req(80, 1, W + 10) for _ in range(10)]
    reqs += [req(80, 1, W + 50), req(80, 1, W + 109), req(80, 1, W + 110), req(80, 1, W + 209)]
    # 10 allows; the 10th puts newCount 10 >= max at W+10. W+50, W+109: getIfPresent hits
    # (age 40, 99 < 100) -> rejected without Redis, remaining = 10 - est(10) = 0. W+110: age
    # 100 -> expired -> est 10 -> deny, put 10 at W+110. W+209: age 99 -> hit again.
    exp = [[1, 9 - i, None] for i in range(10)] + [[0, 0, None]] * 4
    out.append(case(
        "ref:cache:rejectFromCache",
        "SlidingWindowRateLimiter.java:93-100: a cached count >= maxPermits rejects without a"
        " Redis read; put on allow (:119-121) and on deny (:106-108); expireAfterWrite(100 ms)"
        " (:57-64) returns an entry iff its age < 100 ms.",
        LC, reqs, exp))

    reqs = [req(81, 1, W + 900) for _ in range(10)]
    reqs += [req(81, 1, W + 999), req(81, 1, W + 1000), req(81, 1, W + 1050),
             req(81, 1, W + 1100), req(81, 1, W + 1101)]
    # W+900 x10 -> allows, put 10 at W+900. W+999: hit -> deny 0. W+1000 (new window): age
    # 100 -> expired; prev = 10 (alive to W+1900), pw 1.0 -> est 10 -> deny, put 10 at W+1000.
    # W+1050: hit (age 50) -> deny although Redis alone would allow: est = trunc(10 * 0.95) =
    # 9 -> remaining 1. W+1100: age 100 -> expired; est = trunc(10 * 0.9) = 9 -> allow, INCR
    # -> 1, put 1; after: trunc(9.0 + 1) = 10 -> 0. W+1101: pw 0.899, 8.99 + 1 -> 9 -> allow,
    # after trunc(8.99 + 2) = 10 -> 0.
    exp = [[1, 9 - i, None] for i in range(10)]
    exp += [[0, 0, None], [0, 0, None], [0, 1, None], [1, 0, None], [1, 0, None]]
    out.append(case(
        "hand:cache:outlivesWindowRollover",
        "the cache is keyed by the raw key (SlidingWindowRateLimiter.java:94), not by window,"
        " so a cached rejection outlives the window rollover for up to its TTL: at W+1050 the"
        " weighted estimate (9) would admit the request, the cached count (10) rejects it.",
        LC, reqs, exp))

    reqs = [req(82, 1, W + 10) for _ in range(9)]
    reqs += [req(82, 2, W + 20), req(82, 1, W + 30), req(82, 1, W + 40), req(82, 0, W + 45, op=1)]
    # 9 allows (remaining 9..1). W+20, permits 2: est 9 + 2 > 10 -> deny, put 9 (< max: no
    # short-circuit later). W+30: cached 9 < 10 -> Redis path, est 9 -> allow, put 10. W+40:
    # hit -> deny 0. The peek (getAvailablePermits :133-137) never consults the cache: 0.
    exp = [[1, 9 - i, None] for i in range(9)]
    exp += [[0, 1, None], [1, 0, None], [0, 0, None], [0, 0, None]]
    out.append(case(
        "hand:cache:putBelowMaxDoesNotReject",
        "a deny caches the estimate (:106-108); only a cached value >= maxPermits"
        " short-circuits (:95), so a permits-2 denial at est 9 leaves the next permits-1"
        " request to Redis.",
        LC, reqs, exp))

    reqs = [req(83, 1, W + 10) for _ in range(10)]
    reqs += [req(83, 1, W + 15), req(83, 0, W + 20, op=2), req(83, 1, W + 30)]
    exp = [[1, 9 - i, None] for i in range(10)] + [[0, 0, None], [0, 0, None], [1, 9, None]]
    out.append(case(
        "hand:cache:resetInvalidates",
        "reset deletes both buckets and invalidates the cached count"
        " (SlidingWindowRateLimiter.java:139-153): the next request is admitted at once.",
        LC, reqs, exp))

    # ---------- documented outputs of the reference (README / API_EXAMPLES) ----------
    API = [[SW, 100, 60000, 0.0]]     # apiRateLimiter, RateLimiterConfig.java:51-56
    AUTH = [[SW, 10, 60000, 0.0]]     # authRateLimiter, RateLimiterConfig.java:70-74
    BURST = [[TB, 50, 60000, 10.0]]   # burstRateLimiter, RateLimiterConfig.java:88-92
    Wa = W60 + 60000
    out.append(case(
        "doc:apiRemaining97",
        "API_EXAMPLES.md:39-47 / README.md:83-88: GET /api/data as one user, the third"
        " request answers remaining 97 = getAvailablePermits after tryAcquire"
        " (DemoController.java:45-51). The api limiter's local cache only short-circuits at"
        " >= maxPermits (SlidingWindowRateLimiter.java:95), so it does not change this.",
        API, [req(70, 1, Wa + 1000) for _ in range(3)],
        [[1, 99, None], [1, 98, None], [1, 97, None]]))
    reqs = [req(71, 1, Wa + 2000) for _ in range(101)]
    out.append(case(
        "doc:rateLimitExceededRemaining0",
        "API_EXAMPLES.md:50-56 / README.md:90-95: past 100 requests in the minute the 429"
        " body reports remaining 0 (DemoController.java:131-135).",
        API, reqs, [[1, 99 - i, None] for i in range(100)] + [[0, 0, None]]))
    out.append(case(
        "doc:loginRemainingAttempts7",
        "API_EXAMPLES.md:61-77: POST /api/login (10/min, no cache) answers"
        " remaining_attempts 7 on the third attempt (DemoController.java:67-75).",
        AUTH, [req(72, 1, Wa + 3000) for _ in range(3)],
        [[1, 9, None], [1, 8, None], [1, 7, None]]))
    out.append(case(
        "doc:batchTokensRemaining30",
        "API_EXAMPLES.md:84-101: POST /api/batch size 20 on a fresh bucket (cap 50, 10/s)"
        " answers tokens_remaining 30 (DemoController.java:92-99): the Lua reply"
        " {1, 50 - 20} and the build-defined peek right after it.",
        BURST, [req(73, 20, T0), req(73, 0, T0, op=1)], [[1, 30, 30.0], [0, 30, 30.0]]))
    return out


def lua_expect(seq, cap=50.0, rate=10.0 / 1000.0, ttl=2000):
    """Step-by-step evaluation of the Lua script text for one key (used only for the
    FMA-flip KATs, whose expected balances are long to write by hand). Each line maps to
    TokenBucketRateLimiter.java:46-67; Python floats round every op separately."""
    tokens = last = None
    exp_at = None
    out = []
    for (t, p) in seq:
        if p > cap:
            out.append([0, UNK, None])
            continue
        now = float(t)
        if tokens is None or t > exp_at:
            tk, lr = cap, now
        else:
            tk, lr = tokens, last
        elapsed = now - lr
        add = elapsed * rate
        x = tk + add
        tk = x if x < cap else cap
        if tk >= p:
            tk = tk - p
            tokens, last, exp_at = tk, now, t + ttl
            out.append([1, int(tk), tk])
        else:
            out.append([0, int(tk), tk])
    return out


# ---------------------------------------------------------------- random traces
def make_trace(seed, n, n_keys, limiters, t_span_ms, op_rate=0.0, invalid_rate=0.0,
               zipf=1.1, permits_max=4):
    rng = np.random.default_rng(seed)
    ranks = np.minimum(rng.zipf(zipf, size=n), n_keys) - 1 if zipf else rng.integers(0, n_keys, n)
    keys = (ranks.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(seed)
    lim = (ranks % len(limiters)).astype(np.uint16)   # disjoint key space per limiter
    t = np.sort(rng.integers(0, t_span_ms * NS, n)) + T0 * NS
    permits = rng.integers(1, permits_max + 1, n).astype(np.int32)
    ops = np.zeros(n, np.uint8)
    if op_rate:
        r = rng.random(n)
        ops[r < op_rate] = 1
        ops[r < op_rate / 4] = 2
    if invalid_rate:
        bad = rng.random(n) < invalid_rate
        permits[bad] = rng.integers(-3, 1, int(bad.sum()))
    return keys, permits, t.astype(np.int64), lim, ops


TRACES = {
    "sw_small": dict(seed=11, n=4000, n_keys=60, t_span_ms=150_000,
                     limiters=[[SW, 10, 60000, 0.0], [SW, 100, 60000, 0.0], [SW, 5, 1000, 0.0]],
                     op_rate=0.05, invalid_rate=0.01),
    "tb_small": dict(seed=12, n=4000, n_keys=40, t_span_ms=20_000,
                     limiters=[[TB, 50, 60000, 10.0], [TB, 20, 1000, 3.0], [TB, 7, 500, 13.0]],
                     op_rate=0.05, invalid_rate=0.01),
    "mixed_small": dict(seed=13, n=6000, n_keys=300, t_span_ms=200_000,
                        limiters=[[SW, 10, 60000, 0.0], [SW, 100, 60000, 0.0],
                                  [TB, 50, 60000, 10.0], [SW, 1000, 3600000, 0.0],
                                  [TB, 5, 1000, 1.0]],
                        op_rate=0.03, invalid_rate=0.005),
    "hot_small": dict(seed=14, n=5000, n_keys=5, t_span_ms=30_000,
                      limiters=[[SW, 50, 10000, 0.0], [TB, 30, 10000, 2.0]], zipf=2.0),
}


def main():
    from oracle.coracle import COracle, build
    build()
    cases = kats()
    for c in cases:
        for impl in ("py", "c"):
            o = PyOracle() if impl == "py" else COracle()
            for spec in c["limiters"]:
                o.add_limiter(*spec)
            r = np.array(c["requests"], dtype=object)
            args = (np.array(r[:, 0], np.uint64), np.array(r[:, 1], np.int32),
                    np.array(r[:, 2], np.int64), np.array(r[:, 3], np.uint16),
                    np.array(r[:, 4], np.uint8))
            res = o.run(*args)
            a, rem, tok = res[0], res[1], res[2]
            for i, (ea, er, et) in enumerate(c["expected"]):
                ok = int(a[i]) == ea and int(rem[i]) == er
                if et is not None:
                    ok &= float(tok[i]) == et
                if not ok:
                    raise SystemExit(f"{impl} oracle disagrees with KAT {c['name']}[{i}]: "
                                     f"got {(int(a[i]), int(rem[i]), float(tok[i]))}, "
                                     f"expected {(ea, er, et)}")
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": cases}, f, indent=0)
    print(f"kats.json: {len(cases)} cases, all reproduced by both oracles")

    arrays = {}
    for name, spec in TRACES.items():
        spec = dict(spec)
        limiters = spec.pop("limiters")
        keys, permits, now, lim, ops = make_trace(limiters=limiters, **spec)
        py = PyOracle()
        co = COracle()
        for l in limiters:
            py.add_limiter(*l)
            co.add_limiter(*l)
        pa, pr, pt = py.run(keys, permits, now, lim, ops)
        ca, cr, ct, _ = co.run(keys, permits, now, lim, ops)
        pa, pr, pt = np.array(pa, np.uint8), np.array(pr, np.int64), np.array(pt, np.float64)
        assert (pa == ca).all() and (pr == cr).all(), name
        assert np.array_equal(pt.view(np.uint64)[~np.isnan(pt)],
                              ct.view(np.uint64)[~np.isnan(ct)]), name
        for k, v in (("keys", keys), ("permits", permits), ("now_ns", now), ("limiter", lim),
                     ("op", ops), ("allowed", pa), ("remaining", pr), ("tokens", pt),
                     ("limiters", np.array(limiters, np.float64))):
            arrays[f"{name}__{k}"] = v
        print(f"{name}: n={len(keys)} allowed={int(pa.sum())} invalid={int((pr == -2).sum())}")
    np.savez_compressed(os.path.join(HERE, "traces.npz"), **arrays)


if __name__ == "__main__":
    main()
