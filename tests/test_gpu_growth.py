"""On-demand state-table growth (rl_grow_limiter / automatic doubling), checked against the
oracle. Redis creates keys as they come (RedisRateLimitStorage.java:38-49, INCR/HMSET on a
missing key), so a drop-in engine must not run out of slots: a limiter whose regions fill
past 62.5 % is doubled (every region split in two by the next tag bit, k_grow) before its
next batch, with every key's state carried over bit for bit."""
import numpy as np
import pytest

import rl_amd
from oracle.coracle import COracle
from test_gpu_parity import NS, T0, assert_same

pytestmark = pytest.mark.gpu

LIMS = [[rl_amd.TB, 7, 2_000, 3.0, 1, 0],          # TB: balances in fp64
        [rl_amd.SW, 5, 1_000, 0.0, 1, 0],          # SW, cache off (parity mode)
        [rl_amd.SW, 4, 1_000, 0.0, 1, 40]]         # SW with the Caffeine local cache (40 ms)


def engine(**kw):
    e = rl_amd.Engine(max_batch=1 << 18, capacity=1, **kw)
    for l in LIMS:
        e.add_limiter(l[0], l[1], l[2], l[3], capacity=l[4], local_cache_ttl_ms=l[5])
    return e


def batch(rng, known, fresh, t_ms, n_old):
    """n_old requests on already-seen keys plus `fresh` new keys (3 requests each)."""
    keys = [rl_amd.mix64(np.arange(known, known + fresh, dtype=np.uint64) + np.uint64(7 << 40))]
    keys = np.repeat(keys[0], 3)
    if known and n_old:
        old = rl_amd.mix64(rng.integers(0, known, n_old).astype(np.uint64) + np.uint64(7 << 40))
        keys = np.concatenate([keys, old])
    keys = keys[rng.permutation(keys.size)]
    n = keys.size
    lim = (rl_amd.mix64(keys) % np.uint64(len(LIMS))).astype(np.uint16)   # a key keeps its limiter
    now = (t_ms * NS + np.sort(rng.integers(0, 300 * NS, n))).astype(np.int64)
    permits = rng.integers(1, 3, n).astype(np.int32)
    return keys, permits, now, lim


def test_automatic_growth_matches_oracle():
    rng = np.random.default_rng(11)
    e = engine()
    o = COracle(LIMS)
    slots0 = [e.limiter_slots(i) for i in range(len(LIMS))]
    known, t = 0, T0
    for b in range(14):
        # each batch brings about 1/8 of the smallest current table as new keys
        fresh = min(e.limiter_slots(i) for i in range(len(LIMS))) // 8 * len(LIMS)
        k, p, now, lim = batch(rng, known, fresh, t, 4000)
        known += fresh
        t += 250
        a, r, tok, st = e.execute(k, p, now, lim)
        assert st == rl_amd.RL_OK, (b, rl_amd.strerror(st))
        assert_same((a, r, tok), o.run(k, p, now, lim), f"batch {b}")
    st = e.stats()
    assert st["table_grows"] >= 3
    assert all(e.limiter_slots(i) > slots0[i] for i in range(len(LIMS)))
    assert st["capacity_errors"] == 0
    o.close()


def test_explicit_grow_keeps_keyspace():
    rng = np.random.default_rng(12)
    e = engine()
    o = COracle(LIMS)
    k, p, now, lim = batch(rng, 0, 300, T0, 0)
    assert_same(e.execute(k, p, now, lim)[:3], o.run(k, p, now, lim)[:3], "before")
    at = int(now[-1])
    before = np.sort(e.export_state(at), order=["limiter", "key_hash", "kind", "window_start_ms"])
    for li in range(len(LIMS)):
        e.grow_limiter(li, 200_000)
        assert e.limiter_slots(li) >= 400_000
    after = np.sort(e.export_state(at), order=["limiter", "key_hash", "kind", "window_start_ms"])
    assert before.size > 0 and np.array_equal(before, after)
    # the grown tables continue the trace exactly (incl. local-cache words moved with slots)
    k2, p2, now2, lim2 = batch(rng, 300, 500, T0 + 100, 3000)
    assert_same(e.execute(k2, p2, now2, lim2)[:3], o.run(k2, p2, now2, lim2)[:3], "after grow")
    o.close()


def test_overflow_then_growth():
    """A burst larger than the table overflows (RL_E_CAPACITY, those requests untouched);
    the table then doubles twice and the same keys go through on the next batch."""
    e = rl_amd.Engine(max_batch=1 << 16, capacity=1)
    e.add_limiter(rl_amd.TB, 5, 60_000, 1.0, capacity=1)
    n = 3000
    keys = rl_amd.mix64(np.arange(n, dtype=np.uint64))
    slots = e.limiter_slots(0)
    a, r, _, st = e.execute(keys, np.ones(n, np.int32), np.full(n, T0 * NS, np.int64))
    assert st == rl_amd.RL_E_CAPACITY
    assert e.limiter_slots(0) == 4 * slots
    failed = r == rl_amd.REM_ERROR
    assert failed.sum() > 0
    a2, r2, _, st2 = e.execute(keys, np.ones(n, np.int32), np.full(n, (T0 + 1) * NS, np.int64))
    assert st2 == rl_amd.RL_OK
    # keys that failed before start from a full bucket; the others have spent one token
    assert np.array_equal(r2[failed], np.full(failed.sum(), 4))
    assert np.array_equal(r2[~failed], np.full((~failed).sum(), 3))


def test_fixed_capacity_does_not_grow():
    e = rl_amd.Engine(max_batch=1 << 16, capacity=1, fixed_capacity=True)
    e.add_limiter(rl_amd.TB, 5, 60_000, 1.0, capacity=1)
    slots = e.limiter_slots(0)
    keys = rl_amd.mix64(np.arange(3000, dtype=np.uint64))
    _, _, _, st = e.execute(keys, np.ones(3000, np.int32), np.full(3000, T0 * NS, np.int64))
    assert st == rl_amd.RL_E_CAPACITY
    assert e.limiter_slots(0) == slots and e.stats()["table_grows"] == 0
