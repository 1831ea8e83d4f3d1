"""State export / import in the Redis keyspace layout (rl_export_state / rl_import_state,
SURVEY §8(f) row 4) against the oracle's own Redis keyspace, bit-exact.

The oracle (oracle/rl_oracle.py) keeps the reference's literal keyspace: "rl:<key>:<W>"
counters with their PEXPIRE deadlines (SlidingWindowRateLimiter.java:185-188,
RedisRateLimitStorage.java:38-49) and "tb:<key>" hashes (TokenBucketRateLimiter.java:46-64).
After the same trace, the engine's export must equal the oracle's live keys, and an engine
seeded by import must continue the trace exactly as the oracle does.
"""
import numpy as np
import pytest

import rl_amd
from oracle.rl_oracle import PyOracle

pytestmark = pytest.mark.gpu

NS = 1_000_000
T0 = 1_700_000_000_000
LIMS = [(rl_amd.SW, 5, 1000, 0.0), (rl_amd.TB, 10, 1000, 5.0),
        (rl_amd.SW, 3, 500, 0.0), (rl_amd.TB, 4, 300, 20.0)]


def make(lims=LIMS, **kw):
    e = rl_amd.Engine(max_batch=1 << 18, capacity=1 << 12, **kw)
    o = PyOracle()
    for l in lims:
        e.add_limiter(*l)
        o.add_limiter(*l)
    return e, o


def trace(seed, n, t_lo, t_hi, n_keys=300, resets=True):
    rng = np.random.default_rng(seed)
    lim = rng.integers(0, len(LIMS), n).astype(np.uint16)
    keys = (rng.integers(0, n_keys, n).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
            + lim.astype(np.uint64))
    now = np.sort(rng.integers(t_lo * NS, t_hi * NS, n)).astype(np.int64)
    permits = rng.integers(1, 4, n).astype(np.int32)
    ops = np.zeros(n, np.uint8)
    if resets:
        ops[rng.random(n) < 0.01] = rl_amd.OP_RESET
    return keys, permits, now, lim, ops


def run_both(e, o, tr):
    keys, permits, now, lim, ops = tr
    a, r, t, st = e.execute(keys, permits, now, lim, ops)
    wa, wr, wt = o.run(keys, permits, now, lim, ops)
    assert st == rl_amd.RL_OK
    np.testing.assert_array_equal(a, np.asarray(wa, np.uint8))
    np.testing.assert_array_equal(r, np.asarray(wr, np.int64))
    return a, r


def as_tuples(ex):
    return [(int(x["limiter"]), int(x["key_hash"]), int(x["kind"]), int(x["window_start_ms"]),
             int(x["count"]), float(x["tokens"]), int(x["last_refill_ms"]), int(x["expire_at_ms"]))
            for x in ex]


def assert_keyspace(got, want):
    assert len(got) == len(want), (len(got), len(want))
    for g, w in zip(got, want):
        assert g[:5] == w[:5] and g[6:] == w[6:], (g, w)
        assert np.float64(g[5]).view(np.uint64) == np.float64(w[5]).view(np.uint64), (g, w)


@pytest.mark.parametrize("lag_ms", [0, 250, 700, 2500])
def test_export_matches_oracle_keyspace(lag_ms):
    e, o = make()
    run_both(e, o, trace(1, 20000, T0, T0 + 3000))
    run_both(e, o, trace(2, 20000, T0 + 3000, T0 + 6000))
    now_ms = T0 + 6000 + lag_ms
    got = as_tuples(e.export_state(now_ms * NS))
    want = o.keyspace(now_ms)
    if lag_ms <= 700:
        assert len(want) > 100
    assert_keyspace(got, want)
    kinds = {g[2] for g in got}
    if lag_ms == 0:
        assert kinds == {0, 1}


def test_import_continues_like_the_oracle():
    e, o = make()
    run_both(e, o, trace(3, 30000, T0, T0 + 4000))
    cut = T0 + 4000
    dump = e.export_state(cut * NS)
    assert_keyspace(as_tuples(dump), o.keyspace(cut))
    # a fresh engine seeded from the dump continues exactly like the oracle
    e2, o2 = make()
    st, taken = e2.import_state(dump)
    assert st == rl_amd.RL_OK and taken == dump.shape[0]
    o2.load_keyspace(o.keyspace(cut))
    tr = trace(4, 30000, cut, cut + 3000)
    a1, r1 = run_both(e, o, tr)
    a2, r2 = run_both(e2, o2, tr)
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(r1, r2)
    assert_keyspace(as_tuples(e2.export_state((cut + 3000) * NS)), o.keyspace(cut + 3000))


def test_import_replaces_existing_keys_and_round_trips():
    e, o = make()
    run_both(e, o, trace(5, 10000, T0, T0 + 2000))
    dump = e.export_state((T0 + 2000) * NS)
    # importing the engine's own state back is a no-op
    st, taken = e.import_state(dump)
    assert st == rl_amd.RL_OK and taken == dump.shape[0]
    assert_keyspace(as_tuples(e.export_state((T0 + 2000) * NS)), as_tuples(dump))
    # overwrite one TB balance and one SW counter
    tb = np.nonzero(dump["kind"] == rl_amd.STATE_TB_BUCKET)[0][0]
    sw = np.nonzero(dump["kind"] == rl_amd.STATE_SW_BUCKET)[0][-1]
    patch = dump[[tb, sw]].copy()
    patch["tokens"][0] = 0.25
    patch["count"][1] = 1
    assert e.import_state(patch)[0] == rl_amd.RL_OK
    after = e.export_state((T0 + 2000) * NS)
    d = {(int(x["limiter"]), int(x["key_hash"]), int(x["window_start_ms"])): x for x in after}
    assert d[(int(patch[0]["limiter"]), int(patch[0]["key_hash"]), 0)]["tokens"] == 0.25
    assert d[(int(patch[1]["limiter"]), int(patch[1]["key_hash"]),
              int(patch[1]["window_start_ms"]))]["count"] == 1
    assert after.shape == dump.shape


def test_import_rejects_what_redis_could_not_hold():
    e, _ = make()
    x = np.zeros(1, rl_amd.STATE_DTYPE)
    x["key_hash"], x["limiter"], x["kind"] = 7, 1, rl_amd.STATE_SW_BUCKET   # limiter 1 is TB
    assert e.import_state(x)[0] == rl_amd.RL_E_INVALID_ARG
    x["kind"], x["tokens"], x["last_refill_ms"] = rl_amd.STATE_TB_BUCKET, 3.5, T0
    x["expire_at_ms"] = T0 + 1000                                          # TB TTL is 2w = 2000
    assert e.import_state(x)[0] == rl_amd.RL_E_INVALID_ARG
    x["expire_at_ms"] = T0 + 2000
    assert e.import_state(x) == (rl_amd.RL_OK, 1)
    y = np.zeros(1, rl_amd.STATE_DTYPE)
    y["key_hash"], y["limiter"], y["kind"], y["count"] = 9, 0, rl_amd.STATE_SW_BUCKET, 2
    y["window_start_ms"] = T0 + 1                                          # not a multiple of w
    y["expire_at_ms"] = T0 + 1001
    assert e.import_state(y)[0] == rl_amd.RL_E_INVALID_ARG
    y["window_start_ms"], y["expire_at_ms"] = T0, T0 + 2000                # deadline > W + 2w - 1
    assert e.import_state(y)[0] == rl_amd.RL_E_INVALID_ARG
    y["expire_at_ms"] = T0 + 1500
    assert e.import_state(y) == (rl_amd.RL_OK, 1)
    x[0]["limiter"] = 200
    assert e.import_state(x)[0] == rl_amd.RL_E_INVALID_ARG
    # the valid ones are visible through the read path
    avail, st = e.available(1, np.array([7], np.uint64), np.array([T0 * NS], np.int64))
    assert st == rl_amd.RL_OK and avail[0] == 3
    assert as_tuples(e.export_state(T0 * NS)) == [
        (0, 9, 0, T0, 2, 0.0, 0, T0 + 1500), (1, 7, 1, 0, 0, 3.5, T0, T0 + 2000)]


def test_sharded_import_takes_only_owned_keys():
    e, o = make()
    run_both(e, o, trace(6, 10000, T0, T0 + 2000))
    dump = e.export_state((T0 + 2000) * NS)
    owners = rl_amd.owner_of(dump["key_hash"], 2)
    got = []
    for s in range(2):
        es, _ = make(shard_index=s, shard_count=2)
        st, taken = es.import_state(dump)
        assert st == rl_amd.RL_OK and taken == int((owners == s).sum())
        got += as_tuples(es.export_state((T0 + 2000) * NS))
    got.sort(key=lambda x: (x[0], x[1], x[3]))
    assert_keyspace(got, as_tuples(dump))


def test_ttl_sweep_frees_exactly_the_dead_slots():
    e, o = make()
    run_both(e, o, trace(7, 20000, T0, T0 + 3000))
    now_ms = T0 + 3400
    before = e.export_state(now_ms * NS)
    e.sweep_expired(now_ms * NS)
    assert e.sweep_expired(now_ms * NS) == 0                 # idempotent
    after = e.export_state(now_ms * NS)
    assert_keyspace(as_tuples(after), as_tuples(before))     # live state untouched
    assert_keyspace(as_tuples(after), o.keyspace(now_ms))
    live_keys = len({(int(x["limiter"]), int(x["key_hash"])) for x in after})
    assert live_keys > 100
    # far in the future every remaining slot is dead: exactly the live keys are freed
    assert e.sweep_expired((now_ms + 10_000) * NS) == live_keys
    assert e.export_state(now_ms * NS).shape[0] == 0
    # a swept table keeps deciding like the oracle
    run_both(e, o, trace(8, 20000, now_ms + 10_000, now_ms + 12_000))


@pytest.mark.parametrize("algo", [rl_amd.SW, rl_amd.TB])
def test_export_after_hot_regions(algo):
    """Hot keys are applied by the hot-region chain (k_hot_summ / hot_chain / k_hot_fill);
    the state it writes back must export exactly like the oracle's keyspace."""
    from test_gpu_hot import hot_trace
    lims = [(algo, 50, 1000, 10.0 if algo == rl_amd.TB else 0.0)]
    e, o = make(lims)
    e.tune("hot_threshold", 256)
    tr = hot_trace(11, 60000, 2000, 0.4, [0], 4000, hot_keys=3, ops=0.002)
    for sl in (slice(0, 30000), slice(30000, 60000)):
        part = tuple(x[sl] for x in tr)
        a, r, t, st = e.execute(*part)
        wa, wr, wt = o.run(*part)
        assert st == rl_amd.RL_OK
        np.testing.assert_array_equal(a, np.asarray(wa, np.uint8))
        np.testing.assert_array_equal(r, np.asarray(wr, np.int64))
    end_ms = int(tr[2][-1]) // NS
    for lag in (0, 600):
        assert_keyspace(as_tuples(e.export_state((end_ms + lag) * NS)), o.keyspace(end_ms + lag))
