"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit-exact.

Decisions and remaining are compared exactly; TB balances (tokens_after) are
compared bit-for-bit (stricter than north_star's 1e-9 relative bound).
"""
import numpy as np
import pytest

import rl_amd
from golden_io import kat_arrays, load_kats, load_traces
from oracle.coracle import COracle

pytestmark = pytest.mark.gpu

NS = 1_000_000
T0 = 1_700_000_000_000


def engine(limiters, **kw):
    kw.setdefault("max_batch", 1 << 21)
    kw.setdefault("capacity", 1 << 14)
    e = rl_amd.Engine(**kw)
    for l in limiters:
        e.add_limiter(*l)
    return e


def assert_same(got, want, what=""):
    ga, gr, gt = got[0], got[1], got[2]
    wa, wr, wt = want[0], want[1], want[2]
    ga = np.asarray(ga); wa = np.asarray(wa, np.uint8)
    gr = np.asarray(gr); wr = np.asarray(wr, np.int64)
    bad = np.nonzero((ga != wa) | (gr != wr))[0]
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first at {bad[:5]}: " \
                          f"got {list(zip(ga[bad[:5]], gr[bad[:5]]))} " \
                          f"want {list(zip(wa[bad[:5]], wr[bad[:5]]))}"
    if gt is not None and wt is not None:
        gt = np.asarray(gt, np.float64); wt = np.asarray(wt, np.float64)
        assert np.array_equal(np.isnan(gt), np.isnan(wt)), what
        m = ~np.isnan(wt)
        assert np.array_equal(gt[m].view(np.uint64), wt[m].view(np.uint64)), what


# ------------------------------------------------------------------ golden vectors
@pytest.mark.parametrize("case", load_kats(), ids=[c["name"] for c in load_kats()])
def test_kat(case):
    e = engine(case["limiters"])
    a, r, t, st = e.execute(*kat_arrays(case))
    exp = case["expected"]
    want_t = np.array([np.nan if x[2] is None else x[2] for x in exp])
    got_t = t.copy()
    got_t[np.isnan(want_t)] = np.nan           # KATs leave some balances unspecified
    assert_same((a, r, got_t), ([x[0] for x in exp], [x[1] for x in exp], want_t), case["name"])
    expect_invalid = any(x[1] == -2 for x in exp)
    assert st == (rl_amd.RL_E_INVALID_REQUEST if expect_invalid else rl_amd.RL_OK)


@pytest.mark.parametrize("name", sorted(load_traces()))
def test_golden_trace(name):
    d = load_traces()[name]
    e = engine(d["limiters"])
    got = e.execute(d["keys"], d["permits"], d["now_ns"], d["limiter"], d["op"])
    assert_same(got, (d["allowed"], d["remaining"], d["tokens"]), name)


# ------------------------------------------------------------------ seeded random traces
def trace(seed, n, n_keys, n_lim, span_ms, zipf=None, permits_max=4, ops=0.0, invalid=0.0):
    rng = np.random.default_rng(seed)
    if zipf:
        ranks = np.minimum(rng.zipf(zipf, n), n_keys) - 1
    else:
        ranks = rng.integers(0, n_keys, n)
    keys = rl_amd.mix64(ranks.astype(np.uint64) + np.uint64(seed << 40))
    lim = (ranks % n_lim).astype(np.uint16)
    now = (T0 * NS + np.sort(rng.integers(0, span_ms * NS, n))).astype(np.int64)
    permits = rng.integers(1, permits_max + 1, n).astype(np.int32)
    op = np.zeros(n, np.uint8)
    if ops:
        u = rng.random(n)
        op[u < ops] = 1
        op[u < ops / 3] = 2
    if invalid:
        bad = rng.random(n) < invalid
        permits[bad] = 0
    return keys, permits, now, lim, op


def run_both(limiters, tr, batches=1, **kw):
    e = engine(limiters, **kw)
    o = COracle(limiters)
    n = len(tr[0])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    got = [[], [], []]
    for b in range(batches):
        sl = slice(cuts[b], cuts[b + 1])
        a, r, t, st = e.execute(*(x[sl] for x in tr))
        assert st in (rl_amd.RL_OK, rl_amd.RL_E_INVALID_REQUEST), rl_amd.strerror(st)
        got[0].append(a); got[1].append(r); got[2].append(t)
    want = o.run(*tr)
    return tuple(np.concatenate(g) for g in got), want, e


def test_tb_uniform_1m():
    lims = [[rl_amd.TB, 50, 60000, 10.0]]
    tr = trace(1, 1_000_000, 20_000, 1, 2_000)
    got, want, e = run_both(lims, tr)
    assert_same(got, want, "tb_uniform")
    s = e.stats()
    assert s["allowed"] == int(want[0].sum())
    assert s["distinct_keys"] == len(np.unique(tr[0]))


def test_sw_zipf_hot_keys_1m():
    lims = [[rl_amd.SW, 1000, 60000, 0.0]]
    tr = trace(2, 1_000_000, 200_000, 1, 90_000, zipf=1.1, permits_max=1)
    got, want, _ = run_both(lims, tr, capacity=1 << 17)
    assert_same(got, want, "sw_zipf")


def test_mixed_limiters_ops_multi_batch():
    lims = [[rl_amd.SW, 10, 60000, 0.0], [rl_amd.SW, 100, 60000, 0.0],
            [rl_amd.TB, 50, 60000, 10.0], [rl_amd.SW, 5, 1000, 0.0], [rl_amd.TB, 3, 500, 7.0],
            [rl_amd.SW, 1000, 3_600_000, 0.0]]
    tr = trace(3, 600_000, 30_000, len(lims), 300_000, zipf=1.3, ops=0.04, invalid=0.002)
    got, want, _ = run_both(lims, tr, batches=7)
    assert_same(got, want, "mixed multi-batch")


def test_state_persists_across_many_small_batches():
    lims = [[rl_amd.TB, 20, 2000, 5.0], [rl_amd.SW, 30, 2000, 0.0]]
    tr = trace(4, 40_000, 500, 2, 20_000)
    got, want, _ = run_both(lims, tr, batches=40)
    assert_same(got, want, "many batches")


def test_ttl_reclamation_reuses_slots():
    # tiny table (1 region = REGION_SLOTS slots): 3 waves of 0.6*slots distinct keys each,
    # 10 s apart with a 1 s window -> earlier keys expire and their slots must be reclaimed
    # (two waves together would not fit).
    lims = [[rl_amd.TB, 5, 1000, 2.0, 1], [rl_amd.SW, 5, 1000, 0.0, 1]]
    parts = []
    nk = int(rl_amd.REGION_SLOTS * rl_amd.MIN_REGIONS * 0.6)
    for w in range(3):
        k = rl_amd.mix64(np.arange(nk, dtype=np.uint64) + np.uint64(w * 1000))
        k = np.repeat(k, 3)
        now = np.full(k.shape, (T0 + w * 10_000) * NS, np.int64) + np.arange(k.size) * 1000
        parts.append((k, np.ones(k.size, np.int32), now, (np.arange(k.size) % 2).astype(np.uint16)))
    # capacity 1 -> each limiter has exactly one bin of regions; fixed, so slots are reused
    e = rl_amd.Engine(max_batch=1 << 16, capacity=1, fixed_capacity=True)
    for l in lims:
        e.add_limiter(*l[:4], capacity=1)
    o = COracle([l[:4] for l in lims])
    for p in parts:
        a, r, t, st = e.execute(*p)
        assert st == rl_amd.RL_OK, rl_amd.strerror(st)
        assert_same((a, r, t), o.run(*p), "reclaim")


def test_capacity_overflow_reported():
    e = rl_amd.Engine(max_batch=1 << 16, capacity=1)
    e.add_limiter(rl_amd.TB, 5, 60000, 1.0, capacity=1)     # MIN_REGIONS regions
    n = 3000
    keys = rl_amd.mix64(np.arange(n, dtype=np.uint64))
    a, r, t, st = e.execute(keys, np.ones(n, np.int32), np.full(n, T0 * NS, np.int64))
    assert st == rl_amd.RL_E_CAPACITY
    # region = top log2(MIN_REGIONS) bits of mix64(key); each holds REGION_SLOTS keys
    bits = rl_amd.MIN_REGIONS.bit_length() - 1
    region = (rl_amd.mix64(keys) >> np.uint64(64 - bits)).astype(np.int64)
    per = np.bincount(region, minlength=rl_amd.MIN_REGIONS)
    overflow = np.maximum(per - rl_amd.REGION_SLOTS, 0).sum()
    assert overflow > 0
    assert (r == rl_amd.REM_ERROR).sum() == overflow
    assert a.sum() == n - overflow


def test_wide_records_large_max():
    lims = [[rl_amd.SW, 5_000_000, 60000, 0.0], [rl_amd.TB, 1 << 40, 60000, 1e9]]
    rng = np.random.default_rng(5)
    n = 200_000
    keys = rl_amd.mix64(rng.integers(0, 1000, n).astype(np.uint64))
    permits = rng.integers(1, 3_000_000, n).astype(np.int32)
    now = (T0 * NS + np.sort(rng.integers(0, 100_000 * NS, n))).astype(np.int64)
    lim = rng.integers(0, 2, n).astype(np.uint16)
    got, want, _ = run_both(lims, (keys, permits, now, lim, np.zeros(n, np.uint8)))
    assert_same(got, want, "wide")


def test_two_pass_partition_many_regions():
    # 4M-key capacity -> 16384 regions (14 bits) -> two partition passes
    lims = [[rl_amd.TB, 50, 60000, 10.0], [rl_amd.SW, 100, 60000, 0.0]]
    e_kw = dict(capacity=1 << 22)
    tr = trace(6, 800_000, 300_000, 2, 60_000, ops=0.01)
    got, want, _ = run_both(lims, tr, batches=2, **e_kw)
    assert_same(got, want, "two-pass")


def test_time_span_overflow():
    """A batch spanning more than the compact record's 2^32 ms: the device entry point
    rejects it whole before any state is touched (RL_E_INVALID_ARG, every request -2);
    the host entry point then re-runs it in 32-B records, exactly; rl_tune wide_records
    makes the device entry point take it too."""
    import torch
    lims = [[rl_amd.TB, 50, 60000, 10.0]]
    e = engine(lims)
    o = COracle(lims)
    k = rl_amd.mix64(np.arange(10, dtype=np.uint64))
    ok = (k, np.ones(10, np.int32), np.full(10, T0 * NS, np.int64), None, None)
    e.execute(*ok)
    o.run(k, ok[1], ok[2])
    far = np.full(10, T0 * NS, np.int64)
    far[5] = (T0 + (1 << 33)) * NS                   # ~99 days later
    dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda()
           for x in (k.view(np.int64), np.ones(10, np.int32), far)]
    a = torch.empty(10, dtype=torch.uint8, device="cuda")
    r = torch.empty(10, dtype=torch.int64, device="cuda")
    e.execute_device(10, *dev, None, None, a, r)
    assert e.last_status() == rl_amd.RL_E_INVALID_ARG
    assert (r.cpu().numpy() == rl_amd.REM_INVALID).all()
    got = e.execute(k, np.full(10, 2, np.int32), far)     # host entry: exact, in wide records
    assert got[3] == rl_amd.RL_OK
    assert_same(got[:3], o.run(k, np.full(10, 2, np.int32), far)[:3], "span retry")
    e.tune("wide_records", 1)
    nxt = (k, np.ones(10, np.int32), far + NS)
    dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k.view(np.int64), nxt[1], nxt[2])]
    e.execute_device(10, *dev, None, None, a, r)
    assert e.last_status() == rl_amd.RL_OK
    want = o.run(*nxt)
    assert_same((a.cpu().numpy(), r.cpu().numpy(), None), want[:3], "wide_records")


def test_invalid_requests():
    lims = [[rl_amd.SW, 10, 1000, 0.0]]
    e = engine(lims)
    keys = np.arange(6, dtype=np.uint64)
    permits = np.array([1, 0, -5, 2, 1, 1], np.int32)
    lim = np.array([0, 0, 0, 7, 0, 0], np.uint16)
    ops = np.array([0, 0, 0, 0, 9, 1], np.uint8)
    now = np.full(6, T0 * NS, np.int64)
    a, r, t, st = e.execute(keys, permits, now, lim, ops)
    assert st == rl_amd.RL_E_INVALID_REQUEST
    assert list(r) == [9, -2, -2, -2, -2, 10]
    assert list(a) == [1, 0, 0, 0, 0, 0]


def test_available_and_reset_entry_points():
    lims = [[rl_amd.SW, 10, 1000, 0.0], [rl_amd.TB, 10, 1000, 4.0]]
    e = engine(lims)
    o = COracle(lims)
    k = np.array([11, 12, 13], np.uint64)
    now = np.full(3, T0 * NS, np.int64)
    for lid in (0, 1):
        tr = (k, np.array([3, 1, 4], np.int32), now, np.full(3, lid, np.uint16))
        e.execute(*tr)
        o.run(*tr)
        av, st = e.available(lid, k, now + 100 * NS)
        want = o.run(k, np.ones(3, np.int32), now + 100 * NS, np.full(3, lid, np.uint16),
                     np.full(3, 1, np.uint8))
        assert st == rl_amd.RL_OK and np.array_equal(av, want[1])
        assert e.reset(lid, k[:1], now + 200 * NS) == rl_amd.RL_OK
        o.run(k[:1], np.ones(1, np.int32), now[:1] + 200 * NS, np.full(1, lid, np.uint16),
              np.full(1, 2, np.uint8))
        av, _ = e.available(lid, k, now + 300 * NS)
        want = o.run(k, np.ones(3, np.int32), now + 300 * NS, np.full(3, lid, np.uint16),
                     np.full(3, 1, np.uint8))
        assert np.array_equal(av, want[1])


def test_device_entry_point_matches_host():
    import torch
    lims = [[rl_amd.TB, 50, 60000, 10.0], [rl_amd.SW, 100, 60000, 0.0]]
    tr = trace(7, 300_000, 5_000, 2, 10_000)
    e1 = engine(lims)
    host = e1.execute(*tr)
    e2 = engine(lims)
    dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in
           (tr[0].view(np.int64), tr[1], tr[2], tr[3].view(np.int16), tr[4])]
    n = len(tr[0])
    allowed = torch.empty(n, dtype=torch.uint8, device="cuda")
    remaining = torch.empty(n, dtype=torch.int64, device="cuda")
    tokens = torch.empty(n, dtype=torch.float64, device="cuda")
    e2.execute_device(n, *dev, allowed, remaining, tokens)
    assert e2.last_status() == rl_amd.RL_OK
    assert_same((allowed.cpu().numpy(), remaining.cpu().numpy(), tokens.cpu().numpy()),
                host[:3], "device vs host")


def test_synth_trace_matches_oracle():
    import torch
    n = 1 << 20
    e = engine([[rl_amd.TB, 50, 60000, 10.0]], max_batch=n)
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    permits = torch.empty(n, dtype=torch.int32, device="cuda")
    now = torch.empty(n, dtype=torch.int64, device="cuda")
    e.synth_trace(n, keys, permits, now, None, seed=0x5EED0002, n_keys=1 << 14)
    e.sync()
    k = keys.cpu().numpy().view(np.uint64)
    assert 0.95 * (1 << 14) < len(np.unique(k)) <= (1 << 14)
    assert np.all(np.diff(now.cpu().numpy()) >= 0)
    p = permits.cpu().numpy()
    assert p.min() == 1 and p.max() == 4
    a, r, t, st = e.execute(k, p, now.cpu().numpy())
    want = COracle([[rl_amd.TB, 50, 60000, 10.0]]).run(k, p, now.cpu().numpy())
    assert_same((a, r, t), want, "synth")


def test_zipf_trace_is_skewed():
    import torch
    n = 1 << 20
    e = engine([[rl_amd.SW, 1000, 60000, 0.0]], max_batch=n)
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    permits = torch.empty(n, dtype=torch.int32, device="cuda")
    now = torch.empty(n, dtype=torch.int64, device="cuda")
    e.synth_trace(n, keys, permits, now, None, seed=0x5EED0003, n_keys=100_000_000,
                  dist=rl_amd.DIST_ZIPF, zipf_s=1.1, permits_max=1)
    e.sync()
    _, c = np.unique(keys.cpu().numpy(), return_counts=True)
    top = c.max() / n
    assert 0.09 < top < 0.13, top          # SURVEY: top key ~11.1% at s=1.1 over 100M keys


@pytest.mark.parametrize("maxp,window", [(40, 1000), (1000, 60000), (3, 200)])
def test_sw_same_key_runs_in_groups(maxp, window):
    # few keys, dense arrivals: groups of 64 hold long same-key runs that mix allows,
    # denials and window roll-overs (exercises both round hypotheses of wave_apply)
    lims = [[rl_amd.SW, maxp, window, 0.0]]
    rng = np.random.default_rng(maxp)
    n = 400_000
    keys = rl_amd.mix64(rng.integers(0, 40, n).astype(np.uint64) + np.uint64(99))
    now = (T0 * NS + np.sort(rng.integers(0, 30 * window * NS, n))).astype(np.int64)
    permits = rng.integers(1, 4, n).astype(np.int32)
    op = np.where(rng.random(n) < 0.01, 1, 0).astype(np.uint8)
    got, want, _ = run_both(lims, (keys, permits, now, np.zeros(n, np.uint16), op), batches=3)
    assert_same(got, want, "sw runs")


@pytest.mark.parametrize("ttl", [1, 50, 700])
def test_sw_local_cache_random(ttl):
    """SlidingWindowRateLimiter's Caffeine cache (:57-64,93-121,148-150) emulated on the GPU:
    few hot keys at their limits (cache hits, rollovers), peeks and resets, several batches,
    a cache-less SW limiter and a TB limiter (no cache, TokenBucketRateLimiter) beside it."""
    lims = [[rl_amd.SW, 10, 1000, 0.0, 0, ttl], [rl_amd.SW, 40, 5000, 0.0],
            [rl_amd.TB, 20, 1000, 5.0, 0, ttl], [rl_amd.SW, 3, 200, 0.0, 0, ttl]]
    tr = trace(100 + ttl, 300_000, 2_000, len(lims), 60_000, zipf=1.2, permits_max=3,
               ops=0.02)
    got, want, e = run_both(lims, tr, batches=4)
    assert_same(got, want, f"local cache ttl={ttl}")
    o = COracle(lims)
    o.run(*tr)
    hits = o.cache_hits()
    assert hits > 0
    # the engine's counter covers the last batch only: replay the last batch's share
    e2 = engine(lims)
    n = len(tr[0])
    cuts = np.linspace(0, n, 5).astype(int)
    tot = 0
    for b in range(4):
        e2.execute(*(x[cuts[b]:cuts[b + 1]] for x in tr))
        tot += e2.stats()["cache_hits"]
    assert tot == hits


def test_pinned_host_buffers_match_pageable():
    """rl_pin_host: page-locked caller buffers give the same results as pageable ones, over
    several batches that reuse the same buffers (the micro-batcher's pattern)."""
    lims = [(rl_amd.TB, 50, 60_000, 10.0), (rl_amd.SW, 20, 1_000, 0.0)]
    n = 50_000
    bufs = dict(keys=np.zeros(n, np.uint64), permits=np.zeros(n, np.int32),
                now=np.zeros(n, np.int64), lim=np.zeros(n, np.uint16))
    e = engine(lims)
    ref = engine(lims)
    o = COracle(lims)
    for b in bufs.values():
        assert e.pin_host(b) == rl_amd.RL_OK
        assert e.pin_host(b) == rl_amd.RL_OK          # idempotent
    for it in range(3):
        k, p, t, l, _ = trace(900 + it, n, 5_000, 2, 4_000)
        t = t + it * 4_000 * NS
        bufs["keys"][:] = k; bufs["permits"][:] = p; bufs["now"][:] = t; bufs["lim"][:] = l
        got = e.execute(bufs["keys"], bufs["permits"], bufs["now"], bufs["lim"])
        want = ref.execute(k, p, t, l)
        assert_same(got, want[:3], f"pinned batch {it}")
        oa, orem, ot, _ = o.run(k, p, t, l)
        assert_same(got, (oa, orem, ot), f"pinned batch {it} vs oracle")
    for b in bufs.values():
        assert e.unpin_host(b) == rl_amd.RL_OK
    assert e.unpin_host(bufs["keys"]) == rl_amd.RL_E_INVALID_ARG   # no longer pinned
    o.close()


@pytest.mark.parametrize("algo", [rl_amd.SW, rl_amd.TB])
def test_medium_hot_keys_across_windows(algo):
    """Keys just below the hot-path threshold with 1-s windows: a 64-request group spans
    window boundaries (per-window allow prefixes) and long allow chains (per-key chains)."""
    rng = np.random.default_rng(77 + algo)
    lims = [[algo, 100, 1_000, 60.0 if algo == rl_amd.TB else 0.0],
            [algo, 5, 1_000, 2.0 if algo == rl_amd.TB else 0.0]]
    n = 400_000
    hot = rl_amd.mix64(np.arange(12, dtype=np.uint64) + np.uint64(99 << 40))
    cold = rl_amd.mix64(rng.integers(0, 50_000, n).astype(np.uint64))
    keys = np.where(rng.random(n) < 0.9, hot[rng.integers(0, 12, n)], cold)
    lim = (rl_amd.mix64(keys) & np.uint64(1)).astype(np.uint16)
    now = (T0 * NS + np.sort(rng.integers(0, 20_000 * NS, n))).astype(np.int64)
    permits = rng.integers(1, 3, n).astype(np.int32)
    op = np.zeros(n, np.uint8)
    op[rng.random(n) < 0.002] = 1
    got, want, _ = run_both(lims, (keys, permits, now, lim, op), batches=3,
                            capacity=1 << 16)
    assert_same(got, want, "medium-hot")


@pytest.mark.parametrize("maxp,start", [(100, 0), (64, 0), (37, 27)])
def test_sw_local_cache_allow_run_sets_entry(maxp, start):
    """One key with the cache on: an allow run inside a 64-request group whose last allow's
    newCount reaches max puts the blocking entry (:119-121); the rest of the window is
    rejected from the cache (hits), exactly as the reference."""
    lims = [[rl_amd.SW, maxp, 60_000, 0.0, 0, 1000]]
    n = 300
    keys = np.full(n, rl_amd.mix64(np.array([5], np.uint64))[0], np.uint64)
    t0 = (T0 // 60_000) * 60_000 + 1_000
    now = ((t0 + start + np.arange(n) // 4) * NS).astype(np.int64)      # 4 requests per ms
    got, want, e = run_both(lims, (keys, np.ones(n, np.int32), now, np.zeros(n, np.uint16),
                                   np.zeros(n, np.uint8)), batches=1)
    assert_same(got, want, "allow run -> cache entry")
    assert want[0].sum() == maxp
    o = COracle(lims)
    o.run(keys, np.ones(n, np.int32), now, np.zeros(n, np.uint16))
    assert e.stats()["cache_hits"] == o.cache_hits() == n - maxp
