"""Time regression on the GPU path (front-ends with skewed clocks).

* Sliding window: a request whose now falls back into the previous window must INCR that
  window's bucket and leave the newer one intact (Redis keys every window separately,
  SlidingWindowRateLimiter.java:185-188, RedisRateLimitStorage.java:38-49). The engine keeps
  a key's two newest buckets, so it is exact whenever the bucket two windows before the
  key's newest is absent at the regressed now; the traces below give every key a life of
  two windows, which guarantees that, and jitter the arrival times by up to 0.6 w.
* Token bucket: elapsed < 0 is not clamped (Lua :56-58), so balances and their reply
  integers go far below zero; results below the packed width's range travel through the
  escape code and the int64 side array (kResEscape) and must come back exactly, on the
  1-byte, 2-byte and wide result paths.
"""
import numpy as np
import pytest

import rl_amd
from oracle.coracle import COracle
from test_gpu_parity import NS, T0, assert_same

pytestmark = pytest.mark.gpu


def two_window_lives(seed, n, n_keys, w_ms, jitter_ms, n_lim=1):
    """Key k lives in [s_k, s_k + 2w) for a staggered start s_k (a window start), so no
    request ever reaches more than one window behind the key's newest bucket."""
    rng = np.random.default_rng(seed)
    ranks = rng.integers(0, n_keys, n)
    start = (T0 // w_ms) * w_ms + (ranks % 97) * w_ms        # staggered window starts
    off = rng.integers(0, 2 * w_ms, n)
    order = np.argsort(start + off, kind="stable")
    ranks, start, off = ranks[order], start[order], off[order]
    jit = rng.integers(-jitter_ms, jitter_ms + 1, n)
    t = np.clip(off + jit, 0, 2 * w_ms - 1) + start           # stays inside the key's life
    keys = rl_amd.mix64(ranks.astype(np.uint64) + np.uint64(seed << 40))
    now = (t * NS + rng.integers(0, NS, n)).astype(np.int64)
    permits = rng.integers(1, 3, n).astype(np.int32)
    lim = (ranks % n_lim).astype(np.uint16)
    return keys, permits, now, lim, np.zeros(n, np.uint8)


def run(limiters, tr, batches=1, tune=None, **kw):
    kw.setdefault("max_batch", 1 << 21)
    kw.setdefault("capacity", 1 << 14)
    e = rl_amd.Engine(**kw)
    for l in limiters:
        e.add_limiter(*l)
    for k, v in (tune or {}).items():
        e.tune(k, v)
    n = len(tr[0])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    got = [[], [], []]
    for b in range(batches):
        sl = slice(cuts[b], cuts[b + 1])
        a, r, t, st = e.execute(*(x[sl] for x in tr))
        assert st == rl_amd.RL_OK, rl_amd.strerror(st)
        got[0].append(a); got[1].append(r); got[2].append(t)
    return tuple(np.concatenate(g) for g in got), COracle(limiters).run(*tr)


@pytest.mark.parametrize("hot", [False, True])
@pytest.mark.parametrize("maxp", [5, 60])
def test_sw_jitter_across_window_boundaries(maxp, hot):
    lims = [[rl_amd.SW, maxp, 200, 0.0], [rl_amd.TB, maxp, 200, 40.0]]
    tr = two_window_lives(11 + maxp, 300_000, 3_000, 200, 120, n_lim=2)
    # sanity: the trace really regresses across window boundaries for some keys
    o = np.argsort(tr[0], kind="stable")
    kk, ww = tr[0][o], (tr[2] // NS // 200)[o]
    assert np.any((kk[1:] == kk[:-1]) & (ww[1:] < ww[:-1]))
    tune = {"hot_threshold": 64} if hot else None
    got, want = run(lims, tr, batches=3, tune=tune)
    assert_same(got, want, f"sw jitter maxp={maxp} hot={hot}")


def test_sw_regression_keeps_newer_bucket():
    """Newer counts survive a regressed request (the round-1 engine reset the record to the
    older window and over-admitted afterwards)."""
    lims = [[rl_amd.SW, 10, 1000, 0.0]]
    W = (T0 // 1000) * 1000
    k = np.full(16, 5, np.uint64)
    t = [W + 1100] * 8 + [W + 990] + [W + 1200] * 7           # 8 in W+1000, 1 back in W
    now = np.array(t, np.int64) * NS
    got, want = run(lims, (k, np.ones(16, np.int32), now, np.zeros(16, np.uint16),
                           np.zeros(16, np.uint8)))
    assert_same(got, want, "newer bucket kept")
    # 8 in W+1000, the late one counts in bucket W (prev of W+1000: weight 0.8 at W+1200),
    # then trunc(0.8 + 8) = 8 and trunc(0.8 + 9) = 9 still admit two more -> 11
    assert got[0].sum() == want[0].sum() == 11


@pytest.mark.parametrize("maxp", [50, 5000, 1 << 22])       # 1-byte, 2-byte, wide results
def test_tb_deep_negative_balances(maxp):
    lims = [[rl_amd.TB, maxp, 60_000, 10.0]]
    rng = np.random.default_rng(3)
    n = 200_000
    keys = rl_amd.mix64(rng.integers(0, 500, n).astype(np.uint64))
    t = np.sort(rng.integers(0, 30_000 * NS, n))
    back = rng.random(n) < 0.05                             # 5% arrive up to 20 s late
    t[back] -= rng.integers(0, 20_000 * NS, back.sum())
    now = (T0 * NS + t).astype(np.int64)
    permits = rng.integers(1, int(min(maxp, 1 << 30)) // 4 + 2, n).astype(np.int32)
    got, want = run(lims, (keys, permits, now, np.zeros(n, np.uint16), np.zeros(n, np.uint8)),
                    batches=2)
    assert (want[1] < -3).sum() > 10                         # the escape path is exercised
    assert_same(got, want, f"tb negative maxp={maxp}")


def test_tb_deep_negative_two_pass_and_device_entry():
    """Escapes through the two-pass unpermute (mid gather) and without tokens_after."""
    import torch
    lims = [[rl_amd.TB, 20, 60_000, 1.0], [rl_amd.SW, 30, 60_000, 0.0]]
    rng = np.random.default_rng(9)
    n = 400_000
    ranks = rng.integers(0, 200_000, n)
    keys = rl_amd.mix64(ranks.astype(np.uint64))
    t = np.sort(rng.integers(0, 60_000 * NS, n))
    tb = (ranks % 2) == 0
    back = (rng.random(n) < 0.1) & tb                       # only TB keys regress
    t[back] -= rng.integers(0, 60_000 * NS, back.sum())
    now = (T0 * NS + t).astype(np.int64)
    permits = rng.integers(1, 6, n).astype(np.int32)
    lim = (ranks % 2).astype(np.uint16)
    e = rl_amd.Engine(max_batch=n, capacity=1 << 22)        # 2 x 16384 regions: two passes
    for l in lims:
        e.add_limiter(*l)
    want = COracle(lims).run(keys, permits, now, lim, want_tokens=False)
    dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda()
           for x in (keys.view(np.int64), permits, now, lim.view(np.int16))]
    allowed = torch.empty(n, dtype=torch.uint8, device="cuda")
    remaining = torch.empty(n, dtype=torch.int64, device="cuda")
    e.execute_device(n, *dev, None, allowed, remaining)
    assert e.last_status() == rl_amd.RL_OK
    assert (want[1] < -3).sum() > 100
    assert_same((allowed.cpu().numpy(), remaining.cpu().numpy(), None), want[:3], "two-pass esc")


@pytest.mark.parametrize("skew_ms", [0, 5_000])
def test_max_skew_retains_state_for_globally_late_batches(skew_ms):
    """Per-key time is monotone, but batch 3 carries requests older than batch 2's earliest
    one (a lagging front-end). With rl_opts.max_skew_ms covering the lag, the buckets that
    batch 2's region loads would have dropped (dead at its earliest now) are kept and batch 3
    matches the oracle; with 0 (batches in global time order) they are reclaimed."""
    lims = [[rl_amd.TB, 10, 1000, 1.0], [rl_amd.SW, 5, 1000, 0.0]]   # TB ttl 2 s, SW ttl 1 s
    nk = 400
    ka = rl_amd.mix64(np.arange(nk, dtype=np.uint64) + np.uint64(1 << 40))       # lagging keys
    kb = rl_amd.mix64(np.arange(nk, dtype=np.uint64) + np.uint64(2 << 40))       # others
    la = (np.arange(nk) % 2).astype(np.uint16)
    mk = lambda k, l, t, p: (k, np.full(len(k), p, np.int32), np.full(len(k), t * NS, np.int64),
                             l, np.zeros(len(k), np.uint8))
    b1 = mk(ka, la, T0, 4)                               # A drains 4 tokens / counts 1
    b2 = mk(kb, la, T0 + 2_500, 1)                       # earliest now of batch 2: T0 + 2.5 s
    b3 = mk(ka, la, T0 + 900, 3)                         # A again, 0.9 s after its last request
    tr = tuple(np.concatenate(x) for x in zip(b1, b2, b3))
    e = rl_amd.Engine(max_batch=1 << 12, capacity=1, max_skew_ms=skew_ms)
    for l in lims:
        e.add_limiter(*l[:4], capacity=1)                # 8 regions per limiter: all loaded
    got = [e.execute(*b)[:3] for b in (b1, b2, b3)]
    want = COracle(lims).run(*tr)
    g3 = got[2]
    w3 = tuple(x[2 * nk:] for x in want[:3])
    if skew_ms:
        assert_same(g3, w3, "skew retained")
    else:
        assert not np.array_equal(g3[1], w3[1])          # reclaimed: batch 3 sees fresh state
