"""CPU check of the allow-walk algorithm (tools/walk_model.py, the model of rl_hot.hpp's `walk`
and k_hot_fill's walk verdicts): for one key's record stream the walk (next allow from the
state and the per-ms table of first acquires; chunk verdicts with up to 4 allows; remaining-0
chunks; specials, bursts and fifth allows detailed) must give the sequential semantics'
results record by record (SlidingWindowRateLimiter.java:85-180, TokenBucketRateLimiter Lua
:38-68, restated exactly by the model's SW / TB classes). The GPU code is checked against the
oracle by tests/test_gpu_walk.py; this pins the algorithm itself on dense and sparse keys."""
import importlib.util
import os
import random

import pytest

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("walk_model", os.path.join(_ROOT, "tools", "walk_model.py"))
wm = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(wm)


def _trace(seed, n, per_ms, specials, pmax):
    rnd = random.Random(seed)
    t0 = 1_700_000_000_000
    span = max(1, int(n / per_ms))
    ts = sorted(t0 + rnd.randrange(span) for _ in range(n))
    return [(t, rnd.randint(1, pmax), (rnd.choice([1, 2]) if rnd.random() < specials else 0)) for t in ts]


def _check(algo, recs, mk, w):
    want = []
    s = mk()
    for r in recs:
        mine = len(r) < 4 or r[3]
        want.append(s.step(r[0], r[1], r[2]) if mine else None)
    stats = {"detail": 0, "allows": 0, "conflict": 0, "burst": 0}
    got = wm.walk(recs, mk(), algo, w, stats)
    bad = [j for j in range(len(recs)) if got[j] != want[j]]
    assert not bad, (algo, stats, bad[:5], [recs[j] for j in bad[:3]])
    return stats


@pytest.mark.parametrize("per_ms", [20.0, 3.0, 0.7])
@pytest.mark.parametrize("specials", [0.0, 0.003])
@pytest.mark.parametrize("pmax", [1, 2])
def test_walk_model_token_bucket(per_ms, specials, pmax):
    # mixed_tenants' TB 1000 @ 100/s (a full bucket, then one allow per 10-20 ms) and a small
    # bucket that empties and refills within a chunk
    for seed, (cap, rate, w) in enumerate([(1000, 100.0, 60000), (20, 50.0, 2000)]):
        recs = _trace(100 + seed, 6000, per_ms, specials, pmax)
        _check("tb", recs, lambda: wm.TB(cap, rate, w), w)


@pytest.mark.parametrize("per_ms", [20.0, 2.0, 0.5])
@pytest.mark.parametrize("specials", [0.0, 0.003])
@pytest.mark.parametrize("pmax", [1, 2])
def test_walk_model_sliding_window(per_ms, specials, pmax):
    # perSecond(100) (a new window every second, allows as the previous window decays) and a
    # 2-second window of 50
    for seed, (mx, w) in enumerate([(100, 1000), (50, 2000)]):
        recs = _trace(200 + seed, 6000, per_ms, specials, pmax)
        _check("sw", recs, lambda: wm.SW(mx, w), w)


def test_walk_model_dense_key_uses_remaining_zero_verdicts():
    # a key far above its limit: nearly every chunk takes the remaining-0 verdict
    recs = _trace(7, 20000, 40.0, 0.0, 1)
    stats = _check("tb", recs, lambda: wm.TB(1000, 100.0, 60000), 60000)
    assert stats.get("rem0", 0) > 10000 and stats["detail"] < 50


def _sparse_trace(seed, n, per_ms, share, pmax, reset_chunks):
    # the walked key's records (share of them) among other keys' records, as in a hot region;
    # in `reset_chunks` random chunks the key's only record is a reset (after the acquires of
    # the chunks before were denied under the old state)
    rnd = random.Random(seed)
    t0 = 1_700_000_000_000
    span = max(1, int(n / per_ms))
    ts = sorted(t0 + rnd.randrange(span) for _ in range(n))
    recs = [(t, rnd.randint(1, pmax), 0, rnd.random() < share) for t in ts]
    nch = (n + 63) // 64
    for c in rnd.sample(range(2, nch - 2), reset_chunks):
        for j in range(c * 64, min(n, c * 64 + 64)):
            t, p, _, _ = recs[j]
            recs[j] = (t, p, 0, False)
        j = c * 64 + rnd.randrange(64)
        recs[j] = (recs[j][0], 1, 2, True)
    return recs


@pytest.mark.parametrize("algo", ["tb", "sw"])
@pytest.mark.parametrize("share", [0.5, 0.08])
def test_walk_model_reset_only_chunks(algo, share):
    # a chunk whose only record of the key is a reset, after chunks whose
    # acquires were denied under the old state. The search must start again after the key's
    # last plain acquire (not where the old state's search stopped), so that it neither allows
    # a record of a decided chunk nor skips the acquires the reset frees; a sparse key also
    # meets chunks without any of its records right after a boundary (`must` persists).
    for seed in range(6):
        recs = _sparse_trace(300 + seed, 12000, 6.0, share, 2, 12)
        if algo == "tb":
            _check("tb", recs, lambda: wm.TB(40, 20.0, 30000), 30000)
        else:
            _check("sw", recs, lambda: wm.SW(60, 2000), 2000)
