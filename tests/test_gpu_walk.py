"""GPU parity of the hot chains' allow walk (rl_hot.hpp `walk`, k_hot_summ's per-ms tables,
k_hot_fill's walk verdicts): dense hot keys at their limit, whose allows the chain finds from
the key's state and the per-ms table of first acquires instead of detailing a chunk per
allow. Every case is compared bit-exactly with the CPU oracle (decisions, remaining, TB
balances bit-for-bit), with the walk on (the default) and off (rl_tune walk=0).

Batches span at most kWalkSpan (131072 ms) so that the tables are built, and walk_min is 0 so
that keys expecting fewer than kWalkMinAllows allows are walked too; the cases also cover
what sends a chain back to the chunk-by-chunk path: peeks / resets of the hot key, acquires
of more than 2 permits, token-bucket time regression, bursts (a full bucket, a fresh window)
and TB early rejects (permits > max)."""
import numpy as np
import pytest

import rl_amd
from test_gpu_hot import hot_trace, run
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def both(lims, tr, batches, tune=None, walks=True, **kw):
    # walk_min 0: every key dense enough is walked, not only those expecting >= 4000 allows.
    # The last batch's per-region debug words (rl_tune debug_regions; word 20 = walked allows)
    # show whether the walk ran: `walks` says whether it must have (it never may with walk 0).
    for walk in (1, 0):
        got, want, e = run(lims, tr, batches=batches,
                           tune=dict(tune or {}, walk=walk, walk_min=0, debug_regions=1), **kw)
        assert_same(got, want, f"walk={walk}")
        walked = int(e.debug_region_times(1 << 16)[:, 20].sum())
        if walk and walks:
            assert walked > 0, "the walk did not run"
        else:
            assert walked == 0, f"walk={walk}: {walked} walked allows"



@pytest.mark.parametrize("permits_max", [1, 2])
def test_walk_tb_dense_key_at_limit(permits_max):
    # mixed_tenants' limiter 8 (TB 1000 @ 100/s): a full bucket (a burst of ~1000 allows),
    # then one allow per 10-20 ms among ~20 requests per ms of the key
    lims = [[rl_amd.TB, 1000, 60_000, 100.0]]
    tr = hot_trace(41, 2_000_000, 20_000, 0.6, [0], 60_000, permits_max=permits_max)
    both(lims, tr, batches=2, capacity=1 << 16)


@pytest.mark.parametrize("permits_max", [1, 2])
def test_walk_sw_dense_key_at_limit(permits_max):
    # mixed_tenants' perSecond(100) (RateLimitConfig.java:61-66): a new window every second,
    # allows as the previous window's weight decays
    lims = [[rl_amd.SW, 100, 1_000, 0.0]]
    tr = hot_trace(42, 2_000_000, 20_000, 0.6, [0], 60_000, permits_max=permits_max)
    both(lims, tr, batches=2, capacity=1 << 16)


def test_walk_sw_minute_window_and_tb_beside():
    # SW 1000/min (configs[2]) and TB 50 @ 10/s (configs[1]) hot keys in one engine, several
    # hot keys, 3 batches (state carried across them)
    lims = [[rl_amd.SW, 1000, 60_000, 0.0], [rl_amd.TB, 50, 60_000, 10.0]]
    tr = hot_trace(43, 2_400_000, 40_000, 0.5, [0, 1], 90_000, permits_max=2, hot_keys=4)
    both(lims, tr, batches=3, capacity=1 << 16)


@pytest.mark.parametrize("algo", ["tb", "sw"])
def test_walk_with_peeks_and_resets(algo):
    # the hot key's peeks / resets (specials) are detailed; the walk resumes after each
    lims = [[rl_amd.TB, 200, 20_000, 20.0]] if algo == "tb" else [[rl_amd.SW, 50, 2_000, 0.0]]
    tr = hot_trace(44, 1_500_000, 10_000, 0.6, [0], 40_000, permits_max=2, ops=0.0005)
    both(lims, tr, batches=2, capacity=1 << 15)


def test_walk_off_for_large_permits_and_regression():
    # permits up to 4 (group flag: more than 2) and TB time regression (out-of-order flag):
    # the chains stay on the chunk path, results unchanged
    lims = [[rl_amd.TB, 500, 30_000, 50.0], [rl_amd.SW, 300, 5_000, 0.0]]
    tr = hot_trace(45, 1_200_000, 10_000, 0.6, [0, 1], 40_000, permits_max=4, hot_keys=2)
    both(lims, tr, batches=2, capacity=1 << 15, walks=False)
    lims = [[rl_amd.TB, 300, 20_000, 30.0]]
    tr = hot_trace(46, 1_200_000, 10_000, 0.6, [0], 40_000, permits_max=2, regress=True)
    both(lims, tr, batches=2, capacity=1 << 15, walks=False)


def test_walk_tb_early_rejects():
    # TB cap 1: every 2-permit acquire is rejected before the script (remaining -1, :110-116)
    lims = [[rl_amd.TB, 1, 60_000, 20.0]]
    tr = hot_trace(47, 1_000_000, 10_000, 0.6, [0], 30_000, permits_max=2)
    both(lims, tr, batches=2, capacity=1 << 15)


def test_walk_two_pass_routed():
    # > 8192 regions (two partition passes): hot regions routed in pass 0, walked
    lims = [[rl_amd.TB, 1000, 60_000, 100.0], [rl_amd.SW, 100, 1_000, 0.0]]
    tr = hot_trace(48, 2_000_000, 400_000, 0.5, [0, 1], 60_000, permits_max=2, hot_keys=2)
    both(lims, tr, batches=3, capacity=1 << 21, tune={"hot_threshold": 16384})


@pytest.mark.parametrize("algo", ["sw", "tb"])
def test_walk_two_keys_one_region(algo):
    # two heavy keys in one region (chains of the dominant and the second key, slots 2 i and
    # 2 i + 1 of the walk tables), light keys beside them, peeks / resets of every key
    from test_gpu_hot import NS, T0, same_region_keys
    lims = [[rl_amd.SW, 500, 30_000, 0.0]] if algo == "sw" else [[rl_amd.TB, 40, 30_000, 6.0]]
    n = 1_500_000
    rng = np.random.default_rng(60)
    same = same_region_keys(6, 10, 61)                     # capacity 2^17: 2^10 regions
    keys = rl_amd.mix64(rng.integers(0, 100_000, n).astype(np.uint64) + np.uint64(9 << 40))
    u = rng.random(n)
    keys[u < 0.30] = same[0]
    keys[(u >= 0.30) & (u < 0.50)] = same[1]
    light = (u >= 0.50) & (u < 0.51)
    keys[light] = same[2 + rng.integers(0, 4, int(light.sum()))]
    now = (T0 * NS + np.sort(rng.integers(0, 90_000 * NS, n))).astype(np.int64)
    permits = rng.integers(1, 3, n).astype(np.int32)
    op = np.zeros(n, np.uint8)
    v = rng.random(n)
    op[v < 0.002] = 1
    op[v < 0.0005] = 2
    tr = (keys, permits, now, np.zeros(n, np.uint16), op)
    both(lims, tr, batches=3, capacity=1 << 17)


@pytest.mark.parametrize("algo", ["tb", "sw"])
def test_walk_reset_only_chunks(algo):
    # chunks of the walked key's region whose only record of the key is a
    # reset, after chunks whose acquires the old state denied. Every record of the trace is in
    # one region (6 keys), so region chunk c of a batch is records 64c .. 64c + 63 of it; in 24
    # chunks per batch the dominant key's records are replaced by other keys' and one of its
    # records becomes a reset. The walk must search again from the key's last plain acquire
    # (tools/walk_model.py, tests/test_walk_model.py::test_walk_model_reset_only_chunks).
    from test_gpu_hot import NS, T0
    from test_gpu_hot import same_region_keys
    lims = [[rl_amd.TB, 40, 30_000, 20.0]] if algo == "tb" else [[rl_amd.SW, 60, 2_000, 0.0]]
    n = 1_500_000
    rng = np.random.default_rng(64)
    same = same_region_keys(6, 10, 65)                     # capacity 2^17: 2^10 regions
    u = rng.random(n)
    keys = np.where(u < 0.35, same[0], same[1 + rng.integers(0, 5, n)]).astype(np.uint64)
    now = (T0 * NS + np.sort(rng.integers(0, 60_000 * NS, n))).astype(np.int64)
    permits = rng.integers(1, 3, n).astype(np.int32)
    op = np.zeros(n, np.uint8)
    cuts = np.linspace(0, n, 3).astype(int)
    for b in range(2):
        nch = (cuts[b + 1] - cuts[b]) // 64
        for c in rng.choice(np.arange(4, nch - 4), 24, replace=False):
            j0 = cuts[b] + 64 * int(c)
            blk = slice(j0, j0 + 64)
            mine = keys[blk] == same[0]
            keys[blk] = np.where(mine, same[1], keys[blk])
            j = j0 + int(rng.integers(0, 64))
            keys[j] = same[0]
            op[j] = 2
            permits[j] = 1
    tr = (keys, permits, now, np.zeros(n, np.uint16), op)
    both(lims, tr, batches=2, capacity=1 << 17)
