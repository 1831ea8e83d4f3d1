"""GPU parity of the hot-region path (k_hot_summ / k_hot_chain / k_hot_fill): regions
holding a hot key are decided chunk by chunk through the threshold fast path, the
wavefront-per-key sequential run and, for their other keys, wave_apply. Everything is
compared bit-exactly with the CPU oracle, as in test_gpu_parity.py.

`hot_threshold` is lowered in most cases so that the hot path also takes ordinary
regions (the largest 1024 per batch), which exercises its general path on every trace
shape the main suite uses."""
import numpy as np
import pytest

import rl_amd
from oracle.coracle import COracle
from test_gpu_parity import NS, T0, assert_same, trace

pytestmark = pytest.mark.gpu


def run(limiters, tr, batches=1, tune=None, **kw):
    kw.setdefault("max_batch", 1 << 22)
    kw.setdefault("capacity", 1 << 14)
    e = rl_amd.Engine(**kw)
    for l in limiters:
        e.add_limiter(*l)
    for k, v in (tune or {}).items():
        e.tune(k, v)
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


def hot_trace(seed, n, n_keys, hot_share, lim_ids, span_ms, permits_max=4, ops=0.0,
              hot_keys=1, regress=False):
    """Uniform background traffic plus `hot_keys` keys that draw `hot_share` of it."""
    rng = np.random.default_rng(seed)
    ranks = rng.integers(hot_keys, n_keys, n)
    hot = rng.random(n) < hot_share
    ranks[hot] = rng.integers(0, hot_keys, hot.sum())
    keys = rl_amd.mix64(ranks.astype(np.uint64) + np.uint64(seed << 40))
    lim = np.asarray(lim_ids, np.uint16)[ranks % len(lim_ids)]
    t = np.sort(rng.integers(0, span_ms * NS, n))
    if regress:           # TB has no monotone-time precondition: shuffle some times locally
        j = rng.integers(0, n - 1, n // 50)
        t[j], t[j + 1] = t[j + 1].copy(), t[j].copy()
    now = (T0 * NS + t).astype(np.int64)
    permits = rng.integers(1, permits_max + 1, n).astype(np.int32)
    op = np.zeros(n, np.uint8)
    if ops:
        u = rng.random(n)
        op[u < ops] = 1
        op[u < ops / 3] = 2
    return keys, permits, now, lim, op


@pytest.mark.parametrize("algo", ["sw", "tb"])
def test_hot_key_at_limit(algo):
    # one key with 40 % of 1.5M requests over 3 minutes: long deny runs between allows
    lims = [[rl_amd.SW, 1000, 60000, 0.0]] if algo == "sw" else [[rl_amd.TB, 50, 60000, 10.0]]
    tr = hot_trace(11, 1_500_000, 50_000, 0.4, [0], 180_000, permits_max=1 if algo == "sw" else 4)
    got, want, e = run(lims, tr, batches=3, capacity=1 << 17)
    assert_same(got, want, f"hot {algo}")


def test_hot_keys_mixed_limiters_ops():
    # several hot keys over SW and TB limiters, peeks and resets, tokens compared bit-exactly
    lims = [[rl_amd.SW, 100, 10_000, 0.0], [rl_amd.TB, 20, 5_000, 3.0], [rl_amd.SW, 5, 1000, 0.0],
            [rl_amd.TB, 500, 60_000, 50.0]]
    tr = hot_trace(12, 1_200_000, 20_000, 0.6, [0, 1, 2, 3], 120_000, ops=0.01, hot_keys=8)
    got, want, _ = run(lims, tr, batches=4, tune={"hot_threshold": 4096})
    assert_same(got, want, "hot mixed")


def test_hot_key_under_limit_runs_sequentially():
    # a hot key that is almost always allowed: every request changes state (wave-per-key run)
    lims = [[rl_amd.TB, 1_000_000, 60_000, 100_000.0], [rl_amd.SW, 2_000_000, 60_000, 0.0]]
    tr = hot_trace(13, 400_000, 1_000, 0.5, [0, 1], 30_000, hot_keys=2)
    got, want, _ = run(lims, tr, batches=2, tune={"hot_threshold": 8192})
    assert_same(got, want, "hot under limit")


def test_hot_tb_time_regression():
    # TB accepts non-monotone time (negative elapsed, no clamp: Lua :56)
    lims = [[rl_amd.TB, 30, 20_000, 5.0]]
    tr = hot_trace(14, 600_000, 5_000, 0.5, [0], 60_000, regress=True)
    got, want, _ = run(lims, tr, batches=2, tune={"hot_threshold": 4096})
    assert_same(got, want, "hot regress")


@pytest.mark.parametrize("case", ["tb_uniform", "sw_zipf", "mixed_ops"])
def test_every_region_through_hot_kernel(case):
    # hot_threshold = 1: the 1024 largest regions of every batch take the hot path
    if case == "tb_uniform":
        lims = [[rl_amd.TB, 50, 60000, 10.0]]
        tr = trace(21, 300_000, 3_000, 1, 2_000)
    elif case == "sw_zipf":
        lims = [[rl_amd.SW, 1000, 60000, 0.0]]
        tr = trace(22, 300_000, 50_000, 1, 90_000, zipf=1.1, permits_max=1)
    else:
        lims = [[rl_amd.SW, 10, 60000, 0.0], [rl_amd.TB, 50, 60000, 10.0],
                [rl_amd.SW, 5, 1000, 0.0], [rl_amd.TB, 3, 500, 7.0]]
        tr = trace(23, 300_000, 10_000, len(lims), 200_000, zipf=1.3, ops=0.04, invalid=0.002)
    got, want, _ = run(lims, tr, batches=3, tune={"hot_threshold": 1})
    assert_same(got, want, case)


def test_hot_two_pass_partition():
    # > 8192 bins: two partition passes, bin bounds from k_bin_bounds, plus hot regions
    lims = [[rl_amd.SW, 100, 60000, 0.0], [rl_amd.TB, 50, 60000, 10.0]]
    tr = hot_trace(15, 1_000_000, 200_000, 0.3, [0, 1], 60_000, hot_keys=4)
    got, want, e = run(lims, tr, batches=2, capacity=1 << 22, tune={"hot_threshold": 16384})
    assert_same(got, want, "hot two-pass")


def test_hot_stats_and_device_entry():
    import torch
    lims = [[rl_amd.SW, 1000, 60000, 0.0]]
    tr = hot_trace(16, 500_000, 10_000, 0.4, [0], 60_000, permits_max=1)
    n = len(tr[0])
    e = rl_amd.Engine(max_batch=n, capacity=1 << 14, stage_timing=True)
    e.add_limiter(*lims[0])
    e.tune("hot_threshold", 4096)
    dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda()
           for x in (tr[0].view(np.int64), tr[1], tr[2])]
    allowed = torch.empty(n, dtype=torch.uint8, device="cuda")
    remaining = torch.empty(n, dtype=torch.int64, device="cuda")
    e.execute_device(n, *dev, None, None, allowed, remaining)
    assert e.last_status() == rl_amd.RL_OK
    want = COracle(lims).run(*tr[:3])
    assert_same((allowed.cpu().numpy(), remaining.cpu().numpy(), None), want, "device hot")
    s = e.stats()
    assert s["allowed"] == int(want[0].sum())
    assert s["distinct_keys"] == len(np.unique(tr[0]))
    assert e.stage_times()["hot_fill"] > 0


# ---- hot-region routing (two-pass tables): from the second batch on, the previous batch's
# hot regions get pass-0 bins of their own, skip pass 1 and are read by the chains from
# their pass-0 positions; the unpermute maps their results back without pass 1.
def run_grow(limiters, tr, batches, grow_at, **kw):
    """run() with an explicit rl_grow_limiter before batch `grow_at` (region ids change, so
    the route list is dropped)."""
    kw.setdefault("max_batch", 1 << 22)
    e = rl_amd.Engine(**kw)
    for l in limiters:
        e.add_limiter(*l)
    o = COracle(limiters)
    n = len(tr[0])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    got = [[], [], []]
    for b in range(batches):
        if b == grow_at:
            for li in range(len(limiters)):
                e.grow_limiter(li, 2 * e.limiter_slots(li))
        sl = slice(cuts[b], cuts[b + 1])
        a, r, t, st = e.execute(*(x[sl] for x in tr))
        assert st in (rl_amd.RL_OK, rl_amd.RL_E_INVALID_REQUEST), rl_amd.strerror(st)
        got[0].append(a); got[1].append(r); got[2].append(t)
    return tuple(np.concatenate(g) for g in got), o.run(*tr), e


@pytest.mark.parametrize("algo", ["sw", "tb"])
@pytest.mark.parametrize("route", [1, 0])
def test_hot_routed_two_pass(algo, route):
    # hot keys at their limits over 5 batches of a two-pass table, with peeks / resets /
    # invalid requests; routing on and off give the oracle's results (tokens bit-exact)
    lims = ([[rl_amd.SW, 200, 20_000, 0.0], [rl_amd.SW, 5, 1000, 0.0]] if algo == "sw" else
            [[rl_amd.TB, 50, 60_000, 10.0], [rl_amd.TB, 20, 5_000, 3.0]])
    tr = hot_trace(31, 2_000_000, 300_000, 0.5, [0, 1], 100_000, ops=0.005, hot_keys=6)
    tr[1][::997] = 0                                     # invalid (permits 0)
    got, want, _ = run(lims, tr, batches=5, capacity=1 << 22,
                       tune={"hot_threshold": 8192, "route": route})
    assert_same(got, want, f"routed {algo} route={route}")


@pytest.mark.parametrize("segs", [3, 16])
@pytest.mark.parametrize("algo", ["sw", "tb"])
def test_hot_routed_two_pass_segmented(algo, segs):
    # the pass-0 output in segments ([segment][bin]; 16 > the batch's 7 tiles: one per tile)
    lims = ([[rl_amd.SW, 200, 20_000, 0.0], [rl_amd.SW, 5, 1000, 0.0]] if algo == "sw" else
            [[rl_amd.TB, 50, 60_000, 10.0], [rl_amd.TB, 20, 5_000, 3.0]])
    tr = hot_trace(31, 2_000_000, 300_000, 0.5, [0, 1], 100_000, ops=0.005, hot_keys=6)
    tr[1][::997] = 0
    got, want, _ = run(lims, tr, batches=5, capacity=1 << 22,
                       tune={"hot_threshold": 8192, "segments": segs})
    assert_same(got, want, f"segmented {algo} segs={segs}")


def test_hot_routed_every_region_segmented():
    lims = [[rl_amd.SW, 50, 30_000, 0.0], [rl_amd.TB, 40, 30_000, 8.0]]
    tr = trace(33, 1_200_000, 400_000, 2, 150_000, zipf=1.2, ops=0.02, invalid=0.001)
    got, want, _ = run(lims, tr, batches=4, capacity=1 << 22, tune={"hot_threshold": 1, "segments": 4})
    assert_same(got, want, "routed every region segmented")


def test_hot_routed_shifting_hot_set():
    # the hot keys change every batch: regions routed because of the previous batch are
    # small (or empty) in this one and still go through the chains
    lims = [[rl_amd.SW, 100, 10_000, 0.0], [rl_amd.TB, 30, 20_000, 5.0]]
    parts = [hot_trace(40 + b, 400_000, 200_000, 0.6, [0, 1], 20_000, hot_keys=5) for b in range(4)]
    off = np.int64(0)
    cols = [[], [], [], [], []]
    for b, p in enumerate(parts):
        for c in range(5):
            x = p[c]
            if c == 2:
                x = x + np.int64(b) * 20_000 * NS        # consecutive time slices
            cols[c].append(x)
    tr = tuple(np.concatenate(c) for c in cols)
    got, want, _ = run(lims, tr, batches=4, capacity=1 << 22, tune={"hot_threshold": 4096})
    assert_same(got, want, "routed shifting")


def test_hot_routed_every_region():
    # hot_threshold 1 on a two-pass table: the 1024 largest regions of every batch are listed
    # and routed in the next (routed regions of every size, many with one or two records)
    lims = [[rl_amd.SW, 50, 30_000, 0.0], [rl_amd.TB, 40, 30_000, 8.0]]
    tr = trace(33, 1_200_000, 400_000, 2, 150_000, zipf=1.2, ops=0.02, invalid=0.001)
    got, want, _ = run(lims, tr, batches=4, capacity=1 << 22, tune={"hot_threshold": 1})
    assert_same(got, want, "routed every region")


def test_hot_routed_growth_clears_routes():
    # growth renumbers regions: the route list of the batch before is dropped, not misapplied
    lims = [[rl_amd.SW, 300, 60_000, 0.0], [rl_amd.TB, 50, 60_000, 10.0]]
    tr = hot_trace(34, 1_500_000, 200_000, 0.4, [0, 1], 90_000, hot_keys=4)
    got, want, e = run_grow(lims, tr, batches=4, grow_at=2, capacity=1 << 22)
    assert_same(got, want, "routed growth")


@pytest.mark.parametrize("order", [1, 0])
def test_region_order_knob(order):
    # largest-first region dispatch (default) and identity order give the oracle's results
    lims = [[rl_amd.SW, 20, 10_000, 0.0], [rl_amd.TB, 30, 20_000, 5.0]]
    tr = trace(35, 800_000, 60_000, 2, 60_000, zipf=1.15, ops=0.01)
    got, want, _ = run(lims, tr, batches=3, capacity=1 << 16, tune={"region_order": order})
    assert_same(got, want, f"region_order={order}")


def same_region_keys(n_keys, region_bits, seed):
    """n_keys distinct key hashes whose tags (mix64) share one region of a table with
    2^region_bits regions (one shard): the top region_bits bits of mix64(key)."""
    rng = np.random.default_rng(seed)
    cand = rng.integers(1, 2**63, 1 << 20, dtype=np.int64).astype(np.uint64)
    top = rl_amd.mix64(cand) >> np.uint64(64 - region_bits)
    vals, counts = np.unique(top, return_counts=True)
    r = vals[np.argmax(counts)]
    keys = cand[top == r][:n_keys]
    assert len(keys) == n_keys
    return keys


@pytest.mark.parametrize("algo", ["sw", "tb"])
@pytest.mark.parametrize("cap_log2", [17, 22])
def test_hot_two_keys_one_region(algo, cap_log2):
    # two heavy keys in one region: the dominant one's chain (wave 0), the second's (wave 2)
    # and every other key of the region (wave 1) at once; one- and two-pass tables (routed)
    region_bits = max(3, (cap_log2 + 1) - 8)             # capacity * 2 / 256 slots per region
    lims = [[rl_amd.SW, 500, 30_000, 0.0]] if algo == "sw" else [[rl_amd.TB, 40, 30_000, 6.0]]
    n = 1_500_000
    rng = np.random.default_rng(50 + cap_log2)
    same = same_region_keys(6, region_bits, 51)           # 2 heavy + 4 light keys of that region
    keys = rl_amd.mix64(rng.integers(0, 100_000, n).astype(np.uint64) + np.uint64(7 << 40))
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
    lim = np.zeros(n, np.uint16)
    tr = (keys, permits, now, lim, op)
    got, want, _ = run(lims, tr, batches=3, capacity=1 << cap_log2)
    assert_same(got, want, f"two keys {algo} cap 2^{cap_log2}")


def test_hot_routed_device_entry_ragged():
    # device entry without balances (the unpermute's two-level gather: normal records through
    # pass 1, routed ones read in place), ragged batch sizes (partial last tiles)
    import torch
    lims = [[rl_amd.SW, 300, 30_000, 0.0], [rl_amd.TB, 30, 20_000, 5.0]]
    tr = hot_trace(36, 1_700_000, 300_000, 0.5, [0, 1], 90_000, hot_keys=6)
    e = rl_amd.Engine(max_batch=1 << 20, capacity=1 << 22)
    for l in lims:
        e.add_limiter(*l)
    cuts = [0, 333_333, 833_334, 1_611_111, 1_700_000]
    ga, gr = [], []
    for b in range(len(cuts) - 1):
        sl = slice(cuts[b], cuts[b + 1])
        m = cuts[b + 1] - cuts[b]
        k, p, t, li = (torch.from_numpy(np.ascontiguousarray(x[sl])).cuda()
                       for x in (tr[0].view(np.int64), tr[1], tr[2], tr[3].view(np.int16)))
        a = torch.empty(m, dtype=torch.uint8, device="cuda")
        r = torch.empty(m, dtype=torch.int64, device="cuda")
        e.execute_device(m, k, p, t, li, None, a, r)
        assert e.last_status() in (rl_amd.RL_OK, rl_amd.RL_E_INVALID_REQUEST)
        ga.append(a.cpu().numpy()); gr.append(r.cpu().numpy())
    want = COracle(lims).run(*tr[:4])
    assert_same((np.concatenate(ga), np.concatenate(gr), None), want, "routed device ragged")


def test_hot_chain_launch_smaller_than_hot_list():
    # the chain launch is sized from an earlier batch's hot count (RegionArgs::chain_grid):
    # batch 1 has no hot region (next launch: 64 workgroups), batch 2 makes the largest
    # 1024+ regions hot, so each chain workgroup loops over many hot-list entries
    lims = [[rl_amd.SW, 100, 60000, 0.0], [rl_amd.TB, 50, 60000, 10.0]]
    tr = hot_trace(31, 600_000, 20_000, 0.2, [0, 1], 60_000, hot_keys=3)
    e = rl_amd.Engine(max_batch=1 << 22, capacity=1 << 14)
    for l in lims:
        e.add_limiter(*l)
    e.tune("chain_split", 0)                  # (two-wave chains launch one workgroup per entry)
    o = COracle(lims)
    cut = 200_000
    got = [[], [], []]
    for b, sl in enumerate((slice(0, cut), slice(cut, None))):
        if b == 1:
            e.tune("hot_threshold", 1)
        a, r, t, st = e.execute(*(x[sl] for x in tr))
        assert st == rl_amd.RL_OK, rl_amd.strerror(st)
        got[0].append(a); got[1].append(r); got[2].append(t)
    want = o.run(*tr)
    assert_same(tuple(np.concatenate(g) for g in got), want, "chain grid")


@pytest.mark.parametrize("two_pass", [False, True])
def test_hot_path_beside_cache_on_limiter(two_pass):
    """The hot path is gated per limiter (rl_engine.cpp, k_hot_select): a Zipf-hot token
    bucket keeps its chains — and, on two-pass tables, its pass-0 routing — while a sliding
    window with the Caffeine local cache (RateLimitConfig.java:37-38, the api limiter of
    RateLimiterConfig.java:54-55) shares the engine. The cache-on limiter has its own hot key
    (k_solo + its region wave) and ~8k live keys, under Caffeine's maximumSize(10000)
    (SlidingWindowRateLimiter.java:60), so the emulation is exact."""
    lims = [[rl_amd.TB, 50, 60_000, 10.0], [rl_amd.SW, 100, 10_000, 0.0, 0, 50]]
    tr = hot_trace(31, 1_200_000, 16_000, 0.5, [0, 1], 120_000, permits_max=2, hot_keys=2)
    kw = dict(capacity=1 << 21) if two_pass else {}
    got, want, e = run(lims, tr, batches=4, tune={"hot_threshold": 16384}, **kw)
    assert_same(got, want, f"hot beside cache ({'two' if two_pass else 'one'}-pass)")
    st = e.stats()
    assert st["hot_regions"] >= 1, st                 # the TB hot key ran as a chain
    assert st["cache_hits"] > 0, st                   # and the cache-on limiter was live
    if two_pass:
        assert st["routed"] > 0, st                   # its region was routed in pass 0


@pytest.mark.parametrize("case", ["mixed_ops", "every_region", "two_keys", "walk_tb", "sw_limit"])
def test_hot_chain_split(case):
    # chain_split off (one wave per chain, pass 2 after pass 1); on is the default every other
    # hot test runs
    tune = {"chain_split": 0, "hot_threshold": 4096}
    kw = {}
    if case == "mixed_ops":
        lims = [[rl_amd.SW, 100, 10_000, 0.0], [rl_amd.TB, 20, 5_000, 3.0], [rl_amd.SW, 5, 1000, 0.0],
                [rl_amd.TB, 500, 60_000, 50.0]]
        tr = hot_trace(12, 1_200_000, 20_000, 0.6, [0, 1, 2, 3], 120_000, ops=0.01, hot_keys=8)
    elif case == "every_region":
        lims = [[rl_amd.SW, 10, 60000, 0.0], [rl_amd.TB, 50, 60000, 10.0],
                [rl_amd.SW, 5, 1000, 0.0], [rl_amd.TB, 3, 500, 7.0]]
        tr = trace(23, 300_000, 10_000, len(lims), 200_000, zipf=1.3, ops=0.04, invalid=0.002)
        tune["hot_threshold"] = 1
    elif case == "two_keys":
        lims = [[rl_amd.TB, 50, 60000, 10.0]]
        tr = hot_trace(17, 1_000_000, 30_000, 0.5, [0], 60_000, hot_keys=2)
        kw["capacity"] = 1 << 17
    elif case == "walk_tb":
        # a dense TB key at its limit (walked) beside background keys of its region
        lims = [[rl_amd.TB, 1000, 60000, 100.0]]
        tr = hot_trace(18, 2_000_000, 5_000, 0.7, [0], 120_000, permits_max=2)
        tune["walk_min"] = 0
    else:
        lims = [[rl_amd.SW, 1000, 60000, 0.0]]
        tr = hot_trace(11, 1_500_000, 50_000, 0.4, [0], 180_000, permits_max=1)
        kw["capacity"] = 1 << 17
    got, want, _ = run(lims, tr, batches=3, tune=tune, **kw)
    assert_same(got, want, f"chain split {case}")
