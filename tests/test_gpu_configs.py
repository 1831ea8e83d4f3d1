"""Parity on the bench's exact workloads (BASELINE.json configs; bench.py CONFIGS).

Every case draws its requests from the very generator bench.py times (k_synth, same seed,
key population, Zipf exponent, permits and time axis as a default `bench.py --config X`
run), runs them through the HIP path in several batches, and compares every decision and
remaining bit-exactly with the C oracle (key-sharded over 16 host threads):

* mixed_tenants (configs[3]): the 10-limiter set, 16M requests in 2 batches — two
  partition passes (1.3M regions), the hot path (top key ~10% of the traffic) and
  10 limiters with TB + SW, 1-byte and 2-byte results;
* zipf_1b (configs[4]): TB(50, 10/s) + SW(1000/min), 16M requests in 2 batches;
* sw_zipf (configs[2]): ONE full 256M-request batch, so the hot chain of its top region
  (~29.8M records) is compared end to end, not a prefix; and three consecutive whole
  batches, so the routed steady state (pass 0 routes the previous batch's hot regions)
  is compared too;
* the steady state of configs[3]/[4]: six (mixed_tenants) and four (zipf_1b) consecutive
  whole bench batches, each compared with a persistent oracle right after it runs, and one
  whole zipf_1b batch with its TB balances;
* config 1 (configs[0], RateLimiterBenchmark.java:48-71): the single-key SW 100000/min
  stream of 100,000 tryAcquire("user123"), as one batch and as 100 batches.
"""
import os

import numpy as np
import pytest
import torch

import rl_amd
from oracle.coracle import COracle
from test_gpu_parity import NS, T0, assert_same

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16


def bench_configs():
    import bench
    return bench.CONFIGS, bench.T0_NS


def synth(eng, cfg, t0_ns, n, index_base=0, steps=13):
    """The first n requests of a default bench run's step 0 (warmup 3 + steps 10), i.e.
    bench.py's synth_trace call with ws = 1."""
    dev = torch.device("cuda", 0)
    batch = cfg["batch"]
    n_lim = len(cfg["limiters"])
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    permits = torch.empty(n, dtype=torch.int32, device=dev)
    now = torch.empty(n, dtype=torch.int64, device=dev)
    lim = torch.empty(n, dtype=torch.int16, device=dev) if n_lim > 1 else None
    eng.synth_trace(n, keys, permits, now, lim, seed=cfg["seed"], n_keys=cfg["n_keys"],
                    dist=cfg["dist"], zipf_s=cfg.get("zipf_s", 1.1),
                    permits_max=cfg["permits_max"], t0_ns=t0_ns, span_ns=cfg["span_ns"] * steps,
                    index_base=index_base, n_total=steps * batch, n_limiters=n_lim)
    return keys, permits, now, lim


def run_config(name, n, batches, pipeline=False, cuts=None, cfg=None, tune=()):
    """`pipeline`: RL_OPT_PIPELINE, every batch submitted back-to-back with no sync in between
    (batch b+1's partition overlaps batch b's decisions); `cuts`: explicit batch boundaries;
    `cfg`: a workload of bench.CONFIGS' shape not in it. Token-bucket balances
    (tokens_after) are compared bit-for-bit with the oracle's (Lua reply,
    TokenBucketRateLimiter.java:56-67; north_star asks 1e-9 relative)."""
    cfgs, t0_ns = bench_configs()
    cfg = cfg or cfgs[name]
    has_tb = any(l[0] == rl_amd.TB for l in cfg["limiters"])
    if cuts is None:
        per = (n + batches - 1) // batches
        cuts = [min(n, b * per) for b in range(batches + 1)]
    per = max(b - a for a, b in zip(cuts, cuts[1:]))
    eng = rl_amd.Engine(device=0, max_batch=per, capacity=cfg["capacity"], pipeline=pipeline)
    for l in cfg["limiters"]:
        eng.add_limiter(*l)
    for k, v in tune:
        eng.tune(k, v)
    keys, permits, now, lim = synth(eng, cfg, t0_ns, n)
    allowed = torch.empty(n, dtype=torch.uint8, device="cuda")
    remaining = torch.empty(n, dtype=torch.int64, device="cuda")
    tokens = torch.empty(n, dtype=torch.float64, device="cuda") if has_tb else None
    torch.cuda.synchronize()                    # inputs complete before the (pipelined) calls
    for a, b in zip(cuts, cuts[1:]):
        sl = slice(a, b)
        m = sl.stop - sl.start
        eng.execute_device(m, keys[sl], permits[sl], now[sl], None if lim is None else lim[sl],
                           None, allowed[sl], remaining[sl], None if tokens is None else tokens[sl])
        if not pipeline:
            assert eng.last_status() == rl_amd.RL_OK, rl_amd.strerror(eng.last_status())
    eng.sync()
    assert eng.last_status() == rl_amd.RL_OK, rl_amd.strerror(eng.last_status())
    st = eng.stats()
    k = keys.cpu().numpy().view(np.uint64)
    p = permits.cpu().numpy()
    t = now.cpu().numpy()
    li = None if lim is None else lim.cpu().numpy().view(np.uint16)
    got = (allowed.cpu().numpy(), remaining.cpu().numpy(),
           None if tokens is None else tokens.cpu().numpy())
    del keys, permits, now, lim, allowed, remaining, tokens
    eng.close()
    o = COracle(cfg["limiters"], nthreads=ORACLE_THREADS)
    want = o.run(k, p, t, li, None, want_tokens=has_tb)
    if has_tb:
        assert got[2] is not None and want[2] is not None
        assert np.isfinite(want[2]).sum() > 0          # balances really compared
    o.close()
    assert_same(got, want, name)
    return k, got, st


def run_stream(name, batches, n=None, tune=(), timing=False):
    """Consecutive whole bench batches (bench.py steps 0 .. batches-1 of a default run:
    same generator, index base and time axis), each compared with a persistent C oracle
    right after it runs, so the engine's state after many batches — the steady state the
    bench's numbers come from — is checked, not just a prefix of batch 0. Returns the
    per-batch engine stats (and stage times with `timing`)."""
    cfgs, t0_ns = bench_configs()
    cfg = cfgs[name]
    n = n or cfg["batch"]
    has_tb = any(l[0] == rl_amd.TB for l in cfg["limiters"])
    eng = rl_amd.Engine(device=0, max_batch=n, capacity=cfg["capacity"], stage_timing=timing)
    for l in cfg["limiters"]:
        eng.add_limiter(*l)
    for k, v in tune:
        eng.tune(k, v)
    o = COracle(cfg["limiters"], nthreads=ORACLE_THREADS)
    dev = torch.device("cuda", 0)
    allowed = torch.empty(n, dtype=torch.uint8, device=dev)
    remaining = torch.empty(n, dtype=torch.int64, device=dev)
    tokens = torch.empty(n, dtype=torch.float64, device=dev) if has_tb else None
    out = []
    for b in range(batches):
        keys, permits, now, lim = synth(eng, cfg, t0_ns, n, index_base=b * cfg["batch"])
        torch.cuda.synchronize()
        eng.execute_device(n, keys, permits, now, lim, None, allowed, remaining, tokens)
        st = eng.last_status()
        assert st == rl_amd.RL_OK, f"{name} batch {b}: {rl_amd.strerror(st)}"
        stats = eng.stats()
        if timing:
            stats["stage_ms"] = eng.stage_times()
        got = (allowed.cpu().numpy(), remaining.cpu().numpy(),
               None if tokens is None else tokens.cpu().numpy())
        k = keys.cpu().numpy().view(np.uint64)
        li = None if lim is None else lim.cpu().numpy().view(np.uint16)
        want = o.run(k, permits.cpu().numpy(), now.cpu().numpy(), li, None, want_tokens=has_tb)
        del keys, permits, now, lim
        if has_tb:
            assert np.isfinite(want[2]).sum() > 0
        assert_same(got, want, f"{name} batch {b}")
        assert 0 < got[0].sum() < n
        print(f"{name} batch {b}: {int(got[0].sum())} allowed, hot regions {stats['hot_regions']}, "
              f"routed {stats['routed']}"
              + (f", region stage {stats['stage_ms'].get('region', -1):.2f} ms" if timing else ""),
              flush=True)
        out.append(stats)
    eng.close()
    o.close()
    return out


@pytest.mark.timeout(600)
def test_config_mixed_tenants_steady_state():
    """configs[3]'s per-GPU share for six consecutive 2^27-request bench batches (6 minutes of
    trace time): from batch ~3 on, the SW perSecond(100) limiter's hot key lets one request
    through every ~10 ms as its previous bucket's weight decays (SlidingWindowRateLimiter.java:
    170-174), so its hot chain re-derives the denied interval [T0, T1) thousands of times per
    batch — the regime that bounds the config's step time, compared request by request."""
    stats = run_stream("mixed_tenants", 6, timing=True)
    assert all(s["hot_regions"] > 0 for s in stats)


@pytest.mark.timeout(400)
def test_config_zipf_1b_full_batch():
    """configs[4]'s per-GPU share, one whole 2^27-request bench batch (TB + SW, Zipf over
    125M keys), decisions, remaining and TB balances bit-for-bit."""
    cfgs, _ = bench_configs()
    n = cfgs["zipf_1b"]["batch"]
    k, got, st = run_config("zipf_1b", n, 1)
    assert st["hot_regions"] > 0
    assert np.isfinite(got[2]).sum() > n // 4


@pytest.mark.timeout(600)
def test_config_sw_zipf_routed_batches():
    """configs[2] (the headline) as three consecutive whole 2^28-request bench batches: from
    batch 1 on, pass 0 routes the previous batch's hot regions straight to their final bins
    (hot-region routing), which is the regime every timed bench step runs in."""
    stats = run_stream("sw_zipf", 3)
    assert stats[0]["routed"] == 0
    assert all(s["routed"] > (1 << 26) for s in stats[1:]), [s["routed"] for s in stats]


@pytest.mark.parametrize("segs", [8, 16])
def test_config_sw_zipf_segmented(segs):
    """The headline's routed whole batches with the pass-0 output segmented
    (rl_tune "segments"): bins laid out [segment][bin], grouped from their runs."""
    stats = run_stream("sw_zipf", 2, tune=(("segments", segs),))
    assert stats[1]["routed"] > (1 << 26)


@pytest.mark.timeout(600)
def test_config_zipf_1b_steady_state():
    """configs[4]'s per-GPU share over four consecutive whole bench batches (routing on)."""
    stats = run_stream("zipf_1b", 4)
    assert all(s["routed"] > 0 for s in stats[1:])


def test_config_mixed_tenants_16m():
    k, got, st = run_config("mixed_tenants", 1 << 24, 2)
    _, c = np.unique(k, return_counts=True)
    assert c.max() > 16384                       # the hot path fired (hot_threshold)
    assert 0 < got[0].sum() < len(k)


def test_config_tb_uniform_pipelined():
    """configs[1] (the default bench line) in 4 back-to-back batches with RL_OPT_PIPELINE."""
    k, got, st = run_config("tb_uniform", 1 << 24, 4, pipeline=True)
    assert 0 < got[0].sum() < len(k)


@pytest.mark.timeout(400)
def test_config_sw_zipf_pipelined_routed():
    """configs[2]'s workload in 8 back-to-back pipelined batches of 2^24: with RL_OPT_PIPELINE
    batch k routes the hot regions of batch k - 2 (the route table of its scratch set, round 6),
    so from batch 2 on pass 0 sends them straight to their final bins while batch k - 1's region
    stage still runs."""
    k, got, st = run_config("sw_zipf", 1 << 27, 8, pipeline=True)
    assert st["routed"] > 0 and st["hot_regions"] > 0, st
    assert 0 < got[0].sum() < len(k)


def test_config_mixed_tenants_pipelined_ragged():
    """Pipelined batches of ragged, growing sizes: each scratch set is regrown mid-stream
    (two passes, hot path, 10 limiters), and a tiny batch sits between large ones."""
    n = 3 << 22
    cuts = [0, 1 << 20, (1 << 20) + 777, 3 << 21, (3 << 21) + (1 << 22) + 5, n]
    k, got, _ = run_config("mixed_tenants", n, 0, pipeline=True, cuts=cuts)
    assert 0 < got[0].sum() < len(k)


def test_config_zipf_1b_16m():
    k, got, _ = run_config("zipf_1b", 1 << 24, 2)
    assert 0 < got[0].sum() < len(k)


def test_config_tb_uniform_one_batch_balances():
    """configs[1] exactly as bench.py's step 0: one whole 64M-request batch, balances and all."""
    cfgs, _ = bench_configs()
    n = cfgs["tb_uniform"]["batch"]
    k, got, _ = run_config("tb_uniform", n, 1)
    assert 0 < got[0].sum() < len(k)
    assert np.isfinite(got[2]).all()


def test_tb_hot_keys_at_limit():
    """Token-bucket hot keys at their limit through the hot chains (k_hot_chains, default
    hot_threshold): TB 50 at 10/s, Zipf s=1.1 over 1M keys, 8M requests over 4 s in 2
    batches — the top key draws ~1M requests, hundreds of regions go hot, and the chains'
    "denied by time alone" blocks and [T0, T1) runs are checked balance by balance
    (Lua TokenBucketRateLimiter.java:46-67)."""
    cfg = dict(limiters=[(rl_amd.TB, 50, 60_000, 10.0)], n_keys=1_000_000, dist=rl_amd.DIST_ZIPF,
               zipf_s=1.1, batch=1 << 22, span_ns=2_000 * 1_000_000,
               permits_max=3, seed=0x5EED00B1, capacity=1 << 20)
    k, got, st = run_config("tb_hot", 1 << 23, 2, cfg=cfg)
    _, c = np.unique(k, return_counts=True)
    assert c.max() > 16384 * 4                   # several hot regions per batch
    a = got[0]
    assert 0 < a.sum() < len(k)


def test_tb_hot_keys_forced_chains():
    """Every region with >= 64 records through the hot path (hot_threshold 64): mixed
    time-regressing-free TB traffic where most regions run the chains, balances bit-exact."""
    cfg = dict(limiters=[(rl_amd.TB, 50, 60_000, 10.0), (rl_amd.TB, 1000, 60_000, 100.0)],
               n_keys=200_000, dist=rl_amd.DIST_ZIPF, zipf_s=1.1, batch=1 << 21,
               span_ns=4_000 * 1_000_000, permits_max=4, seed=0x5EED00B2, capacity=1 << 18)
    k, got, _ = run_config("tb_forced", 1 << 22, 2, cfg=cfg, tune=(("hot_threshold", 64),))
    assert 0 < got[0].sum() < len(k)


@pytest.mark.timeout(400)
def test_config_sw_zipf_full_batch():
    cfgs, _ = bench_configs()
    n = cfgs["sw_zipf"]["batch"]                 # 2^28: one whole bench batch
    k, got, _ = run_config("sw_zipf", n, 1)
    _, c = np.unique(k, return_counts=True)
    assert c.max() > 25_000_000                  # the ~29.8M-record hot chain, end to end


def config1_trace():
    """RateLimiterBenchmark.benchmarkSlidingWindow_SingleKey (:48-71): 10 threads x 10,000
    tryAcquire("user123"), maxPermits 100000 per minute; arrivals 12.5 us apart (the
    published 80,192 req/s run took ~1.25 s, README.md:174-181)."""
    n = 100_000
    t0 = (T0 // 60000) * 60000 + 5000
    keys = np.full(n, rl_amd.key_hash("user123"), np.uint64)
    now = (t0 * NS + np.arange(n, dtype=np.int64) * 12_500).astype(np.int64)
    return keys, np.ones(n, np.int32), now


def test_config1_single_key_stream():
    # RateLimiterBenchmark.java:50-55: enableLocalCache(true), localCacheTtl 50 ms
    lims = [[rl_amd.SW, 100_000, 60_000, 0.0, 0, 50]]
    keys, permits, now = config1_trace()
    want = COracle(lims).run(keys, permits, now, want_tokens=False)
    assert want[0].sum() == 100_000 and want[1][-1] == 0     # README.md:179: 100% success
    for batches in (1, 100):
        e = rl_amd.Engine(max_batch=1 << 17, capacity=1 << 10)
        e.add_limiter(*lims[0])
        got = [[], []]
        for sl in np.array_split(np.arange(len(keys)), batches):
            a, r, _, st = e.execute(keys[sl], permits[sl], now[sl], want_tokens=False)
            assert st == rl_amd.RL_OK
            got[0].append(a); got[1].append(r)
        assert_same((np.concatenate(got[0]), np.concatenate(got[1]), None), want[:3],
                    f"config1 x{batches}")
        assert e.stats()["cache_hits"] == 0


def test_solo_runs_cache_on():
    """Cache-on sliding windows: large regions' leading allow runs decided by k_solo
    (rl_solo.hip) with a low threshold, so that runs end every way the pass allows — a denial,
    a put reaching max, a cache entry still valid at the batch start, another key, a peek, a
    window change — over several batches (state and cache words carried in HBM)."""
    NSV = 1_000_000
    rng = np.random.default_rng(0x50105)
    lims = [[rl_amd.SW, 600, 1_000, 0.0, 0, 40], [rl_amd.SW, 100_000, 60_000, 0.0, 0, 50],
            [rl_amd.SW, 5, 200, 0.0, 0, 300]]
    n = 400_000
    t0 = (T0 // 60_000) * 60_000 + 55_000
    # few keys (large regions), skewed; limiter by key; bursts that cross the limits
    keys_u = rng.integers(1, 2**63, 40, dtype=np.uint64)
    kid = np.minimum(rng.zipf(1.6, n) - 1, 39)
    keys = keys_u[kid]
    lim = (kid % 3).astype(np.uint16)
    now = (t0 * NSV + np.sort(rng.integers(0, 9_000 * NSV, n))).astype(np.int64)
    permits = rng.integers(1, 3, n).astype(np.int32)
    ops = np.where(rng.random(n) < 0.0005, rl_amd.OP_PEEK, rl_amd.OP_ACQUIRE).astype(np.uint8)
    want = COracle(lims).run(keys, permits, now, lim, ops, want_tokens=False)
    for thr in (64, 0):
        e = rl_amd.Engine(max_batch=1 << 17, capacity=1 << 10)
        for l in lims:
            e.add_limiter(*l)
        e.tune("solo_threshold", thr)
        got = [[], []]
        for sl in np.array_split(np.arange(n), 5):
            a, r, _, st = e.execute(keys[sl], permits[sl], now[sl], lim[sl], ops[sl], want_tokens=False)
            assert st == rl_amd.RL_OK, rl_amd.strerror(st)
            got[0].append(a); got[1].append(r)
        assert_same((np.concatenate(got[0]), np.concatenate(got[1]), None), want[:3], f"solo thr {thr}")
        e.close()
    assert 0 < want[0].sum() < n


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [("scatter_split", 0), ("unpermute_split", 0), ("unpermute_split", 1),
                                  ("mid_xcd", 1), ("region_order", 0)])
def test_config_partition_knobs(knob):
    """Every partition/unpermute variant the engine keeps behind rl_tune stays bit-exact on
    the two-pass headline table (routing from batch 1): the non-split scatter, the plain and
    split unpermute on both passes, the XCD-mapped mid gather, the plain dispatch order."""
    run_config("zipf_1b", 1 << 22, 3, tune=(knob,))
