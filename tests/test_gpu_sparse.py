"""Sparse regions on the GPU path: a region that receives few records probes and updates
single 4-slot buckets in HBM instead of loading its 8 KB image (rl_tune "sparse_max").

The HBM probe chains must stay exact across batches however a region is visited (sparse,
as an image, through the hot path, the TTL sweep): dead slots are tombstones that are
reused by inserts, long chains are compacted, and the one key whose dead state is
all-zero (key hash 0 after a token-bucket reset) never leaves a hole. Everything is
compared bit-exactly with the oracle.
"""
import numpy as np
import pytest

import rl_amd
from oracle.coracle import COracle
from test_gpu_parity import NS, T0, assert_same

pytestmark = pytest.mark.gpu

EVERY = 1 << 30          # sparse_max: every region sparse


def run_batches(limiters, parts, sparse_max, capacity, max_batch=1 << 20):
    e = rl_amd.Engine(max_batch=max_batch, capacity=capacity)
    for l in limiters:
        e.add_limiter(*l)
    e.tune("sparse_max", sparse_max)
    o = COracle(limiters)
    for i, p in enumerate(parts):
        got = e.execute(*p)
        assert got[3] in (rl_amd.RL_OK, rl_amd.RL_E_INVALID_REQUEST), \
            f"batch {i}: {rl_amd.strerror(got[3])}"
        assert_same(got[:3], o.run(*p)[:3], f"sparse_max={sparse_max} batch {i}")
        s = e.stats()
        assert s["capacity_errors"] == 0
    return e


def churn_trace(seed, batches, per_batch, n_keys, n_lim, gap_ms, zipf=None, ops=0.0):
    """Batches gap_ms apart; keys drawn from a large population so most of them live for
    one batch and die (their slots become tombstones for the sparse regions)."""
    rng = np.random.default_rng(seed)
    parts = []
    for b in range(batches):
        if zipf:
            ranks = np.minimum(rng.zipf(zipf, per_batch), n_keys) - 1
        else:
            ranks = rng.integers(0, n_keys, per_batch)
        keys = rl_amd.mix64(ranks.astype(np.uint64) + np.uint64(seed << 40))
        t = T0 + b * gap_ms
        now = (t * NS + np.sort(rng.integers(0, gap_ms * NS, per_batch))).astype(np.int64)
        permits = rng.integers(1, 3, per_batch).astype(np.int32)
        lim = (ranks % n_lim).astype(np.uint16)
        op = np.zeros(per_batch, np.uint8)
        if ops:
            u = rng.random(per_batch)
            op[u < ops] = 1
            op[u < ops / 3] = 2
        parts.append((keys, permits, now, lim, op))
    return parts


LIMS = [[rl_amd.SW, 3, 1000, 0.0], [rl_amd.TB, 4, 2000, 1.5], [rl_amd.SW, 50, 60_000, 0.0],
        [rl_amd.TB, 50, 60_000, 10.0]]


@pytest.mark.parametrize("sparse_max", [0, 96, EVERY])
def test_sparse_churn_multi_batch(sparse_max):
    # 2048 regions per limiter, ~4 records per region per batch: sparse unless disabled;
    # 1-2 s TTLs against 1.7 s between batches make most slots die and get reused
    parts = churn_trace(11, 12, 40_000, 3_000_000, len(LIMS), 1_700, zipf=1.05, ops=0.02)
    run_batches(LIMS, parts, sparse_max, capacity=1 << 18)


def test_sparse_and_image_batches_interleave():
    # batch sizes alternate so regions switch between sparse and image mode (and the hot
    # path for the Zipf head) from one batch to the next
    rng = np.random.default_rng(12)
    parts = []
    t = T0
    for b in range(10):
        n = 400_000 if b % 3 == 0 else 8_000
        ranks = np.minimum(rng.zipf(1.2, n), 500_000) - 1
        keys = rl_amd.mix64(ranks.astype(np.uint64) + np.uint64(12 << 40))
        now = (t * NS + np.sort(rng.integers(0, 900 * NS, n))).astype(np.int64)
        t += 900
        parts.append((keys, rng.integers(1, 3, n).astype(np.int32), now,
                      (ranks % len(LIMS)).astype(np.uint16), np.zeros(n, np.uint8)))
    e = rl_amd.Engine(max_batch=1 << 20, capacity=1 << 16)
    for l in LIMS:
        e.add_limiter(*l)
    e.tune("hot_threshold", 4096)
    o = COracle(LIMS)
    for i, p in enumerate(parts):
        got = e.execute(*p)
        assert got[3] == rl_amd.RL_OK, rl_amd.strerror(got[3])
        assert_same(got[:3], o.run(*p)[:3], f"interleave batch {i}")


def test_sparse_local_cache_limiter():
    # the api limiter with its Caffeine cache on (k_regions<..., CACHE>): cache words move
    # with their slots through faults, tombstone reuse and compaction
    lims = [[rl_amd.SW, 5, 1000, 0.0, 0, 300], [rl_amd.TB, 4, 2000, 1.5]]
    parts = churn_trace(13, 10, 30_000, 400_000, 2, 700, zipf=1.1)
    run_batches(lims, parts, EVERY, capacity=1 << 16)


def test_tombstone_chains_compact():
    # a small table (32 regions per limiter) and keys that live for one batch: every region
    # stays sparse, tombstones pile up, probe chains grow and get compacted; the live
    # keyspace always fits, so no request may fail
    lims = [[rl_amd.SW, 2, 1000, 0.0], [rl_amd.TB, 2, 500, 1.0]]
    rng = np.random.default_rng(14)
    parts = []
    for b in range(60):
        nk = 3000
        ranks = np.arange(b * nk, (b + 1) * nk, dtype=np.uint64)
        keys = np.repeat(rl_amd.mix64(ranks + np.uint64(14 << 40)), 2)
        lim = np.repeat((ranks % 2).astype(np.uint16), 2)
        t = T0 + b * 1500
        now = (t * NS + np.sort(rng.integers(0, 400 * NS, keys.size))).astype(np.int64)
        parts.append((keys, np.ones(keys.size, np.int32), now, lim, np.zeros(keys.size, np.uint8)))
    run_batches(lims, parts, EVERY, capacity=1 << 12)


def colliders(n, region_bits):
    """Keys whose tag lies in region 0 with home bucket 0 (the home of tag 0 = key 0)."""
    cand = np.arange(1, 4_000_000, dtype=np.uint64)
    t = rl_amd.mix64(cand)
    m = ((t >> np.uint64(64 - region_bits)) == 0) & ((t & np.uint64(0xFC)) == 0)
    return cand[m][:n]


@pytest.mark.parametrize("sparse_max", [0, EVERY])
def test_key_zero_reset_leaves_no_hole(sparse_max):
    # capacity 1 -> MIN_REGIONS regions. Key 0 (tag 0) and 7 keys sharing its home bucket:
    # after key 0's bucket is deleted (TB reset) its slot must still chain to the keys
    # placed behind it
    bits = rl_amd.MIN_REGIONS.bit_length() - 1
    others = colliders(7, bits)
    assert others.size == 7
    keys = np.concatenate([[np.uint64(0)], others]).astype(np.uint64)
    lims = [[rl_amd.TB, 50, 60_000, 0.001]]
    n = keys.size
    z8, one = np.zeros(n, np.uint16), np.ones(n, np.int32)
    parts = [
        (keys, np.full(n, 7, np.int32), np.full(n, T0 * NS, np.int64), z8, np.zeros(n, np.uint8)),
        (keys[:1], one[:1], np.full(1, (T0 + 10) * NS, np.int64), z8[:1], np.full(1, 2, np.uint8)),
        (keys[1:], one[1:], np.full(n - 1, (T0 + 20) * NS, np.int64), z8[1:], np.zeros(n - 1, np.uint8)),
        (keys, one, np.full(n, (T0 + 30) * NS, np.int64), z8, np.zeros(n, np.uint8)),
    ]
    e = rl_amd.Engine(max_batch=1 << 16, capacity=1)
    e.add_limiter(*lims[0], capacity=1)
    e.tune("sparse_max", sparse_max)
    o = COracle(lims)
    for i, p in enumerate(parts):
        got = e.execute(*p)
        assert got[3] == rl_amd.RL_OK, rl_amd.strerror(got[3])
        assert_same(got[:3], o.run(*p)[:3], f"key0 batch {i}")
    # the colliders kept their balances (50 - 7 - 1 - 1 = 41 left, 42 after batch 2)
    assert (got[1][1:] == 41).all()


def test_sweep_then_sparse():
    # the TTL sweep rebuilds regions (no tombstones left); sparse batches after it must still
    # find every live key
    parts = churn_trace(15, 8, 30_000, 200_000, len(LIMS), 800)
    e = rl_amd.Engine(max_batch=1 << 20, capacity=1 << 16)
    for l in LIMS:
        e.add_limiter(*l)
    e.tune("sparse_max", EVERY)
    o = COracle(LIMS)
    for i, p in enumerate(parts):
        got = e.execute(*p)
        assert got[3] == rl_amd.RL_OK
        assert_same(got[:3], o.run(*p)[:3], f"sweep batch {i}")
        if i % 2 == 1:
            e.sweep_expired(int(p[2][-1]))
