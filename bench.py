#!/usr/bin/env python3
"""bench.py — rate-limit decisions/s of the MI355X engine (BASELINE.json metric).

A "step" is one batch of N timestamped requests, resident in HBM, pushed through the
whole hot path (partition -> per-region sequential semantics -> results in caller
order). Steps are consecutive slices of one synthetic trace, so state carries over
and time moves forward exactly as in a replay.

Default workload (N=1): BASELINE.json configs[2], the largest single-GPU configuration —
sliding window 1000/min (SlidingWindowRateLimiter.java:158-180), 100M keys Zipf s=1.1,
256M-request batches spanning 60 s each. The same JSON line carries configs[1] (token
bucket cap 50 at 10/s, 1M keys uniform, 64M-request batches; `tb_uniform`), the per-GPU
share of configs[4] (TB 50@10/s + SW 1000/min, Zipf s=1.1, 125M keys, 2^27 requests per
step; `zipf_1b`), the per-GPU share of configs[3] (10 limiters, 125M keys, 2^27 requests per
step; `mixed_tenants`) and configs[0] (the reference's single-key benchmark; `config1`) as
extra keys, each with its own roofline, CPU baseline and parity check.

Multi-GPU (torchrun, one rank per GPU): weak scaling. Every rank is a front-end that
receives its own slice of the global stream; requests are routed to the owner shard
(top bits of mix64(key), or the hot-key directory) by the C-ABI router (rl_router_*,
the path a JNI caller uses) over RCCL all-to-all, decided there, and the decisions
return by a second all-to-all.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rl_amd  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec per GPU
NS = 1_000_000
T0_NS = 1_700_000_000_000 * NS

CONFIGS = {
    # configs[1]: TB cap=50 refill=10/s, 1M keys uniform, 64M-request batch, 1 MI355X
    "tb_uniform": dict(limiters=[(rl_amd.TB, 50, 60_000, 10.0)], n_keys=1_000_000,
                       dist=rl_amd.DIST_UNIFORM, batch=1 << 26, span_ns=2_000 * NS,
                       permits_max=4, seed=0x5EED0002, capacity=1_000_000,
                       desc="TB cap=50 refill=10/s window=60s; 1M keys uniform; 64M-request "
                            "batches over 2 s"),
    # configs[2]: SW 1000/min, 100M keys Zipf s=1.1, 256M requests over 60 s
    "sw_zipf": dict(limiters=[(rl_amd.SW, 1000, 60_000, 0.0)], n_keys=100_000_000,
                    dist=rl_amd.DIST_ZIPF, zipf_s=1.1, batch=1 << 28, span_ns=60_000 * NS,
                    permits_max=1, seed=0x5EED0003, capacity=30_000_000,
                    desc="SW 1000/min window 60s; 100M keys Zipf s=1.1; 256M requests over 60 s"),
    # configs[3]: 10 limiter configs (RateLimiterConfig.java:51-92 + RateLimitConfig.java:61-80
    # factories + TB variants), each key owned by one limiter (rank % 10), Zipf s=1.1; the
    # config is 500M keys on 4 GPUs: 125M keys and 128M requests per GPU per step
    "mixed_tenants": dict(limiters=[(rl_amd.SW, 10, 60_000, 0.0),        # login / authRateLimiter
                                    (rl_amd.SW, 100, 60_000, 0.0),       # api (cache off)
                                    (rl_amd.TB, 50, 60_000, 10.0),       # burst
                                    (rl_amd.SW, 5, 1_000, 0.0),          # perSecond(5)
                                    (rl_amd.SW, 100, 1_000, 0.0),        # perSecond(100)
                                    (rl_amd.SW, 1000, 60_000, 0.0),      # perMinute(1000)
                                    (rl_amd.SW, 5000, 3_600_000, 0.0),   # perHour(5000)
                                    (rl_amd.TB, 10, 10_000, 1.0),
                                    (rl_amd.TB, 1000, 60_000, 100.0),
                                    (rl_amd.TB, 100, 300_000, 0.5)],
                          n_keys=125_000_000, dist=rl_amd.DIST_ZIPF, zipf_s=1.1, batch=1 << 27,
                          span_ns=60_000 * NS, permits_max=2, seed=0x5EED0004,
                          capacity=16_000_000,
                          desc="10 limiters (login 10/min, api 100/min, burst TB 50@10/s, 7 "
                               "variants); Zipf s=1.1; 125M keys + 128M requests per GPU per "
                               "step over 60 s (500M keys at 4 GPUs)"),
    # configs[4]: 1B keys over 8 GPUs, TB(50, 10/s) + SW(1000/min) by key rank, Zipf s=1.1,
    # 2^30 requests per step: 125M keys and 2^27 requests per GPU
    "zipf_1b": dict(limiters=[(rl_amd.TB, 50, 60_000, 10.0), (rl_amd.SW, 1000, 60_000, 0.0)],
                    n_keys=125_000_000, dist=rl_amd.DIST_ZIPF, zipf_s=1.1, batch=1 << 27,
                    span_ns=60_000 * NS, permits_max=1, seed=0x5EED0005, capacity=24_000_000,
                    desc="TB 50@10/s + SW 1000/min; Zipf s=1.1; 125M keys + 2^27 requests per "
                         "GPU per step over 60 s (1B keys, 2^30 requests at 8 GPUs)"),
}

# algorithmic bytes per request / per distinct key
REQ_IN = 8 + 8 + 4             # key 8 + now 8 + permits 4 (+ limiter 2 when there are several)
REQ_OUT = 1 + 8                # allowed 1 + remaining 8
KEY_BYTES = 32 + 32            # state slot read + written

# Bytes each pipeline kernel must move as designed (its own I/O, per request), for the
# per-kernel bandwidth fractions; the headline roofline is the whole step's ALGORITHMIC
# bytes over the whole step's time. Pass 1 of a routed two-pass batch
# partitions only the n_normal records that pass 0 did not route to their final place
# (DESIGN.md §4 "Hot-region routing"), so k_group is charged for those alone.
def kernel_io_bytes(name, n, u, n_lim, res_bytes, n_normal=None):
    lim = 2 if n_lim > 1 else 0
    nn = n if n_normal is None else n_normal
    return {
        "upsweep0": n * (8 + lim),
        "scatter0": n * (REQ_IN + lim + 16 + 4),          # request in; record 16 + position 4 out
        # k_group: the normal records read twice (count, place), written once + positions
        "group": nn * (16 + 16 + 16 + 4),
        "region": n * (16 + res_bytes) + u * KEY_BYTES,   # records in, packed results out, slots
        "unpermute": n * (4 + res_bytes + REQ_OUT),        # positions + gathered results in, decisions out
    }.get(name)


# ---- per-GPU HBM footprint (the driver's --gpus 8 run must fit 288 GB per GPU) ----------
HBM_BYTES_PER_GPU = 288e9              # MI355X_MICROARCH.md: 288 GB HBM3E per GPU
_TILE, _TILE_THREADS, _DIGIT_BINS = 65536, 512, 1 << 13     # rl_device.hpp kTile / kTileThreads
_REGION_BYTES = 256 * 32               # kRegionSlots x sizeof(Slot)
_HOT_MAX, _HOT_CHUNK = 1024, 64        # rl_launch.hpp kHotMax / kHotChunk
_WALK_TAB_ENTRIES = 1 << 26                # rl_launch.hpp kWalkTabEntries (uint2 each)
_ROUTER_EXC = 4096                     # rl_router.cpp kExcCap


_WALK_MIN_ALLOWS, _WALK_SPAN_MS = 4000, 1 << 17   # rl_launch.hpp kWalkMinAllows / kWalkSpan


def walk_possible(cfg):
    """Could a key of this config be walked (rl_hot.hpp walk_dense: at least kWalkMinAllows
    expected allows over a batch's span)? The engine holds the 512-MiB walk tables only then."""
    span = cfg["span_ns"] / NS
    if span >= _WALK_SPAN_MS:
        return False
    for algo, mx, w, refill in cfg["limiters"]:
        e = mx + refill / 1000.0 * span if algo == rl_amd.TB else mx * (span / w + 2.0)
        if e >= _WALK_MIN_ALLOWS:
            return True
    return False


def engine_max_batch(n, ws, router="capi"):
    """max_batch of a rank's engine in run(): its per-exchange receive capacity."""
    return n * ws if (ws > 1 and router == "python") else n * min(ws, 2)


def hbm_footprint(name, n, ws, steps, warm, router="capi", recv_cap=0, table_scale=1,
                  parity_tokens=False, pipeline=False):
    """Device bytes one rank of `bench.py --gpus ws --config name` holds at its peak, from
    the allocation sizes in rl_engine.cpp (rl_add_limiter_ex, ensure_scratch, ensure_regions,
    ensure_hot_summ, ensure_hot_mark) and rl_router.cpp (rl_router_create_ex), plus the
    inputs and outputs run() keeps resident. Tables are counted at their creation size
    (test_gpu_bench_footprint checks the model against hipMemGetInfo after a run)."""
    cfg = CONFIGS[name]
    n_lim = len(cfg["limiters"])
    req_in = 8 + 8 + 4 + (2 if n_lim > 1 else 0)
    out = {"inputs": (steps + warm) * n * req_in,
           "outputs": n * (1 + 8) + (n * 8 if parity_tokens else 0)}
    cap = engine_max_batch(n, ws, router)
    rcap = min(recv_cap or cap, cap) if ws > 1 else n
    # engine scratch: sized to the largest batch it decides (+1/8, at most max_batch)
    m = rcap if ws > 1 else n
    sc_n = max(m, min(cap, max(m + m // 8, 1 << 20)))
    padn = sc_n + _TILE_THREADS
    per_rec = 16 + 2 + 16 + 4 + 4 + 8 + 8 + 8     # rec0 digit rec1 pos0 pos1 res tok ext
    tiles = (sc_n + _TILE - 1) // _TILE
    sets = 2 if pipeline else 1
    out["engine_scratch"] = sets * (padn * per_rec + _DIGIT_BINS * tiles * 4)
    # state tables (rl_add_limiter_ex: load <= 0.5 at capacity, whole bins of 8 regions)
    cap_keys = cfg["capacity"] * ws * table_scale
    per_shard = -(-cap_keys // ws)
    regions = 0
    for _ in cfg["limiters"]:
        r = max(-(-per_shard * 2 // 256), 1)
        k = max((r - 1).bit_length(), 3)
        regions += 1 << k
    out["tables"] = regions * _REGION_BYTES
    out["region_arrays"] = sets * regions * 8 + regions * (4 + 4 + 1) + 4 * (regions + 1)
    l1 = m // _HOT_CHUNK + _HOT_MAX + 1
    out["hot_summaries"] = (l1 + l1 // 64 + _HOT_MAX + 1) * 8
    # allow-walk tables: allocated once a batch lists a key dense enough to walk (k_hot_scan)
    out["walk_tables"] = _WALK_TAB_ENTRIES * 8 if walk_possible(cfg) else 0
    if ws > 1 and router == "capi":
        ret = lambda t: t * 8 + ws * (8 + 8 + 16 * _ROUTER_EXC)   # ret_bound (rl_router.cpp)
        send = n * (4 + 16 + 2 + 8 + 4 + 8 + 8) + ret(n)
        recv = rcap * (16 + 2 + 8 + 4 + 8 + 1 + 8 + 8) + ret(rcap)
        out["router"] = send + recv
    elif ws > 1:
        out["router"] = ws * n * 48            # python router: device exchange buffers (bound)
    out["total"] = sum(out.values())
    out["fits_288GB"] = out["total"] <= HBM_BYTES_PER_GPU
    return out


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def load_pmc(config_name, kernel, batch, world):
    """(HBM traffic per launch, the profile directory it came from) from the committed
    rocprofv3 PMC summary (profiles/pmc_summary.json, tools/pmc_json.py), or (None, None)
    unless that profile was taken on this exact workload: the same config, requests per GPU
    per step and world size. The directory is the summary's _meta[config] (pmc_json always
    records it; tests/test_pmc_provenance.py recomputes the values from it)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None, None
    try:
        s = json.load(open(path))
        d = s.get(config_name, {})
        if d.get("batch") != batch or d.get("world", 1) != world:
            return None, None
        # the step's traffic in the steady state (batches 1..: the timed steps all route hot
        # regions; batch 0 does not), else over every profiled batch
        k = d.get(kernel + "_steady", d.get(kernel)) if kernel == "step" else d.get(kernel)
        return (None, None) if k is None else (float(k["hbm_bytes_per_launch"]),
                                               s.get("_meta", {}).get(config_name))
    except Exception:
        return None, None


def config1_line(dev):
    """BASELINE configs[0] (RateLimiterBenchmark.java:48-71): the single-key SW 100000/min
    stream of 100,000 tryAcquire("user123"). The Java + Redis reference cannot run here; its
    published 80,192 req/s (README.md:174-181) is context. Times the C oracle (1 thread, the
    CPU port) and the engine on the same stream as one HBM-resident batch."""
    from oracle.coracle import COracle
    n = 100_000
    t0 = (1_700_000_000_000 // 60000) * 60000 + 5000
    keys = np.full(n, rl_amd.key_hash("user123"), np.uint64)
    now = (t0 * NS + np.arange(n, dtype=np.int64) * 12_500).astype(np.int64)
    permits = np.ones(n, np.int32)
    lim = [(rl_amd.SW, 100_000, 60_000, 0.0, 0, 50)]      # cache on, TTL 50 ms (:50-55)
    o = COracle(lim)
    c0 = time.perf_counter()
    oa, orem, _, _ = o.run(keys, permits, now, want_tokens=False)
    cpu_s = time.perf_counter() - c0
    o.close()
    d = [torch.from_numpy(x).to(dev) for x in (keys.view(np.int64), permits, now)]
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    r = torch.empty(n, dtype=torch.int64, device=dev)
    best = None
    for rep in range(3):                       # a fresh engine (empty state) per repetition
        e = rl_amd.Engine(device=dev.index or 0, max_batch=n, capacity=1 << 10)
        e.add_limiter(*lim[0])
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        e.execute_device(n, *d, None, None, a, r)
        e.sync()
        dt = time.perf_counter() - g0
        best = dt if best is None else min(best, dt)
        e.close()
    ok = bool(np.array_equal(a.cpu().numpy(), oa) and np.array_equal(r.cpu().numpy(), orem))
    return {"workload": "RateLimiterBenchmark sliding window single key user123, max 100000/min, "
                        "100,000 requests (RateLimiterBenchmark.java:48-71)",
            "allowed": int(oa.sum()), "parity": "bit-exact" if ok else "MISMATCH",
            "engine_value": n / best, "engine_ms": best * 1e3,
            "cpu_port_value": n / cpu_s, "cpu_port_cores": 1,
            "reference_published": 80192, "unit": "decisions/s",
            "note": "engine = one HBM-resident batch: the 100k requests share one key, so one "
                    "region wave applies them 64 at a time (each group's allow run in one round, "
                    "local cache on); the micro-batched host path is timed by "
                    "tests/cpp/test_host_api (config1)"}


def cpu_baseline(cfg, keys, permits, now, lim, sample_n, gpu_allowed, gpu_remaining, gpu_tokens,
                 single_thread=True):
    """The C oracle (oracle/rl_oracle.c, the CPU restatement: kind "port") on the first
    sample_n requests of batch 0, key-sharded over the box's host-core share, and (unless
    single_thread=False) the exact 1-thread replay; both double as the parity check of the
    GPU's batch 0 on that prefix: decisions, remaining and — token buckets — the fp64
    balance bit-for-bit (north_star: within 1e-9 relative; Lua TokenBucketRateLimiter.java:56-67)."""
    from oracle.coracle import COracle
    n = min(sample_n, keys.shape[0])
    k = keys[:n].cpu().numpy().view(np.uint64)
    p = permits[:n].cpu().numpy()
    t = now[:n].cpu().numpy()
    l = None if lim is None else lim[:n].cpu().numpy().view(np.uint16)
    has_tb = any(x[0] == rl_amd.TB for x in cfg["limiters"])
    threads = max(1, min(16, os.cpu_count() or 1))
    oT = COracle(cfg["limiters"], nthreads=threads)
    t0 = time.perf_counter()
    aT, rT, tT, _ = oT.run(k, p, t, l, None, want_tokens=has_tb)
    dtT = time.perf_counter() - t0
    oT.close()
    dt1 = None
    if single_thread:
        o1 = COracle(cfg["limiters"])
        t0 = time.perf_counter()
        a1, r1, _, _ = o1.run(k, p, t, l, None, want_tokens=False)
        dt1 = time.perf_counter() - t0
        o1.close()
        ok_1 = bool(np.array_equal(aT, a1) and np.array_equal(rT, r1))
    else:
        ok_1 = True
    ga = gpu_allowed[:n]
    gr = gpu_remaining[:n]
    dec_ok = bool(np.array_equal(ga, aT) and np.array_equal(gr, rT)) and ok_1
    bal = None
    if has_tb and gpu_tokens is not None:
        gt = gpu_tokens[:n]
        m = ~np.isnan(tT)
        bal = bool(np.array_equal(np.isnan(gt), ~m) and
                   np.array_equal(gt[m].view(np.uint64), tT[m].view(np.uint64)))
    cpu_model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    out = {
        "value": n / dtT, "unit": "decisions/s", "cores": threads, "kind": "port",
        "cpu_model": cpu_model,
        "sample": f"first {n} requests of batch 0 (same synthetic trace), oracle/rl_oracle.c "
                  f"key-sharded over {threads} threads",
        "sharded_seconds": dtT,
    }
    if dt1 is not None:
        out["single_thread_value"] = n / dt1
        out["single_thread_seconds"] = dt1
    return out, dec_ok, bal, n


def parity_text(dec_ok, bal, n):
    s = f"{'bit-exact' if dec_ok else 'MISMATCH'} decisions + remaining vs oracle on the first {n} " \
        f"requests of batch 0"
    if bal is not None:
        s += f"; token-bucket balances {'bit-exact' if bal else 'MISMATCH'}"
    return s


def make_inputs(eng, cfg, n, ws, rank, total_steps, dev):
    n_global_total = total_steps * ws * n
    n_lim = len(cfg["limiters"])
    inputs = []
    for s in range(total_steps):
        keys = torch.empty(n, dtype=torch.int64, device=dev)
        permits = torch.empty(n, dtype=torch.int32, device=dev)
        now = torch.empty(n, dtype=torch.int64, device=dev)
        lim = torch.empty(n, dtype=torch.int16, device=dev) if n_lim > 1 else None
        eng.synth_trace(n, keys, permits, now, lim, seed=cfg["seed"], n_keys=cfg["n_keys"] * ws,
                        dist=cfg["dist"], zipf_s=cfg.get("zipf_s", 1.1),
                        permits_max=cfg["permits_max"], t0_ns=T0_NS,
                        span_ns=cfg["span_ns"] * total_steps,
                        index_base=(s * ws + rank) * n, n_total=n_global_total, n_limiters=n_lim)
        inputs.append((keys, permits, now, lim))
    return inputs


def plan_directory(router, cfg, inputs, n, k=4096, sample=1 << 22):
    """Hot-key directory (rl_router_plan_directory) from this rank's first batch: the top
    keys of a sample of its requests (Zipf configs; BASELINE north_star's skew)."""
    keys = inputs[0][0][:min(sample, n)]
    u, c = torch.unique(keys, return_counts=True)
    top = torch.topk(c, min(k, c.numel()))
    kk = u[top.indices].cpu().numpy().view(np.uint64)
    cc = top.values.cpu().numpy().astype(np.uint64)
    return router.plan_directory(kk, cc, int(keys.numel()), k)


def run(name, args, ws, rank, local, dev, rehearse, steps, warm, parity_tokens):
    """Time `steps` steps of config `name` after `warm` warmup steps; returns the line's
    dict and what the CPU baseline needs (batch 0's inputs and GPU results)."""
    cfg = CONFIGS[name]
    n = (args.batch if name == args.config else 0) or cfg["batch"]
    total_steps = steps + warm
    # weak scaling: each shard owns 1/ws of the keys but sees ws x n requests' worth of
    # key space across ranks, i.e. the same number of requests per GPU; a shard's table
    # is sized for its share of the global key population. The C-ABI router's owner decides
    # at most its receive capacity (min(ws, 2) x n) per exchange round and splits a step
    # into rounds when an owner receives more (a skewed step); the python router hands an
    # owner everything it receives (up to ws x n).
    cap = engine_max_batch(n, ws, args.router)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0 = torch.cuda.mem_get_info(dev)[0]
    eng = rl_amd.Engine(device=local, max_batch=cap,
                        capacity=cfg["capacity"] * ws * args.table_scale, stage_timing=False,
                        shard_index=rank, shard_count=ws,
                        pipeline=ws == 1 and args.pipeline)
    for l in cfg["limiters"]:
        eng.add_limiter(*l)
    for kv in args.tune:
        k, v = kv.split("=")
        eng.tune(k, int(v))
    n_lim = len(cfg["limiters"])
    inputs = make_inputs(eng, cfg, n, ws, rank, total_steps, dev)
    allowed = torch.empty(n, dtype=torch.uint8, device=dev)
    remaining = torch.empty(n, dtype=torch.int64, device=dev)
    has_tb = any(x[0] == rl_amd.TB for x in cfg["limiters"])
    tokens0 = torch.empty(n, dtype=torch.float64, device=dev) if (parity_tokens and has_tb) else None
    eng.sync()
    torch.cuda.synchronize()

    router = None
    directory = 0
    if ws > 1:
        if args.router == "python":
            from rl_amd.router import DeviceOps, Router
            router = Router(DeviceOps(eng, ws, dev, n), ws, rank,
                            exchange_device="cpu" if rehearse else None)

            def step(s, tok=None):
                k, p, t, li = inputs[s]
                router.step(k, p, t, allowed, remaining, li)
        else:
            from rl_amd.capi_router import CRouter
            router = CRouter(eng, ws, rank, n, transport="host" if rehearse else "rccl",
                             device=local, recv_cap=args.recv_cap)
            if cfg["dist"] == rl_amd.DIST_ZIPF and not args.no_directory:
                directory = plan_directory(router, cfg, inputs, n)

            def step(s, tok=None):
                k, p, t, li = inputs[s]
                router.step(n, k, p, t, li, allowed, remaining)
    else:
        def step(s, tok=None):
            k, p, t, li = inputs[s]
            eng.execute_device(n, k, p, t, li, None, allowed, remaining, tok)

    # Warmup steps. Step 0 also returns the TB balances (parity); steps 1.. of the warmup
    # carry hipEvents between the stages (the per-stage breakdown); the timed steps below
    # run without them.
    keep0 = None
    stages = {}
    for s in range(warm):
        if s == 1:
            eng.tune("stage_timing", 1)
        step(s, tokens0 if s == 0 else None)
        if s == 0:
            eng.sync()
            torch.cuda.synchronize()
            keep0 = (allowed.cpu().numpy(), remaining.cpu().numpy(),
                     None if tokens0 is None else tokens0.cpu().numpy())
    if warm > 1:
        stages = eng.stage_times()
    warm_stats = eng.stats()          # the batch whose stage times were just read (routed count)
    eng.tune("stage_timing", 1 if args.stage_timing else 0)
    del tokens0

    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(warm, total_steps):
        step(s)
    eng.sync()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if ws > 1:
        router.finish()                    # collective: raises on every rank on an engine error
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    st = eng.last_status()
    stats = eng.stats()
    used = free0 - torch.cuda.mem_get_info(dev)[0]     # this rank's device bytes at the end
    if args.stage_timing:
        stages = eng.stage_times()
    ms_per_step = elapsed / steps * 1e3
    value = ws * n * steps / elapsed

    kern = {k: v for k, v in stages.items() if k not in ("total", "region_offsets") and v > 0}
    # the pass-1 marks bracket empty time (one pass; two passes group per bin since round 6)
    for k in ("scan1", "scatter1"):
        kern.pop(k, None)
    if kern.get("group", 0.0) < 0.01 * kern.get("scatter0", 1.0):
        kern.pop("group", None)
    U = stats["distinct_keys"]
    req_bytes = REQ_IN + (2 if n_lim > 1 else 0) + REQ_OUT
    algo_bytes = n * req_bytes + U * KEY_BYTES            # per GPU per step
    step_s = elapsed / steps
    achieved = algo_bytes * ws / step_s / 1e9             # whole node
    peak = HBM_PEAK_GBS * ws
    traffic, traffic_dir = load_pmc(name, "step", n, ws)
    res_b = eng.result_width()
    kernels = {}
    n_normal = n - warm_stats["routed"] if warm > 1 else n
    for k, ms in kern.items():
        io = kernel_io_bytes(k, n, U, n_lim, res_b, n_normal)
        kernels[k] = {"ms": round(ms, 4), "io_bytes": io,
                      "io_frac": None if io is None else round(io / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    dom = max(kern, key=kern.get) if kern else None
    out = {
        "metric": "rate-limit decisions/sec (whole node)",
        "value": value,
        "unit": "decisions/s",
        "n_gpus": ws,
        "steps": steps,
        "warmup": warm,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if all(l[0] == rl_amd.TB for l in cfg["limiters"]) else
                 ("int64" if not has_tb else "int64+f64"),
        "data": "synthetic (deterministic splitmix64 trace generated on device)",
        "config": {"workload": f"{name}: {cfg['desc']}", "requests_per_gpu_per_step": n,
                   "n_keys": cfg["n_keys"] * ws, "n_limiters": n_lim,
                   "parallelism": f"key-hash shards x{ws}"
                   + (f" + {'C-ABI rl_router' if args.router == 'capi' else 'python router'} "
                      f"all-to-all ({'host rehearsal' if rehearse else 'RCCL'})"
                      + (f", hot-key directory {directory} keys" if directory else "")
                      if ws > 1 else "")},
        # Headline: the whole step's ALGORITHMIC bytes (N x (in + out) + U x
        # (slot read + write)) over the whole step's wall time, against 8 TB/s per GPU. The
        # step is one launch sequence of the pipeline kernels; `kernels` breaks it down.
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "traffic_source": None if traffic is None else
                     f"{traffic_dir} (rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this config, {n} "
                     f"requests/GPU, world {ws}; folded into profiles/pmc_summary.json[{name}])",
                     "kernel": "pipeline (one step)",
                     "algorithmic_bytes_per_step": algo_bytes,
                     "bytes_per_request": req_bytes, "distinct_keys_per_step": U,
                     "dominant_kernel": dom, "kernels": kernels},
        "stage_ms": {k: round(v, 4) for k, v in stages.items()},
        "batch_stats": {k: stats[k] for k in ("allowed", "distinct_keys", "invalid",
                                              "capacity_errors", "regions_touched")},
        "status": rl_amd.strerror(st),
    }
    fp = hbm_footprint(name, n, ws, steps, warm, args.router, args.recv_cap, args.table_scale,
                       parity_tokens and has_tb, ws == 1 and args.pipeline)
    out["hbm_footprint_gb"] = {k: (round(v / 1e9, 3) if not isinstance(v, bool) else v)
                               for k, v in fp.items()}
    out["hbm_footprint_gb"]["tables_now"] = round(
        sum(eng.limiter_slots(i) for i in range(n_lim)) * 32 / 1e9, 3)   # after on-demand growth
    out["hbm_footprint_gb"]["measured"] = round(used / 1e9, 3)           # hipMemGetInfo delta
    if router is not None and hasattr(router, "stats"):
        rs = router.stats()
        out["router"] = {"rounds_per_step": rs["rounds"] / max(1, rs["steps"]),
                         "split_steps": rs["split_steps"], "max_recv": rs["max_recv"],
                         "recv_cap": rs["recv_cap"], "reserved_gb": rs["reserved_bytes"] / 1e9,
                         "header_sync_ms_per_step": rs["header_sync_ns"] * 1e-6 / max(1, rs["steps"])}
    if router is not None and hasattr(router, "close"):
        router.close()
    eng.close()
    return out, inputs[0], keep0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="sw_zipf", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="requests per GPU per step (override)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="N=1: skip the extra tb_uniform / zipf_1b / mixed_tenants / config1 keys of the line")
    ap.add_argument("--cpu-sample", type=int, default=1 << 26)
    ap.add_argument("--tune", action="append", default=[],
                    help="engine knob key=value (rl_tune), e.g. hot_threshold=32768")
    ap.add_argument("--table-scale", type=int, default=1,
                    help="size the state tables for this many times the config's key count "
                         "(engine sizing: lower load, more and smaller regions)")
    ap.add_argument("--pipeline", action="store_true",
                    help="N=1: overlap batch s+1's partition with batch s's decisions (RL_OPT_PIPELINE)")
    ap.add_argument("--stage-timing", action="store_true",
                    help="also record hipEvents inside the timed steps (diagnostics only)")
    ap.add_argument("--router", choices=("capi", "python"), default="capi",
                    help="N>1: the C-ABI router (product path) or the torch.distributed one")
    ap.add_argument("--recv-cap", type=int, default=0,
                    help="N>1: requests an owner decides per exchange round (0: min(N, 2) x batch)")
    ap.add_argument("--no-directory", action="store_true",
                    help="N>1: hash owners only (no hot-key directory on Zipf configs)")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    if ws != args.gpus and not (ws == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
    # RL_BENCH_REHEARSE=1: every rank on cuda:0, exchanges through gloo on the host — a
    # functional rehearsal of the N>1 path on a one-GPU box (its numbers mean nothing)
    rehearse = ws > 1 and os.environ.get("RL_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    if ws > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    # CPU baseline + parity on rank 0's slice of batch 0. The global stream is rank-major, so
    # that slice is the head of the whole trace: the oracle's sequential replay of it alone is
    # exact at any world size. At N>1 the router returns no token balances (decisions and
    # remaining are compared).
    baseline = rank == 0 and not args.no_cpu_baseline
    out, in0, keep0 = run(args.config, args, ws, rank, local, dev, rehearse, args.steps,
                          args.warmup, parity_tokens=baseline and ws == 1)
    if baseline:
        k0, p0, t0_, l0 = in0
        cb, dec_ok, bal, m = cpu_baseline(CONFIGS[args.config], k0, p0, t0_, l0, args.cpu_sample,
                                          keep0[0], keep0[1], keep0[2])
        if ws > 1:
            cb["sample"] += f" (rank 0's slice: the head of the {ws}-rank global stream)"
        out["cpu_baseline"] = cb
        out["parity"] = parity_text(dec_ok, bal, m)
    else:
        out["cpu_baseline"] = None
    del in0
    if baseline and ws == 1 and not args.no_extra:
        torch.cuda.empty_cache()
        # BASELINE configs[1] (tb_uniform) and the per-GPU share of configs[4] (zipf_1b: the
        # north-star 1B-key TB + SW trace at 8 GPUs) on the same box, each with its own
        # roofline, CPU baseline and batch-0 parity (TB balances bit-for-bit)
        for extra in ("tb_uniform", "zipf_1b", "mixed_tenants"):
            if extra == args.config:
                continue
            xo, xin0, xkeep0 = run(extra, args, 1, 0, local, dev, False, args.steps,
                                   args.warmup, parity_tokens=True)
            cbx, dec_x, bal_x, mx = cpu_baseline(CONFIGS[extra], *xin0, args.cpu_sample,
                                                 xkeep0[0], xkeep0[1], xkeep0[2], single_thread=False)
            out[extra] = {k: xo[k] for k in ("value", "unit", "ms_per_step", "config", "stage_ms",
                                             "batch_stats", "status", "roofline", "hbm_footprint_gb")}
            out[extra]["roofline_frac"] = xo["roofline"]["frac"]
            out[extra]["cpu_baseline"] = cbx
            out[extra]["parity"] = parity_text(dec_x, bal_x, mx)
            del xin0, xkeep0
            torch.cuda.empty_cache()
        out["config1"] = config1_line(dev)
    if rank == 0:
        print(json.dumps(out))
    if ws > 1:
        dist.barrier()                     # rank 0's CPU baseline ran after the timed steps
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
