// rl_hot.hpp — 4b. hot regions: dominant-key chains, their summaries and fills (templates;
// rl_hot.hip holds the untemplated kernels and the launchers, rl_rt_*.hip the instantiations).
#pragma once
#include "rl_region.hpp"

#pragma clang fp contract(off)

namespace rl {

// ------------------------------------------------------------------ 4b. hot regions
// A region far above the average share (a hot Zipf key: at s = 1.1 over 100M keys the
// top key draws 11 % of all requests) would serialise one wave, and one CU's memory
// bandwidth, for the whole batch. Its dominant key (the HOT key) gets a fast path:
//  * a deny never changes state (SlidingWindowRateLimiter.java:104-111,
//    TokenBucketRateLimiter.java:61-67);
//  * for a fixed state the SW estimate (:158-180) is non-increasing in `now` for `now`
//    at or after the newest bucket, and the TB balance (Lua :46-58) is non-decreasing.
// So one threshold pair [T0, T1) per state holds exactly the times at which a request is
// denied with remaining 0 (SW: est >= max; TB: 0 <= balance < 1), whatever its permits.
// Inside an undecided chunk the further thresholds T_2.. decide the other denials by
// integer compares (hot_pred_k below); the allowed request, a peek or a reset runs the
// exact step alone, and after each state change the thresholds are found again by an
// exact search that evaluates the very same arithmetic (tb_refill, sw_estimate) at 64
// times per wave instruction. Three phases:
//  A  k_hot_summ  (all CUs)  per 64 records: time range of the hot key's plain acquires,
//                             count of records that need the exact path;
//  B  k_hot_chain (one wave per hot region, beside k_regions) walks the summaries with
//                             [T0, T1), decides whole chunks unread, processes the rest
//                             record by record (other keys through wave_apply);
//  C  k_hot_fill  (all CUs)  writes the results of the decided chunks.
// Start of the range on which the thresholds (hot_pred_k) are monotone and valid.
template <int ALGO>
__device__ inline int64_t hot_t0(int64_t lo, int64_t hi, uint64_t a, uint64_t b, uint64_t c) {
    if constexpr (ALGO == kAlgoTB) {
        if (!(c & 1u)) return lo;                               // absent: full at every t
        if (!(__longlong_as_double((long long)a) >= 0.0)) return hi + 1;
        return (int64_t)b > lo ? (int64_t)b : lo;               // t >= last: balance >= 0
    } else {
        const SW2 s = sw_unpack(a, b, c);
        if (s.b1_cnt == 0 && s.b0_cnt == 0) return lo;
        return s.b1_start > lo ? s.b1_start : lo;
    }
}

// First t in [s, hi] with pred(t) for a predicate monotone (false..true) on [s, hi];
// hi + 1 if none. One wave: an exponential bracket (64 probes in one instruction), then
// 64-ary narrowing. Arguments are wave-uniform.
template <class P>
__device__ inline int64_t wave_first_true(int64_t s, int64_t hi, uint32_t lane, P pred) {
    if (s > hi) return hi + 1;
    int64_t t = lane == 0 ? s : (lane < 63 ? s + ((int64_t)1 << (lane - 1)) : hi);
    if (t > hi) t = hi;
    const uint64_t m = __ballot(pred(t));
    if (m == 0) return hi + 1;
    const uint32_t k = (uint32_t)__builtin_ctzll(m);
    if (k == 0) return s;
    int64_t lo = __shfl(t, (int)k - 1, 64) + 1;                 // pred(t_{k-1}) false
    int64_t h = __shfl(t, (int)k, 64);                          // pred(t_k) true
    while (h > lo) {
        const int64_t step = (h - lo + 64) / 64;
        int64_t u = lo + ((int64_t)lane + 1) * step - 1;
        if (u > h) u = h;
        const uint64_t mm = __ballot(pred(u));
        if (mm == 0) return h;                                  // (monotone: not reached)
        const uint32_t kk = (uint32_t)__builtin_ctzll(mm);
        const int64_t uk = __shfl(u, (int)kk, 64);
        const int64_t ukm = __shfl(u, kk ? (int)kk - 1 : 0, 64);
        lo = kk ? ukm + 1 : lo;
        h = uk;
    }
    return lo;
}

// For a fixed state and t >= hot_t0, an acquire of k permits at t is allowed iff t >= T_k,
// the first t with (TB) balance >= k or (SW) estimate <= max - k: the predicate below is
// monotone in t (nested in k).
template <int ALGO>
__device__ inline bool hot_pred_k(const DevLimiter& L, int64_t t, uint64_t a, uint64_t b, uint64_t c,
                                  int64_t k) {
    if constexpr (ALGO == kAlgoTB) {
        return tb_refill(L, t, a, b, c) >= (double)k;
    } else {
        const SW2 s = sw_unpack(a, b, c);
        return sw_estimate(s, sw_geo(t, L), t, L.window_ms) + k <= L.max_permits;
    }
}

// A starting point for T_k from the closed forms (hot_t1_lb checks it exactly).
template <int ALGO>
__device__ inline int64_t hot_tk_guess(const DevLimiter& L, int64_t s, uint64_t a, uint64_t b,
                                       uint64_t c, int64_t k) {
    if constexpr (ALGO == kAlgoTB) {
        if (!(c & 1u)) return s;                                // absent: full at every t
        const double tok0 = __longlong_as_double((long long)a);
        const int64_t last = (int64_t)b;
        if (!(tok0 < (double)k) || !(L.rate_per_ms > 0.0)) return s;
        const double te = (double)last + ceil(((double)k - tok0) * L.inv_rate);
        const int64_t g = te < 4.0e18 ? (int64_t)te : INT64_MAX / 4;
        const int64_t full = last + L.ttl_ms + 1;               // expired: full again
        return g < full ? g : full;
    } else {
        const int64_t m = L.max_permits - k + 1;                // allowed iff estimate < m
        const int64_t w = L.window_ms;
        const SW2 st = sw_unpack(a, b, c);
        const SWGeo g0 = sw_geo(s, L);
        const int64_t C = sw_get(st, g0.curr_start, s, w);
        const int64_t P = sw_get(st, g0.prev_start, s, w);
        const int64_t wend = g0.curr_start + w;                 // next window: a new geometry
        if (m <= 0) return s;
        if (C < m) {
            if (P == 0) return s;
            // estimate = P * pw + C < m  <=>  now % w > w (1 - (m - C) / P)
            const double rr = (double)w * (1.0 - (double)(m - C) * __builtin_amdgcn_rcp((double)P));
            int64_t g = g0.curr_start + (int64_t)floor(rr) + 1;
            int64_t lastp = INT64_MAX / 4;                      // previous bucket's TTL lapse
            if (st.b1_start == g0.prev_start) lastp = st.b1_start + st.b1_off;
            else if (st.b1_start == g0.curr_start) lastp = g0.prev_start + st.b0_off;
            if (g > lastp + w + 1) g = lastp + w + 1;
            if (g < wend) return g > s ? g : s;
        }
        // not in this window: in the next one the current bucket (C) is the previous one,
        // weighted by pw, until its TTL lapses (last INCR + w)
        if (C < m) return wend;
        const int64_t lastc = st.b1_start == g0.curr_start ? st.b1_start + st.b1_off : wend;
        const double rr = (double)w * (1.0 - (double)m * __builtin_amdgcn_rcp((double)C));
        int64_t g = wend + (int64_t)floor(rr) + 1;
        if (g > lastc + w + 1) g = lastc + w + 1;
        return g;
    }
}

// A lower bound T1 > T0 of the first t >= T0 at which an acquire of one permit is
// allowed, from the closed-form guess g checked exactly at g - 1 (the predicate is monotone
// on [T0, hi]); T0 (an empty range) when the check fails. [T0, T1) then holds only denials
// with remaining 0; whatever lies beyond it is processed exactly.
template <int ALGO>
__device__ inline int64_t hot_t1_lb(const DevLimiter& L, uint64_t a, uint64_t b, uint64_t c,
                                    int64_t T0, int64_t hi) {
    if (T0 > hi) return T0;
    int64_t g = hot_tk_guess<ALGO>(L, T0, a, b, c, 1);
    if (g > hi + 1) g = hi + 1;
    if (g <= T0 + 1) return T0;
    return hot_pred_k<ALGO>(L, g - 1, a, b, c, 1) ? T0 : g;
}

// prev * pw of the sliding-window estimate at `now` (:170-174, rounded as Java rounds) for
// the key state (a, b, c), off the hot chains' fast paths: a call, so that the compiler cannot
// hoist the window geometry and its fp64 division into them (inlined, they were computed for
// every request of every detailed chunk, used or not).
__device__ __attribute__((noinline)) double sw_prev_weighted(int64_t now, uint64_t a, uint64_t b,
                                                             uint64_t c, int64_t w, double inv_w) {
    DevLimiter L{};
    L.window_ms = w;
    L.inv_window = inv_w;
    const SWGeo g = sw_geo(now, L);
    return (double)sw_get(sw_unpack(a, b, c), g.prev_start, now, w) * g.prev_weight;
}

// Wave-uniform values made visibly so (v_readfirstlane into SGPRs): the chains' control flow
// on them then compiles to scalar branches instead of exec-mask regions around 64-bit VALU
// compares, which a lone wave pays for at every step.
__device__ inline uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ inline int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ inline uint64_t uni(uint64_t x) {
    return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | (uint64_t)uni((uint32_t)x);
}
__device__ inline int64_t uni(int64_t x) { return (int64_t)uni((uint64_t)x); }
__device__ inline double uni(double x) {
    return __longlong_as_double((long long)uni((uint64_t)__double_as_longlong(x)));
}
__device__ inline HotInfo uni(const HotInfo& f) {
    HotInfo u;
    u.tag = uni(f.tag); u.bin = uni(f.bin); u.start = uni(f.start); u.end = uni(f.end);
    u.n_chunks = uni(f.n_chunks); u.chunk_base = uni(f.chunk_base); u.ok = uni(f.ok);
    u.n_groups = uni(f.n_groups); u.group_base = uni(f.group_base); u.tag2 = uni(f.tag2);
    return u;
}
__device__ inline DevLimiter uni(const DevLimiter& l) {
    DevLimiter u;
    u.algo = uni(l.algo); u.region_bits = uni(l.region_bits); u.region_base = uni(l.region_base);
    u.lflags = uni(l.lflags); u.max_permits = uni(l.max_permits); u.window_ms = uni(l.window_ms);
    u.ttl_ms = uni(l.ttl_ms); u.rate_per_ms = uni(l.rate_per_ms); u.capacity = uni(l.capacity);
    u.table = uni(l.table); u.inv_window = uni(l.inv_window); u.cache_table = uni(l.cache_table);
    u.cache_ttl_ms = uni(l.cache_ttl_ms); u.inv_rate = uni(l.inv_rate);
    return u;
}

// Lane order = arrival order; chunk g of the listed regions -> (region i, chunk c).
__device__ inline uint32_t hot_region_of(const uint32_t* s_base, uint32_t hc, uint32_t g) {
    uint32_t lo = 0, hi = hc;                        // last i with s_base[i] <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (s_base[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

// Phase 0 (one wave per listed region): bounds, chunks and the dominant key of a sample
// of the region's first 64 records (a hot region is dominated by its hot key), and a
// second key when the sample says it holds >= kHot2MinRecords of the region.
constexpr uint32_t kHot2MinSample = 4;
constexpr uint32_t kHot2MinRecords = 32768;
template <class Codec>
__global__ __launch_bounds__(64) void k_hot_prep(RegionArgs a) {
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t i = blockIdx.x, lane = threadIdx.x;
    if (i == 0 && lane == 0) a.ctl->n_hot = hc;
    if (i >= hc) return;
    const uint32_t e = a.hot_list[i];
    uint32_t bin, start, end;
    if (e & kHotRoutedBit) {                      // routed: its own pass-0 bin
        const uint32_t r = e & ~kHotRoutedBit;
        bin = a.route_list[r];
        start = a.route_start[r];
        end = start + a.route_cnt[r];
    } else {
        bin = e;
        start = a.rstart[bin];
        end = start + (a.rend ? a.rend[bin] - start : a.rcount[bin]);
    }
    const typename Codec::Rec* recs = (const typename Codec::Rec*)a.rec;
    const int64_t base = a.ctl->base_ms;
    const uint32_t n0 = min(end - start, 64u);
    const bool act = lane < n0;
    uint64_t h = 0;
    bool ok = false;
    if (act) {
        const Req q = Codec::dec(recs[start + lane], base);
        h = q.h;
        ok = !q.invalid;
    }
    uint32_t cnt = 0;
    for (uint32_t k = 0; k < n0; ++k) cnt += (__shfl(h, (int)k, 64) == h) ? 1u : 0u;
    uint32_t key = (act && ok) ? (cnt << 6) | (63u - lane) : 0u;
    for (int o = 32; o > 0; o >>= 1) key = max(key, (uint32_t)__shfl_xor((int)key, o, 64));
    const uint64_t tag = __shfl(h, (int)(63u - (key & 63u)), 64);
    // a second heavy key (two hot Zipf keys in one region): its own chain, or wave 1 would
    // apply its ~10^5 records 64 at a time (sw_zipf: a 398K-record region set the stage)
    uint32_t key2 = (act && ok && h != tag) ? (cnt << 6) | (63u - lane) : 0u;
    for (int o = 32; o > 0; o >>= 1) key2 = max(key2, (uint32_t)__shfl_xor((int)key2, o, 64));
    const uint64_t tag2 = __shfl(h, (int)(63u - (key2 & 63u)), 64);
    const uint32_t c1 = key >> 6, c2 = key2 >> 6;
    const bool two = c1 >= 2u && c2 >= kHot2MinSample &&
                     (uint64_t)(end - start) * c2 >= (uint64_t)kHot2MinRecords * n0;
    if (lane == 0) {
        HotInfo f;
        f.tag = tag; f.bin = bin; f.start = start; f.end = end;
        f.n_chunks = (end - start + kHotChunk - 1) / kHotChunk;
        f.chunk_base = 0;
        f.ok = (c1 >= 2u ? 1u : 0u) | (two ? 2u : 0u);
        f.n_groups = (f.n_chunks + 63) / 64;
        f.group_base = 0;
        f.tag2 = two ? tag2 : 0;
        a.hot_info[i] = f;
    }
}



// Phase A (one wave per group of 64 chunks, all CUs): what a chain needs to decide its key's
// records of a chunk (64 records) or a group (4096) without reading them: the time range of
// its plain acquires, and how many of its records need the exact path (peek / reset). Eight
// words per chunk, four per key (key k at 4k): [0] min now, [1] max now, [2] n_special |
// n_hot << 8 | n_early << 16 | n_rest << 24, [3] verdict: bit 0 = the key's records decided
// by the thresholds (words 0-2 then hold its state), bit 1 = TB early rejects among them,
// bits 8-15 = n_rest. n_rest counts the records of other keys: for the dominant key every
// other record, for the second key those of neither (the records wave 1 applies). Group
// words: the same over the group's chunks, with 0/1 flags for the counts. The wave keeps
// four chunks' records in flight.
__device__ inline uint64_t wave_min64(uint64_t v) { return wave_min_dpp<uint64_t>(v); }
__device__ inline uint64_t wave_max64(uint64_t v) { return wave_max_dpp<uint64_t>(v); }
__device__ inline uint32_t wave_min32(uint32_t v) { return wave_min_dpp<uint32_t>(v); }
__device__ inline uint32_t wave_max32(uint32_t v) { return wave_max_dpp<uint32_t>(v); }

// A key the walk pays for, from its expected allows e (an upper estimate: TB a full bucket plus
// the refill over the batch's span; SW the limit per window over the windows the span
// touches): at least walk_min of them (kWalkMinAllows), so that the chain is long, and at most
// 2.5 per 64-record chunk: denser keys allow several times per chunk, which the chunk-by-chunk
// path decides at one detail per chunk.
__device__ inline bool walk_dense(const HotInfo& f, const DevLimiter& L, int64_t lo, int64_t hi,
                                  uint32_t walk_min) {
    const double span = (double)(hi - lo + 1);
    const double e = L.algo == kAlgoTB ? L.capacity + L.rate_per_ms * span
                                       : (double)L.max_permits * (span / (double)L.window_ms + 2.0);
    return e >= (double)walk_min && 2.0 * e <= 5.0 * (double)f.n_chunks;
}

// Allow walks (hot_chain): is region i's key table built in this batch (slot 2 i + key)?
__device__ inline bool walk_table_on(const RegionArgs& a, uint32_t i, const HotInfo& f,
                                     const DevLimiter& L, int64_t lo, int64_t hi) {
    return a.walk_tab && i < walk_regions(lo, hi) && f.end - f.start < (1u << 31) &&
           walk_dense(f, L, lo, hi, a.walk_min);
}

template <class Codec>
__global__ __launch_bounds__(256) void k_hot_summ(RegionArgs a) {
    using Rec = typename Codec::Rec;
    __shared__ uint32_t s_base[kHotMax + 1];
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t total = a.hot_total[1];
    for (uint32_t i = threadIdx.x; i < hc; i += 256) s_base[i] = a.hot_info[i].group_base;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const Rec* recs = (const Rec*)a.rec;
    const int64_t base = a.ctl->base_ms;
    const int64_t lo = batch_lo(a.ctl), hi = batch_hi(a.ctl);
    const uint64_t lanes_below = (1ULL << lane) - 1;
    for (uint32_t gg = blockIdx.x * 4 + wid; gg < total; gg += gridDim.x * 4) {
        const uint32_t i = hot_region_of(s_base, hc, gg);
        const HotInfo f = a.hot_info[i];
        const DevLimiter& L = a.lims[a.region_lim[f.bin]];
        const bool tb = L.algo == kAlgoTB;
        const int64_t maxp = L.max_permits;
        const bool two = (f.ok & 2u) != 0;
        const uint32_t c0 = (gg - s_base[i]) * 64, c1 = min(c0 + 64, f.n_chunks);
        uint64_t gmn[2] = {~0ULL, ~0ULL}, gmx[2] = {0ULL, 0ULL};
        uint32_t gfl[2] = {0u, 0u};                      // flags: special, hot, early, rest
        // allow-walk table of each key (slot 2 i + k): the first plain acquire of 1 and of at
        // most 2 permits in each ms, found once per (chunk, ms) and merged by atomicMin over
        // the chunks. Group flags (word 2, bits 24-25): the key's plain acquires are not in
        // time order (bit 24, judged against the chunks before in the group: wcarry), or
        // some ask for more than 2 permits (bit 25); either keeps the chain off the walk.
        const bool walk_on = walk_table_on(a, i, f, L, lo, hi);
        int64_t wcarry[2] = {INT64_MIN, INT64_MIN};
        uint32_t wflag[2] = {0u, 0u};
        auto load = [&](uint32_t c) { return recs[min(f.start + c * kHotChunk + lane, f.end - 1)]; };
        auto chunk = [&](const Rec& r, uint32_t c) {
            const uint32_t j = f.start + c * kHotChunk + lane;
            const bool valid = j < f.end;
            const Req q = Codec::dec(r, base);
            const bool acq = q.op == (uint32_t)kOpAcquire;
            const bool hot0 = valid && (f.ok & 1u) && !q.invalid && q.h == f.tag;
            const bool hot1 = two && valid && !q.invalid && q.h == f.tag2;
            uint64_t w[8];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (k == 1 && !two) {                     // (wave-uniform) no second key: its words
                    const uint64_t no = w[2] >> 24;       // hold only key 0's rest count
                    w[4] = (uint64_t)INT64_MAX; w[5] = (uint64_t)INT64_MIN;
                    w[6] = no << 24; w[7] = no << 8;
                    gfl[1] |= no ? 8u : 0u;
                    break;
                }
                const bool hot = k ? hot1 : hot0;
                const bool early = hot && acq && tb && (int64_t)q.permits > maxp;
                const bool plain = hot && acq && !early;
                const bool special = hot && !acq;         // the key's peek / reset
                // n_rest: not the dominant key / neither key (invalid records included)
                const bool rest = valid && !hot0 && (k == 0 || !hot1);
                uint64_t mn = ~0ULL, mx = 0ULL;
                if (k == 0 || two) {                      // (wave-uniform)
                    if constexpr (std::is_same<Codec, CodecC>::value) {
                        // compact records: now = base + now_rel, so the 32-bit offsets order
                        // the same way and the reductions move half the bits
                        const uint32_t m32 = wave_min32(plain ? r.now_rel : ~0u);
                        const uint32_t x32 = wave_max32(plain ? r.now_rel : 0u);
                        if (__ballot(plain)) {
                            mn = ord_key(base + (int64_t)m32);
                            mx = ord_key(base + (int64_t)x32);
                        }
                    } else {
                        mn = wave_min64(plain ? ord_key(q.now_ms) : ~0ULL);
                        mx = wave_max64(plain ? ord_key(q.now_ms) : 0ULL);
                    }
                }
                if (walk_on && (k == 0 || two)) {                // (wave-uniform)
                    const uint64_t pm = __ballot(plain);
                    if (pm) {
                        const uint64_t bp = pm & lanes_below;
                        const int64_t tp = shfl64(q.now_ms, bp ? 63 - __builtin_clzll(bp) : (int)lane);
                        const bool ooo = plain && (bp ? tp : wcarry[k]) > q.now_ms;
                        wflag[k] |= (__ballot(ooo) ? 1u : 0u) | (__ballot(plain && q.permits > 2) ? 2u : 0u);
                        uint2* wt = a.walk_tab + (size_t)(2 * i + k) * walk_stride(lo, hi);
                        const uint32_t ix = (uint32_t)(q.now_ms - lo), rel = j - f.start;
                        const uint64_t b1 = __ballot(plain && q.permits == 1) & lanes_below;
                        const uint64_t b2 = __ballot(plain && q.permits <= 2) & lanes_below;
                        const int64_t t1 = shfl64(q.now_ms, b1 ? 63 - __builtin_clzll(b1) : (int)lane);
                        const int64_t t2 = shfl64(q.now_ms, b2 ? 63 - __builtin_clzll(b2) : (int)lane);
                        if (plain && q.permits == 1 && (!b1 || t1 != q.now_ms))
                            atomicMin(&wt[ix].x, rel);
                        if (plain && q.permits <= 2 && (!b2 || t2 != q.now_ms))
                            atomicMin(&wt[ix].y, rel);
                        wcarry[k] = (int64_t)readlane64((uint64_t)q.now_ms, 63u - (uint32_t)__builtin_clzll(pm));
                    }
                }
                const uint32_t ns = (uint32_t)__popcll(__ballot(special));
                const uint32_t nh = (uint32_t)__popcll(__ballot(hot));
                const uint32_t ne = (uint32_t)__popcll(__ballot(early));
                const uint32_t no = (uint32_t)__popcll(__ballot(rest));
                w[4 * k + 0] = mn == ~0ULL ? (uint64_t)INT64_MAX : (mn ^ 0x8000000000000000ULL);
                w[4 * k + 1] = mx == 0ULL ? (uint64_t)INT64_MIN : (mx ^ 0x8000000000000000ULL);
                w[4 * k + 2] = ns | (nh << 8) | (ne << 16) | (no << 24);
                w[4 * k + 3] = (uint64_t)no << 8;
                gmn[k] = mn < gmn[k] ? mn : gmn[k];
                gmx[k] = mx > gmx[k] ? mx : gmx[k];
                gfl[k] |= (ns ? 1u : 0u) | (nh ? 2u : 0u) | (ne ? 4u : 0u) | (no ? 8u : 0u);
            }
            uint64_t v = w[0];                            // lanes 0-7: one 64-B store
#pragma unroll
            for (int k = 1; k < 8; ++k) v = lane == (uint32_t)k ? w[k] : v;
            if (lane < 8) a.hot_summ[(size_t)(f.chunk_base + c) * 8 + lane] = v;
        };
        Rec q0 = load(c0), q1 = load(c0 + 1), q2 = load(c0 + 2), q3 = load(c0 + 3);
        for (uint32_t c = c0; c < c1; c += 4) {
            chunk(q0, c);     q0 = load(c + 4);
            if (c + 1 >= c1) break;
            chunk(q1, c + 1); q1 = load(c + 5);
            if (c + 2 >= c1) break;
            chunk(q2, c + 2); q2 = load(c + 6);
            if (c + 3 >= c1) break;
            chunk(q3, c + 3); q3 = load(c + 7);
        }
        uint64_t v = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint64_t gw0 = gmn[k] ^ 0x8000000000000000ULL, gw1 = gmx[k] ^ 0x8000000000000000ULL;
            const uint64_t gw2 = (gfl[k] & 1u) | ((gfl[k] >> 1 & 1u) << 8) | ((gfl[k] >> 2 & 1u) << 16) |
                                 ((uint64_t)wflag[k] << 24);
            const uint64_t gw3 = (uint64_t)(gfl[k] >> 3 & 1u) << 8;   // rest: kept through the verdict
            v = lane == 4u * k ? gw0 : lane == 4u * k + 1 ? gw1 : lane == 4u * k + 2 ? gw2 :
                lane == 4u * k + 3 ? gw3 : v;
        }
        if (lane < 8) a.hot_summ2[(size_t)gg * 8 + lane] = v;
    }
}

// Phase B (one single-wave workgroup per listed region, beside k_regions). Pass 1 walks the
// region's summaries in arrival order with the hot key's threshold pair: a group of 64
// chunks, or a chunk, whose hot-key times all lie in [T0, T1) has its hot records decided
// without being read (verdict + the key's state go back into the summary for k_hot_fill);
// the other chunks are processed one by one (fast check, then the sequential run of the
// key's state changes). Pass 1 runs again for a second dominant key when the region
// holds one (HotInfo::ok bit 1). Pass 2 then applies every other key of the region in
// arrival order, 64 records at a time through wave_apply. (A workgroup of one wave per pass
// waited for its wave slots on one CU beside the normal regions: sw_zipf's later chains
// started ~4 ms into the stage.)
// SPLIT (two-wave workgroups): wave 0 loads the region and runs pass 1, wave 1 runs pass 2
// beside it on the same LDS image (pass 1 touches only its keys' slots, pass 2 never those)
// and exits, handing its debug words over in LDS; wave 0 waits for it and writes back.
template <class Codec, class Res, bool TOK, bool SPLIT>
__device__ inline void hot_chain(const RegionArgs& a, uint32_t i, RegionLds<Codec, true>& S) {
    using Rec = typename Codec::Rec;
    constexpr uint32_t NS = kRegionSlots;
    __shared__ int32_t s_hslot[2];
    __shared__ uint64_t s_p2[3];                      // SPLIT: wave 1 done, its cycles, records
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = SPLIT ? threadIdx.x >> 6 : 0u;
    if (i >= hc) return;
    // the passes are sequential critical paths beside thousands of normal-region waves
    __builtin_amdgcn_s_setprio(3);
    const HotInfo f = a.hot_info[i];
    const uint32_t region = f.bin;                    // a bin is one region
    const DevLimiter L = a.lims[a.region_lim[region]];
    const int64_t base = uni(a.ctl->base_ms);
    const int64_t lo = uni(batch_lo(a.ctl));
    const int64_t hi = uni(batch_hi(a.ctl));
    const Rec* recs = (const Rec*)a.rec;
    Res* res = (Res*)a.res;
    const uint32_t pad = a.n_total + lane;
    if (a.ctl->span_overflow != 0) {                  // whole batch rejected (see k_regions)
        for (uint32_t j = f.start + threadIdx.x; j < f.end; j += blockDim.x) {
            res[j] = (Res)pack_result(false, kRemInvalid);
            if (TOK) a.tok[j] = __builtin_nan("");
        }
        return;
    }
    const uint64_t t_start = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    RL_GLOBAL Slot* tab = as_global((Slot*)L.table + (size_t)(region - L.region_base) * NS);
    if (wv == 0) {
        // ---- load + rebuild the region (as k_regions), find or insert the hot key's slot
        Slot img[NS / 64];
#pragma unroll
        for (uint32_t k = 0; k < NS / 64; ++k) {
            S.occ[lane + 64 * k] = 0;
            S.pm[lane + 64 * k] = 0;
            img[k] = tab[lane + 64 * k];
        }
        wave_fence();
#pragma unroll
        for (uint32_t k = 0; k < NS / 64; ++k) {
            const Slot v = img[k];
            if (slot_live(L, v, keep_from(a))) {
                uint32_t p = slot_home(v.tag);
                while (atomicCAS(&S.occ[p], 0u, 1u) != 0u) p = (p + 1) & (NS - 1);
                S.tag[p] = v.tag; S.sa[p] = v.a; S.sb[p] = v.b; S.sc[p] = v.c;
            }
        }
        wave_fence();
        int32_t hsl[2] = {-1, -1};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (!((f.ok >> k) & 1u)) continue;              // (wave-uniform)
            const uint64_t tg = k ? f.tag2 : f.tag;
            const uint32_t p0 = slot_home(tg);
            int32_t hslot = -1;
            for (uint32_t m = 0; m < NS; ++m) {             // linear probing, as the rebuild
                const uint32_t p = (p0 + m) & (NS - 1);
                const uint32_t o = S.occ[p];
                if (!(o & 1u) || S.tag[p] == tg) { hslot = (int32_t)p; break; }
            }
            if (hslot >= 0 && !(S.occ[hslot] & 1u) && lane == 0) {
                S.occ[hslot] = 1u; S.tag[hslot] = tg; S.sa[hslot] = 0; S.sb[hslot] = 0; S.sc[hslot] = 0;
            }
            wave_fence();
            hsl[k] = hslot;
        }
        if (lane == 0) { s_hslot[0] = hsl[0]; s_hslot[1] = hsl[1]; }
        if (SPLIT && lane == 0) s_p2[0] = 0;
    }
    if (SPLIT) __syncthreads();
    else wave_fence();
    // hot_ok false (no dominant key, or its region is full): pass 2 takes every record; the
    // second key has a chain only beside the first's
    const int32_t hsl0 = s_hslot[0];
    const int32_t hsl1 = hsl0 >= 0 ? s_hslot[1] : -1;
    const bool hot_ok = hsl0 >= 0, hot_ok2 = hsl1 >= 0;
    auto is_hot = [&](const Req& q, bool valid) {
        return valid && !q.invalid && ((hot_ok && q.h == f.tag) || (hot_ok2 && q.h == f.tag2));
    };
    // summary words of chunk c / group g (8 per entry: 4 per key)
    auto summ_at = [&](uint32_t c) {
        return a.hot_summ + (size_t)(f.chunk_base + (c < f.n_chunks ? c : 0)) * 8;
    };
    auto grp_at = [&](uint32_t g) {
        return a.hot_summ2 + (size_t)(f.group_base + (g < f.n_groups ? g : 0)) * 8;
    };
    // the verdict word holding wave 1's "records of neither key" count in bits 8-15
    const uint32_t rest_w = hot_ok2 ? 7u : 3u;

    uint32_t n_allowed = 0, n_invalid = 0, n_caperr = 0, n_rounds = 0, n_detail = 0, n_other = 0;
    uint32_t n_internal = 0;                          // walk logic errors (RL_E_INTERNAL, uniform)
    uint32_t n_changed = 0, n_tk = 0, n_fb = 0;       // debug: changes, [T0, T1) updates,
    uint32_t n_late = 0;                              // detailed chunks starting before T0 / ending past T1
    uint32_t n_prehit = 0;                            // debug: chunks whose records were prefetched
    uint32_t n_bisect = 0;                            // debug: SW table entries found by bisection
    uint64_t cyc_build = 0;                           // debug: SW table builds
    uint64_t cyc_run = 0, cyc_search = 0, cyc_detail = 0, cyc_pass2 = 0;   // debug stamps
    uint64_t cyc_pre = 0, cyc_pass1 = 0;
    uint64_t cyc_sw[4] = {0, 0, 0, 0};                // debug: SW run: setup, greedy, remaining, commit
    uint32_t n_sw_it = 0;                             // debug: SW greedy steps
    uint32_t n_walk = 0, n_find = 0, n_enter = 0;     // debug: walked allows, table steps, block loads
    uint64_t cyc_find = 0, cyc_walk = 0;              // debug: walk cycles (finding / all)
    uint64_t cyc_close = 0, cyc_allow = 0;            // debug: walk cycles (verdicts / allows)
    bool any_hot = false;
    auto pass1 = [&](auto algo, const uint32_t kk) {
        constexpr int A = decltype(algo)::value;
        const uint32_t ow = 4u * kk;                      // this key's summary words
        const uint32_t hs = (uint32_t)(kk ? hsl1 : hsl0);
        const uint64_t tag = kk ? f.tag2 : f.tag;
        auto is_key = [&](const Req& q, bool valid) { return valid && !q.invalid && q.h == tag; };
        // the hot key's state (registers; written to LDS when it changes) and the range
        // [T0, T1) in which every acquire is denied with remaining 0 (whole chunks and groups
        // inside it are decided without being read)
        uint64_t sa = uni(S.sa[hs]), sb = uni(S.sb[hs]), sc = uni(S.sc[hs]);
        // T1 from the closed-form guess verified at g - 1; when the guess overshoots (the
        // check fails), the exact first allowed time by a search on the same arithmetic
        auto t1_of = [&](int64_t t0) {
            int64_t g = hot_tk_guess<A>(L, t0, sa, sb, sc, 1);
            if (g > hi + 1) g = hi + 1;
            if (g <= t0 + 1) return t0;
            auto pred = [&](int64_t t) { return hot_pred_k<A>(L, t, sa, sb, sc, 1); };
            if (!pred(g - 1)) return g;
            return wave_first_true(t0, g - 1, lane, pred);
        };
        const uint64_t c_p1 = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
        int64_t T0 = hot_t0<A>(lo, hi, sa, sb, sc);
        int64_t T1 = t1_of(T0);
        // Sliding window: the allow-time table of the key's current window W. P(t) (the
        // previous bucket, with its TTL lapse) is the same for every state the key passes
        // through inside W (allows only INCR the current bucket, :114-116), so the first
        // times at which an acquire of 1 or 2 permits is allowed with C = thr_c + lane in the
        // current bucket, thr1 / thr2 (per lane; W + w = not in this window), hold until W
        // ends: the allows of W are then found by integer compares, and [T0, T1) after a
        // change is a table read instead of one lone wave's fp64 chain (the reference's
        // arithmetic is only evaluated where the table is built, each entry verified there
        // by the exact predicate, :158-180).
        int64_t thr_w = INT64_MIN, thr_c = 0;           // table for window thr_w, counts thr_c + lane
        int64_t w_cache = INT64_MIN / 2;                 // the window of the last chunk detailed
        int64_t thr1 = 0, thr2 = 0;
        auto thr_build = [&](int64_t W, int64_t C) {     // (W, C wave-uniform; state sa, sb, sc)
            const uint64_t c_b = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
            const int64_t w = L.window_ms;
            // the state after C - (its count in W) allows inside W: every lane's own count
            SW2 s1 = sw_unpack(sa, sb, sc);
            const int64_t cnt = C + (int64_t)lane;
            if (s1.b1_start != W) {                      // roll into W (as sw_commit_allows)
                if (s1.b1_start == W - w) { s1.b0_cnt = s1.b1_cnt; s1.b0_off = s1.b1_off; }
                else { s1.b0_cnt = 0; s1.b0_off = 0; }
                s1.b1_start = W;
                s1.b1_off = 0;                           // (alive through W whatever it is)
            }
            s1.b1_cnt = (uint32_t)cnt;
            const uint64_t la = (uint64_t)s1.b1_start;
            const uint64_t lb = (uint64_t)s1.b1_cnt | ((uint64_t)s1.b0_cnt << 32);
            const uint64_t lc = (uint64_t)(uint32_t)s1.b1_off | ((uint64_t)(uint32_t)s1.b0_off << 32);
            const int64_t end = W + w;
            auto first = [&](int64_t q) {                // first t in [W, W + w) allowing q
                auto pred = [&](int64_t t) { return hot_pred_k<kAlgoSW>(L, t, la, lb, lc, q); };
                int64_t g = hot_tk_guess<kAlgoSW>(L, W, la, lb, lc, q);
                g = g < W ? W : g > end ? end : g;
                // the guess is exact but at rounding edges: verify, step, else bisect
                for (int it = 0; it < 2; ++it) {
                    if (g > W && pred(g - 1)) --g;
                    else if (g < end && !pred(g)) ++g;
                    else return g;
                }
                if ((g == W || !pred(g - 1)) && (g == end || pred(g))) return g;
                ++n_bisect;
                int64_t l = W, h = end;                  // pred false below l... true at h
                while (l < h) {
                    const int64_t m = l + (h - l) / 2;
                    if (pred(m)) h = m; else l = m + 1;
                }
                return l;
            };
            thr1 = cnt + 1 <= L.max_permits ? first(1) : end;
            thr2 = cnt + 2 <= L.max_permits ? first(2) : end;
            thr_w = W;
            thr_c = C;
            if (a.dbg) cyc_build += __builtin_amdgcn_s_memtime() - c_b;
        };
        // [T0, T1) for the current state from the table, when it covers it
        auto t1_table = [&](int64_t t0, int64_t& t1) {
            if constexpr (A != kAlgoSW) return false;
            const SW2 s0 = sw_unpack(sa, sb, sc);
            const int64_t W = s0.b1_start, w = L.window_ms;
            if (W != thr_w || t0 < W || t0 >= W + w) return false;
            const int64_t k = (int64_t)s0.b1_cnt - thr_c;
            if (k < 0 || k > 63) return false;
            const int64_t T = (int64_t)readlane64((uint64_t)thr1, (uint32_t)k);
            t1 = T > hi + 1 ? hi + 1 : T;
            if (t1 < t0) t1 = t0;
            return true;
        };
        // The hot records of one chunk (lane = arrival order inside the chunk). The next chunk
        // the walk details is prefetched (found from the group summaries once [T0, T1) is
        // known), so its records are in flight while this chunk's results are stored.
        Rec pre = recs[min(f.start + lane, f.end - 1)];
        uint32_t pre_c = 0;
        // mn_l / mx_l / ns_l: this lane's chunk summary in the walked group; todo_after: the
        // group's chunks still to walk after this one
        auto detail = [&](uint32_t c, int64_t mn_l, int64_t mx_l, uint32_t ns_l, uint64_t todo_after) {
            ++n_detail;
            const uint64_t c_det = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
            const uint32_t j = f.start + c * kHotChunk + lane;
            const bool valid = j < f.end;
            const bool use_pre = pre_c == c;
            n_prehit += use_pre ? 1u : 0u;
            const Rec r = use_pre ? pre : recs[valid ? j : f.start];
            const Req q = Codec::dec(r, base);
            const bool hot = is_key(q, valid);
            bool oa = false;
            int64_t orem = 0;
            double tk = __builtin_nan("");
            bool pend = hot;
            if (A == kAlgoTB && hot && q.op == (uint32_t)kOpAcquire && (int64_t)q.permits > L.max_permits) {
                orem = kRemUnknown;                       // :110-116, no state access
                pend = false;
            }
            // the pending prefix inside [T0, T1): denied, remaining 0
            auto fast_prefix = [&]() {
                const bool fast = q.op == (uint32_t)kOpAcquire && q.now_ms >= T0 && q.now_ms < T1;
                const uint64_t m = __ballot(pend && !fast);
                const uint32_t first = m ? (uint32_t)__builtin_ctzll(m) : 64u;
                if (pend && lane < first) {
                    orem = 0;
                    if (TOK && A == kAlgoTB) tk = tb_refill(L, q.now_ms, sa, sb, sc);
                    pend = false;
                }
            };
            fast_prefix();
            bool changed = false;
            bool t_fresh = false;                         // [T0, T1) is for the current state
            const uint64_t c_run = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
            if (a.dbg) cyc_pre += c_run - c_det;
            if constexpr (A == kAlgoTB) {
                // token bucket: rounds; each applies the prefix up to the first state change
                // (every earlier pending request is denied and leaves the state alone, Lua
                // :61-67), so a chunk costs 1 + its allows (the balance is a sequential fp64
                // recurrence, Lua :56-63)
                if (std::is_same<Codec, CodecC>::value && !__any(pend && q.op != (uint32_t)kOpAcquire)) {
                    // acquires only (the common case): tb_step in straight-line code. The
                    // request time as a double is base + now_rel, exact (integers below 2^53),
                    // so elapsed = now - last_refill is one exact subtraction of doubles
                    // (Lua :56), the same value as the integer difference converted
                    const double td = (double)base + (double)(q.now_ms - base);
                    const double pd = (double)q.permits;
                    const double cap = L.capacity, rate = L.rate_per_ms, ttld = (double)L.ttl_ms;
                    while (__any(pend)) {
                        const double tok = __longlong_as_double((long long)sa);
                        const double lastd = (double)(int64_t)sb;
                        const bool ex = (sc & 1u) != 0;
                        const double x = tok + (td - lastd) * rate;          // Lua :57-58
                        const double rf = (!ex || td > lastd + ttld) ? cap : (x < cap ? x : cap);
                        const bool ok = rf >= pd;                              // Lua :61
                        const double nt = ok ? rf - pd : rf;
                        const uint64_t mut = __ballot(pend && ok);
                        const uint32_t fm = mut ? (uint32_t)__builtin_ctzll(mut) : 64u;
                        if (pend && lane <= fm) {
                            oa = ok;
                            orem = d2l(nt);                                   // {allowed, tokens}
                            tk = nt;
                            n_allowed += ok ? 1u : 0u;
                            pend = false;
                        }
                        if (fm < 64u) {                                        // persist (:62-64)
                            // (the lanes after it: the next round, ~20 instructions, decides
                            // them; [T0, T1) is derived once the chunk is done)
                            sa = readlane64((uint64_t)__double_as_longlong(nt), fm);
                            sb = readlane64((uint64_t)q.now_ms, fm);
                            sc = 1;
                            changed = true;
                        }
                    }
                }
                while (__any(pend)) {
                    Outcome o{};
                    if (pend) o = tb_step(L, q.op, q.permits, q.now_ms, sa, sb, sc);
                    const uint64_t mut = __ballot(pend && o.mutate);
                    const uint32_t fm = mut ? (uint32_t)__builtin_ctzll(mut) : 64u;
                    if (pend && lane <= fm) {
                        oa = o.allowed;
                        orem = o.remaining;
                        tk = o.tokens;
                        n_allowed += o.allowed ? 1u : 0u;
                        pend = false;
                    }
                    if (fm < 64u) {                        // fm is wave-uniform: read lanes
                        sa = readlane64(o.a, fm);
                        sb = readlane64(o.b, fm);
                        sc = readlane64(o.c, fm);
                        changed = true;
                        t_fresh = false;
                        // the later requests inside the new state's [T0, T1) are denied
                        // with remaining 0 by time alone (a key at its limit: the balance
                        // stays below 1 for a while after an allow), not by another round
                        if (__any(pend)) {
                            T0 = hot_t0<A>(lo, hi, sa, sb, sc);
                            T1 = t1_of(T0);
                            t_fresh = true;
                            ++n_tk;
                            fast_prefix();
                        }
                    }
                }
            } else {
                // sliding window: inside one window W the acquires only INCR the current
                // bucket (:114-116), so with k allows before it an acquire of p permits at t
                // is allowed iff t >= T_p(C0 + k) (C0: the bucket's count before the chunk;
                // the estimate is non-increasing in t inside W). The allows follow by a greedy
                // scan: the k-th is the first request after the (k-1)-th at or past its
                // threshold. Thresholds come from the window's table (p <= 2) or, per request,
                // from the largest allowed k (K) by the closed form corrected by the exact
                // predicate. Requests the scan cannot take (another window, before the newest
                // bucket, near the epoch, a peek or a reset) run the exact step alone.
                const int64_t w = L.window_ms, mx = L.max_permits;
                while (__any(pend)) {
                    const uint64_t c_it = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
                    const uint32_t f0 = (uint32_t)__builtin_ctzll(__ballot(pend));
                    const int64_t t_f = (int64_t)readlane64((uint64_t)q.now_ms, f0);
                    // t_f's window: the last one seen, or one division
                    if (!(t_f >= w_cache && t_f - w_cache < w)) {
                        int64_t rr;
                        w_cache = jdiv(t_f, w, L.inv_window, &rr) * w;
                    }
                    const int64_t W0 = w_cache;
                    // (window membership by compares: no per-request division)
                    const bool in_w = q.now_ms >= W0 && q.now_ms - W0 < w;
                    const bool scan = pend && q.op == (uint32_t)kOpAcquire && in_w &&
                                      (int64_t)sa <= W0 && t_f >= w;
                    const uint64_t und = __ballot(pend && !scan);
                    const uint32_t stop = und ? (uint32_t)__builtin_ctzll(und) : 64u;
                    const bool in = scan && lane < stop;
                    if (__any(in)) {
                        const SW2 s0 = sw_unpack(sa, sb, sc);
                        const int64_t C0 = s0.b1_start == W0 ? (int64_t)s0.b1_cnt : 0;
                        const bool small = !__any(in && q.permits > 2);
                        if (small && (thr_w != W0 || C0 < thr_c || C0 - thr_c > 63)) {
                            thr_build(W0, C0);
                            ++n_tk;
                        }
                        int64_t kk = 0, na = 0;
                        bool al = false;
                        uint32_t cur = 0, last = 0;
                        const uint64_t c_g = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
                        if (a.dbg) cyc_sw[0] += c_g - c_it;
                        const uint64_t inm = __ballot(in);
                        if (small) {
                            // greedy scan on the table: the na-th allow is the first request
                            // at or past T_p(C0 + na); rebuilt when the window fills it. (One
                            // step per allow, thresholds by readlane: a chain's allows are
                            // mostly one per chunk, where allow runs through per-lane table
                            // reads measured slower.)
                            for (;;) {
                                if (C0 + na - thr_c > 63) {     // (wave-uniform) table exhausted
                                    thr_build(W0, C0 + na);
                                    ++n_tk;
                                }
                                ++n_sw_it;
                                const uint32_t ix = (uint32_t)(C0 + na - thr_c);
                                const int64_t u1 = (int64_t)readlane64((uint64_t)thr1, ix);
                                const int64_t u2 = (int64_t)readlane64((uint64_t)thr2, ix);
                                const bool cnd = in && lane >= cur;
                                const uint64_t m = __ballot(cnd && q.now_ms >= (q.permits == 1 ? u1 : u2));
                                if (cnd) kk = na;
                                if (!m) break;
                                const uint32_t fa = (uint32_t)__builtin_ctzll(m);
                                if (lane == fa) al = true;
                                last = fa;
                                ++na;
                                cur = fa + 1;
                            }
                            const uint64_t c_r = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
                            if (a.dbg) cyc_sw[1] += c_r - c_g;
                            // remaining after the request: max - est(C0 + kk (+1)) = the number
                            // of q <= 2 with T_q at or before t; 2 or more: the exact estimate
                            const int64_t cc = C0 + kk + (al ? 1 : 0);
                            const int64_t ixl = cc - thr_c;
                            const bool tab = ixl >= 0 && ixl <= 63;
                            const int src = (int)(tab ? ixl : 0);
                            const int64_t v1 = (int64_t)(((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uint64_t)thr1 >> 32), src, 64) << 32) |
                                                         (uint32_t)__shfl((int)(uint32_t)thr1, src, 64));
                            const int64_t v2 = (int64_t)(((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uint64_t)thr2 >> 32), src, 64) << 32) |
                                                         (uint32_t)__shfl((int)(uint32_t)thr2, src, 64));
                            if (in) {
                                int64_t rem;
                                if (tab && q.now_ms < v1) rem = 0;
                                else if (tab && q.now_ms < v2) rem = 1;
                                else {
                                    const double t = sw_prev_weighted(q.now_ms, sa, sb, sc, w, L.inv_window);
                                    const int64_t e = d2l(t + (double)cc);
                                    rem = mx - e > 0 ? mx - e : 0;
                                }
                                oa = al;
                                orem = rem;
                                n_allowed += al ? 1u : 0u;
                                pend = false;
                            }
                            if (a.dbg) cyc_sw[2] += __builtin_amdgcn_s_memtime() - c_r;
                        } else {
                            const double tv = in ? sw_prev_weighted(q.now_ms, sa, sb, sc, w, L.inv_window)
                                                 : 0.0;                                // :174, rounded
                            auto est = [&](int64_t k) { return d2l(tv + (double)(C0 + k)); };
                            int64_t K = -1;
                            if (in) {
                                K = mx - (int64_t)q.permits - C0 - (int64_t)tv;      // ~ largest k
                                if (K >= 0 && est(K) + q.permits > mx) --K;         // rounding edges
                                if (K >= 0 && est(K) + q.permits > mx) --K;
                                if (est(K + 1) + q.permits <= mx) ++K;
                                if (K < -1) K = -1;
                            }
                            {                             // the greedy scan as a fixpoint (wave_apply)
                                bool x = in && K >= (int64_t)popc_below(inm);
                                for (;;) {
                                    ++n_sw_it;
                                    kk = (int64_t)popc_below(__ballot(x) & inm);
                                    const bool nx = in && K >= kk;
                                    if (!__any(nx != x)) break;
                                    x = nx;
                                }
                                al = x;
                                const uint64_t am = __ballot(al);
                                na = (int64_t)__popcll(am);
                                if (am) last = 63u - (uint32_t)__builtin_clzll(am);
                            }
                            if (in) {
                                const int64_t e = est(al ? kk + 1 : kk);             // after the request
                                oa = al;
                                orem = mx - e > 0 ? mx - e : 0;
                                n_allowed += al ? 1u : 0u;
                                pend = false;
                            }
                        }
                        const uint64_t c_c = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
                        if (na > 0) {
                            const int64_t t_last = (int64_t)readlane64((uint64_t)q.now_ms, last);
                            SWGeo gl{};
                            gl.curr_start = W0;
                            sw_commit_allows(L, gl, sa, sb, sc, (uint32_t)na, t_last);
                            changed = true;
                        }
                        if (a.dbg) cyc_sw[3] += __builtin_amdgcn_s_memtime() - c_c;
                    }
                    if (stop < 64u) {
                        // the exact step of request `stop` alone (wave-uniform arithmetic)
                        const uint32_t op_s = (uint32_t)__builtin_amdgcn_readlane((int)q.op, (int)stop);
                        const int32_t p_s = __builtin_amdgcn_readlane(q.permits, (int)stop);
                        const int64_t t_s = (int64_t)readlane64((uint64_t)q.now_ms, stop);
                        const Outcome o = sw_step_g(L, op_s, p_s, t_s, sw_geo(t_s, L), sa, sb, sc);
                        if (lane == stop) {
                            oa = o.allowed;
                            orem = o.remaining;
                            n_allowed += o.allowed ? 1u : 0u;
                            pend = false;
                        }
                        if (o.mutate) {
                            sa = o.a; sb = o.b; sc = o.c;
                            changed = true;
                            thr_w = INT64_MIN;               // P may have changed: rebuild
                        }
                    }
                }
            }
            if (changed) {
                wave_fence();
                if (lane == 0) { S.sa[hs] = sa; S.sb[hs] = sb; S.sc[hs] = sc; }
                wave_fence();
                ++n_changed;
            }
            // [T0, T1) for the next chunks, after every change (measured: leaving it empty
            // through runs of changing chunks read the chunk after each of them needlessly)
            const uint64_t c_srch = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
            if (t_fresh) {
                // computed after the last change
            } else if (changed) {
                T0 = hot_t0<A>(lo, hi, sa, sb, sc);
                if (!t1_table(T0, T1)) T1 = t1_of(T0);
                ++n_tk;
            } else if (T1 < hi && __any(hot && q.op == (uint32_t)kOpAcquire && q.now_ms >= T1)) {
                // no change although requests lay past T1: T1 was only a lower bound of the
                // first allowed time (the guess undershot); without this the chunks up to
                // the real one would all be read and decided one by one. Exact, from T0.
                T1 = wave_first_true(T0, hi, lane,
                                     [&](int64_t t) { return hot_pred_k<A>(L, t, sa, sb, sc, 1); });
                ++n_tk;
            }
            // the next chunk the walk will detail: the first one left in the group that the
            // new [T0, T1) does not decide (else the next chunk); its loads go out now
            {
                const bool skip_l = ns_l == 0 && mn_l >= T0 && mx_l < T1;
                const uint64_t nx = todo_after & ~__ballot(skip_l);
                pre_c = nx ? (c & ~63u) + (uint32_t)__builtin_ctzll(nx) : c + 1;
                pre = recs[min(f.start + pre_c * kHotChunk + lane, f.end - 1)];
            }
            if (a.dbg) {
                const uint64_t c_end = __builtin_amdgcn_s_memtime();
                cyc_run += c_srch - c_run;
                cyc_search += c_end - c_srch;
            }
            if (hot && !(a.ablate & kAblNoChainStores)) {
                put_res<Res>(a, j, oa, orem);
                if (TOK) a.tok[j] = tk;
            }
            if (a.dbg) cyc_detail += __builtin_amdgcn_s_memtime() - c_det;
        };
        // level 1: the chunks of one group of 64
        auto walk_group = [&](uint32_t grp) {
            const uint32_t c = grp * 64 + lane;
            const bool has = c < f.n_chunks;
            uint64_t* sm = summ_at(c) + ow;
            const ulonglong2 v01 = *(const ulonglong2*)sm;
            const uint64_t v2 = sm[2];
            int64_t mn = INT64_MAX, mx = INT64_MIN;
            uint32_t ns = 0, ne = 0, nh = 0;
            if (has) {
                mn = (int64_t)v01.x;
                mx = (int64_t)v01.y;
                const uint32_t w = (uint32_t)v2;
                ns = w & 0xFFu;
                nh = (w >> 8) & 0xFFu;
                ne = (w >> 16) & 0xFFu;
                any_hot |= nh != 0;
            }
            uint64_t todo = __ballot(has && nh != 0);
            while (todo) {
                const bool skip = ns == 0 && mn >= T0 && mx < T1;
                const uint64_t nsk = todo & ~__ballot(skip);
                const uint32_t fst = nsk ? (uint32_t)__builtin_ctzll(nsk) : 64u;
                if (((todo >> lane) & 1u) && lane < fst) {  // decided: the key's state is constant here
                    sm[0] = sa; sm[1] = sb; sm[2] = sc;
                    sm[3] = (((v2 >> 24) & 0xFFu) << 8) | (ne ? 3u : 1u);
                }
                if (fst == 64u) break;
                todo &= fst == 63u ? 0ULL : ~((2ULL << fst) - 1);
                if (a.dbg) {
                    const int64_t fmn = (int64_t)readlane64((uint64_t)mn, fst);
                    const int64_t fmx = (int64_t)readlane64((uint64_t)mx, fst);
                    n_fb += fmn < T0 ? 1u : 0u;
                    n_late += fmx >= T1 ? 1u : 0u;
                }
                detail(grp * 64 + fst, mn, mx, ns, todo);
            }
        };
        // ---- Allow walk. A key at its limit is allowed about once per refill interval (TB) or
        // per decay step of its estimate (SW); detailing the chunk of every such allow cost a
        // lone wave ~3.6K cycles (mixed_tenants: ~6000 allows per key and batch). The walk
        // finds each next allow from the key's state alone: the first ms t >= ts at which the
        // key's first plain acquire asking for at most q(t) permits exists — q(t) being what
        // the state grants at t (TB: the refilled balance, Lua :56-61, one lane per ms; SW: the
        // window's allow-time table, :104) — 64 ms per step with k_hot_summ's per-ms table (the
        // first acquire of 1 and of at most 2 permits) in registers. Chunks are decided by verdicts k_hot_fill applies: every record
        // of the key denied under the chunk's state but up to 4 allowed (offsets), the records
        // after each under the state it leaves; chunks (or whole groups) whose acquires all
        // precede the first ms the state grants take the chains' remaining-0 verdict. The
        // verdicts of the cursor's block of 64 chunks are kept in registers and stored when the
        // cursor leaves it. A chunk holding a peek / reset, a fifth allow, or an allow after which
        // the next request of the same ms could be allowed too (a burst) is detailed as before.
        // Needs the key's plain acquires in time order with at most 2 permits (k_hot_summ's group
        // flags); tools/walk_model.py is a CPU model of this loop.
        auto walk = [&]() -> bool {
            if (!walk_table_on(a, i, f, L, lo, hi)) return false;
            if constexpr (A == kAlgoSW) {
                if (lo < L.window_ms) return false;           // near the epoch (:170-172)
                if ((int64_t)sa > lo) return false;           // the state is newer than the batch
            }
            auto up64 = [&](int64_t v, uint32_t o) { return shfl64(v, lane >= o ? (int)(lane - o) : (int)lane); };
            {   // eligibility over the key's groups; any_hot as the group walk sets it
                int64_t carry = INT64_MIN;
                for (uint32_t g0 = 0; g0 < f.n_groups; g0 += 64) {
                    const uint32_t g = g0 + lane;
                    const bool has = g < f.n_groups;
                    const uint64_t* sg = grp_at(g) + ow;
                    const int64_t mn = has ? (int64_t)sg[0] : INT64_MAX;
                    const int64_t mx = has ? (int64_t)sg[1] : INT64_MIN;
                    const uint32_t w2 = has ? (uint32_t)sg[2] : 0u;
                    any_hot |= ((w2 >> 8) & 0xFFu) != 0;
                    if (__any((w2 >> 24) & 3u)) return false;
                    int64_t pmx = mx;                         // max over the groups up to mine
                    for (uint32_t o = 1; o < 64; o <<= 1) {
                        const int64_t y = up64(pmx, o);
                        if (lane >= o && y > pmx) pmx = y;
                    }
                    int64_t before = up64(pmx, 1);
                    if (lane == 0) before = INT64_MIN;
                    if (carry > before) before = carry;
                    if (__any(mn != INT64_MAX && mn < before)) return false;
                    const int64_t top = (int64_t)readlane64((uint64_t)pmx, 63);
                    if (top > carry) carry = top;
                }
            }
            const uint32_t span = (uint32_t)(hi - lo) + 1u;
            const uint2* wt = a.walk_tab + (size_t)(2 * i + kk) * walk_stride(lo, hi);
            auto tab = [&](int64_t t) { return wt[min((uint32_t)(t - lo), span - 1u)]; };
            // the table window: lane l holds ms wb + l (A), wb + 64 + l (B), wb + 128 + l (C, in flight)
            int64_t wb = lo;
            uint2 tA = tab(wb + lane), tB = tab(wb + 64 + lane), tC = tab(wb + 128 + lane);
            // group window: lane l holds group gwb + l's summary (max plain time, flags, rest word)
            uint32_t gwb = kNone, g_w2 = 0;
            int64_t g_mx = INT64_MIN;
            uint64_t g_w3 = 0;
            auto gwin = [&](uint32_t g) {
                if ((g & ~63u) == gwb) return;
                gwb = g & ~63u;
                const bool has = gwb + lane < f.n_groups;
                const uint64_t* sg = grp_at(has ? gwb + lane : 0u) + ow;
                g_mx = has ? (int64_t)sg[1] : INT64_MIN;
                g_w2 = has ? (uint32_t)sg[2] : 0u;
                g_w3 = has ? sg[3] : 0ULL;
            };
            // the register block: lane l holds chunk cb + l's summary and its pending verdict
            // (vF: word 3's flags in bits 0-7, the allows' offsets from bit 8 on, 6 bits each)
            uint32_t cb = kNone, b_w2 = 0, vF = 0;
            int64_t b_mx = INT64_MIN;
            uint64_t vA = 0, vB = 0, vC = 0;
            auto flush = [&]() {
                const uint32_t c = cb + lane;
                if (cb != kNone && vF != 0 && c < f.n_chunks && ((b_w2 >> 8) & 0xFFu)) {
                    uint64_t* sm = summ_at(c) + ow;
                    sm[0] = vA; sm[1] = vB; sm[2] = vC;
                    sm[3] = (uint64_t)(vF & 0xFFu) | ((uint64_t)((b_w2 >> 24) & 0xFFu) << 8) |
                            ((uint64_t)(vF >> 8) << 16);
                }
            };
            // (the block after it is loaded on entry, so that it is in registers when the
            // cursor gets there)
            uint32_t nb = kNone, n_w2 = 0;
            int64_t n_mx = INT64_MIN;
            auto load_blk = [&](uint32_t b, uint32_t& w2, int64_t& mx) {
                const uint32_t c = b + lane;
                const bool has = c < f.n_chunks;
                const uint64_t* sm = summ_at(has ? c : 0u) + ow;
                w2 = has ? (uint32_t)sm[2] : 0u;
                mx = has ? (int64_t)sm[1] : INT64_MIN;
            };
            auto enter = [&](uint32_t b) {
                if (b == cb) return;
                flush();
                cb = b;
                if (b == nb) { b_w2 = n_w2; b_mx = n_mx; }
                else { load_blk(b, b_w2, b_mx); ++n_enter; }
                vF = 0;
                nb = b + 64;
                load_blk(nb, n_w2, n_mx);
            };
            auto cinfo = [&](uint32_t c, uint32_t& w2, int64_t& mxc) {
                enter(c & ~63u);
                w2 = (uint32_t)__builtin_amdgcn_readlane((int)b_w2, (int)(c - cb));
                mxc = (int64_t)readlane64((uint64_t)b_mx, c - cb);
            };
            // the verdict of a denied chunk of the register block (this lane's): remaining 0 when
            // its acquires all precede q1
            auto deny_fl = [&](int64_t q1) {
                return b_mx < q1 ? 1u | (((b_w2 >> 16) & 0xFFu) ? 2u : 0u) : 5u;
            };
            // chunks [c0, c1) denied under (x0, x1, x2): whole groups outside the register block
            // whose acquires all precede q1 take group verdicts, 64 groups per store
            auto deny = [&](uint32_t c0, uint32_t c1, uint64_t x0, uint64_t x1, uint64_t x2, int64_t q1) {
                while (c0 < c1) {
                    const uint32_t b = c0 & ~63u;
                    if (c0 == b && c1 >= b + 64 && b != cb) {
                        const uint32_t G0 = b / 64, G1 = min(c1 / 64, (b & ~4095u) / 64 + 64);
                        gwin(G0);
                        const uint32_t g = gwb + lane;
                        const bool in = g >= G0 && g < G1;
                        const uint64_t bad = __ballot(in && !(g_mx < q1 && !(g_w2 & 0xFFu) && g * 64 != cb));
                        const uint32_t stop = bad ? gwb + (uint32_t)__builtin_ctzll(bad) : G1;
                        if (in && g < stop && ((g_w2 >> 8) & 0xFFu)) {
                            uint64_t* sg = grp_at(g) + ow;
                            sg[0] = x0; sg[1] = x1; sg[2] = x2;
                            sg[3] = (g_w3 & 0xFF00u) | (((g_w2 >> 16) & 0xFFu) ? 3u : 1u);
                        }
                        if (stop > G0) { c0 = stop * 64; continue; }
                    }
                    const uint32_t e = min(c1, b + 64);
                    enter(b);
                    const uint32_t c = cb + lane;
                    const uint32_t fl = deny_fl(q1);
                    if (c >= c0 && c < e) { vA = x0; vB = x1; vC = x2; vF = fl; }
                    c0 = e;
                }
            };
            // the first chunk >= from holding a peek / reset of the key (group flags first)
            auto first_special = [&](uint32_t from) -> uint32_t {
                for (uint32_t G = from / 64; G < f.n_groups;) {
                    gwin(G);
                    const uint32_t g = gwb + lane;
                    const uint64_t m = __ballot(g >= G && g < f.n_groups && (g_w2 & 0xFFu));
                    if (!m) { G = gwb + 64; continue; }
                    const uint32_t gs = gwb + (uint32_t)__builtin_ctzll(m);
                    const uint32_t c = gs * 64 + lane;
                    const uint64_t* sm = summ_at(c < f.n_chunks ? c : 0u) + ow;
                    const uint32_t w2 = c < f.n_chunks ? (uint32_t)sm[2] : 0u;
                    const uint64_t mm = __ballot(c >= from && (w2 & 0xFFu));
                    if (mm) return gs * 64 + (uint32_t)__builtin_ctzll(mm);
                    G = gs + 1;
                }
                return kNone;
            };
            auto allowed1 = [&](int64_t t) { return hot_pred_k<A>(L, t, sa, sb, sc, 1); };
            uint32_t cc = 0;                                  // cursor: chunks before it are decided
            uint64_t ka = sa, kb = sb, kc = sc;               // the state at cc's start
            uint32_t pc = 0, pofs = 0;                        // cc's walked allows: count, offsets
            int64_t ts = lo;                                  // the next allow is at ms >= ts
            bool must = false;                                // cc must be detailed (see detail_at)
            // the latest ms of the key's plain acquires in the chunks detail_at has passed
            // (the boundary ms whose later acquires the table cannot show; INT64_MIN: none)
            int64_t mlast = INT64_MIN;
            int64_t W = 0;                                    // SW: the window of the thresholds in use
            if constexpr (A == kAlgoSW) {
                int64_t rr;
                W = uni(jdiv(ts, L.window_ms, L.inv_window, &rr) * L.window_ms);
            }
            // A bound no correct walk reaches (every step moves the cursor chunk or ts forward):
            // past it the walk stops and flags the batch (RL_E_CAPACITY) instead of spinning.
            uint32_t guard = 4u * (span + f.n_chunks) + 4096u;
            auto spin = [&]() {
                if (guard != 0) --guard;
                return guard == 0;
            };
            // The latest ms of the key's plain acquires in the chunks before c (INT64_MIN: none),
            // from the records themselves (the summaries of decided chunks hold verdicts by
            // now). Plain acquires are in time order (k_hot_summ's flags), so it is the last
            // one found going back. Only after a chunk whose key records are specials alone.
            auto plain_before = [&](uint32_t c) -> int64_t {
                for (uint32_t k = c; k-- > 0;) {
                    const uint32_t j = f.start + k * kHotChunk + lane;
                    const bool valid = j < f.end;
                    const Req q = Codec::dec(recs[valid ? j : f.start], base);
                    const bool plain = is_key(q, valid) && q.op == (uint32_t)kOpAcquire &&
                                       !(A == kAlgoTB && (int64_t)q.permits > L.max_permits);
                    const uint64_t m = __ballot(plain);
                    if (m) return uni((int64_t)readlane64((uint64_t)q.now_ms, 63u - (uint32_t)__builtin_clzll(m)));
                }
                return INT64_MIN;
            };
            // a chunk detailed from the current state (the group walk's path), then the cursor past it
            auto detail_at = [&](uint32_t c) {
                T0 = hot_t0<A>(lo, hi, sa, sb, sc);
                if (!t1_table(T0, T1)) T1 = t1_of(T0);
                detail(c, INT64_MAX, INT64_MIN, 1u, 0ULL);
                sa = uni(sa); sb = uni(sb); sc = uni(sc);
                uint32_t w2;
                int64_t mxc;
                cinfo(c, w2, mxc);
                cc = c + 1; ka = sa; kb = sb; kc = sc; pc = 0; pofs = 0;
                const bool special = (w2 & 0xFFu) != 0u;
                // the boundary: this chunk's last plain acquire, else (specials only) the last
                // one before it; a chunk without the key's records (reached as a `must` chunk
                // right after the boundary's own) leaves it as it is
                if (mxc != INT64_MIN) mlast = mxc;
                else if (special) mlast = plain_before(c);
                mlast = uni(mlast);
                if (special) {
                    // a reset may grant acquires the old state denied: the search starts again
                    // right after the boundary (every later plain acquire is at or after it)
                    ts = mlast == INT64_MIN ? lo : mlast + 1;
                } else if (mlast != INT64_MIN && mlast + 1 > ts) {
                    ts = mlast + 1;
                }
                // the next chunks' acquires in the boundary ms come after every table entry of
                // that ms: while the state grants there, the next chunk is detailed too
                must = mlast != INT64_MIN && uni((uint32_t)allowed1(mlast)) != 0u;
            };
            // back to the cursor chunk's start state, to detail it (the detail counts its
            // walked allows again)
            auto undo_cursor = [&]() {
                if (lane == 0) n_allowed -= pc;
                sa = ka; sb = kb; sc = kc;
            };
            // (every chunk to detail goes through one call site: `detail` is inlined, and a
            // copy per call site made the kernel's code several times larger)
            uint32_t dc = kNone;
            uint32_t spn = first_special(1);                  // the next special after the cursor
            const uint64_t c_w0 = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
            for (;;) {
                // (the loop-carried scalars re-declared uniform: a value the compiler cannot
                // prove uniform turns every branch on it into an exec-mask region)
                dc = uni(dc); cc = uni(cc); pc = uni(pc); pofs = uni(pofs); ts = uni(ts);
                wb = uni(wb); guard = uni(guard); spn = uni(spn); cb = uni(cb); nb = uni(nb);
                gwb = uni(gwb); must = uni((uint32_t)must) != 0u;
                ka = uni(ka); kb = uni(kb); kc = uni(kc); sa = uni(sa); sb = uni(sb); sc = uni(sc);
                if constexpr (A == kAlgoSW) W = uni(W);
                if (dc != kNone) { detail_at(dc); dc = kNone; }
                if (cc >= f.n_chunks || spin()) break;
                if (spn <= cc) spn = first_special(cc + 1);   // (kNone is above every chunk)
                // the cursor chunk: detailed when it must be or holds a special
                if (pc == 0) {
                    uint32_t w2;
                    int64_t mxc;
                    cinfo(cc, w2, mxc);
                    if (must || (w2 & 0xFFu)) { must = false; dc = cc; continue; }
                }
                // The common path as a loop of its own (find, verdicts, allow: the cursor chunk
                // always holds a walked allow here), so that the register allocator weighs the
                // values it uses above the rest of the chain's; anything else leaves it.
                bool done = false;
                for (;;) {
                    cc = uni(cc); pc = uni(pc); pofs = uni(pofs); ts = uni(ts); cb = uni(cb);
                    ka = uni(ka); kb = uni(kb); kc = uni(kc); sa = uni(sa); sb = uni(sb); sc = uni(sc);
                    // the next allow: the first ms >= ts with an acquire the state grants; q1: the
                    // first ms >= ts the state grants anything at
                    int64_t tf = INT64_MIN, q1 = INT64_MAX;
                    uint32_t rf = 0, pf = 1;
                    const uint64_t c_f0 = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
                    for (;;) {
                        ++n_find;
                        ts = uni(ts); wb = uni(wb); guard = uni(guard); q1 = uni(q1);
                        if (ts > hi || spin()) break;
                        if (ts < wb || ts >= wb + 192) {              // far ahead (or searched again
                                                                      // after a special): refill the window
                            wb = lo + ((ts - lo) & ~(int64_t)63);
                            tA = tab(wb + lane); tB = tab(wb + 64 + lane); tC = tab(wb + 128 + lane);
                        }
                        while (ts >= wb + 64) {
                            wb += 64; tA = tB; tB = tC; tC = tab(wb + 128 + lane);
                        }
                        int64_t lim_t = hi;                           // SW: the window's end - 1
                        int64_t Q1 = 0, Q2 = 0;                       // SW: the window's thresholds
                        if constexpr (A == kAlgoSW) {
                            const int64_t w = L.window_ms;
                            if (!(ts >= W && ts - W < w)) {
                                int64_t rr;
                                W = uni(jdiv(ts, w, L.inv_window, &rr) * w);
                            }
                            const SW2 s0 = sw_unpack(sa, sb, sc);
                            const int64_t C = s0.b1_start == W ? (int64_t)s0.b1_cnt : 0;
                            if (thr_w != W || C < thr_c || C - thr_c > 63) { thr_build(W, C); ++n_tk; }
                            Q1 = (int64_t)readlane64((uint64_t)thr1, (uint32_t)(C - thr_c));
                            Q2 = (int64_t)readlane64((uint64_t)thr2, (uint32_t)(C - thr_c));
                            if (W + w - 1 < lim_t) lim_t = W + w - 1;
                        }
                        // one 64-ms view: what the state grants per ms (q), the first candidate
                        auto view = [&](int64_t tb, const uint2 e) -> bool {
                            const int64_t t = tb + (int64_t)lane;
                            uint32_t q;
                            if constexpr (A == kAlgoTB) {
                                // tb_refill per lane, its elapsed time as (tb - last) + lane (exact:
                                // integers below 2^53), no contraction (Lua :56-58)
                                const int64_t last = (int64_t)sb;
                                const double el = (double)(tb - last) + (double)lane;
                                const double x = __longlong_as_double((long long)sa) + el * L.rate_per_ms;
                                double bal = x < L.capacity ? x : L.capacity;
                                if (!(sc & 1u) || t > last + L.ttl_ms) bal = L.capacity;
                                q = bal >= 2.0 ? 2u : bal >= 1.0 ? 1u : 0u;
                            } else {
                                q = t >= Q2 ? 2u : t >= Q1 ? 1u : 0u;
                            }
                            if (!(t >= ts && t <= lim_t)) q = 0;
                            const uint64_t mq = __ballot(q != 0);
                            if (mq && q1 == INT64_MAX) q1 = tb + (int64_t)__builtin_ctzll(mq);
                            const uint32_t cnd = q >= 2u ? e.y : q == 1u ? e.x : kWalkNone;
                            const uint64_t m = __ballot(cnd != kWalkNone);
                            if (!m) return false;
                            const uint32_t l = (uint32_t)__builtin_ctzll(m);
                            rf = (uint32_t)__builtin_amdgcn_readlane((int)cnd, (int)l);
                            const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)e.x, (int)l);
                            pf = rf != ex ? 2u : 1u;                  // (q >= 2 and a 2-permit acquire first)
                            tf = tb + (int64_t)l;
                            return true;
                        };
                        if (view(wb, tA) || view(wb + 64, tB)) break;
                        ts = lim_t < wb + 127 ? lim_t + 1 : wb + 128;  // (SW: the next window)
                    }
                    if (a.dbg) cyc_find += __builtin_amdgcn_s_memtime() - c_f0;
                    // (no allow before the batch ends: the rest is denied, up to the next special)
                    const uint32_t cs = tf == INT64_MIN ? f.n_chunks - 1u : rf / kHotChunk;
                    const uint32_t cfl = 13u | ((pc - 1u) << 4) | (pofs << 8);   // cc's verdict, pc > 0
                    const uint64_t c_c0 = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
                    if (spn <= cs || tf == INT64_MIN) {               // a special in (cc, cs] / the end
                        enter(cc & ~63u);
                        const uint32_t fl = pc ? cfl : deny_fl(q1);
                        if (cb + lane == cc) { vA = ka; vB = kb; vC = kc; vF = fl; }
                        const uint32_t e = spn <= cs ? spn : f.n_chunks;
                        deny(cc + 1, e, sa, sb, sc, q1);
                        if (e == f.n_chunks) { done = true; break; }
                        dc = spn;
                        break;
                    }
                    if (cs < cc) {
                        // a table entry in a decided chunk: the search bound (ts above every
                        // plain acquire before the cursor) excludes it, so this is a logic
                        // error; the batch reports RL_E_INTERNAL and the cursor is detailed
                        ++n_internal;
                        if (pc > 0) undo_cursor();
                        dc = cc;
                        break;
                    }
                    if (cs == cc && pc > 0) {                         // another allow in the cursor chunk
                        if (pc == 4) { undo_cursor(); dc = cc; break; }
                    } else if (cs > cc) {
                        const uint32_t fl = pc ? cfl : deny_fl(q1);
                        if (cc >= cb && cs < cb + 64) {               // (the common case: one block)
                            const uint32_t c = cb + lane;
                            const uint32_t dfl = deny_fl(q1);
                            if (c == cc) { vA = ka; vB = kb; vC = kc; vF = fl; }
                            else if (c > cc && c < cs) { vA = sa; vB = sb; vC = sc; vF = dfl; }
                        } else {
                            enter(cc & ~63u);
                            const uint32_t fl2 = pc ? cfl : deny_fl(q1);
                            if (cb + lane == cc) { vA = ka; vB = kb; vC = kc; vF = fl2; }
                            deny(cc + 1, cs, sa, sb, sc, q1);
                        }
                        cc = cs; ka = sa; kb = sb; kc = sc; pc = 0; pofs = 0;
                    }
                    const uint64_t c_a0 = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
                    if (a.dbg) cyc_close += c_a0 - c_c0;
                    pofs |= (rf % kHotChunk) << (6 * pc);
                    ++pc;
                    // the allow (Lua :61-64 / SlidingWindowRateLimiter :114-116) at ms tf
                    bool burst;
                    if constexpr (A == kAlgoTB) {
                        const double nt = uni(tb_refill(L, tf, sa, sb, sc) - (double)pf);
                        sa = (uint64_t)__double_as_longlong(nt);
                        sb = (uint64_t)tf;
                        sc = 1;
                        burst = nt >= 1.0;                            // (elapsed 0: the balance is nt)
                    } else {
                        SWGeo gl{};
                        gl.curr_start = W;
                        sw_commit_allows(L, gl, sa, sb, sc, 1u, tf);
                        sa = uni(sa); sb = uni(sb); sc = uni(sc);
                        // the window's table at the new count, when it holds it
                        const int64_t C = (int64_t)sw_unpack(sa, sb, sc).b1_cnt;
                        if (thr_w == W && C >= thr_c && C - thr_c <= 63)
                            burst = tf >= (int64_t)readlane64((uint64_t)thr1, (uint32_t)(C - thr_c));
                        else
                            burst = allowed1(tf);
                    }
                    if (lane == 0) ++n_allowed;
                    ++n_changed;
                    ++n_walk;
                    ts = tf + 1;
                    if (a.dbg) cyc_allow += __builtin_amdgcn_s_memtime() - c_a0;
                    if (burst) {                                      // the next request of ms tf too: detail
                        undo_cursor();
                        dc = cc;
                        break;
                    }
                }
                if (done) break;
            }
            flush();
            if (guard == 0) ++n_internal;                // the step bound: a walk that would not end
            if (a.dbg) cyc_walk += __builtin_amdgcn_s_memtime() - c_w0;
            wave_fence();
            if (lane == 0) { S.sa[hs] = sa; S.sb[hs] = sb; S.sc[hs] = sc; }
            wave_fence();
            return true;
        };
        if (walk()) {
            if (a.dbg) cyc_pass1 += __builtin_amdgcn_s_memtime() - c_p1;
            return;
        }
        // level 2: 64 groups per test, the next 64 in flight
        ulonglong2 nx01 = *(const ulonglong2*)(grp_at(lane) + ow);
        uint64_t nx2 = grp_at(lane)[ow + 2], nx3 = grp_at(lane)[ow + 3];
        for (uint32_t g0 = 0; g0 < f.n_groups; g0 += 64) {
            const uint32_t g = g0 + lane;
            const bool has = g < f.n_groups;
            uint64_t* sg = grp_at(g) + ow;
            const ulonglong2 v01 = nx01;
            const uint64_t v2 = nx2, v3 = nx3;
            nx01 = *(const ulonglong2*)(grp_at(g + 64) + ow);
            nx2 = grp_at(g + 64)[ow + 2];
            nx3 = grp_at(g + 64)[ow + 3];
            const int64_t mn = (int64_t)v01.x, mx = (int64_t)v01.y;
            const uint32_t w = (uint32_t)v2;
            const bool ns = (w & 0xFFu) != 0, nh = ((w >> 8) & 0xFFu) != 0, ne = ((w >> 16) & 0xFFu) != 0;
            any_hot |= has && nh;
            uint64_t todo = __ballot(has && nh);
            while (todo) {
                const bool skip = !ns && mn >= T0 && mx < T1;
                const uint64_t nsk = todo & ~__ballot(skip);
                const uint32_t fst = nsk ? (uint32_t)__builtin_ctzll(nsk) : 64u;
                if (((todo >> lane) & 1u) && lane < fst) {  // a whole group decided
                    sg[0] = sa; sg[1] = sb; sg[2] = sc;
                    sg[3] = (v3 & 0xFF00u) | (ne ? 3u : 1u);
                }
                if (fst == 64u) break;
                todo &= fst == 63u ? 0ULL : ~((2ULL << fst) - 1);
                walk_group(g0 + fst);
            }
        }
        if (a.dbg) cyc_pass1 += __builtin_amdgcn_s_memtime() - c_p1;
    };
    auto pass2 = [&](auto algo) {
        constexpr int A = decltype(algo)::value;
        const uint64_t c_p2 = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
        uint32_t head = 0, count = 0;                     // LDS ring (wave-uniform)
        SparseSrc sp{nullptr, nullptr, 0, false};         // the whole image is in LDS
        auto apply64 = [&](uint32_t valid_n) {
            const bool v = lane < valid_n;
            const uint32_t ri = (head + (v ? lane : 0u)) % kRing;
            uint32_t n_hits = 0;                          // (no local cache on the hot path)
            const Applied ap = wave_apply<Codec, A, false>(a, S, L, lane, S.ring[ri], v, S.ring_pos[ri], base,
                                                    pad, n_allowed, n_invalid, n_caperr, n_rounds, n_hits, sp);
            if (v && !(a.ablate & kAblNoChainStores)) {
                put_res<Res>(a, ap.j, ap.alw, ap.rem);
                if (TOK) a.tok[ap.j] = ap.tok;
            }
        };
        auto take = [&](const Rec& r, uint32_t j, bool valid) {   // append other keys' records
            const bool other = valid && !is_hot(Codec::dec(r, base), valid);
            const uint64_t bal = __ballot(other);
            if (other) {
                const uint32_t k = (head + count + popc_below(bal)) % kRing;
                S.ring[k] = r;
                S.ring_pos[k] = j;
            }
            count += (uint32_t)__popcll(bal);
            n_other += lane == 0 ? (uint32_t)__popcll(bal) : 0u;
            wave_fence();
            if (count >= 64) {
                apply64(64);
                head = (head + 64) % kRing;
                count -= 64;
            }
        };
        // The chunks holding other keys' records, in arrival order, across groups: a
        // wave-uniform cursor over (block of 64 groups, group, chunk). Four chunks' records
        // are in flight (unrolled, so the prefetch registers rotate without moves): a region
        // whose second key is itself hot runs thousands of chunks through here, and one
        // chunk in flight left each of them waiting on its load (sw_zipf: a 398K-record
        // region ended the region stage 3.5 ms after the normal regions).
        uint32_t cg0 = 0, cgrp = 0;
        uint64_t cgtodo = 0, ctodo = 0;
        bool cdone = f.n_groups == 0;
        auto group_mask = [&](uint32_t g0) {
            const uint32_t g = g0 + lane;
            return __ballot(g < f.n_groups && (!hot_ok || ((grp_at(g)[rest_w] >> 8) & 1u)));
        };
        if (!cdone) cgtodo = group_mask(0);
        auto next_chunk = [&]() -> uint32_t {
            while (!cdone && ctodo == 0) {
                if (cgtodo == 0) {
                    cg0 += 64;
                    if (cg0 >= f.n_groups) { cdone = true; break; }
                    cgtodo = group_mask(cg0);
                    continue;
                }
                cgrp = cg0 + (uint32_t)__builtin_ctzll(cgtodo);
                cgtodo &= cgtodo - 1;
                const uint32_t c = cgrp * 64 + lane;
                uint32_t no = 0;
                if (c < f.n_chunks) no = hot_ok ? (uint32_t)(summ_at(c)[rest_w] >> 8) & 0xFFu : 64u;
                ctodo = __ballot(no != 0);
            }
            if (cdone) return kNone;
            const uint32_t cc = cgrp * 64 + (uint32_t)__builtin_ctzll(ctodo);
            ctodo &= ctodo - 1;
            return cc;
        };
        auto rec_of = [&](uint32_t cc) {
            return recs[cc == kNone ? f.start : min(f.start + cc * kHotChunk + lane, f.end - 1)];
        };
        auto take_chunk = [&](const Rec& r, uint32_t cc) {
            const uint32_t j = f.start + cc * kHotChunk + lane;
            take(r, j, j < f.end);
        };
        uint32_t k0 = next_chunk(), k1 = next_chunk(), k2 = next_chunk(), k3 = next_chunk();
        Rec r0 = rec_of(k0), r1 = rec_of(k1), r2 = rec_of(k2), r3 = rec_of(k3);
        while (k0 != kNone) {
            take_chunk(r0, k0); k0 = next_chunk(); r0 = rec_of(k0);
            if (k1 == kNone) break;
            take_chunk(r1, k1); k1 = next_chunk(); r1 = rec_of(k1);
            if (k2 == kNone) break;
            take_chunk(r2, k2); k2 = next_chunk(); r2 = rec_of(k2);
            if (k3 == kNone) break;
            take_chunk(r3, k3); k3 = next_chunk(); r3 = rec_of(k3);
        }
        if (count > 0) apply64(count);
        if (a.dbg) cyc_pass2 += __builtin_amdgcn_s_memtime() - c_p2;
    };
    if (L.algo == kAlgoTB) {
        if (wv == 0 && hot_ok) pass1(std::integral_constant<int, kAlgoTB>{}, 0u);
        if (wv == 0 && hot_ok2) pass1(std::integral_constant<int, kAlgoTB>{}, 1u);
        if (!SPLIT || wv == 1) pass2(std::integral_constant<int, kAlgoTB>{});
    } else {
        if (wv == 0 && hot_ok) pass1(std::integral_constant<int, kAlgoSW>{}, 0u);
        if (wv == 0 && hot_ok2) pass1(std::integral_constant<int, kAlgoSW>{}, 1u);
        if (!SPLIT || wv == 1) pass2(std::integral_constant<int, kAlgoSW>{});
    }
    for (int off = 32; off > 0; off >>= 1) {
        n_allowed += __shfl_xor(n_allowed, off, 64);
        n_invalid += __shfl_xor(n_invalid, off, 64);
        n_caperr += __shfl_xor(n_caperr, off, 64);
    }
    if (lane == 0) {
        unsigned long long* st = a.stats + (size_t)(blockIdx.x & (kStatSlots - 1)) * kStWords;
        if (n_allowed) atomicAdd(st + kStAllowed, (unsigned long long)n_allowed);
        if (n_invalid) atomicAdd(st + kStInvalid, (unsigned long long)n_invalid);
        if (n_caperr) atomicAdd(st + kStCapErr, (unsigned long long)n_caperr);
        if (n_internal) atomicOr(&a.ctl->internal_err, 1u);
    }
    if (SPLIT) {
        if (wv == 1) {                                // hand over, then leave the SIMD
            if (lane == 0) {
                s_p2[1] = cyc_pass2; s_p2[2] = n_other;
                __atomic_store_n(&s_p2[0], 1ULL, __ATOMIC_RELEASE);
            }
            return;
        }
        while (__atomic_load_n(&s_p2[0], __ATOMIC_ACQUIRE) == 0) __builtin_amdgcn_s_sleep(2);
        cyc_pass2 = s_p2[1];
        n_other = (uint32_t)s_p2[2];
    }
    // ---- write the region back, statistics
    const bool hot_touched = __any(any_hot);
    if (lane == 0 && hot_ok && hot_touched) S.occ[hsl0] |= 2u;
    if (lane == 0 && hot_ok2 && hot_touched) S.occ[hsl1] |= 2u;
    wave_fence();
    uint32_t touched = 0, used = 0;
    for (uint32_t sl = lane; sl < NS; sl += 64) {
        const uint32_t o = S.occ[sl];
        Slot v{0, 0, 0, 0};
        if (o & kOccUsed) v = slot_used(Slot{S.tag[sl], S.sa[sl], S.sb[sl], S.sc[sl]});
        tab[sl] = v;
        touched += (o >> 1) & 1u;
        used += o & kOccUsed;
    }
    for (int off = 32; off > 0; off >>= 1) {
        touched += __shfl_xor(touched, off, 64);
        used += __shfl_xor(used, off, 64);
        n_bisect += __shfl_xor(n_bisect, off, 64);
    }
    if (lane == 0) {
        note_fill(a, region, used, n_caperr != 0);
        unsigned long long* st = a.stats + (size_t)(blockIdx.x & (kStatSlots - 1)) * kStWords;
        atomicAdd(st + kStDistinct, (unsigned long long)touched);
        atomicAdd(st + kStRegions, 1ULL);
        atomicAdd(st + kStTableBytes, (unsigned long long)(2u * NS * 32u));
        if (a.dbg) {
            uint64_t* d = a.dbg + (size_t)region * kDbgWords;
            // top bit: a hot region; bits 0-31: detailed chunks, 32-62: other-key records
            d[0] = t_start; d[1] = __builtin_amdgcn_s_memrealtime(); d[2] = f.end - f.start;
            d[3] = (uint64_t)n_detail | (uint64_t)min(n_tk, 0xFFFFu) << 32 | (uint64_t)min(n_fb, 0x7FFFu) << 48 | (1ULL << 63);
            d[4] = cyc_detail; d[5] = cyc_run; d[6] = cyc_search;
            d[7] = min((uint64_t)n_changed, (uint64_t)0xFFFFFF) | min((uint64_t)n_late, (uint64_t)0xFFFFFF) << 24;
            d[8] = cyc_pre; d[9] = cyc_pass1; d[10] = cyc_pass2; d[11] = n_other; d[12] = n_prehit;
            d[13] = cyc_build; d[14] = n_bisect;
            d[15] = cyc_sw[0]; d[16] = cyc_sw[1]; d[17] = cyc_sw[2]; d[18] = cyc_sw[3]; d[19] = n_sw_it;
            d[20] = n_walk; d[21] = n_find; d[22] = cyc_find; d[23] = cyc_walk;
            d[24] = cyc_close; d[25] = cyc_allow; d[26] = n_enter;
        }
    }
}

// The hot chains alone (single-wave workgroups), launched on a side stream of the device's
// highest priority just before the normal regions' launch, so they start first. They are a
// few hundred lone waves beside ~10^6 normal-region waves: a larger register budget costs
// no occupancy that matters: one wave per SIMD gives the walk's registers room (512 VGPRs,
// no spills).
constexpr int kChainMinWaves = 1;
template <class Codec, class Res, bool TOK, bool SPLIT>
__global__ __launch_bounds__(SPLIT ? 128 : 64, kChainMinWaves) void k_hot_chains(RegionArgs a) {
    __shared__ RegionLds<Codec, true> S;
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    if (SPLIT) {
        // one chain per workgroup: wave 1 leaves after its pass (the grid covers the list)
        if (blockIdx.x < hc) hot_chain<Codec, Res, TOK, true>(a, blockIdx.x, S);
        return;
    }
    for (uint32_t i = blockIdx.x; i < hc; i += gridDim.x) {       // (workgroup-uniform)
        wave_fence();                                             // the last chain's LDS users
        hot_chain<Codec, Res, TOK, false>(a, i, S);
    }
}

// A chunk a chain's allow walk decided (verdict bit 2): the key's records under the state in
// sm[0..2], but the allowed ones (bit 3: bits 4-5 hold their count - 1, bits 16-39 their
// offsets, 6 bits each, ascending) and, after each, the state that allow leaves (TB: Lua
// :56-64; SW: the INCR of :114-116). Every lane runs it (the allowed records' times and
// permits are read from their lanes); `mine`: this lane holds the key's record.
template <class Res, bool TOK>
__device__ inline void walk_fill_key(const RegionArgs& a, const DevLimiter& L, const uint64_t* sm,
                                     uint64_t v, const Req& q, bool mine, uint32_t lane, uint32_t j) {
    const bool tb = L.algo == kAlgoTB;
    uint64_t ya = sm[0], yb = sm[1], yc = sm[2];        // the state after the allows so far
    uint64_t sa = ya, sb = yb, sc = yc;                  // this lane's: after the last allow before it
    bool at = false;
    double nt = 0.0, nt_at = 0.0;
    const uint32_t na = (v & 8u) ? (uint32_t)((v >> 4) & 3u) + 1u : 0u;
#pragma unroll 1
    for (uint32_t k = 0; k < na; ++k) {
        const uint32_t o = (uint32_t)(v >> (16 + 6 * k)) & 63u;
        const int64_t t_o = (int64_t)readlane64((uint64_t)q.now_ms, o);
        const int32_t p_o = __builtin_amdgcn_readlane(q.permits, (int)o);
        if (tb) {
            nt = tb_refill(L, t_o, ya, yb, yc) - (double)p_o;
            ya = (uint64_t)__double_as_longlong(nt); yb = (uint64_t)t_o; yc = 1;
        } else {
            sw_commit_allows(L, sw_geo(t_o, L), ya, yb, yc, 1u, t_o);
        }
        if (lane == o) { at = true; nt_at = nt; }
        if (lane >= o) { sa = ya; sb = yb; sc = yc; }
    }
    if (!mine) return;
    bool alw = false;
    int64_t rem;
    double tk = __builtin_nan("");
    if (tb && (int64_t)q.permits > L.max_permits) {
        rem = kRemUnknown;                                  // :110-116
    } else {
        alw = at;
        if (tb) {
            tk = at ? nt_at : tb_refill(L, q.now_ms, sa, sb, sc);
            rem = d2l(tk);
        } else {
            const int64_t r = L.max_permits - sw_estimate(sw_unpack(sa, sb, sc), sw_geo(q.now_ms, L),
                                                          q.now_ms, L.window_ms);
            rem = r > 0 ? r : 0;
        }
    }
    put_res<Res>(a, j, alw, rem);
    if (TOK) a.tok[j] = tk;
}

// Phase C (one wave per group of 64 chunks, all CUs): results of the chunks the chains
// decided. The group's chunk verdicts come in with one load per lane; a chunk holding only
// the dominant key's records is written without reading them (unless TB balances are out).
// WALK: the chunks of allow walks' verdicts only (bit 2), which the other instance skips —
// their exact per-record arithmetic would otherwise set the register budget of every fill
// wave (80 VGPRs instead of 38).
template <class Codec, class Res, bool TOK, bool WALK>
__global__ __launch_bounds__(256) void k_hot_fill(RegionArgs a) {
    __shared__ uint32_t s_base[kHotMax + 1];
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t total = a.hot_total[1];
    for (uint32_t i = threadIdx.x; i < hc; i += 256) s_base[i] = a.hot_info[i].group_base;
    __syncthreads();
    if (a.ctl->span_overflow != 0) return;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const typename Codec::Rec* recs = (const typename Codec::Rec*)a.rec;
    const int64_t base = a.ctl->base_ms;
    Res* res = (Res*)a.res;
    for (uint32_t gg = blockIdx.x * 4 + wid; gg < total; gg += gridDim.x * 4) {
        const uint32_t i = hot_region_of(s_base, hc, gg);
        const HotInfo f = a.hot_info[i];
        const uint32_t c0 = (gg - s_base[i]) * 64, c1 = min(c0 + 64, f.n_chunks);
        const uint64_t* s2 = a.hot_summ2 + (size_t)gg * 8;
        const uint64_t g0 = s2[3], g1 = s2[7];
        // lane l: chunk c0 + l's verdict words of both keys
        const uint64_t* s1l = a.hot_summ + (size_t)(f.chunk_base + min(c0 + lane, c1 - 1)) * 8;
        const uint64_t cv0 = s1l[3], cv1 = s1l[7];
        const uint64_t any = WALK ? __ballot(c0 + lane < c1 && ((((g0 & 1u) ? 0u : cv0) | ((g1 & 1u) ? 0u : cv1)) & 4u))
                                  : __ballot(c0 + lane < c1 && (((g0 | cv0) & 1u) || ((g1 | cv1) & 1u)));
        if (!any) continue;
        const DevLimiter& L = a.lims[a.region_lim[f.bin]];
        for (uint64_t m = any; m; m &= m - 1) {
            const uint32_t l = (uint32_t)__builtin_ctzll(m);
            const uint32_t c = c0 + l;
            const uint64_t c0w = readlane64(cv0, l), c1w = readlane64(cv1, l);
            // per key k: decided as part of its group (state in the group summary), or alone
            const uint64_t v0 = (g0 & 1u) ? ((g0 & 3u) | (c0w & 0xFF00u)) : c0w;
            const uint64_t v1 = (g1 & 1u) ? (g1 & 3u) : c1w;
            const uint32_t j = f.start + c * kHotChunk + lane;
            if ((v0 | v1) & 4u) {                        // an allow walk's verdict (chunk level)
                if constexpr (!WALK) continue;
                const bool valid = j < f.end;
                const Req q = Codec::dec(recs[valid ? j : f.start], base);
                const uint64_t* s1 = a.hot_summ + (size_t)(f.chunk_base + c) * 8;
                const bool ok = valid && !q.invalid;
                if (v0 & 4u) walk_fill_key<Res, TOK>(a, L, s1, v0, q, ok && q.h == f.tag, lane, j);
                if (v1 & 4u) walk_fill_key<Res, TOK>(a, L, s1 + 4, v1, q, ok && q.h == f.tag2, lane, j);
                // (a key with a plain verdict beside a walked one: as below)
                if (((v0 & 5u) == 1u && q.h == f.tag) || ((v1 & 5u) == 1u && q.h == f.tag2)) {
                    if (ok) {
                        const uint64_t* sm = (q.h == f.tag ? ((g0 & 1u) ? s2 : s1) : ((g1 & 1u) ? s2 : s1) + 4);
                        const bool early = L.algo == kAlgoTB && (int64_t)q.permits > L.max_permits;
                        res[j] = (Res)pack_result(false, early ? kRemUnknown : 0);
                        if (TOK) a.tok[j] = (L.algo == kAlgoTB && !early) ? tb_refill(L, q.now_ms, sm[0], sm[1], sm[2])
                                                                         : __builtin_nan("");
                    }
                }
                continue;
            }
            if constexpr (WALK) continue;
            if (j >= f.end) continue;
            // the decided keys' records here are acquires (n_special == 0); TB permits > max
            // (verdict bit 1) are the only ones not (deny, 0); other records are the chains'
            if (!TOK && (v0 & 1u) && !(v0 & 0xFF02u)) {  // every record is the dominant key's
                res[j] = (Res)pack_result(false, 0);
                continue;
            }
            const Req q = Codec::dec(recs[j], base);
            if (q.invalid) continue;
            const uint64_t* s1 = a.hot_summ + (size_t)(f.chunk_base + c) * 8;
            const uint64_t* sm;
            if ((v0 & 1u) && q.h == f.tag) sm = (g0 & 1u) ? s2 : s1;
            else if ((v1 & 1u) && q.h == f.tag2) sm = ((g1 & 1u) ? s2 : s1) + 4;   // (ok bit 1)
            else continue;                               // another key
            const bool early = L.algo == kAlgoTB && (int64_t)q.permits > L.max_permits;
            res[j] = (Res)pack_result(false, early ? kRemUnknown : 0);
            if (TOK) a.tok[j] = (L.algo == kAlgoTB && !early) ? tb_refill(L, q.now_ms, sm[0], sm[1], sm[2])
                                                             : __builtin_nan("");
        }
    }
}

// The chain launch on the side stream hs: single-wave workgroups looping over the hot list,
// or (chain_split) one two-wave workgroup per possible hot region.
template <class Codec, class Res>
hipError_t hot_chains_t(const RegionArgs& a, hipStream_t hs) {
    if (a.chain_split) {
        const dim3 g(kHotMax);
        if (a.tok) hipLaunchKernelGGL((k_hot_chains<Codec, Res, true, true>), g, dim3(128), 0, hs, a);
        else hipLaunchKernelGGL((k_hot_chains<Codec, Res, false, true>), g, dim3(128), 0, hs, a);
        return hipGetLastError();
    }
    const dim3 g(a.chain_grid ? min(a.chain_grid, kHotMax) : kHotMax);
    if (a.tok) hipLaunchKernelGGL((k_hot_chains<Codec, Res, true, false>), g, dim3(64), 0, hs, a);
    else hipLaunchKernelGGL((k_hot_chains<Codec, Res, false, false>), g, dim3(64), 0, hs, a);
    return hipGetLastError();
}
template <class Codec, class Res>
hipError_t hot_fill_t(const RegionArgs& a, hipStream_t s) {
    const dim3 gp(persistent_grid(1u << 30, 4));
    if (a.tok) hipLaunchKernelGGL((k_hot_fill<Codec, Res, true, false>), gp, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_hot_fill<Codec, Res, false, false>), gp, dim3(256), 0, s, a);
    if (a.walk_tab) {                                 // (allow walks on: their verdicts)
        if (a.tok) hipLaunchKernelGGL((k_hot_fill<Codec, Res, true, true>), gp, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((k_hot_fill<Codec, Res, false, true>), gp, dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace rl
