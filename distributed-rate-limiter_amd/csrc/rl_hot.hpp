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
__device__ inline uint64_t wave_min64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) { const uint64_t x = __shfl_xor(v, o, 64); v = x < v ? x : v; }
    return v;
}
__device__ inline uint64_t wave_max64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) { const uint64_t x = __shfl_xor(v, o, 64); v = x > v ? x : v; }
    return v;
}

__device__ inline uint32_t wave_min32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) { const uint32_t x = __shfl_xor(v, o, 64); v = x < v ? x : v; }
    return v;
}
__device__ inline uint32_t wave_max32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) { const uint32_t x = __shfl_xor(v, o, 64); v = x > v ? x : v; }
    return v;
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
            const uint64_t gw2 = (gfl[k] & 1u) | ((gfl[k] >> 1 & 1u) << 8) | ((gfl[k] >> 2 & 1u) << 16);
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
template <class Codec, class Res, bool TOK>
__device__ inline void hot_chain(const RegionArgs& a, uint32_t i, RegionLds<Codec, true>& S) {
    using Rec = typename Codec::Rec;
    constexpr uint32_t NS = kRegionSlots;
    __shared__ int32_t s_hslot[2];
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t lane = threadIdx.x & 63;
    if (i >= hc) return;
    // the passes are sequential critical paths beside thousands of normal-region waves
    __builtin_amdgcn_s_setprio(3);
    const HotInfo f = a.hot_info[i];
    const uint32_t region = f.bin;                    // a bin is one region
    const DevLimiter L = a.lims[a.region_lim[region]];
    const int64_t base = a.ctl->base_ms;
    const int64_t lo = batch_lo(a.ctl);
    const int64_t hi = batch_hi(a.ctl);
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
    {
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
    }
    wave_fence();
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
    uint32_t n_changed = 0, n_tk = 0, n_fb = 0;       // debug: changes, [T0, T1) updates,
    uint32_t n_late = 0;                              // detailed chunks starting before T0 / ending past T1
    uint32_t n_prehit = 0;                            // debug: chunks whose records were prefetched
    uint32_t n_bisect = 0;                            // debug: SW table entries found by bisection
    uint64_t cyc_build = 0;                           // debug: SW table builds
    uint64_t cyc_run = 0, cyc_search = 0, cyc_detail = 0, cyc_pass2 = 0;   // debug stamps
    uint64_t cyc_pre = 0, cyc_pass1 = 0;
    uint64_t cyc_sw[4] = {0, 0, 0, 0};                // debug: SW run: setup, greedy, remaining, commit
    uint32_t n_sw_it = 0;                             // debug: SW greedy steps
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
        uint64_t sa = S.sa[hs], sb = S.sb[hs], sc = S.sc[hs];
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
        if (hot_ok) pass1(std::integral_constant<int, kAlgoTB>{}, 0u);
        if (hot_ok2) pass1(std::integral_constant<int, kAlgoTB>{}, 1u);
        pass2(std::integral_constant<int, kAlgoTB>{});
    } else {
        if (hot_ok) pass1(std::integral_constant<int, kAlgoSW>{}, 0u);
        if (hot_ok2) pass1(std::integral_constant<int, kAlgoSW>{}, 1u);
        pass2(std::integral_constant<int, kAlgoSW>{});
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
        }
    }
}

// The hot chains alone (single-wave workgroups), launched on a side stream of the device's
// highest priority just before the normal regions' launch, so they start first. They are a
// few hundred lone waves beside ~10^6 normal-region waves: a larger register budget costs
// no occupancy that matters.
#ifndef RL_CHAIN_MIN_WAVES
#define RL_CHAIN_MIN_WAVES 2
#endif
template <class Codec, class Res, bool TOK>
__global__ __launch_bounds__(64, RL_CHAIN_MIN_WAVES) void k_hot_chains(RegionArgs a) {
    __shared__ RegionLds<Codec, true> S;
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    for (uint32_t i = blockIdx.x; i < hc; i += gridDim.x) {       // (workgroup-uniform)
        wave_fence();                                             // the last chain's LDS users
        hot_chain<Codec, Res, TOK>(a, i, S);
    }
}

// Phase C (one wave per group of 64 chunks, all CUs): results of the chunks the chains
// decided. The group's chunk verdicts come in with one load per lane; a chunk holding only
// the dominant key's records is written without reading them (unless TB balances are out).
template <class Codec, class Res, bool TOK>
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
        const uint64_t any = __ballot(c0 + lane < c1 && (((g0 | cv0) & 1u) || ((g1 | cv1) & 1u)));
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

// The chain launch: single-wave workgroups on the side stream hs.
template <class Codec, class Res>
hipError_t hot_chains_t(const RegionArgs& a, hipStream_t hs) {
    const dim3 g(a.chain_grid ? min(a.chain_grid, kHotMax) : kHotMax);
    if (a.tok) hipLaunchKernelGGL((k_hot_chains<Codec, Res, true>), g, dim3(64), 0, hs, a);
    else hipLaunchKernelGGL((k_hot_chains<Codec, Res, false>), g, dim3(64), 0, hs, a);
    return hipGetLastError();
}
template <class Codec, class Res>
hipError_t hot_fill_t(const RegionArgs& a, hipStream_t s) {
    const dim3 gp(persistent_grid(1u << 30, 4));
    if (a.tok) hipLaunchKernelGGL((k_hot_fill<Codec, Res, true>), gp, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_hot_fill<Codec, Res, false>), gp, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace rl
