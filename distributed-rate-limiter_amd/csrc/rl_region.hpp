// rl_region.hpp — the per-region sequential semantics (wave_apply, region_body_t), shared by
// the normal-region kernels (rl_region.hip) and the hot chains (rl_hot.hip).
#pragma once
#include "rl_kcommon.hpp"

#pragma clang fp contract(off)

namespace rl {

// ------------------------------------------------------------------ 4. regions
// One single-wave workgroup per REGION (a partition bin is one region). The region's 256
// slots (8 KB) live in the wave's LDS for the whole batch, loaded in place (or, for a sparse
// region, only the 4-slot buckets its probes reach); the wave streams the region's records in
// arrival order, kDepth slices of 64 in flight, and applies them 64 at a time; the slots the
// batch touched or changed go back to HBM. No barriers anywhere.


struct RegionTable {
    static constexpr bool kCache = false;
    alignas(16) uint64_t tag[kRegionSlots];
    uint64_t sa[kRegionSlots];
    uint64_t sb[kRegionSlots];
    uint64_t sc[kRegionSlots];
    alignas(16) uint32_t occ[kRegionSlots];   // bit0 occupied, bit1 touched by this batch
    uint64_t pm[kRegionSlots];                // the lanes of the group in flight holding the
                                              // slot's key (wave_apply; zero between groups)
};
// With a sliding-window local cache (SlidingWindowRateLimiter.java:57-64): every slot also
// carries its key's cache state (block-until ms, sw_step_cache), moved with the slot.
struct RegionTableX : RegionTable {
    static constexpr bool kCache = true;
    uint64_t sx[kRegionSlots];
};

template <class Codec, bool RING>
struct RegionLds : RegionTable {
    using Rec = typename Codec::Rec;
    Rec ring[kRing];                  // pending requests of the other keys (hot chains)
    uint32_t ring_pos[kRing];         // ... and their result index
};
template <class Codec>
struct RegionLds<Codec, false> : RegionTable {};

// Image regions keep dead slots as tombstones until live + dead slots exceed this many (of
// 256), then drop them and relink (the sparse path rebuilds on long probe chains instead).
constexpr uint32_t kTombCrowd = 192;
// Token-bucket rounds: allows decided per key and round (wave_apply)
constexpr int kTbSteps = 3;
constexpr bool kSparseOn = true;                 // (rl_tune ablate kAblNoProbe turns it off at run time)

// Sparse region (few records): the LDS table starts with every bucket kOccUnloaded and a
// probe that reaches such a bucket faults it in from HBM (128 B, + 32 B of cache words);
// dead slots come in as tombstones. tab == nullptr: the whole image is in LDS.
struct SparseSrc {
    const RL_GLOBAL Slot* tab;
    const RL_GLOBAL uint64_t* xtab;   // local-cache words (nullable)
    int64_t keep;                     // slot_live threshold (keep_from)
    bool long_chain;                  // per lane: a probe went past two used buckets
    int64_t wref = -1;                // a window start near the stream's requests (SW; uniform)
    uint32_t n_it = 0, n_probe = 0;   // debug: greedy steps, probe bucket steps (uniform)
};

template <class LdsT>
__device__ inline void fault_bucket(const SparseSrc& sp, const DevLimiter& L, LdsT& S, uint32_t p) {
    Slot v[4];
    uint64_t x[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = sp.tab[p + k];
    if constexpr (LdsT::kCache)
        if (sp.xtab) {
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = sp.xtab[p + k];
        }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool fr = slot_free(v[k], x[k]);
        const bool lv = !fr && slot_live(L, v[k], sp.keep, x[k]);
        S.tag[p + k] = v[k].tag; S.sa[p + k] = v[k].a; S.sb[p + k] = v[k].b; S.sc[p + k] = v[k].c;
        if constexpr (LdsT::kCache) S.sx[p + k] = x[k];
        S.occ[p + k] = fr ? 0u : lv ? kOccUsed : (kOccUsed | kOccTomb);
    }
}

// After an in-place load dropped some slots: a key whose probe sequence from its home now
// meets a free slot before it moves to the first such slot (the invariant of linear probing:
// a key sits before the first free slot from its home), until no key moves. Both slots of a
// move are kOccDirty. A move only shortens its key's probe, so the loop ends.
template <class LdsT>
__device__ inline void relink(LdsT& S, uint32_t lane) {
    constexpr uint32_t NS = kRegionSlots;
    for (;;) {
        bool again = false;
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) {
            const uint32_t s = lane + 64 * i;
            if (S.occ[s] & kOccUsed) {
                uint32_t p = slot_home(S.tag[s]);
                while (p != s && (S.occ[p] & kOccUsed)) p = (p + 1) & (NS - 1);
                if (p != s) {
                    again = true;
                    const uint32_t o = S.occ[p];
                    if (!(o & kOccUsed) && atomicCAS(&S.occ[p], o, kOccUsed | kOccDirty) == o) {
                        S.tag[p] = S.tag[s]; S.sa[p] = S.sa[s]; S.sb[p] = S.sb[s]; S.sc[p] = S.sc[s];
                        if constexpr (LdsT::kCache) S.sx[p] = S.sx[s];
                        S.occ[s] = kOccDirty;
                    }
                }
            }
            wave_fence();
        }
        if (!__any(again)) break;
    }
}

struct Applied {
    uint32_t j;                       // result index (padding slot for idle lanes)
    bool alw;                         // allowed
    int64_t rem;                      // remaining
    double tok;
};

// Result store in partition order: packed in the width Res, or the escape code plus the
// exact value in the int64 side array when remaining is outside Res's range (a TB
// balance below -3 after time regression; see kResEscape).
template <class Res>
__device__ inline void put_res(const RegionArgs& a, uint32_t j, bool alw, int64_t rem) {
    Res* res = (Res*)a.res;
    if (res_fits<Res>(rem)) {
        res[j] = (Res)pack_result(alw, rem);
    } else {
        res[j] = (Res)kResEscape;
        a.ext[j] = rem;
        atomicAdd(&a.ctl->n_esc, 1u);
    }
}

// Growth signal of a region after its batch (lane 0): `used` live keys, or an overflow.
__device__ inline void note_fill(const RegionArgs& a, uint32_t region, uint32_t used, bool overflow) {
    if (used > kGrowUsed || overflow) {
        const uint32_t li = a.region_lim[region];
        atomicOr(&a.ctl->grow[li >> 6], 1ULL << (li & 63));
    }
}

// Apply one group of up to 64 requests (lane order = arrival order; `valid` lanes only).
// SP: the region may be sparse (unloaded buckets, tombstones); image regions (SP = false)
// compile those checks out of the probe loop.
template <class Codec, int ALGO, bool SP, class LdsT>
__device__ inline Applied wave_apply(const RegionArgs& a, LdsT& S, const DevLimiter& L,
                                     uint32_t lane, const typename Codec::Rec& cur, bool valid,
                                     uint32_t j, int64_t base, uint32_t pad, uint32_t& n_allowed,
                                     uint32_t& n_invalid, uint32_t& n_caperr, uint32_t& n_rounds,
                                     uint32_t& n_hits, SparseSrc& sp) {
    constexpr uint32_t NS = kRegionSlots;
    constexpr bool tb = ALGO == kAlgoTB;        // per-algorithm code: nothing of the other
    constexpr bool CACHE = LdsT::kCache && !tb;
    const bool cache_on = CACHE && L.cache_ttl_ms > 0;
    Applied r;
    r.j = valid ? j : pad;
    const Req q = Codec::dec(cur, base);
    const bool live = valid && !q.invalid;
    r.alw = false;
    r.rem = kRemInvalid;
    r.tok = __builtin_nan("");
    n_invalid += (valid && q.invalid) ? 1u : 0u;
    // ---- find or insert the key's slot (lookup phase, then claim phase)
    int32_t slot = -1;
    bool need = live, failed = false;
    const uint32_t home = slot_home(q.h);
    if (a.ablate & kAblNoProbe) { if (need) slot = (int32_t)home; need = false; }
    for (;;) {
        if (!__any(need)) break;
        ++sp.n_probe;
        uint32_t cand = kNone, fault = kNone;
        bool cand_tomb = false;
        if (need) {
            // linear probing from a 4-aligned home, one 4-slot bucket per step: the key
            // is in the chain before its first free slot (nothing is deleted mid-batch).
            // A sparse region may reach a bucket not loaded yet (fault it in, retry) and
            // holds tombstones (never a hit; the first one before the free slot is reused).
            uint32_t p = home, tomb = kNone;
            for (uint32_t step = 0; step < NS / 4; ++step) {
                const uint4 o4 = *(const uint4*)&S.occ[p];
                if (SP && (o4.x & kOccUnloaded)) {  // a bucket is loaded whole
                    fault = p;
                    sp.long_chain |= step >= 2;
                    break;
                }
                const ulonglong2 t01 = *(const ulonglong2*)&S.tag[p];
                const ulonglong2 t23 = *(const ulonglong2*)&S.tag[p + 2];
                const uint32_t occm = (o4.x & 1u) | (o4.y & 1u) << 1 | (o4.z & 1u) << 2 |
                                      (o4.w & 1u) << 3;
                const uint32_t tombm = !SP ? 0u : (o4.x >> 3 & 1u) | (o4.y >> 3 & 1u) << 1 |
                                                         (o4.z >> 3 & 1u) << 2 | (o4.w >> 3 & 1u) << 3;
                const uint32_t hit = occm & ~tombm &
                                     ((t01.x == q.h ? 1u : 0u) | (t01.y == q.h ? 2u : 0u) |
                                      (t23.x == q.h ? 4u : 0u) | (t23.y == q.h ? 8u : 0u));
                const uint32_t freem = ~occm & 15u;
                // first free slot vs first hit in scan order
                const uint32_t ff = freem ? (uint32_t)__builtin_ctz(freem) : 4u;
                const uint32_t fh = hit ? (uint32_t)__builtin_ctz(hit) : 4u;
                if (fh < ff) { slot = (int32_t)(p + fh); need = false; break; }
                const uint32_t tm = tombm & ((1u << ff) - 1u);
                if (tomb == kNone && tm) tomb = p + (uint32_t)__builtin_ctz(tm);
                if (ff < 4u) {
                    cand = tomb != kNone ? tomb : p + ff;
                    cand_tomb = tomb != kNone;
                    sp.long_chain |= step >= 2;
                    break;
                }
                p = (p + 4) & (NS - 1);
            }
            if (need && cand == kNone && fault == kNone) {
                if (tomb != kNone) { cand = tomb; cand_tomb = true; }   // wrapped: reuse a tombstone
                else { need = false; failed = true; }
            }
        }
        if (SP && __any(fault != kNone)) {
            // lanes faulting the same bucket write the same words; nothing else in the
            // wave touches an unloaded bucket
            if (fault != kNone) fault_bucket(sp, L, S, fault);
        }
        wave_fence();
        // (a free slot may carry kOccDirty: a slot the in-place load dropped)
        const uint32_t expect = cand_tomb ? (kOccUsed | kOccTomb) : need && cand != kNone ? (S.occ[cand] & kOccDirty) : 0u;
        if (need && cand != kNone && atomicCAS(&S.occ[cand], expect, kOccUsed) == expect) {
            S.tag[cand] = q.h; S.sa[cand] = 0; S.sb[cand] = 0; S.sc[cand] = 0;
            if constexpr (LdsT::kCache) S.sx[cand] = 0;
            slot = (int32_t)cand;
            need = false;
        }
        wave_fence();
        // a lane that lost the claim to another request of its own key (a new key with several
        // requests in the group) finds it there without probing again
        if (need && cand != kNone && (S.occ[cand] & (kOccUsed | kOccTomb)) == kOccUsed && S.tag[cand] == q.h) {
            slot = (int32_t)cand;
            need = false;
        }
    }
    if (failed) {
        r.rem = kRemError;
        ++n_caperr;
    }
    if (slot >= 0) atomicOr(&S.occ[slot], 2u);
    // ---- apply in arrival order. Per round, two hypotheses about a key's pending requests
    // are tested at once against its current state: (D) every earlier one is denied (no
    // state change: SlidingWindowRateLimiter.java:104-111, Lua :61-67) -> the prefix up to
    // and including the first state-changing request is final; (A, sliding window only)
    // every earlier one is allowed (the current bucket counts them: :114-116) -> the prefix
    // up to and including the first denied request is final. The longer prefix is taken,
    // so a run of denials or a run of allows costs one round, not one per request.
    // my key's lanes: one LDS OR per lane into its slot's word, read back, cleared
    const bool one_round = (a.ablate & kAblNoRounds) != 0;
    uint64_t peers = 1ULL << lane;
    if (!one_round) {
        if (slot >= 0) atomicOr((unsigned long long*)&S.pm[slot], 1ULL << lane);
        wave_fence();
        if (slot >= 0) peers = S.pm[slot];
        wave_fence();
        if (slot >= 0) S.pm[slot] = 0;
    }
    bool pending = slot >= 0;
    SWGeo geo{};
    uint64_t same_w = 0, elig_m = 0;        // (A): lanes in my window / acquires
    if constexpr (!tb) {
        // the wave's reference window follows its first request (requests of a region come
        // in arrival order: it moves about once per window)
        const uint64_t lm = __ballot(slot >= 0);
        if (lm) {
            const int64_t n0 = (int64_t)readlane64((uint64_t)q.now_ms, (uint32_t)__builtin_ctzll(lm));
            const int64_t w = L.window_ms;
            if (!(sp.wref >= 0 && n0 >= sp.wref && n0 - sp.wref < 2 * w)) {
                int64_t rr;
                sp.wref = n0 >= 0 ? jdiv(n0, w, L.inv_window, &rr) * w : -1;
            }
        }
        if (slot >= 0) geo = sw_geo_ref(q.now_ms, L, sp.wref);
        // window index relative to the wave's first window (2 bits; 3 = "far")
        const int64_t wmin = wave_min_dpp<int64_t>(slot >= 0 ? geo.curr_start : INT64_MAX);
        // (window starts are multiples of w: compares instead of a 64-bit division)
        const int64_t dw = geo.curr_start - wmin, w1 = L.window_ms;
        const int64_t wi = slot < 0 ? 3 : dw == 0 ? 0 : dw == w1 ? 1 : dw == 2 * w1 ? 2 : 3;
        const uint64_t b0 = __ballot(wi & 1), b1 = __ballot(wi & 2);
        same_w = ((wi & 1) ? b0 : ~b0) & ((wi & 2) ? b1 : ~b1);
        elig_m = __ballot(slot >= 0 && wi < 3 && q.op == (uint32_t)kOpAcquire);
    }
    if constexpr (!tb) if (!cache_on) {
        // Sliding window: a greedy scan per key instead of one round per state change. Inside
        // the window W0 of a key's first pending request, its acquires only INCR the current
        // bucket (:114-116), so with k allows before it a request's estimate is
        // d2l(tv + (C0 + k)), tv = prev * pw at its own time (:174): it is allowed iff k <= K,
        // its largest such k (denials change nothing, :104-111). One pass computes K per lane;
        // the allows then follow by integer compares (the j-th allow of a key is its first
        // request after the (j-1)-th with K >= j - 1), every key of the group at once. The
        // first request of a key the scan cannot take (another window, before the key's newest
        // bucket, near the epoch, a peek or a reset) runs the exact step alone; its later
        // requests go to the next pass. (The rounds below remain for the token bucket, whose
        // allows are a sequential fp64 recurrence, and for a limiter with the local cache; a
        // cache-off sliding window takes the scan in the cache kernel variant too.)
        {
            const int64_t w = L.window_ms, mx = L.max_permits;
            while (__any(pending)) {
                ++n_rounds;
                const uint64_t kp = peers & __ballot(pending);
                const uint32_t f0 = kp ? (uint32_t)__builtin_ctzll(kp) : lane;
                const int64_t W0 = __shfl(geo.curr_start, (int)f0, 64);
                uint64_t sa = 0, sb = 0, sc = 0;
                if (pending) { sa = S.sa[slot]; sb = S.sb[slot]; sc = S.sc[slot]; }
                const bool scan = pending && q.op == (uint32_t)kOpAcquire && geo.curr_start == W0 &&
                                  (int64_t)sa <= W0 && geo.prev_start != geo.curr_start;
                const uint64_t und = __ballot(pending && !scan) & peers;
                const uint32_t stop = und ? (uint32_t)__builtin_ctzll(und) : 64u;
                const bool in = scan && lane < stop;
                const SW2 s0 = sw_unpack(sa, sb, sc);
                const uint32_t C0 = s0.b1_start == W0 ? s0.b1_cnt : 0u;
                const double C0d = (double)C0;
                double tv = 0.0;
                int64_t K = -1;
                // (double)(C0 + kk) as one exact sum of doubles (counts are u32, kk < 2^31)
                auto est = [&](int64_t kk) { return d2l(tv + (C0d + (double)(int32_t)kk)); };
                if (in) {
                    const int64_t P = sw_get(s0, geo.prev_start, q.now_ms, w);
                    tv = (double)(uint32_t)P * geo.prev_weight;            // :174, rounded
                    K = mx - (int64_t)q.permits - (int64_t)C0 - d2l(tv);   // ~ largest k
                    if (K < -1) K = -1;           // (then no k >= 0 is allowed: est(0) > mx - p)
                    // rounding edges: K is exact when est(K) fits and est(K + 1) does not
                    if (K >= 0 && est(K) + q.permits > mx) {
                        --K;
                        if (K >= 0 && est(K) + q.permits > mx) --K;
                    } else if (est(K + 1) + q.permits <= mx) {
                        ++K;
                    }
                }
                // the greedy scan as a fixpoint: a lane is allowed iff its key's allows before
                // it (kk) are <= K. Starting from "every earlier one allowed", each step
                // recounts; the r-th lane of a key is final once its r earlier lanes are, so
                // the iteration ends at the sequential result after at most (the busiest key's
                // lanes) steps — one or two when K grows with time, as inside a window
                const uint64_t my = peers & __ballot(in);
                bool al = in && K >= (int64_t)popc_below(my);
                int64_t kk = 0;
                for (;;) {
                    ++sp.n_it;
                    kk = (int64_t)popc_below(__ballot(al) & my);
                    const bool nal = in && K >= kk;
                    if (!__any(nal != al)) break;
                    al = nal;
                }
                const uint64_t am = __ballot(al) & peers;
                const int64_t k = (int64_t)__popcll(am);
                const uint32_t last = am ? 63u - (uint32_t)__builtin_clzll(am) : 64u;
                if (in) {
                    const int64_t e = est(al ? kk + 1 : kk);                // after the request
                    r.alw = al;
                    r.rem = mx - e > 0 ? mx - e : 0;
                    r.tok = __builtin_nan("");
                    n_allowed += al ? 1u : 0u;
                    pending = false;
                }
                if (al && lane == last) {                 // the key's last allow commits them all
                    SWGeo gl{};
                    gl.curr_start = W0;
                    sw_commit_allows(L, gl, sa, sb, sc, (uint32_t)k, q.now_ms);
                    S.sa[slot] = sa; S.sb[slot] = sb; S.sc[slot] = sc;
                }
                wave_fence();
                if (pending && lane == stop) {            // the exact step, after the scan's allows
                    const Outcome o = sw_step_g(L, q.op, q.permits, q.now_ms, geo, S.sa[slot],
                                                S.sb[slot], S.sc[slot]);
                    if (o.mutate) { S.sa[slot] = o.a; S.sb[slot] = o.b; S.sc[slot] = o.c; }
                    r.alw = o.allowed;
                    r.rem = o.remaining;
                    r.tok = __builtin_nan("");
                    n_allowed += o.allowed ? 1u : 0u;
                    pending = false;
                }
                wave_fence();
            }
        }
        return r;
    }
    {
    if constexpr (tb) {
        // Token bucket, acquires only (the common group): tb_step's acquire branch in
        // straight-line code per round (Lua :56-65; elapsed as one exact integer difference,
        // times below 2^53). A round decides each key's requests up to its first allow.
        if (!(a.ablate & kAblNoStep) && !__any(pending && q.op != (uint32_t)kOpAcquire)) {
            if (pending && (int64_t)q.permits > L.max_permits) {       // :110-116, no state access
                r.rem = kRemUnknown;
                pending = false;
            }
            const double pd = (double)q.permits, cap = L.capacity, rate = L.rate_per_ms;
            while (__any(pending)) {
                ++n_rounds;
                uint64_t sa = 0, sb = 0, sc = 0;
                if (pending) { sa = S.sa[slot]; sb = S.sb[slot]; sc = S.sc[slot]; }
                // up to kTbSteps allows per key and round: after a key's first allow (lane fm)
                // its later pending lanes take the state that allow leaves, (tokens, now, 1),
                // from lane fm's registers, as the next round would from the slot. The slot is
                // written once, by the key's last allow of the round.
                double tk = __longlong_as_double((long long)sa);
                int64_t last = (int64_t)sb;
                bool live = (sc & 1u) != 0;
                bool mutated = false;                     // this lane's allow changed the state
                uint32_t from = 0;                        // my key's lanes below it are decided
#pragma unroll
                for (int st = 0; st < kTbSteps; ++st) {
                    const bool cand = pending && lane >= from;
                    const bool ex = live && !(q.now_ms > last + L.ttl_ms);
                    const double x = tk + (double)(q.now_ms - last) * rate;
                    const double rf = !ex ? cap : (x < cap ? x : cap);
                    const bool ok = rf >= pd;
                    const double nt = ok ? rf - pd : rf;
                    const uint64_t mut = __ballot(cand && ok) & peers;
                    const uint32_t fm = mut ? (uint32_t)__builtin_ctzll(mut) : 64u;
                    if (cand && lane <= fm) {
                        mutated = lane == fm;
                        r.alw = ok;
                        r.rem = d2l(nt);
                        r.tok = nt;
                        n_allowed += ok ? 1u : 0u;
                        pending = false;
                    }
                    if (st + 1 == kTbSteps || !__any(pending)) break;
                    const int src = fm < 64u ? (int)fm : (int)lane;
                    const double tk2 = __shfl(nt, src, 64);
                    const int64_t t2 = __shfl(q.now_ms, src, 64);
                    if (fm < 64u) { tk = tk2; last = t2; live = true; }
                    from = fm + 1u;
                }
                const uint64_t mm = __ballot(mutated) & peers;
                if (mutated && lane == 63u - (uint32_t)__builtin_clzll(mm)) {
                    S.sa[slot] = (uint64_t)__double_as_longlong(r.tok);
                    S.sb[slot] = (uint64_t)q.now_ms;
                    S.sc[slot] = 1;
                }
                wave_fence();
            }
            return r;
        }
    }
    while (__any(pending)) {
        ++n_rounds;
        Outcome o{};
        SWAllow al{false, 0};
        bool elig = false, hit = false, xs = false;
        const uint64_t pm = __ballot(pending);
        const uint64_t kp = peers & pm;                        // my key's pending requests
        if (pending) {
            const uint64_t sa = S.sa[slot], sb = S.sb[slot], sc = S.sc[slot];
            if (a.ablate & kAblNoStep) {
                o.mutate = (q.permits & 1) != 0; o.allowed = o.mutate; o.remaining = q.permits;
                o.a = sa; o.b = sb; o.c = sc;
            } else {
                if constexpr (tb) {
                    o = tb_step(L, q.op, q.permits, q.now_ms, sa, sb, sc);
                } else if (cache_on) {
                    if constexpr (CACHE) {
                        const uint64_t x0 = S.sx[slot];
                        o = sw_step_cache(L, q.op, q.permits, q.now_ms, geo, sa, sb, sc, x0, hit);
                        // (A) with the local cache: while the key has no cache entry that
                        // rejects (x0 == 0) a put changes nothing unless its value reaches
                        // max (:106-108, :119-121), so a run of allows is still closed-form;
                        // the request whose put sets the entry (xs) ends the run, inclusive
                        const uint64_t upto = kp & (((1ULL << lane) - 1) | (1ULL << lane));
                        elig = x0 == 0 && (upto & ~(elig_m & same_w)) == 0 &&
                               (int64_t)sa <= geo.curr_start && geo.prev_start != geo.curr_start;
                        if (elig) {
                            const uint32_t k = popc_below(kp);
                            al = sw_try_after_allows(L, q.permits, q.now_ms, geo, sa, sb, sc, k);
                            const SW2 s0 = sw_unpack(sa, sb, sc);
                            const int64_t curr0 = s0.b1_start == geo.curr_start ? (int64_t)s0.b1_cnt : 0;
                            // allow: newCount = curr0 + k + 1; deny: the estimate, >= max iff
                            // its remaining is 0
                            xs = al.allowed ? curr0 + (int64_t)k + 1 >= L.max_permits : al.remaining == 0;
                        }
                    }
                } else {
                    o = sw_step_g(L, q.op, q.permits, q.now_ms, geo, sa, sb, sc);
                    // (A) for this request needs: it and every EARLIER pending peer are
                    // acquires in its window, not before the key's newest bucket (the allows
                    // of one window then only INCR its bucket). A later window's requests
                    // become eligible in the next round, once this window's are final.
                    const uint64_t upto = kp & (((1ULL << lane) - 1) | (1ULL << lane));
                    // (near the epoch, now < w, Java's truncating division makes the previous
                    // window the current one, :170-172: its count then moves with the allows)
                    elig = (upto & ~(elig_m & same_w)) == 0 && (int64_t)sa <= geo.curr_start &&
                           geo.prev_start != geo.curr_start;
                    if (elig) al = sw_try_after_allows(L, q.permits, q.now_ms, geo, sa, sb, sc,
                                                       popc_below(kp));
                }
            }
        }
        const uint64_t mut = __ballot(pending && o.mutate) & peers;
        const uint32_t fm = mut ? (uint32_t)__builtin_ctzll(mut) : 64u;
        bool use_a = false;
        uint32_t fa = 64u, a_end = 0u;
        if constexpr (!tb) {
            // per key: (A) is final up to its first denial (inclusive) or its first pending
            // request that is not eligible (exclusive); (D) up to the first state change
            const uint64_t den = __ballot(pending && elig && (!al.allowed || xs)) & peers;
            const uint64_t nel = __ballot(pending && !elig) & peers;
            const uint32_t fd = den ? (uint32_t)__builtin_ctzll(den) : 64u;
            const uint32_t fs = nel ? (uint32_t)__builtin_ctzll(nel) : 64u;
            fa = fd < fs ? fd : fs;                 // allows: the pending peers below fa
            a_end = fd < fs ? fd + 1u : fs;
            // (cache) the run's last request is itself an allow when its put sets the entry
            if (fd < fs && ((__ballot(pending && elig && al.allowed && xs) & peers) >> fd & 1u)) fa = fd + 1u;
            const uint32_t d_end = fm < 64u ? fm + 1u : 64u;
            use_a = a_end > d_end;               // the allow hypothesis decides more
        }
        if (pending && use_a) {
            if constexpr (!tb) {
                if (lane < a_end) {
                    const uint64_t ok = kp & (fa >= 64u ? ~0ULL : ((1ULL << fa) - 1));   // the allows
                    if (ok && lane == 63u - (uint32_t)__builtin_clzll(ok)) {   // the last allow commits
                        uint64_t na = S.sa[slot], nb = S.sb[slot], nc = S.sc[slot];
                        sw_commit_allows(L, geo, na, nb, nc, (uint32_t)__popcll(ok), q.now_ms);
                        S.sa[slot] = na; S.sb[slot] = nb; S.sc[slot] = nc;
                    }
                    if constexpr (CACHE)
                        if (xs && lane + 1u == a_end)        // this request's put sets the entry
                            S.sx[slot] = (uint64_t)(q.now_ms + L.cache_ttl_ms);
                    r.alw = al.allowed;
                    r.rem = al.remaining;
                    r.tok = __builtin_nan("");
                    n_allowed += al.allowed ? 1u : 0u;
                    pending = false;
                }
            }
        } else if (pending && lane <= fm) {
            if (lane == fm) {
                S.sa[slot] = o.a; S.sb[slot] = o.b; S.sc[slot] = o.c;
                if constexpr (CACHE) if (cache_on) S.sx[slot] = o.x;
            }
            r.alw = o.allowed;
            r.rem = o.remaining;
            r.tok = o.tokens;
            n_allowed += o.allowed ? 1u : 0u;
            n_hits += hit ? 1u : 0u;                   // counted once, when final
            pending = false;
        }
        wave_fence();
    }
    return r;
    }
}

template <class Codec, class Res, bool TOK, class LdsT>
__device__ inline void region_body_t(const RegionArgs& a, uint32_t g, LdsT& S) {
    using Rec = typename Codec::Rec;
    constexpr uint32_t NS = kRegionSlots;

    uint32_t bin = g;
    if (a.order) {
        // largest regions first (k_order_place), after a prefix of the smallest: the first
        // workgroups the machine takes then finish quickly and the hot chains (a side
        // stream of higher priority) get their slots at once instead of behind the longest
        // normal regions
        const uint32_t tot = a.order[a.n_regions];
        if (g >= tot) return;
        const uint32_t k = min(a.order_prefix, tot);
        bin = a.order[g < k ? tot - k + g : g - k];
    }
    const uint32_t n_bins = a.n_regions;
    if (bin >= n_bins) return;
    if (a.hot_mark && a.hot_mark[bin] == a.epoch) return;     // owned by hot_chain
    if (a.ablate & kAblNoNormal) return;
    const uint32_t start = a.rstart[bin];
    const uint32_t cnt = a.rend ? a.rend[bin] - start : a.rcount[bin];
    if (cnt == 0) return;
    const uint32_t end = start + cnt;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t region = bin;
    const DevLimiter L = a.lims[a.region_lim[region]];
    const int64_t base = a.ctl->base_ms;
    const int64_t batch_min = keep_from(a);
    const uint32_t pad = a.n_total + lane;          // padding slot for idle lanes
    const Rec* recs = (const Rec*)a.rec;
    Res* res = (Res*)a.res;

    if (a.ctl->span_overflow != 0) {
        // compact records cannot represent this batch's time span: reject it whole,
        // before any state is touched (the host reports RL_E_INVALID_ARG)
        for (uint32_t j = start + lane; j < end; j += 64) {
            res[j] = (Res)pack_result(false, kRemInvalid);
            if (TOK) a.tok[j] = __builtin_nan("");
        }
        return;
    }
    // kDepth slices of the region's stream in flight (issued while the region image loads);
    // the stream is read once (non-temporal)
    constexpr uint32_t kDepth = 4;
    const uint64_t t_begin = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    auto fetch = [&](uint32_t c) { return ld_rec<kNtRgRec>(recs + min(c + lane, end - 1)); };
    Rec q0 = fetch(start), q1 = fetch(start + 64), q2 = fetch(start + 128), q3 = fetch(start + 192);

    // ---- the region's slots: the whole image in place, or (sparse) buckets on demand
    RL_GLOBAL Slot* tab = as_global((Slot*)L.table + (size_t)(region - L.region_base) * NS);
    RL_GLOBAL uint64_t* xtab = nullptr;             // the slots' local-cache states
    if constexpr (LdsT::kCache)
        if (L.cache_table) xtab = as_global((uint64_t*)L.cache_table + (size_t)(region - L.region_base) * NS);
    // Few records: probe and update single buckets in HBM (128 B read + 32 B written per
    // distinct key) instead of moving the 8 KB image both ways.
    const bool sparse = kSparseOn && cnt <= a.sparse_max && !(a.ablate & kAblNoProbe);
    SparseSrc sp{sparse ? tab : nullptr, xtab, batch_min, false};
    bool tombs = false;                              // an image region kept dead slots as tombstones
    // rebuild the LDS table from registers: linear probing from each key's home
    auto rebuild = [&](const Slot (&img)[NS / 64], const uint64_t (&xim)[NS / 64], const bool (&keep)[NS / 64]) {
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) { S.occ[lane + 64 * i] = 0; S.pm[lane + 64 * i] = 0; }
        wave_fence();
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) {
            const Slot v = img[i];
            if (keep[i]) {
                uint32_t p = slot_home(v.tag);
                while (atomicCAS(&S.occ[p], 0u, 1u) != 0u) p = (p + 1) & (NS - 1);
                S.tag[p] = v.tag; S.sa[p] = v.a; S.sb[p] = v.b; S.sc[p] = v.c;
                if constexpr (LdsT::kCache) S.sx[p] = xim[i];
            }
        }
        wave_fence();
    };
    if (sparse) {
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) { S.occ[lane + 64 * i] = kOccUnloaded; S.pm[lane + 64 * i] = 0; }
        wave_fence();
    } else {
        // load the region in place: live keys keep their slots, so only the slots this batch
        // changes are written back. Entries no request of this batch can see stay where they
        // are as tombstones (claimable by an insert, never a hit; in HBM a dead slot that is
        // not zero already is one): dropping them would need the relink below, which moved
        // most keys of a region whose window rolled over (sw_zipf's steady state: region load
        // 3.6 -> 13 us). Only once live + dead slots crowd the region (> kTombCrowd) are the
        // dead ones dropped and the chains relinked.
        uint32_t n_live = 0, n_dead = 0;
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) {
            const uint32_t s = lane + 64 * i;
            const Slot v = tab[s];
            const uint64_t x = xtab ? xtab[s] : 0;
            const bool fr = slot_free(v, x);
            const bool kp = !fr && slot_live(L, v, batch_min, x);
            S.occ[s] = kp ? kOccUsed : fr ? 0u : (kOccUsed | kOccTomb);
            S.pm[s] = 0;
            S.tag[s] = v.tag; S.sa[s] = v.a; S.sb[s] = v.b; S.sc[s] = v.c;
            if constexpr (LdsT::kCache) S.sx[s] = x;
            n_live += kp ? 1u : 0u;
            n_dead += !fr && !kp ? 1u : 0u;
        }
        for (int o = 32; o > 0; o >>= 1) {
            n_live += __shfl_xor(n_live, o, 64);
            n_dead += __shfl_xor(n_dead, o, 64);
        }
        if (n_dead != 0 && n_live + n_dead > kTombCrowd) {
#pragma unroll
            for (uint32_t i = 0; i < NS / 64; ++i) {
                const uint32_t s = lane + 64 * i;
                if (S.occ[s] & kOccTomb) S.occ[s] = kOccDirty;
            }
            wave_fence();
            relink(S, lane);
            n_dead = 0;
        }
        wave_fence();
        tombs = n_dead != 0;
    }

    uint32_t n_allowed = 0, n_invalid = 0, n_caperr = 0, n_rounds = 0, n_hits = 0;
    const uint64_t t_start = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    // the whole stream is instantiated once per algorithm (uniform per region), so the
    // compiler hoists nothing of the other algorithm into the hot loop
    auto stream = [&](auto algo, auto spc) {
        constexpr int A = decltype(algo)::value;
        constexpr bool SPX = decltype(spc)::value;
        auto slice = [&](const Rec& r, uint32_t c0) {
            // every record of the stream is the region's: applied straight from registers
            const uint32_t idx = c0 + lane;
            const Applied ap = wave_apply<Codec, A, SPX>(a, S, L, lane, r, idx < end, idx, base, pad,
                                                 n_allowed, n_invalid, n_caperr, n_rounds, n_hits, sp);
            put_res<Res>(a, ap.j, ap.alw, ap.rem);
            if (TOK) a.tok[ap.j] = ap.tok;
        };
        // unrolled by kDepth so the prefetch registers rotate without moves (a register move
        // would wait on its load and shrink the effective depth to one slice)
        for (uint32_t c0 = start; c0 < end; c0 += 64 * kDepth) {
            slice(q0, c0);
            q0 = fetch(c0 + 64 * kDepth);
            if (c0 + 64 >= end) break;
            slice(q1, c0 + 64);
            q1 = fetch(c0 + 64 * kDepth + 64);
            if (c0 + 128 >= end) break;
            slice(q2, c0 + 128);
            q2 = fetch(c0 + 64 * kDepth + 128);
            if (c0 + 192 >= end) break;
            slice(q3, c0 + 192);
            q3 = fetch(c0 + 64 * kDepth + 192);
        }
    };
    using SpOn = std::integral_constant<bool, kSparseOn>;
    using SpOff = std::integral_constant<bool, false>;
    // (tombstones need the sparse probe's checks; an image region holds no unloaded bucket)
    if (L.algo == kAlgoTB) {
        if (sparse || tombs) stream(std::integral_constant<int, kAlgoTB>{}, SpOn{});
        else stream(std::integral_constant<int, kAlgoTB>{}, SpOff{});
    } else {
        if (sparse || tombs) stream(std::integral_constant<int, kAlgoSW>{}, SpOn{});
        else stream(std::integral_constant<int, kAlgoSW>{}, SpOff{});
    }
    wave_fence();
    const uint64_t t_stream = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t touched = 0;
    for (uint32_t s = lane; s < NS; s += 64) touched += (S.occ[s] & kOccTouched) ? 1u : 0u;
    bool whole = false;                              // rebuilt: every slot goes back
    if (sparse && __any(sp.long_chain)) {
        // probe chains have grown long (tombstones accumulate while a region only ever sees
        // few records): fault in the rest of the region (one bucket per lane), keep its live
        // keys and rebuild it as an image region does, then write it back whole
        if (S.occ[4 * lane] & kOccUnloaded) fault_bucket(sp, L, S, 4 * lane);
        wave_fence();
        Slot img[NS / 64];
        uint64_t xim[NS / 64];
        bool keep[NS / 64];
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) {
            const uint32_t s = lane + 64 * i;
            const uint32_t o = S.occ[s];
            keep[i] = (o & kOccUsed) && !(o & kOccTomb);
            img[i] = Slot{S.tag[s], S.sa[s], S.sb[s], S.sc[s]};
            xim[i] = 0;
            if constexpr (LdsT::kCache) xim[i] = S.sx[s];
        }
        wave_fence();
        rebuild(img, xim, keep);
        whole = true;
    }
    // ---- write the region back: every slot (free ones as zeros) after a rebuild, else only
    // the slots this batch touched or changed (kOccDirty: dropped, moved by relink)
    const bool full = !sparse || whole;             // every slot is in LDS
    uint32_t used = 0;                               // live keys (full regions only)
    uint32_t moved = 0;                              // table bytes read + written
    const uint32_t xw = xtab ? 8u : 0u;              // local-cache word per slot
    for (uint32_t s = lane; s < NS; s += 64) {
        const uint32_t o = S.occ[s];
        const bool wr = whole || (o & (kOccTouched | kOccDirty));
        used += (full && (o & kOccUsed) && !(o & kOccTomb)) ? 1u : 0u;
        moved += (sparse ? (!(o & kOccUnloaded) && (s & 3u) == 0 ? 4u * (32u + xw) : 0u) : 32u + xw) +
                 (wr ? 32u + xw : 0u);
        if (!wr) continue;
        Slot v{0, 0, 0, 0};
        uint64_t x = 0;
        if (o & kOccUsed) {
            if constexpr (LdsT::kCache) x = S.sx[s];
            v = slot_used(Slot{S.tag[s], S.sa[s], S.sb[s], S.sc[s]}, x);
        }
        tab[s] = v;
        if constexpr (LdsT::kCache)
            if (xtab) xtab[s] = x;
    }
    for (int off = 32; off > 0; off >>= 1) {
        n_allowed += __shfl_xor(n_allowed, off, 64);
        n_invalid += __shfl_xor(n_invalid, off, 64);
        n_caperr += __shfl_xor(n_caperr, off, 64);
        n_hits += __shfl_xor(n_hits, off, 64);
        touched += __shfl_xor(touched, off, 64);
        used += __shfl_xor(used, off, 64);
        moved += __shfl_xor(moved, off, 64);
    }
    if (lane == 0) {
        note_fill(a, region, used, n_caperr != 0);
        unsigned long long* st = a.stats + (size_t)(blockIdx.x & (kStatSlots - 1)) * kStWords;
        atomicAdd(st + kStTableBytes, (unsigned long long)moved);
        if (n_allowed) atomicAdd(st + kStAllowed, (unsigned long long)n_allowed);
        if (n_invalid) atomicAdd(st + kStInvalid, (unsigned long long)n_invalid);
        if (n_caperr) atomicAdd(st + kStCapErr, (unsigned long long)n_caperr);
        atomicAdd(st + kStDistinct, (unsigned long long)touched);
        atomicAdd(st + kStRegions, 1ULL);
        if (n_hits) atomicAdd(st + kStCacheHits, (unsigned long long)n_hits);
        if (a.dbg) {
            uint64_t* d = a.dbg + (size_t)bin * kDbgWords;
            d[0] = t_start; d[1] = __builtin_amdgcn_s_memrealtime(); d[2] = cnt; d[3] = n_rounds;
            d[4] = t_begin; d[5] = t_stream; d[6] = sparse ? 1u : 0u; d[7] = sp.n_it; d[8] = sp.n_probe;
        }
    }
}

// Normal regions (one wave each) at >= kRegionMinWaves waves per SIMD (VGPR budget).
constexpr int kRegionMinWaves = 4;

}  // namespace rl
