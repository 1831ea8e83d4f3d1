// rl_solo.hip — single-key allow runs of sliding-window limiters with the local cache, decided
// by a whole workgroup before the region stage.
//
// With the Caffeine cache on (SlidingWindowRateLimiter.java:57-64,93-121) a denial may change
// state (it puts the estimate), so such regions have no hot-key chain: one region wave applies
// a key's requests 64 at a time. The reference's own benchmark (RateLimiterBenchmark.java:
// 48-71, BASELINE configs[0]) is exactly that case: one key, 100,000 requests, every one
// allowed — 1,563 dependent 64-request groups on one wave.
//
// But a run of allows is closed-form: inside the window W of a key's first request, with no
// rejecting cache entry, the r-th acquire of the run sees the current bucket at C0 + r (each
// allow INCRs it by 1, :114-116, whatever its permits) and the previous bucket's weighted
// count at its own time (:170-174), so whether it is allowed — and its remaining (A4) — is a
// function of r and its own record alone. The run ends at the first request that is denied,
// or that the cache rejects, or whose allow puts a count >= max into the cache (that one is
// still part of it). k_solo finds that end with one block-wide minimum over the region's
// records (all CUs' worth of lanes on a 100k-request region), writes the run's results, stores
// the key's new state (slot and cache word) in HBM and moves the region's start past the run;
// k_regions then applies the rest exactly as before (nothing, when the run is the region).
#include "rl_kcommon.hpp"
#include "rl_region.hpp"

#pragma clang fp contract(off)

namespace rl {

// Regions of cache-on sliding-window limiters with at least `thr` records.
__global__ __launch_bounds__(256) void k_solo_select(const uint32_t* rstart, const uint32_t* rcount,
                                                     const uint32_t* rend, uint32_t n_bins,
                                                     uint32_t thr, const DevLimiter* lims,
                                                     const uint8_t* region_lim, uint32_t* list,
                                                     uint32_t* count) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= n_bins) return;
    const uint32_t cnt = rend ? rend[b] - rstart[b] : rcount[b];
    if (cnt < thr) return;
    const DevLimiter& L = lims[region_lim[b]];
    if (L.algo != kAlgoSW || L.cache_ttl_ms <= 0 || L.cache_table == 0) return;
    const uint32_t k = atomicAdd(count, 1u);
    if (k < kSoloMax) list[k] = b;
}

constexpr uint32_t kSoloThreads = 1024;

template <class Codec, class Res>
__global__ __launch_bounds__(kSoloThreads) void k_solo(RegionArgs a, uint32_t* rstart, uint32_t* rcount,
                                                       const uint32_t* list, const uint32_t* count) {
    using Rec = typename Codec::Rec;
    constexpr uint32_t NS = kRegionSlots;
    __shared__ uint64_t s_h;
    __shared__ int64_t s_w0;
    __shared__ uint32_t s_cut, s_f, s_ok, s_slot;
    __shared__ uint64_t s_st[4];                      // the key's state a, b, c and cache word x
    const uint32_t t = threadIdx.x;
    const uint32_t n_list = min(count[0], kSoloMax);
    if (a.ctl->span_overflow != 0) return;            // the region stage rejects the batch whole
    const Rec* recs = (const Rec*)a.rec;
    const int64_t base = a.ctl->base_ms;
    for (uint32_t li = blockIdx.x; li < n_list; li += gridDim.x) {      // (block-uniform)
        __syncthreads();
        const uint32_t bin = list[li];
        const uint32_t start = rstart[bin];
        const uint32_t end = a.rend ? a.rend[bin] : start + rcount[bin];
        const DevLimiter L = a.lims[a.region_lim[bin]];
        const int64_t w = L.window_ms, mx = L.max_permits;
        RL_GLOBAL Slot* tab = as_global((Slot*)L.table + (size_t)(bin - L.region_base) * NS);
        RL_GLOBAL uint64_t* xtab = as_global((uint64_t*)L.cache_table + (size_t)(bin - L.region_base) * NS);
        if (t == 0) {
            // the run's key and window: the region's first request
            const Req q0 = Codec::dec(recs[start], base);
            int64_t rr;
            s_h = q0.h;
            s_w0 = jdiv(q0.now_ms, w, L.inv_window, &rr) * w;
            s_cut = end - start;
            s_f = end - start;
            // the key's slot: linear probing over 4-slot buckets from its home (the HBM
            // invariant: a key sits before the first free slot of its probe sequence); a dead
            // state (no bucket live for this batch) reads as absent, as a region load drops it
            uint32_t slot = kNone, reuse = kNone;
            const uint32_t home = slot_home(q0.h);
            for (uint32_t m = 0; m < NS; ++m) {
                const uint32_t p = (home + m) & (NS - 1);
                const Slot v = tab[p];
                const uint64_t x = xtab[p];
                if (slot_free(v, x)) { if (reuse == kNone) reuse = p; break; }
                const bool live = slot_live(L, v, keep_from(a), x);
                if (v.tag == q0.h) { slot = p; break; }
                if (!live && reuse == kNone) reuse = p;          // a dead slot may be taken over
            }
            s_ok = !q0.invalid && q0.op == (uint32_t)kOpAcquire && q0.now_ms >= w &&
                   (slot != kNone || reuse != kNone);
            Slot v{q0.h, 0, 0, 0};
            uint64_t x = 0;
            if (slot != kNone) {
                const Slot u = tab[slot];
                const uint64_t ux = xtab[slot];
                if (slot_live(L, u, keep_from(a), ux)) { v = u; x = ux; }
            } else {
                slot = reuse;
            }
            // a key whose newest bucket is past W (time regression) takes the exact path
            if (s_ok && v.b != 0 && (int64_t)v.a > s_w0) s_ok = 0;
            s_slot = slot;
            s_st[0] = v.a; s_st[1] = v.b; s_st[2] = v.c; s_st[3] = x;
        }
        __syncthreads();
        if (!s_ok) continue;
        const uint64_t h = s_h;
        const int64_t W0 = s_w0;
        const SW2 s0 = sw_unpack(s_st[0], s_st[1], s_st[2]);
        const int64_t C0 = s0.b1_start == W0 ? (int64_t)s0.b1_cnt : 0;
        const int64_t x0 = (int64_t)s_st[3];
        const uint32_t n = end - start;
        // 1. the longest prefix of requests the run can take at all: acquires of this key
        // inside W (another key, a peek or a reset, another window: the exact path from there)
        for (uint32_t r = t; r < n; r += kSoloThreads) {
            const Req q = Codec::dec(recs[start + r], base);
            const bool take = !q.invalid && q.op == (uint32_t)kOpAcquire && q.h == h &&
                              q.now_ms >= W0 && q.now_ms - W0 < w;
            if (!take) { atomicMin(&s_cut, r); break; }   // later r of this thread: past it
        }
        __syncthreads();
        const uint32_t cut = s_cut;
        // 2. the run's end: the first request denied (or rejected by a cache entry still
        // valid at its time), or the request after an allow whose put reaches max
        for (uint32_t r = t; r < cut; r += kSoloThreads) {
            const Req q = Codec::dec(recs[start + r], base);
            const int64_t cnt = C0 + (int64_t)r;          // the bucket before this request
            const SWGeo g = sw_geo(q.now_ms, L);
            const double tv = (double)sw_get(s0, g.prev_start, q.now_ms, w) * g.prev_weight;  // :174
            const int64_t est = d2l(tv + (double)cnt);
            const bool hit = r == 0 && x0 != 0 && q.now_ms < x0;                      // :93-100
            uint32_t e = kNone;
            if (hit || est + (int64_t)q.permits > mx) e = r;                           // :104
            else if (cnt + 1 >= mx) e = r + 1;            // its put sets a rejecting entry (:119-121)
            if (e != kNone) { atomicMin(&s_f, e); break; }
        }
        __syncthreads();
        const uint32_t f = min(s_f, cut);
        if (f == 0) continue;
        // 3. the run's results: allowed, remaining after the request (A4)
        for (uint32_t r = t; r < f; r += kSoloThreads) {
            const Req q = Codec::dec(recs[start + r], base);
            const SWGeo g = sw_geo(q.now_ms, L);
            const double tv = (double)sw_get(s0, g.prev_start, q.now_ms, w) * g.prev_weight;
            const int64_t est2 = d2l(tv + (double)(C0 + (int64_t)r + 1));
            put_res<Res>(a, start + r, true, mx - est2 > 0 ? mx - est2 : 0);
            if (a.tok) a.tok[start + r] = __builtin_nan("");
        }
        // 4. the key's state after the run (as sw_commit_allows + the last put) and the rest
        // of the region for k_regions
        if (t == 0) {
            const Req ql = Codec::dec(recs[start + f - 1], base);
            uint64_t sa = s_st[0], sb = s_st[1], sc = s_st[2];
            SWGeo gl{};
            gl.curr_start = W0;
            sw_commit_allows(L, gl, sa, sb, sc, f, ql.now_ms);
            const uint64_t x = C0 + (int64_t)f >= mx ? (uint64_t)(ql.now_ms + L.cache_ttl_ms) : 0;
            tab[s_slot] = slot_used(Slot{h, sa, sb, sc}, x);
            xtab[s_slot] = x;
            rstart[bin] = start + f;
            if (!a.rend) rcount[bin] = n - f;
            unsigned long long* st = a.stats + (size_t)(blockIdx.x & (kStatSlots - 1)) * kStWords;
            atomicAdd(st + kStAllowed, (unsigned long long)f);
            if (f == n) {                                 // no region wave for it
                atomicAdd(st + kStDistinct, 1ULL);
                atomicAdd(st + kStRegions, 1ULL);
                s_ok = 0;                                 // (the fill count below)
            }
        }
        if (f == n) {
            // no region wave runs for this region in this batch, so its growth check (the
            // live keys a region write-back counts, note_fill) is made here: the run's key may
            // have taken a free or dead slot. Slot s_slot holds the key's new state.
            __syncthreads();
            if (t < NS) {
                const Slot v = tab[t];
                const uint64_t x = xtab[t];
                const bool used = t == s_slot || (!slot_free(v, x) && slot_live(L, v, keep_from(a), x));
                if (used) atomicAdd(&s_ok, 1u);
            }
            __syncthreads();
            if (t == 0) note_fill(a, bin, s_ok, false);
        }
    }
}

hipError_t launch_solo_select(const uint32_t* rstart, const uint32_t* rcount, const uint32_t* rend,
                              uint32_t n_bins, uint32_t thr, const DevLimiter* lims,
                              const uint8_t* region_lim, uint32_t* list, uint32_t* count,
                              hipStream_t s) {
    if (n_bins == 0) return hipSuccess;
    hipLaunchKernelGGL(k_solo_select, dim3((n_bins + 255) / 256), dim3(256), 0, s, rstart, rcount,
                       rend, n_bins, thr, lims, region_lim, list, count);
    return hipGetLastError();
}

template <class Codec, class Res>
static hipError_t solo_t(const RegionArgs& a, uint32_t* rstart, uint32_t* rcount, const uint32_t* list,
                         const uint32_t* count, hipStream_t s) {
    hipLaunchKernelGGL((k_solo<Codec, Res>), dim3(kSoloGrid), dim3(kSoloThreads), 0, s, a, rstart,
                       rcount, list, count);
    return hipGetLastError();
}

hipError_t launch_solo(const RegionArgs& a, bool wide, int res_bytes, uint32_t* rstart, uint32_t* rcount,
                       const uint32_t* list, const uint32_t* count, hipStream_t s) {
    if (wide) return solo_t<CodecW, uint64_t>(a, rstart, rcount, list, count, s);
    if (res_bytes == 1) return solo_t<CodecC, uint8_t>(a, rstart, rcount, list, count, s);
    if (res_bytes == 2) return solo_t<CodecC, uint16_t>(a, rstart, rcount, list, count, s);
    return solo_t<CodecC, uint32_t>(a, rstart, rcount, list, count, s);
}

}  // namespace rl
