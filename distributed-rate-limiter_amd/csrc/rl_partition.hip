// rl_partition.hip — stable partition of a batch into region order (upsweep, scans,
// scatter, bin bounds) and the unpermute back to arrival order, for gfx950.
#include "rl_kcommon.hpp"

#pragma clang fp contract(off)

namespace rl {

// ------------------------------------------------------------------ 1. upsweep
// DIG: the pass stores each element's digit for the scatter (routing).
template <class Codec, bool RAW, bool DIG>
__global__ __launch_bounds__(kTileThreads) void k_upsweep(PartArgs a) {
    // dynamic LDS (upsweep_lds_bytes): the histogram of this pass's bins, then the route table
    // when routing; sized to the pass so that 4 workgroups fit a CU at 8192 bins
    extern __shared__ uint32_t dyn_lds[];
    __shared__ LimLds L;
    const uint32_t t = threadIdx.x;
    const uint32_t bins = a.n_bins_pass ? a.n_bins_pass : 1u << a.digit_bits;
    uint32_t* hist = dyn_lds;
    RouteLds& R = *(RouteLds*)(dyn_lds + bins);
    load_lim_lds(L, a);
    if (a.route_list) route_load(R, a.route_list);
    if constexpr (RAW) {
        if (blockIdx.x == 0 && t == 0) {
            BatchCtl* c = a.ctl;
            c->base_ms = floor_div_ms(a.now_ns[0]) - (1LL << 31);
            c->min_now_key = ~0ULL;
            c->max_now_key = 0;
            c->span_overflow = 0;
            c->n_esc = 0;
            c->allowed = c->distinct = c->invalid = c->cap_err = c->regions = c->cache_hits = 0;
            c->grow[0] = c->grow[1] = c->grow[2] = c->grow[3] = 0;
            c->table_bytes = 0;
            c->n_normal = a.n;                           // k_route_ranges lowers it when routing
            c->n_hot = 0;                                // k_hot_prep sets it when the hot path runs
            c->internal_err = 0;
            c->n_walk = 0;                               // k_hot_scan sets it when the hot path runs
        }
    }
    // later passes partition the normal records only (their count is on device)
    const uint32_t n = a.n_dev ? *a.n_dev : a.n;
    for (uint32_t it = 0;; ++it) {
        const uint32_t tile = tile_at(it, a.n_tiles);
        if (tile >= a.n_tiles) break;
        for (uint32_t b = t; b < bins; b += kTileThreads) hist[b] = 0;
        __syncthreads();
        const uint32_t items = a.tile_items, T = items * (uint32_t)kTileThreads;
        if (tile * (uint64_t)T < n) {
#pragma unroll 8
            for (uint32_t r = 0; r < items; ++r) {
                const uint32_t i = tile * T + r * (uint32_t)kTileThreads + t;
                if (i < n) {
                    const uint32_t g = bin_of<Codec, RAW>(a, i, L);
                    const uint32_t d = pass_digit(a, g, R);
                    atomicAdd(&hist[d], 1u);
                    if constexpr (DIG) a.digit[i] = (uint16_t)d;      // the scatter reads it back
                }
            }
        }
        __syncthreads();
        for (uint32_t b = t; b < bins; b += kTileThreads)
            a.counts[(size_t)b * a.n_tiles + tile] = hist[b];
    }
}

// ------------------------------------------------------------------ 2. scans
// Exclusive scan of each row of a [rows][cols] matrix (one block per row).
__global__ __launch_bounds__(256) void k_scan_rows(const uint32_t* in, uint32_t* out,
                                                   uint32_t cols, uint32_t* totals) {
    __shared__ uint32_t tmp[4];
    const size_t row = blockIdx.x;
    const uint32_t* src = in + row * cols;
    uint32_t* dst = out + row * cols;
    const uint32_t chunk = (cols + 255) / 256;
    const uint32_t beg = min(threadIdx.x * chunk, cols);
    const uint32_t end = min(beg + chunk, cols);
    uint32_t sum = 0;
    for (uint32_t k = beg; k < end; ++k) sum += src[k];
    uint32_t tot;
    uint32_t run = block_exclusive_scan<256>(sum, tmp, &tot);
    for (uint32_t k = beg; k < end; ++k) {
        const uint32_t v = src[k];
        dst[k] = run;
        run += v;
    }
    if (threadIdx.x == 0) totals[row] = tot;
}

// Single-block exclusive scan of a short array (<= a few million entries).
__global__ __launch_bounds__(1024) void k_scan_small(const uint32_t* in, uint32_t* out,
                                                     uint32_t len) {
    __shared__ uint32_t tmp[16];
    const uint32_t chunk = (len + 1023) / 1024;
    const uint32_t beg = min(threadIdx.x * chunk, len);
    const uint32_t end = min(beg + chunk, len);
    uint32_t sum = 0;
    for (uint32_t k = beg; k < end; ++k) sum += in[k];
    uint32_t run = block_exclusive_scan<1024>(sum, tmp, nullptr);
    for (uint32_t k = beg; k < end; ++k) {
        const uint32_t v = in[k];
        out[k] = run;
        run += v;
    }
}

__global__ __launch_bounds__(256) void k_add_rows(const uint32_t* row_base, uint32_t* data,
                                                  uint32_t cols) {
    const size_t row = blockIdx.x;
    const uint32_t b = row_base[row];
    for (uint32_t k = threadIdx.x; k < cols; k += 256) data[row * cols + k] += b;
}

// ------------------------------------------------------------------ 3. scatter
// Stable: a tile's elements are ranked in (round, wave, lane) order, which is the
// arrival order; tiles are ordered by the exclusive [bin][tile] scan. The inputs of
// round r+1 are loaded into registers before round r is ranked, so the global-load
// latency hides behind the two LDS barriers of a round.
template <class Codec, bool RAW>
struct ScatterIn;

template <class Codec>
struct ScatterIn<Codec, true> {
    uint64_t key; int64_t now_ns; int32_t permits; uint32_t lim; uint32_t op; uint32_t dig;
    // Every load is unconditional (an absent array reads the key's bytes instead and the
    // value is dropped): a load under a branch leaves the wait-count pass unsure how many
    // loads are in flight, and it then waits for all of them — the whole prefetch ring and
    // every store before it — at the first use of any input.
    __device__ inline void load(const PartArgs& a, uint32_t i) {
        key = ld<kNtScIn>(a.key + i);
        now_ns = ld<kNtScIn>(a.now_ns + i);
        permits = ld<kNtScIn>(a.permits + i);
        const uint16_t* lp = a.limiter ? a.limiter + i : (const uint16_t*)(a.key + i);
        const uint8_t* op_p = a.op ? a.op + i : (const uint8_t*)(a.key + i);
        const uint16_t* dp = a.digit ? a.digit + i : (const uint16_t*)(a.key + i);
        lim = *lp;            // raw: masked where used (a select here would wait for it)
        op = *op_p;
        dig = ld<kNtScIn>(dp);
    }
    __device__ inline uint32_t lim_v(const PartArgs& a) const { return a.limiter ? lim : 0u; }
    __device__ inline uint32_t op_v(const PartArgs& a) const { return a.op ? op : 0u; }
    __device__ inline uint32_t dig_v(const PartArgs& a) const { return a.digit ? dig : 0u; }
};

template <class Codec>
struct ScatterIn<Codec, false> {
    typename Codec::Rec rec;
    __device__ inline void load(const PartArgs& a, uint32_t i) {
        rec = ((const typename Codec::Rec*)a.rec_in)[i];
    }
};

// The record output arrays: routed regions' records go straight to the final array, at a
// uniform element offset from the normal one. Selecting between the two kernel-argument
// pointers per lane let the compiler fold their reads into one vector load from the argument
// segment at a lane-chosen offset, followed by a vmcnt(0) wait in every round (a drain of the
// prefetched loads and of every store in flight); a pointer rebuilt from integers is a flat
// one, whose stores the wait-count pass cannot track either. An offset keeps both out.
template <class Rec>
__device__ inline void scatter_outputs(const PartArgs& a, Rec*& out_norm, int64_t& route_off,
                                       uint32_t& lo_route) {
    out_norm = (Rec*)a.rec_out;
    route_off = a.route_list ? (Rec*)a.rec_out_route - out_norm : 0;
    lo_route = a.route_list ? a.lo_bins : 0xFFFFFFFFu;
}

constexpr int kScatterDepth = 8;   // rounds of inputs in flight (divides tile_items)

template <class Codec, bool RAW>
__global__ __launch_bounds__(kTileThreads) void k_scatter(PartArgs a) {
    using Rec = typename Codec::Rec;
    static_assert(kTileThreads / 64 <= 8, "per-wave counts are packed 8 to a bin");
    // dynamic LDS (scatter_lds_bytes): per bin, this round's per-wave counts packed in one
    // word (cntw), then the next slot (cur); sized to the pass's bins
    extern __shared__ uint64_t dyn_lds64[];
    // this round's count of each wave per bin, the waves' bytes packed in one word: a lane
    // sums the earlier waves' counts for its bin with one read and two v_sad_u8
    __shared__ LimLds L;
    __shared__ uint64_t s_mm[2][kTileThreads / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t bins = a.n_bins_pass ? a.n_bins_pass : 1u << a.digit_bits;
    uint64_t* cntw = dyn_lds64;
    uint32_t* cur = (uint32_t*)(dyn_lds64 + bins);
    load_lim_lds(L, a);
    int64_t base = 0;
    if constexpr (RAW) base = a.ctl->base_ms;
    // later passes partition the normal records only (their count is on device); lanes past
    // it store to the padding past the whole batch (a.n), clear of the routed records
    const uint32_t n = a.n_dev ? *a.n_dev : a.n;
    const uint32_t last = n - 1;
    Rec* out_norm;
    int64_t route_off;
    uint32_t lo_route;
    scatter_outputs(a, out_norm, route_off, lo_route);
    uint64_t mn = ~0ULL, mx = 0;
    bool overflow = false;
    for (uint32_t it = 0;; ++it) {
        const uint32_t tile = tile_at(it, a.n_tiles);
        if (tile >= a.n_tiles) break;
        const uint32_t tile0 = tile * a.tile_items * (uint32_t)kTileThreads;
        if (tile0 >= n) continue;                        // (workgroup-uniform)
        __syncthreads();     // previous tile's LDS users are done
        for (uint32_t b = t; b < bins; b += kTileThreads) {
            cur[b] = cursor_base(a, b, tile) + a.counts[(size_t)b * a.n_tiles + tile];
            cntw[b] = 0;
        }
        // kScatterDepth rounds of inputs in flight; out-of-range lanes re-load element n-1
        // so every wave issues the same loads and stores each round (static vmcnt counting)
        ScatterIn<Codec, RAW> in[kScatterDepth];
#pragma unroll
        for (int k = 0; k < kScatterDepth; ++k) in[k].load(a, min(tile0 + (uint32_t)k * kTileThreads + t, last));
        __syncthreads();
        auto round = [&](const ScatterIn<Codec, RAW>& in, int r) {
            const uint32_t i = tile0 + (uint32_t)r * kTileThreads + t;
            const bool active = i < n;
            Rec rec{};
            uint32_t d = 0;
            if (active) {
                if constexpr (RAW) {
                    uint32_t lim = in.lim_v(a), op = in.op_v(a);
                    const int32_t p = in.permits;
                    const int64_t now_ms = floor_div_ms(in.now_ns);
                    const bool lim_ok = lim < a.n_lim;
                    if (!lim_ok) lim = 0;
                    const bool invalid = !lim_ok || op > 2u || (op == 0u && p <= 0);
                    if (op > 2u) op = 0;
                    const uint64_t h = mix64(in.key);
                    rec = Codec::enc(h, now_ms, base, p, op, lim, invalid);
                    // an invalid request's now is never read: it neither widens the batch's
                    // time range nor rejects the batch for its span
                    if (!invalid) {
                        const int64_t rel = now_ms - base;
                        // only the compact record keeps now relative to base
                        if constexpr (std::is_same<Codec, CodecC>::value)
                            overflow |= rel < 0 || rel > 0xFFFFFFFFLL;
                        const uint64_t k = ord_key(now_ms);
                        mn = k < mn ? k : mn;
                        mx = k > mx ? k : mx;
                    }
                    // routing: the upsweep's digit (route-table lookup done once per request)
                    d = a.digit ? in.dig_v(a)
                                : ((L.base[lim] + region_local(h, a.shard_bits, L.bits[lim]))
                                   >> a.digit_shift) & ((1u << a.digit_bits) - 1);
                } else {
                    rec = in.rec;
                    const uint32_t lim = Codec::limiter_of(rec);
                    d = ((L.base[lim] + region_local(rec.h, a.shard_bits, L.bits[lim]))
                         >> a.digit_shift) & ((1u << a.digit_bits) - 1);
                }
            }
            const uint32_t abl = a.ablate;
            const uint64_t m = (abl & kAblNoMatch) ? (1ULL << lane) : wave_match(d, a.digit_bits, active);
            const uint32_t lr = popc_below(m);
            const uint32_t cnt = (uint32_t)__popcll(m);
            const bool leader = active && lr == 0;
            if (leader) ((uint8_t*)&cntw[d])[wid] = (uint8_t)cnt;
            if (!(abl & kAblNoBarrier)) __syncthreads();
            uint32_t pos = 0;
            if (active) {
                const uint64_t below = wid == 0 ? 0ULL : cntw[d] & ((1ULL << (8 * wid)) - 1);
                pos = cur[d] + lr + __builtin_amdgcn_sad_u8((uint32_t)below, 0u, 0u) +
                      __builtin_amdgcn_sad_u8((uint32_t)(below >> 32), 0u, 0u);
            }
            if (!(abl & kAblNoBarrier)) __syncthreads();
            if (leader) {
                atomicAdd(&cur[d], cnt);
                ((uint8_t*)&cntw[d])[wid] = 0;
            }
            if (abl & (kAblNoMatch | kAblNoBarrier)) pos = min(pos, n - 1);
            // inactive lanes write to the padding slot past n (buffers carry spare entries)
            uint32_t wpos = active ? pos : a.n + t;
            if (abl & kAblSeqRecStore) wpos = active ? i : a.n + t;
            // a routed region's records go straight to the final record array
            Rec* dst = out_norm + ((active && d >= lo_route ? route_off : 0) + wpos);
            if (!(abl & kAblNoRecStore)) st_rec<kNtScRec>(dst, rec);
            if (!(abl & kAblNoPosStore)) st<kNtScPos>(a.pos_out + (active ? i : a.n + t), pos);
        };
        // Unrolled by the prefetch depth so the input registers rotate without moves (a
        // move would wait on its load). vmcnt retires loads and stores in issue order, so
        // waiting for round r's inputs also waits for the scattered stores issued before
        // them: a deep ring spreads that store-ack latency over kScatterDepth rounds.
        for (int r = 0; r < (int)a.tile_items; r += kScatterDepth) {
#pragma unroll
            for (int k = 0; k < kScatterDepth; ++k) {
                round(in[k], r + k);
                in[k].load(a, min(tile0 + (uint32_t)(r + k + kScatterDepth) * kTileThreads + t, last));
            }
        }
    }
    if constexpr (RAW) {
        // min / max now over this workgroup's tiles -> one atomic each
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t a1 = __shfl_xor(mn, o, 64), b1 = __shfl_xor(mx, o, 64);
            mn = a1 < mn ? a1 : mn;
            mx = b1 > mx ? b1 : mx;
        }
        __syncthreads();
        if (lane == 0) { s_mm[0][wid] = mn; s_mm[1][wid] = mx; }
        const bool any_over = __syncthreads_or(overflow);
        if (t == 0) {
            for (int w = 1; w < kTileThreads / 64; ++w) {
                mn = s_mm[0][w] < mn ? s_mm[0][w] : mn;
                mx = s_mm[1][w] > mx ? s_mm[1][w] : mx;
            }
            if (mn != ~0ULL) atomicMin((unsigned long long*)&a.ctl->min_now_key, (unsigned long long)mn);
            if (mx != 0) atomicMax((unsigned long long*)&a.ctl->max_now_key, (unsigned long long)mx);
            if (any_over) atomicOr(&a.ctl->span_overflow, 1u);
        }
    }
}

// ------------------------------------------------------------------ 3b. split scatter
// The same stable partition with the global loads and the stores in different waves. gfx950
// has one vmcnt for vector loads and stores, retired in issue order: in k_scatter a wave's
// wait for its prefetched inputs also waits for the acks of every scattered record store it
// issued before them (no-store ablation on sw_zipf: scatter0 4.8 -> 2.8 ms). Here loader waves
// (threads kTileThreads..2*kTileThreads-1) keep kSplitDepth rounds of inputs in flight,
// encode each round and stage its records and digits in LDS one round ahead; the ranking
// waves (threads 0..kTileThreads-1) read them from LDS, rank, and store — they issue no
// global load inside a tile, so nothing ever waits behind their stores.
constexpr int kSplitDepth = 4;       // loader rounds in flight (divides tile_items)
template <class Codec>
__host__ __device__ inline size_t split_stage_off(uint32_t bins) {     // in u64 words, 16-B aligned
    return ((size_t)bins + (bins + 1) / 2 + 1) & ~(size_t)1;
}
// ABL (measurement-only instantiations, rl_tune ablate bits 20-25; results wrong): 1 no record
// store, 2 no position store, 4 records stored at their input index, 8 no ballot match,
// 16 no encode (the key as the record, digit 0 + lane), 32 whole sectors (each lane its
// record to both halves of its 32-B sector)
template <class Codec, bool RAW, int ABL = 0>
__global__ __launch_bounds__(2 * kTileThreads) void k_scatter_split(PartArgs a) {
    using Rec = typename Codec::Rec;
    constexpr int kRecV = (int)(sizeof(Rec) / 16);
    static_assert(sizeof(Rec) % 16 == 0, "records are whole 16-B vectors");
    extern __shared__ uint64_t dyn_lds64[];
    __shared__ LimLds L;
    __shared__ uint64_t s_mm[2][2 * kTileThreads / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const bool loader = t >= (uint32_t)kTileThreads;          // (wave-uniform)
    const uint32_t lt = loader ? t - (uint32_t)kTileThreads : t;   // element within a round
    const uint32_t bins = a.n_bins_pass ? a.n_bins_pass : 1u << a.digit_bits;
    uint64_t* cntw = dyn_lds64;                               // as k_scatter
    uint32_t* cur = (uint32_t*)(dyn_lds64 + bins);
    Rec* stg = (Rec*)(dyn_lds64 + split_stage_off<Codec>(bins));   // [2][kTileThreads]
    uint16_t* sdg = (uint16_t*)(stg + 2 * kTileThreads);           // [2][kTileThreads]
    load_lim_lds(L, a);
    int64_t base = 0;
    if constexpr (RAW) base = a.ctl->base_ms;
    const uint32_t n = a.n_dev ? *a.n_dev : a.n;
    const uint32_t last = n - 1;
    Rec* out_norm;
    int64_t route_off;
    uint32_t lo_route;
    scatter_outputs(a, out_norm, route_off, lo_route);
    uint64_t mn = ~0ULL, mx = 0;
    bool overflow = false;
    // (loaders) element i's record and digit, as k_scatter's round
    auto encode = [&](const ScatterIn<Codec, RAW>& in, uint32_t i, Rec& rec, uint32_t& d) __attribute__((always_inline)) {
        rec = Rec{};
        d = 0;
        if (i >= n) return;
        if constexpr (RAW && (ABL & 16)) {
            rec.h = in.key;
            d = (i & 63u) % (a.n_bins_pass ? a.n_bins_pass : 1u);
            return;
        }
        if constexpr (RAW) {
            uint32_t lim = in.lim_v(a), op = in.op_v(a);
            const int32_t p = in.permits;
            const int64_t now_ms = floor_div_ms(in.now_ns);
            const bool lim_ok = lim < a.n_lim;
            if (!lim_ok) lim = 0;
            const bool invalid = !lim_ok || op > 2u || (op == 0u && p <= 0);
            if (op > 2u) op = 0;
            const uint64_t h = mix64(in.key);
            rec = Codec::enc(h, now_ms, base, p, op, lim, invalid);
            if (!invalid) {
                const int64_t rel = now_ms - base;
                if constexpr (std::is_same<Codec, CodecC>::value)
                    overflow |= rel < 0 || rel > 0xFFFFFFFFLL;
                const uint64_t k = ord_key(now_ms);
                mn = k < mn ? k : mn;
                mx = k > mx ? k : mx;
            }
            d = a.digit ? in.dig_v(a)
                        : ((L.base[lim] + region_local(h, a.shard_bits, L.bits[lim]))
                           >> a.digit_shift) & ((1u << a.digit_bits) - 1);
        } else {
            rec = in.rec;
            const uint32_t lim = Codec::limiter_of(rec);
            d = ((L.base[lim] + region_local(rec.h, a.shard_bits, L.bits[lim]))
                 >> a.digit_shift) & ((1u << a.digit_bits) - 1);
        }
    };
    for (uint32_t it = 0;; ++it) {
        const uint32_t tile = tile_at(it, a.n_tiles);
        if (tile >= a.n_tiles) break;
        const uint32_t tile0 = tile * a.tile_items * (uint32_t)kTileThreads;
        if (tile0 >= n) continue;                        // (workgroup-uniform)
        __syncthreads();     // previous tile's LDS users are done
        // The two roles run separate loops with the same barriers (1 + 2 per round), so the
        // wait-count pass sees only the loaders' loads on one path and only the rankers'
        // stores on the other. Round r: rankers take round r from stage r & 1 while loaders
        // stage round r + 1 from the register ring (slot (r + 1) % depth) and reload that slot
        // with round r + 1 + depth (past the tile: the next tile's inputs, or element n - 1).
        if (loader) {
            ScatterIn<Codec, RAW> in[kSplitDepth];
            for (uint32_t b = lt; b < bins; b += kTileThreads)
                cur[b] = cursor_base(a, b, tile) + a.counts[(size_t)b * a.n_tiles + tile];
#pragma unroll
            for (int k = 0; k < kSplitDepth; ++k) in[k].load(a, min(tile0 + (uint32_t)k * kTileThreads + lt, last));
            Rec r0;
            uint32_t d0;
            encode(in[0], tile0 + lt, r0, d0);           // round 0 staged before the loop
            stg[lt] = r0;
            sdg[lt] = (uint16_t)d0;
            in[0].load(a, min(tile0 + (uint32_t)kSplitDepth * kTileThreads + lt, last));
            __syncthreads();
            auto stage = [&](int r, ScatterIn<Codec, RAW>& nxt) __attribute__((always_inline)) {
                // (the last round stages the next tile's first, unread: that tile's prologue
                // writes stage 0 again after its first barrier)
                const uint32_t i = tile0 + (uint32_t)(r + 1) * kTileThreads + lt;
                Rec nr;
                uint32_t nd;
                encode(nxt, i, nr, nd);
                const uint32_t sl = (uint32_t)((r + 1) & 1) * kTileThreads + lt;
                stg[sl] = nr;
                sdg[sl] = (uint16_t)nd;
                nxt.load(a, min(i + (uint32_t)kSplitDepth * kTileThreads, last));
                __syncthreads();
                __syncthreads();
            };
            for (int r = 0; r < (int)a.tile_items; r += kSplitDepth) {
#pragma unroll
                for (int k = 0; k < kSplitDepth; ++k) stage(r + k, in[(k + 1) % kSplitDepth]);
            }
        } else {
            for (uint32_t b = lt; b < bins; b += kTileThreads) cntw[b] = 0;
            __syncthreads();
            for (int r = 0; r < (int)a.tile_items; ++r) {
                const uint32_t i = tile0 + (uint32_t)r * kTileThreads + lt;
                const bool active = i < n;
                const uint32_t sl = (uint32_t)(r & 1) * kTileThreads + lt;
                u32x4_t rv[kRecV];                        // the record, kept in registers
#pragma unroll
                for (int k = 0; k < kRecV; ++k) rv[k] = ((const u32x4_t*)stg)[sl * kRecV + k];
                const uint32_t d = sdg[sl];
                const uint64_t m = (ABL & 8) ? (active ? 1ULL << lane : 0ULL) : wave_match(d, a.digit_bits, active);
                const uint32_t lr = popc_below(m);
                const uint32_t cnt = (uint32_t)__popcll(m);
                const bool leader = active && lr == 0;
                if (leader) ((uint8_t*)&cntw[d])[wid] = (uint8_t)cnt;
                __syncthreads();
                uint32_t pos = 0;
                if (active) {
                    const uint64_t below = wid == 0 ? 0ULL : cntw[d] & ((1ULL << (8 * wid)) - 1);
                    pos = cur[d] + lr + __builtin_amdgcn_sad_u8((uint32_t)below, 0u, 0u) +
                          __builtin_amdgcn_sad_u8((uint32_t)(below >> 32), 0u, 0u);
                }
                __syncthreads();
                if (leader) {
                    atomicAdd(&cur[d], cnt);
                    ((uint8_t*)&cntw[d])[wid] = 0;
                }
                const uint32_t wpos = (ABL & 4) ? (active ? i : a.n + lt) : active ? min(pos, last) : a.n + lt;
                Rec* dst = out_norm + ((active && d >= lo_route && !(ABL & 4) ? route_off : 0) + wpos);
                if constexpr ((ABL & 32) && kRecV == 1) {
                    // whole 32-B sectors: the lane writes its record to both halves of its
                    // sector (twice the store lanes, no partial sector)
                    u32x4_t* sec = (u32x4_t*)(out_norm + ((active && d >= lo_route ? route_off : 0) + (wpos & ~1u)));
                    sec[0] = rv[0];
                    sec[1] = rv[0];
                } else if constexpr (!(ABL & 1)) {
#pragma unroll
                    for (int k = 0; k < kRecV; ++k) ((u32x4_t*)dst)[k] = rv[k];
                }
                if constexpr (!(ABL & 2)) st<kNtScPos>(a.pos_out + (active ? i : a.n + lt), pos);
            }
        }
    }
    if constexpr (RAW) {
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t a1 = __shfl_xor(mn, o, 64), b1 = __shfl_xor(mx, o, 64);
            mn = a1 < mn ? a1 : mn;
            mx = b1 > mx ? b1 : mx;
        }
        __syncthreads();
        if (lane == 0) { s_mm[0][wid] = mn; s_mm[1][wid] = mx; }
        const bool any_over = __syncthreads_or(overflow);
        if (t == 0) {
            for (int w = 1; w < 2 * kTileThreads / 64; ++w) {
                mn = s_mm[0][w] < mn ? s_mm[0][w] : mn;
                mx = s_mm[1][w] > mx ? s_mm[1][w] : mx;
            }
            if (mn != ~0ULL) atomicMin((unsigned long long*)&a.ctl->min_now_key, (unsigned long long)mn);
            if (mx != 0) atomicMax((unsigned long long*)&a.ctl->max_now_key, (unsigned long long)mx);
            if (any_over) atomicOr(&a.ctl->span_overflow, 1u);
        }
    }
}

// ------------------------------------------------------------------ 3g. local grouping
// Two-pass batches. Pass 0 partitions by the HIGH dh bits of the region id (bin = region >>
// s0; routed hot regions to bins of their own), so a normal pass-0 bin holds the records of
// 2^s0 consecutive regions in arrival order. The bins are then grouped by region inside their
// own ranges of the final array. A bin is cut into tiles of group_tile_recs records (8192):
//   k_gtiles  tiles per bin (scan) and each tile's bin;
//   k_gcount  one wave per tile: its records per region (wave-private LDS counters);
//   k_gscan   one workgroup per bin: per region, the prefix over the bin's tiles, then the
//             regions' starts (region-major, then tile: stable) -> each tile's cursors and
//             the regions' bounds (rstart / rend: the old k_bin_bounds searches are gone);
//   k_gplace  one wave per tile: rank inside each 64-record round by ballot match, place at
//             the tile's own cursors (no barrier), pos_out[j] = final position.
// A tile's output lands in the bin's window (a few hundred KB) within microseconds, so the
// scattered 16-B record stores complete their sectors while the lines are still in L2 (the
// global second pass spread every bin's runs over the whole batch and left half-written
// sectors: write amplification 1.57x). Tiles rather than one workgroup per bin: the largest
// bins hold ~8x the mean (sw_zipf: 230K records against 30K), and one workgroup per bin made
// the largest set the stage (2.0 ms). pos_out keeps the unpermute's two gathers local.
constexpr int kGroupThreads = 256;
constexpr int kGroupWaves = kGroupThreads / 64;
constexpr int kGroupDepth = 8;                       // rounds of records in flight per wave

__global__ __launch_bounds__(1024) void k_gtiles(GroupArgs a) {
    __shared__ uint32_t tmp[16];
    const uint32_t t = threadIdx.x, nb = a.n_bins0, T = a.tile_recs;
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t b0 = min(t * per, nb), b1 = min(b0 + per, nb);
    const uint32_t S = a.seg_start ? a.n_segs : 1u;
    // (segmented: a bin's runs in segment order, tiles never crossing a run)
    auto run_of = [&](uint32_t b, uint32_t s, uint32_t& st, uint32_t& c) {
        if (a.seg_start) { st = a.seg_start[b * S + s]; c = a.seg_cnt[b * S + s]; }
        else { st = a.bin_base[b]; c = a.bin_total[b]; }
    };
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; ++b)
        for (uint32_t s = 0; s < S; ++s) {
            uint32_t st, c;
            run_of(b, s, st, c);
            sum += (c + T - 1) / T;
        }
    uint32_t tot;
    uint32_t base = block_exclusive_scan<1024>(sum, tmp, &tot);
    for (uint32_t b = b0; b < b1; ++b) {
        a.tile_base[b] = min(base, a.max_tiles);
        for (uint32_t s = 0; s < S; ++s) {
            uint32_t st, c;
            run_of(b, s, st, c);
            const uint32_t nt = (c + T - 1) / T;
            for (uint32_t j = 0; j < nt && base + j < a.max_tiles; ++j) {
                a.tile_bin[base + j] = b;
                if (a.seg_start) {
                    a.tile_beg[base + j] = st + j * T;
                    a.tile_end[base + j] = st + min((j + 1) * T, c);
                }
            }
            base += nt;
        }
    }
    if (t == 0) a.tile_base[nb] = min(tot, a.max_tiles);
}

// (tile t of the batch: bin, first record, end)
__device__ inline void group_tile(const GroupArgs& a, uint32_t t, uint32_t& b, uint32_t& beg,
                                  uint32_t& end) {
    b = a.tile_bin[t];
    if (a.seg_start) {
        beg = a.tile_beg[t];
        end = a.tile_end[t];
        return;
    }
    const uint32_t j = t - a.tile_base[b];
    const uint32_t bb = a.bin_base[b], be = bb + a.bin_total[b];
    beg = bb + j * a.tile_recs;
    end = min(beg + a.tile_recs, be);
}

template <class Codec>
struct GroupSub {                                    // a record's region inside its bin
    uint32_t base[256];
    uint8_t bits[256];
    __device__ inline void load(const GroupArgs& a) {
        for (uint32_t l = threadIdx.x; l < a.n_lim; l += blockDim.x) {
            base[l] = a.lims[l].region_base;
            bits[l] = (uint8_t)a.lims[l].region_bits;
        }
    }
    __device__ inline uint32_t of(const GroupArgs& a, const typename Codec::Rec& r, uint32_t smask) const {
        const uint32_t lim = Codec::limiter_of(r);
        return (base[lim] + region_local(r.h, a.shard_bits, bits[lim])) & smask;
    }
};

template <class Codec>
__global__ __launch_bounds__(kGroupThreads) void k_gcount(GroupArgs a) {
    using Rec = typename Codec::Rec;
    extern __shared__ uint32_t gl[];                 // [waves][2^s0]
    __shared__ GroupSub<Codec> G;
    G.load(a);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t nsub = 1u << a.sub_bits, smask = nsub - 1u;
    uint32_t* cw = gl + wid * nsub;
    const Rec* __restrict__ in = (const Rec*)a.rec_in;
    const uint32_t n_t = a.tile_base[a.n_bins0];
    for (uint32_t t = blockIdx.x * kGroupWaves + wid; t < n_t; t += gridDim.x * kGroupWaves) {
        uint32_t b, beg, end;
        group_tile(a, t, b, beg, end);
        for (uint32_t k = lane; k < nsub; k += 64) cw[k] = 0;
        wave_fence();
        for (uint32_t i0 = beg; i0 < end; i0 += 64 * kGroupDepth) {
            Rec r[kGroupDepth];
#pragma unroll
            for (int k = 0; k < kGroupDepth; ++k) {
                const uint32_t i = i0 + (uint32_t)k * 64 + lane;
                r[k] = ld_rec<kNtRgRec>(in + (i < end ? i : end - 1));
            }
#pragma unroll
            for (int k = 0; k < kGroupDepth; ++k)
                if (i0 + (uint32_t)k * 64 + lane < end) atomicAdd(&cw[G.of(a, r[k], smask)], 1u);
        }
        wave_fence();
        uint32_t* dst = a.tcount + (size_t)t * nsub;
        for (uint32_t k = lane; k < nsub; k += 64) dst[k] = cw[k];
        wave_fence();
    }
}

__global__ __launch_bounds__(kGroupThreads) void k_gscan(GroupArgs a) {
    extern __shared__ uint32_t tot[];                // [2^s0] the regions' record counts
    __shared__ uint32_t tmp[kGroupWaves];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t nsub = 1u << a.sub_bits;
    const uint32_t t0 = a.tile_base[b], t1 = a.tile_base[b + 1 <= a.n_bins0 ? b + 1 : b];
    // per region: the prefix over the bin's tiles (in place)
    for (uint32_t k = t; k < nsub; k += kGroupThreads) {
        uint32_t run = 0;
        for (uint32_t j = t0; j < t1; ++j) {
            uint32_t* c = a.tcount + (size_t)j * nsub + k;
            const uint32_t v = *c;
            *c = run;
            run += v;
        }
        tot[k] = run;
    }
    __syncthreads();
    // the regions' starts: a contiguous chunk of regions per thread, one block scan
    const uint32_t per = (nsub + kGroupThreads - 1) / kGroupThreads;
    const uint32_t k0 = min(t * per, nsub), k1 = min(k0 + per, nsub);
    uint32_t sum = 0;
    for (uint32_t k = k0; k < k1; ++k) sum += tot[k];
    uint32_t run = a.bin_base[b] + block_exclusive_scan<kGroupThreads>(sum, tmp, nullptr);
    const uint32_t g0 = b << a.sub_bits;
    for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t c = tot[k];
        tot[k] = run;
        if (g0 + k < a.n_regions) {
            a.rstart[g0 + k] = run;
            a.rend[g0 + k] = run + c;
        }
        run += c;
    }
    __syncthreads();
    for (uint32_t k = t; k < nsub; k += kGroupThreads) {
        const uint32_t st = tot[k];
        for (uint32_t j = t0; j < t1; ++j) a.tcount[(size_t)j * nsub + k] += st;
    }
}

template <class Codec>
__global__ __launch_bounds__(kGroupThreads) void k_gplace(GroupArgs a) {
    using Rec = typename Codec::Rec;
    extern __shared__ uint32_t gl[];                 // [waves][2^s0]: the tile's cursors
    __shared__ GroupSub<Codec> G;
    G.load(a);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t nsub = 1u << a.sub_bits, smask = nsub - 1u;
    uint32_t* cw = gl + wid * nsub;
    const Rec* __restrict__ in = (const Rec*)a.rec_in;
    Rec* __restrict__ out = (Rec*)a.rec_out;
    const uint32_t n_t = a.tile_base[a.n_bins0];
    // Every lane loads and stores in every round (past the tile's end: the last record again,
    // stored to the padding past the batch), and the next rounds' records are loaded before
    // this round's stores: with no memory operation under a branch the wait-count pass counts
    // statically, so waiting for a round's records does not drain the stores issued before it
    // (one vmcnt for both on gfx950).
    const uint32_t pad = a.pad + lane;
    for (uint32_t t = blockIdx.x * kGroupWaves + wid; t < n_t; t += gridDim.x * kGroupWaves) {
        uint32_t b, beg, end;
        group_tile(a, t, b, beg, end);
        const uint32_t* src = a.tcount + (size_t)t * nsub;
        for (uint32_t k = lane; k < nsub; k += 64) cw[k] = src[k];
        wave_fence();
        auto load = [&](Rec (&r)[kGroupDepth], uint32_t i0) {
#pragma unroll
            for (int k = 0; k < kGroupDepth; ++k) {
                const uint32_t i = i0 + (uint32_t)k * 64 + lane;
                r[k] = ld_rec<kNtRgRec>(in + (i < end ? i : end - 1));
            }
        };
        auto place = [&](const Rec (&r)[kGroupDepth], uint32_t i0) {
#pragma unroll
            for (int k = 0; k < kGroupDepth; ++k) {
                const uint32_t i = i0 + (uint32_t)k * 64 + lane;
                const bool act = i < end;
                const uint32_t sb = act ? G.of(a, r[k], smask) : 0u;
                const uint64_t m = wave_match(sb, (int)a.sub_bits, act);
                const uint32_t lr = popc_below(m);
                const uint32_t pos = cw[sb] + lr;
                wave_fence();                            // every lane has read its cursor
                if (act && lr == 0) cw[sb] = pos + (uint32_t)__popcll(m);
                wave_fence();
                const uint32_t wp = (a.ablate & kAblGroupSeq) ? i : pos;
                st_rec<false>(out + (act ? wp : pad), r[k]);    // (temporal: sectors merge in L2)
                st<kNtScPos>(a.pos_out + (act ? i : pad), act ? pos : 0u);
            }
        };
        Rec ra[kGroupDepth], rb[kGroupDepth];
        load(ra, beg);
        for (uint32_t i0 = beg; i0 < end; i0 += 128 * kGroupDepth) {
            load(rb, i0 + 64 * kGroupDepth);
            place(ra, i0);
            if (i0 + 64 * kGroupDepth >= end) break;     // (wave-uniform)
            load(ra, i0 + 128 * kGroupDepth);
            place(rb, i0 + 64 * kGroupDepth);
        }
        wave_fence();
    }
}

// k_gplace with the tile's records sorted by region in LDS first, in chunks of kGChunk: the
// global stores then go out as runs of consecutive records per region (a wave-instruction
// covers a few lines instead of 64 scattered 16-B pieces: with every record scattered,
// k_gplace ran 1.5 ms on sw_zipf, with the same stores made contiguous 0.9 ms). Each wave
// ranks its own 256 records of the chunk (4 rounds, ballot match, wave-private counts), the
// counts are scanned region-major then wave (stable), records go to their sorted slot in
// LDS, and the chunk is written out in sorted order; the tile's cursors advance per chunk.
// For bins of up to 2^kGLdsMaxSub regions (wider ones take k_gplace).
constexpr int kGPThreads = 512;
constexpr int kGPWaves = kGPThreads / 64;
constexpr uint32_t kGChunk = 2048;                   // records sorted in LDS at once
constexpr uint32_t kGLdsMaxSub = 10;
template <class Rec>
__host__ __device__ inline size_t gplace_lds_bytes(uint32_t sub_bits) {
    const size_t nsub = (size_t)1 << sub_bits;
    return kGChunk * sizeof(Rec) + kGChunk * 2 + kGPWaves * nsub * 2 + 2 * nsub * 4;
}
template <class Codec>
__global__ __launch_bounds__(kGPThreads) void k_gplace_lds(GroupArgs a) {
    using Rec = typename Codec::Rec;
    extern __shared__ uint4 glds[];
    __shared__ GroupSub<Codec> G;
    __shared__ uint32_t s_tmp[kGPWaves];
    const uint32_t t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t nsub = 1u << a.sub_bits, smask = nsub - 1u;
    Rec* stg = (Rec*)glds;                            // [kGChunk] the chunk, sorted
    uint16_t* ssub = (uint16_t*)(stg + kGChunk);      // [kGChunk] their regions
    uint16_t* hist = ssub + kGChunk;                  // [waves][nsub] counts, then wave prefixes
    uint32_t* tsub = (uint32_t*)(hist + kGPWaves * nsub);   // [nsub] chunk-local region starts
    uint32_t* gcur = tsub + nsub;                     // [nsub] the tile's global cursors
    G.load(a);
    const Rec* __restrict__ in = (const Rec*)a.rec_in;
    Rec* __restrict__ out = (Rec*)a.rec_out;
    const uint32_t n_t = a.tile_base[a.n_bins0];
    const uint32_t per = (nsub + kGPThreads - 1) / kGPThreads;
    const uint32_t k0 = min(t * per, nsub), k1 = min(k0 + per, nsub);
    for (uint32_t tt = blockIdx.x; tt < n_t; tt += gridDim.x) {
        uint32_t b, beg, end;
        group_tile(a, tt, b, beg, end);
        __syncthreads();                              // the previous tile's readers are done
        for (uint32_t k = t; k < nsub; k += kGPThreads) gcur[k] = a.tcount[(size_t)tt * nsub + k];
        for (uint32_t c0 = beg; c0 < end; c0 += kGChunk) {
            const uint32_t c1 = min(c0 + kGChunk, end);
            for (uint32_t k = t; k < kGPWaves * nsub; k += kGPThreads) hist[k] = 0;
            // this wave's 256 records of the chunk: 4 rounds, loaded together
            const uint32_t w0 = c0 + wid * 256u;
            Rec r[4];
            uint32_t sb[4], wr[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t j = w0 + (uint32_t)q * 64 + lane;
                r[q] = ld_rec<kNtRgRec>(in + (j < c1 ? j : c1 - 1));
            }
            __syncthreads();                          // hist zeroed (and gcur loaded)
            uint16_t* hw = hist + wid * nsub;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t j = w0 + (uint32_t)q * 64 + lane;
                const bool act = j < c1;
                sb[q] = act ? G.of(a, r[q], smask) : 0u;
                const uint64_t m = wave_match(sb[q], (int)a.sub_bits, act);
                const uint32_t lr = popc_below(m);
                wr[q] = (uint32_t)hw[sb[q]] + lr;    // rank among this wave's records of the region
                wave_fence();
                if (act && lr == 0) hw[sb[q]] = (uint16_t)(wr[q] + (uint32_t)__popcll(m));
                wave_fence();
            }
            __syncthreads();
            // region-major, then wave: each region's start in the chunk, each wave's offset in it
            uint32_t sum = 0;
            for (uint32_t k = k0; k < k1; ++k) {
                uint32_t run = 0;
                for (uint32_t w = 0; w < (uint32_t)kGPWaves; ++w) {
                    const uint32_t v = hist[w * nsub + k];
                    hist[w * nsub + k] = (uint16_t)run;
                    run += v;
                }
                tsub[k] = run;                        // (the region's count, for now)
                sum += run;
            }
            uint32_t base = block_exclusive_scan<kGPThreads>(sum, s_tmp, nullptr);
            for (uint32_t k = k0; k < k1; ++k) {
                const uint32_t c = tsub[k];
                tsub[k] = base;
                base += c;
            }
            __syncthreads();
            // sorted slots in LDS; the final position of every pass-0 position
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t j = w0 + (uint32_t)q * 64 + lane;
                if (j < c1) {
                    const uint32_t o = (uint32_t)hist[wid * nsub + sb[q]] + wr[q];
                    stg[tsub[sb[q]] + o] = r[q];
                    ssub[tsub[sb[q]] + o] = (uint16_t)sb[q];
                    st<kNtScPos>(a.pos_out + j, gcur[sb[q]] + o);
                }
            }
            __syncthreads();
            // the chunk in sorted order: runs of consecutive records per region
            for (uint32_t i = t; i < c1 - c0; i += kGPThreads) {
                const uint32_t k = ssub[i];
                st_rec<false>(out + gcur[k] + (i - tsub[k]), stg[i]);
            }
            __syncthreads();
            // the tile's cursors past this chunk
            for (uint32_t k = k0; k < k1; ++k) {
                const uint32_t nx = k + 1 < nsub ? tsub[k + 1] : c1 - c0;
                gcur[k] += nx - tsub[k];
            }
        }
    }
}

// ------------------------------------------------------------------ segmented pass 0
// From the row-scanned counts (exclusive prefix per bin over the tiles): each (bin, segment)
// run's count, its start — normal bins segment-major over [0, n_normal), routed bins
// bin-major after them, exactly where the unsegmented layout put them — and the cursor
// base a tile of that segment adds to its row prefix (seg_adj = start - prefix at the
// segment's first tile; modular arithmetic).
__global__ __launch_bounds__(1024) void k_seg_base(const uint32_t* __restrict__ counts,
                                                   const uint32_t* __restrict__ bin_total,
                                                   const uint32_t* __restrict__ bin_base,
                                                   uint32_t bins, uint32_t lo, uint32_t nt,
                                                   uint32_t seg_tiles, uint32_t S, uint32_t* seg_adj,
                                                   uint32_t* seg_start, uint32_t* seg_cnt) {
    __shared__ uint32_t tmp[16];
    auto pre = [&](uint32_t b, uint32_t s) -> uint32_t {
        const uint32_t t0 = s * seg_tiles;
        return t0 < nt ? counts[(size_t)b * nt + t0] : bin_total[b];
    };
    const uint32_t N = S * lo;
    const uint32_t per = (N + 1023) / 1024;
    const uint32_t i0 = min(threadIdx.x * per, N), i1 = min(i0 + per, N);
    uint32_t sum = 0;
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t s = i / lo, b = i % lo;
        sum += pre(b, s + 1) - pre(b, s);
    }
    uint32_t run = block_exclusive_scan<1024>(sum, tmp, nullptr);
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t s = i / lo, b = i % lo;
        const uint32_t p0 = pre(b, s), c = pre(b, s + 1) - p0;
        seg_start[b * S + s] = run;
        seg_cnt[b * S + s] = c;
        seg_adj[b * S + s] = run - p0;
        run += c;
    }
    for (uint32_t b = lo + threadIdx.x; b < bins; b += 1024)
        for (uint32_t s = 0; s < S; ++s) {
            const uint32_t p0 = pre(b, s);
            seg_adj[b * S + s] = bin_base[b];
            seg_start[b * S + s] = bin_base[b] + p0;
            seg_cnt[b * S + s] = pre(b, s + 1) - p0;
        }
}

hipError_t launch_seg_base(const uint32_t* counts, const uint32_t* bin_total,
                           const uint32_t* bin_base, uint32_t bins, uint32_t lo_bins,
                           uint32_t n_tiles, uint32_t seg_tiles, uint32_t n_segs,
                           uint32_t* seg_adj, uint32_t* seg_start, uint32_t* seg_cnt, hipStream_t s) {
    if (seg_tiles == 0 || (size_t)(n_segs - 1) * seg_tiles >= n_tiles || lo_bins > bins)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_seg_base, dim3(1), dim3(1024), 0, s, counts, bin_total, bin_base, bins,
                       lo_bins, n_tiles, seg_tiles, n_segs, seg_adj, seg_start, seg_cnt);
    return hipGetLastError();
}

// ------------------------------------------------------------------ routing helpers
// After the pass-0 scan: the routed bins' ranges (pass 1 reuses bin_base / bin_total) and
// the number of normal records, which pass 1 and the unpermute read on device.
__global__ __launch_bounds__(1024) void k_route_ranges(const uint32_t* __restrict__ route_list,
                                                       const uint32_t* __restrict__ bin_base,
                                                       const uint32_t* __restrict__ bin_total,
                                                       uint32_t lo_bins, uint32_t* route_start,
                                                       uint32_t* route_cnt, BatchCtl* ctl) {
    for (uint32_t i = threadIdx.x; i < kRouteSlots; i += blockDim.x) {
        const bool used = route_list[i] != kNone;
        const uint32_t bn = lo_bins + (used ? route_list[kRouteSlots + i] : 0u);
        route_start[i] = used ? bin_base[bn] : 0u;
        route_cnt[i] = used ? bin_total[bn] : 0u;
    }
    if (threadIdx.x == 0) ctl->n_normal = bin_base[lo_bins];
}

// ------------------------------------------------------------------ 5. unpermute
template <class Res>
__global__ __launch_bounds__(kTileThreads) void k_unpermute(UnpermArgs a) {
  const uint32_t t = threadIdx.x;
  const Res* __restrict__ res = (const Res*)a.res;
  const uint32_t* __restrict__ pos0 = a.pos0;
  const uint32_t* __restrict__ pos1 = a.pos1;
  uint8_t* __restrict__ allowed = a.allowed;
  int64_t* __restrict__ remaining = a.remaining;
  constexpr int B = 8;                         // rounds per batch (loads issued together)
  constexpr int NB = kTileItems / B;
  const bool simple = pos1 || a.tokens_out || (a.ablate & kAblNoGather);
  // two-pass batches: mid (res) holds the normal records' results in pass-0 order, res_hi
  // the routed records' results at their own (pass-0) positions >= n_normal
  const Res* __restrict__ res_hi = (const Res*)a.res_hi;
  const uint32_t nn = res_hi ? a.ctl->n_normal : 0u;
  for (uint32_t it = 0;; ++it) {
    const uint32_t tile = tile_at(it, a.n_tiles);
    if (tile >= a.n_tiles) break;
    const uint32_t tbase = tile * (uint32_t)kTile + t;
    if (!simple && tile * (uint64_t)kTile + kTile <= a.n) {
        // Full tile, one result array: software-pipelined so that every wait is for loads
        // issued a batch earlier and never directly behind the previous batch's stores
        // (vmcnt retires loads and stores in issue order).
        uint32_t pE[B], pO[B];
        Res vE[B], vO[B];
        auto load = [&](uint32_t (&p)[B], int b) {
#pragma unroll
            for (int k = 0; k < B; ++k) p[k] = ld<kNtUn>(pos0 + tbase + (uint32_t)(b * B + k) * kTileThreads);
        };
        auto gather = [&](Res (&v)[B], const uint32_t (&p)[B]) {
#pragma unroll
            for (int k = 0; k < B; ++k) v[k] = (res_hi && p[k] >= nn ? res_hi : res)[p[k]];
        };
        auto store = [&](const Res (&v)[B], int b) {
#pragma unroll
            for (int k = 0; k < B; ++k) {
                const uint32_t i = tbase + (uint32_t)(b * B + k) * kTileThreads;
                st<kNtUn>(allowed + i, (uint8_t)(v[k] & 1u));
                st<kNtUn>(remaining + i, (int64_t)(v[k] >> 1) - kResBias);
            }
        };
        load(pE, 0);
        for (int b = 0; b < NB; b += 2) {
            gather(vE, pE);
            load(pO, b + 1);
            if (b > 0) store(vO, b - 1);
            gather(vO, pO);
            load(pE, (b + 2) % NB);                 // unconditional (last one unused)
            store(vE, b);
        }
        store(vO, NB - 1);
        continue;
    }
    for (int r0 = 0; r0 < kTileItems; r0 += B) {
        uint32_t p[B];
        Res v[B];
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const uint32_t i = tile * (uint32_t)kTile + (uint32_t)(r0 + k) * kTileThreads + t;
            p[k] = pos0[i < a.n ? i : 0];
        }
        if (pos1) {
            // pass 1 moved the normal records only; routed ones kept their pass-0 position
            const uint32_t nn = a.ctl->n_normal;
#pragma unroll
            for (int k = 0; k < B; ++k) p[k] = p[k] < nn ? pos1[p[k]] : p[k];
        }
        if (a.ablate & kAblNoGather) {
#pragma unroll
            for (int k = 0; k < B; ++k) v[k] = (Res)p[k];
        } else {
#pragma unroll
            for (int k = 0; k < B; ++k) v[k] = (res_hi && p[k] >= nn ? res_hi : res)[p[k]];
        }
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const uint32_t i = tile * (uint32_t)kTile + (uint32_t)(r0 + k) * kTileThreads + t;
            if (i < a.n) {
                allowed[i] = (uint8_t)(v[k] & 1u);
                remaining[i] = (int64_t)(v[k] >> 1) - kResBias;
                if (a.tokens_out) a.tokens_out[i] = a.tok ? a.tok[p[k]] : __builtin_nan("");
            }
        }
    }
  }
  if (a.ctl && a.ctl->n_esc != 0) {
    // Rare (TB balances below -3 after time regression): the gather above decoded the
    // escape code as (allowed 1, remaining -3); rewrite those results from the side array.
    // Same tiles, same thread per element as above, so the rewrite follows the first store.
    const Res* rf = (const Res*)a.res_final;
    for (uint32_t it = 0;; ++it) {
      const uint32_t tile = tile_at(it, a.n_tiles);
      if (tile >= a.n_tiles) break;
      for (int r = 0; r < kTileItems; ++r) {
        const uint32_t i = tile * (uint32_t)kTile + (uint32_t)r * kTileThreads + t;
        if (i >= a.n) break;
        uint32_t j = pos0[i];
        if (a.pos1_final && j < a.ctl->n_normal) j = a.pos1_final[j];
        if ((uint64_t)rf[j] == kResEscape) {
          allowed[i] = 0;
          remaining[i] = a.ext[j];
        }
      }
    }
  }
}

// Split unpermute (rl_tune unpermute_split): the position reads and result gathers in loader
// waves (threads kTileThreads..), the decision stores in storer waves, one round apart through
// LDS, so that no wait for a gather sits behind the acks of earlier stores (one vmcnt for both
// on gfx950). Loaders keep kUnPosDepth rounds of positions and kUnGatherDepth rounds of
// gathers in flight. One-array batches only (no pos1 pass, no tokens): k_unpermute otherwise.
constexpr int kUnPosDepth = 8, kUnGatherDepth = 4;
template <class Res>
__global__ __launch_bounds__(2 * kTileThreads) void k_unpermute_split(UnpermArgs a) {
    __shared__ Res stage[2][kTileThreads];
    const uint32_t t = threadIdx.x;
    const bool loader = t >= (uint32_t)kTileThreads;          // (wave-uniform)
    const uint32_t lt = loader ? t - (uint32_t)kTileThreads : t;
    const Res* __restrict__ res = (const Res*)a.res;
    const Res* __restrict__ res_hi = (const Res*)a.res_hi;
    const uint32_t nn = res_hi ? a.ctl->n_normal : 0u;
    const uint32_t last = a.n - 1;
    for (uint32_t it = 0;; ++it) {
        const uint32_t tile = tile_at(it, a.n_tiles);
        if (tile >= a.n_tiles) break;
        const uint32_t tbase = tile * (uint32_t)kTile + lt;
        __syncthreads();                                      // last tile's stage readers are done
        if (loader) {
            uint32_t P[kUnPosDepth];
            Res V[kUnGatherDepth];
            auto pos_of = [&](int r) { return ld<kNtUn>(a.pos0 + min(tbase + (uint32_t)r * kTileThreads, last)); };
            auto gather = [&](uint32_t p) { return (res_hi && p >= nn ? res_hi : res)[p]; };
#pragma unroll
            for (int k = 0; k < kUnPosDepth; ++k) P[k] = pos_of(k);
#pragma unroll
            for (int k = 0; k < kUnGatherDepth; ++k) {
                V[k] = gather(P[k]);
                P[k] = pos_of(k + kUnPosDepth);
            }
            // round r: stage round r's results; gather round r + G (its position, slot
            // (r + G) % D, arrived); reload that slot with round r + G + D
            for (int r0 = 0; r0 < kTileItems; r0 += kUnPosDepth) {
#pragma unroll
                for (int k = 0; k < kUnPosDepth; ++k) {
                    const int r = r0 + k;
                    stage[r & 1][lt] = V[k % kUnGatherDepth];
                    V[k % kUnGatherDepth] = gather(P[(k + kUnGatherDepth) % kUnPosDepth]);
                    P[(k + kUnGatherDepth) % kUnPosDepth] = pos_of(r + kUnGatherDepth + kUnPosDepth);
                    __syncthreads();
                }
            }
        } else {
            for (int r = 0; r < kTileItems; ++r) {
                __syncthreads();
                const Res v = stage[r & 1][lt];
                const uint32_t i = tbase + (uint32_t)r * kTileThreads;
                if (i < a.n) {
                    st<kNtUn>(a.allowed + i, (uint8_t)(v & 1u));
                    st<kNtUn>(a.remaining + i, (int64_t)(v >> 1) - kResBias);
                }
            }
        }
    }
    if (!loader && a.ctl && a.ctl->n_esc != 0) {
        // as k_unpermute: the escape code decoded as (allowed 1, remaining -3) is rewritten
        // from the side array by the thread that stored it
        const Res* rf = (const Res*)a.res_final;
        for (uint32_t it = 0;; ++it) {
            const uint32_t tile = tile_at(it, a.n_tiles);
            if (tile >= a.n_tiles) break;
            for (int r = 0; r < kTileItems; ++r) {
                const uint32_t i = tile * (uint32_t)kTile + (uint32_t)r * kTileThreads + t;
                if (i >= a.n) break;
                uint32_t j = a.pos0[i];
                if (a.pos1_final && j < a.ctl->n_normal) j = a.pos1_final[j];
                if ((uint64_t)rf[j] == kResEscape) {
                    a.allowed[i] = 0;
                    a.remaining[i] = a.ext[j];
                }
            }
        }
    }
}

// Two-pass batches: undo the high-digit pass first. mid[j] = res[pos1[j]] for j in
// pass-0 order: pos1 is read in order and, since pass 0 left the records sorted by low
// digit, consecutive j fall into one low-digit run whose elements go to the 2^d1
// high-digit bins in order — the gather walks 2^d1 sequential streams instead of the
// whole result array. k_unpermute then gathers mid[pos0[i]] (2^d0 streams). Two
// local gathers replace the composed res[pos1[pos0[i]]], which hit a random line of a
// 1 GB index and of the result array per request.
// Routed records (pass-0 positions >= ctl->n_normal) skipped pass 1: k_unpermute reads
// their results in place (UnpermArgs::res_hi), so mid covers the normal records only.
template <class Res>
__global__ __launch_bounds__(256) void k_unpermute_mid(const uint32_t* __restrict__ pos1,
                                                       const Res* __restrict__ res,
                                                       Res* __restrict__ mid, uint32_t n,
                                                       const BatchCtl* __restrict__ ctl, uint32_t xcd) {
    constexpr int B = 8;
    // consecutive blocks of j on one XCD: a pass-0 bin's 2^d1 result streams are then read
    // through one L2 instead of being fetched into all eight
    const uint32_t base = (xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x) * (256u * B) + threadIdx.x;
    n = min(n, ctl->n_normal);
    if (base >= n) return;
    uint32_t p[B];
#pragma unroll
    for (int k = 0; k < B; ++k) {
        const uint32_t j = base + (uint32_t)k * 256u;
        p[k] = pos1[j < n ? j : base];
    }
    Res v[B];
#pragma unroll
    for (int k = 0; k < B; ++k) v[k] = res[p[k]];
#pragma unroll
    for (int k = 0; k < B; ++k) {
        const uint32_t j = base + (uint32_t)k * 256u;
        if (j < n) mid[j] = v[k];
    }
}

__global__ void k_fill_invalid(uint8_t* allowed, int64_t* remaining, double* tok, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        allowed[i] = 0;
        remaining[i] = kRemInvalid;
        if (tok) tok[i] = __builtin_nan("");
    }
}


hipError_t launch_upsweep(const PartArgs& a, bool raw, bool wide, hipStream_t s) {
    dim3 grid(persistent_grid(a.n_tiles, a.up_per_cu ? a.up_per_cu : 4)), block(kTileThreads);
    const uint32_t bins = a.n_bins_pass ? a.n_bins_pass : 1u << a.digit_bits;
    if (bins > (1u << kMaxDigitBits)) return hipErrorInvalidValue;
    const size_t lds = bins * sizeof(uint32_t) + (a.route_list ? sizeof(RouteLds) : 0);
    if (raw && a.digit) {
        if (wide) hipLaunchKernelGGL((k_upsweep<CodecW, true, true>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((k_upsweep<CodecC, true, true>), grid, block, lds, s, a);
    } else if (raw) {
        if (wide) hipLaunchKernelGGL((k_upsweep<CodecW, true, false>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((k_upsweep<CodecC, true, false>), grid, block, lds, s, a);
    } else {
        return hipErrorInvalidValue;         // (record-input passes: k_group since round 6)
    }
    return hipGetLastError();
}

hipError_t launch_scatter(const PartArgs& a, bool raw, bool wide, hipStream_t s) {
    dim3 grid(persistent_grid(a.n_tiles, a.sc_per_cu ? a.sc_per_cu : 1)), block(kTileThreads);
    const uint32_t bins = a.n_bins_pass ? a.n_bins_pass : 1u << a.digit_bits;
    if (bins > (1u << kMaxDigitBits)) return hipErrorInvalidValue;
    if (a.sc_split && (a.ablate >> 20) && raw && !wide) {   // measurement-only variants
        const dim3 b2(2 * kTileThreads);
        const size_t lc = split_stage_off<CodecC>(bins) * 8 + 2 * kTileThreads * (sizeof(RecC) + 2);
        switch ((a.ablate >> 20) & 63u) {
            case 1: hipLaunchKernelGGL((k_scatter_split<CodecC, true, 1>), grid, b2, lc, s, a); break;
            case 2: hipLaunchKernelGGL((k_scatter_split<CodecC, true, 2>), grid, b2, lc, s, a); break;
            case 3: hipLaunchKernelGGL((k_scatter_split<CodecC, true, 3>), grid, b2, lc, s, a); break;
            case 4: hipLaunchKernelGGL((k_scatter_split<CodecC, true, 4>), grid, b2, lc, s, a); break;
            case 8: hipLaunchKernelGGL((k_scatter_split<CodecC, true, 8>), grid, b2, lc, s, a); break;
            case 16: hipLaunchKernelGGL((k_scatter_split<CodecC, true, 16>), grid, b2, lc, s, a); break;
            case 27: hipLaunchKernelGGL((k_scatter_split<CodecC, true, 27>), grid, b2, lc, s, a); break;
            case 32: hipLaunchKernelGGL((k_scatter_split<CodecC, true, 32>), grid, b2, lc, s, a); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (a.sc_split && !a.ablate) {
        const dim3 b2(2 * kTileThreads);
        const size_t lc = split_stage_off<CodecC>(bins) * 8 + 2 * kTileThreads * (sizeof(RecC) + 2);
        const size_t lw = split_stage_off<CodecW>(bins) * 8 + 2 * kTileThreads * (sizeof(RecW) + 2);
        if (!raw) return hipErrorInvalidValue;   // (record-input passes: k_group since round 6)
        if (wide) hipLaunchKernelGGL((k_scatter_split<CodecW, true>), grid, b2, lw, s, a);
        else hipLaunchKernelGGL((k_scatter_split<CodecC, true>), grid, b2, lc, s, a);
        return hipGetLastError();
    }
    const size_t lds = bins * (sizeof(uint64_t) + sizeof(uint32_t));
    if (!raw) return hipErrorInvalidValue;
    if (wide) hipLaunchKernelGGL((k_scatter<CodecW, true>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((k_scatter<CodecC, true>), grid, block, lds, s, a);
    return hipGetLastError();
}

hipError_t launch_scan_rows(const uint32_t* in, uint32_t* out, uint32_t rows, uint32_t cols,
                            uint32_t* totals, hipStream_t s) {
    hipLaunchKernelGGL(k_scan_rows, dim3(rows), dim3(256), 0, s, in, out, cols, totals);
    return hipGetLastError();
}

hipError_t launch_scan_small(const uint32_t* in, uint32_t* out, uint32_t len, hipStream_t s) {
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, s, in, out, len);
    return hipGetLastError();
}

hipError_t launch_add_rows(const uint32_t* row_base, uint32_t* data, uint32_t rows,
                           uint32_t cols, hipStream_t s) {
    hipLaunchKernelGGL(k_add_rows, dim3(rows), dim3(256), 0, s, row_base, data, cols);
    return hipGetLastError();
}

// Fold the sharded batch counters into BatchCtl and clear them for the next batch.
__global__ __launch_bounds__(256) void k_stats_reduce(unsigned long long* stats, BatchCtl* ctl) {
    __shared__ unsigned long long part[kStWords][4];
    const uint32_t t = threadIdx.x, lane = t & 63, wid = t >> 6;
    unsigned long long acc[kStCount] = {};
    for (uint32_t s = t; s < kStatSlots; s += 256) {
        unsigned long long* p = stats + (size_t)s * kStWords;
#pragma unroll
        for (int k = 0; k < (int)kStCount; ++k) { acc[k] += p[k]; p[k] = 0; }
    }
#pragma unroll
    for (int k = 0; k < (int)kStCount; ++k) {
        unsigned long long v = acc[k];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) part[k][wid] = v;
    }
    __syncthreads();
    if (t < kStCount) {
        const unsigned long long v = part[t][0] + part[t][1] + part[t][2] + part[t][3];
        unsigned long long* dst = t == kStAllowed ? &ctl->allowed : t == kStInvalid ? &ctl->invalid
                                : t == kStCapErr ? &ctl->cap_err : t == kStDistinct ? &ctl->distinct
                                : t == kStRegions ? &ctl->regions : t == kStCacheHits ? &ctl->cache_hits
                                : &ctl->table_bytes;
        *dst += v;
    }
}

hipError_t launch_stats_reduce(unsigned long long* stats, BatchCtl* ctl, hipStream_t s) {
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(256), 0, s, stats, ctl);
    return hipGetLastError();
}

hipError_t launch_group(const GroupArgs& a, bool wide, hipStream_t s) {
    if (a.n_bins0 == 0 || a.sub_bits > (uint32_t)kMaxDigitBits || a.max_tiles == 0)
        return hipErrorInvalidValue;
    const size_t nsub = (size_t)1 << a.sub_bits;
    const size_t lds = kGroupWaves * nsub * sizeof(uint32_t);
    // one wave per tile: a persistent grid over the (device-counted) tiles
    const dim3 gw(persistent_grid((a.max_tiles + kGroupWaves - 1) / kGroupWaves, 8)), b(kGroupThreads);
    hipLaunchKernelGGL(k_gtiles, dim3(1), dim3(1024), 0, s, a);
    if (wide) hipLaunchKernelGGL(k_gcount<CodecW>, gw, b, lds, s, a);
    else hipLaunchKernelGGL(k_gcount<CodecC>, gw, b, lds, s, a);
    hipLaunchKernelGGL(k_gscan, dim3(a.n_bins0), b, nsub * sizeof(uint32_t), s, a);
    if (a.sub_bits <= kGLdsMaxSub && !(a.ablate & kAblGroupSeq)) {
        const dim3 gp(persistent_grid((a.max_tiles + 1) / 2, 4)), bp(kGPThreads);
        if (wide) hipLaunchKernelGGL(k_gplace_lds<CodecW>, gp, bp, gplace_lds_bytes<RecW>(a.sub_bits), s, a);
        else hipLaunchKernelGGL(k_gplace_lds<CodecC>, gp, bp, gplace_lds_bytes<RecC>(a.sub_bits), s, a);
        return hipGetLastError();
    }
    if (wide) hipLaunchKernelGGL(k_gplace<CodecW>, gw, b, lds, s, a);
    else hipLaunchKernelGGL(k_gplace<CodecC>, gw, b, lds, s, a);
    return hipGetLastError();
}

template <class Res>
static void unpermute_mid(const UnpermArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_unpermute_mid<Res>, dim3((a.n + 2047) / 2048), dim3(256), 0, s, a.pos1,
                       (const Res*)a.res, (Res*)a.mid, a.n, a.ctl, a.mid_xcd);
}

hipError_t launch_route_ranges(const uint32_t* route_list, const uint32_t* bin_base,
                               const uint32_t* bin_total, uint32_t lo_bins, uint32_t* route_start,
                               uint32_t* route_cnt, BatchCtl* ctl, hipStream_t s) {
    hipLaunchKernelGGL(k_route_ranges, dim3(1), dim3(1024), 0, s, route_list, bin_base, bin_total,
                       lo_bins, route_start, route_cnt, ctl);
    return hipGetLastError();
}

hipError_t launch_unpermute(const UnpermArgs& a_in, int res_bytes, hipStream_t s) {
    UnpermArgs a = a_in;
    a.res_final = a.res;
    a.pos1_final = a.pos1;
    if (a.pos1 && a.mid && !a.tokens_out && a.n) {      // two-pass: undo pass 1, then pass 0
        if (res_bytes == 8) unpermute_mid<uint64_t>(a, s);
        else if (res_bytes == 1) unpermute_mid<uint8_t>(a, s);
        else if (res_bytes == 2) unpermute_mid<uint16_t>(a, s);
        else unpermute_mid<uint32_t>(a, s);
        a.res_hi = a.res;
        a.res = a.mid;
        a.pos1 = nullptr;
    }
    dim3 g(persistent_grid(a.n_tiles, a.per_cu ? a.per_cu : 1)), b(kTileThreads);
    if (a.split && !a.pos1 && !a.tokens_out && !a.ablate) {
        const dim3 b2(2 * kTileThreads);
        if (res_bytes == 8) hipLaunchKernelGGL(k_unpermute_split<uint64_t>, g, b2, 0, s, a);
        else if (res_bytes == 1) hipLaunchKernelGGL(k_unpermute_split<uint8_t>, g, b2, 0, s, a);
        else if (res_bytes == 2) hipLaunchKernelGGL(k_unpermute_split<uint16_t>, g, b2, 0, s, a);
        else hipLaunchKernelGGL(k_unpermute_split<uint32_t>, g, b2, 0, s, a);
        return hipGetLastError();
    }
    if (res_bytes == 8) hipLaunchKernelGGL(k_unpermute<uint64_t>, g, b, 0, s, a);
    else if (res_bytes == 1) hipLaunchKernelGGL(k_unpermute<uint8_t>, g, b, 0, s, a);
    else if (res_bytes == 2) hipLaunchKernelGGL(k_unpermute<uint16_t>, g, b, 0, s, a);
    else hipLaunchKernelGGL(k_unpermute<uint32_t>, g, b, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fill_invalid(uint8_t* allowed, int64_t* remaining, double* tok, uint32_t n,
                               hipStream_t s) {
    hipLaunchKernelGGL(k_fill_invalid, dim3((n + 255) / 256), dim3(256), 0, s, allowed,
                       remaining, tok, n);
    return hipGetLastError();
}

}  // namespace rl
