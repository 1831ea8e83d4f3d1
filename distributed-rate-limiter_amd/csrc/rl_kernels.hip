// rl_kernels.hip — the batched rate-limit decision pipeline for gfx950 (MI355X).
//
// One batch = requests in arrival order. The pipeline groups every request with
// the other requests of its (limiter, key) WITHOUT a full sort:
//
//   1. k_upsweep  : per 64K-request tile, histogram of the partition digit of each
//                   request's BIN (bin = 8 consecutive state-table regions; region =
//                   top bits of mix64(key)).
//   2. k_scan_rows/k_scan_small : exclusive scan of the [bin][tile] histogram.
//   3. k_scatter  : stable partition (wave ballot-match ranking) of the requests
//                   into bin order, packed into 16-byte records.
//   (1-3 repeat once more when a limiter set has > 1024 bins.)
//   4. k_regions  : one single-wave workgroup per REGION. The wave loads its region's
//                   256 state slots (8 KB) into LDS once, streams its bin's records
//                   in arrival order, keeps its region's requests in an LDS ring and
//                   applies the reference semantics per key in order, 64 at a time
//                   (deny never mutates, so a group needs 1 + (#state changes of its
//                   busiest key) rounds); the region is written back once.
//   5. k_unpermute: results back to the caller's order (allowed u8, remaining i64).
//
// Partition and unpermute grids are persistent and walk tiles XCD-aware: at any
// time the 32 CUs of an XCD work on 32 consecutive tiles, so the per-bin record runs
// they write (and the result runs they gather) share lines in that XCD's L2.
#include <algorithm>
#include <type_traits>

#include "rl_launch.hpp"

#pragma clang fp contract(off)

namespace rl {

// ------------------------------------------------------------------ helpers
__device__ inline uint32_t xcd_remap(uint32_t b, uint32_t n) {
    // bijective: blocks b, b+8, ... (one XCD under round-robin dispatch) get
    // consecutive tile ids.
    const uint32_t q = n / 8, r = n % 8, x = b % 8;
    const uint32_t base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + b / 8;
}

__device__ inline uint32_t popc_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Lanes of this wave whose `v` (low nbits) equals mine, among `active` lanes.
__device__ inline uint64_t wave_match(uint32_t v, int nbits, bool active) {
    uint64_t m = __ballot(active);
#pragma unroll
    for (int b = 0; b < kMaxDigitBits; ++b) {
        if (b < nbits) {                             // wave-uniform
            const bool bit = (v >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
    }
    return m;
}

__device__ inline uint64_t readlane64(uint64_t v, uint32_t lane) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)lane) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)lane);
}

__device__ inline uint64_t ord_key(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ULL; }

// Earliest / latest now_ms of the batch's valid requests. A batch with no valid request
// has min = INT64_MIN (every stored bucket is kept when a region is loaded) and max = lo.
__device__ inline int64_t batch_lo(const BatchCtl* c) {
    return c->min_now_key == ~0ULL ? INT64_MIN : (int64_t)(c->min_now_key ^ 0x8000000000000000ULL);
}
// Time from which a loaded region keeps a slot: every later request has now >= this
// (batches in global time order, less the caller's declared skew, rl_opts.max_skew_ms).
__device__ inline int64_t keep_from(const RegionArgs& a) {
    const int64_t lo = batch_lo(a.ctl);
    return lo < INT64_MIN + a.skew_ms ? INT64_MIN : lo - a.skew_ms;
}
__device__ inline int64_t batch_hi(const BatchCtl* c) {
    return c->max_now_key == 0ULL ? batch_lo(c) : (int64_t)(c->max_now_key ^ 0x8000000000000000ULL);
}

// Streaming (non-temporal) accesses for data touched once per batch: the scatter's request
// reads and position writes, the region kernel's record stream (one region per bin) and
// unpermute's position reads and output writes. They keep L2 / Infinity Cache for the
// scattered record runs, the state table and the packed results the unpermute gathers
// (tb_uniform 3.33 -> 3.12 ms/step on MI355X). Scattered record stores stay temporal: a
// streaming partial-line store goes to memory on its own (scatter 1.5 -> 3.3 ms).
// A/B builds: -DRL_TEMPORAL=1 turns the streaming accesses off, -DRL_NT_SCATTER_REC on.
#ifndef RL_TEMPORAL
#define RL_TEMPORAL 0
#endif
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <bool NT, class T>
__device__ inline T ld(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, class T>
__device__ inline void st(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <bool NT, class Rec>
__device__ inline void st_rec(Rec* p, const Rec& r) {
    if constexpr (NT && sizeof(Rec) == 16) {
        u32x4_t v;
        __builtin_memcpy(&v, &r, 16);
        __builtin_nontemporal_store(v, (u32x4_t*)p);
    } else {
        *p = r;
    }
}
constexpr bool kNtScIn = !RL_TEMPORAL;
#ifdef RL_NT_SCATTER_REC
constexpr bool kNtScRec = true;
#else
constexpr bool kNtScRec = false;
#endif
constexpr bool kNtScPos = !RL_TEMPORAL;
#ifdef RL_NT_UPSWEEP
constexpr bool kNtUp = true;
#else
constexpr bool kNtUp = false;
#endif
template <bool NT, class Rec>
__device__ inline Rec ld_rec(const Rec* p) {
    if constexpr (NT && sizeof(Rec) == 16) {
        const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
        Rec r;
        __builtin_memcpy(&r, &v, 16);
        return r;
    } else {
        return *p;
    }
}
constexpr bool kNtRgRec = !RL_TEMPORAL;
constexpr bool kNtUn = !RL_TEMPORAL;

template <int NT>
__device__ inline uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_tmp /*[NT/64]*/,
                                                uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) s_tmp[wid] = x;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
    for (int w = 0; w < NT / 64; ++w) {
        const uint32_t s = s_tmp[w];
        if ((uint32_t)w < wid) wpre += s;
        tot += s;
    }
    __syncthreads();
    if (total) *total = tot;
    return wpre + x - v;
}

struct LimLds {
    uint32_t base[256];
    uint8_t bits[256];
};

__device__ inline void load_lim_lds(LimLds& L, const PartArgs& a) {
    for (uint32_t l = threadIdx.x; l < a.n_lim; l += blockDim.x) {
        L.base[l] = a.lims[l].region_base;
        L.bits[l] = (uint8_t)a.lims[l].region_bits;
    }
}

// Tile processed by this workgroup at iteration `it` of a persistent grid: the
// workgroups of one XCD (blocks b, b+8, ...) take consecutive tiles.
// RL_TILE_ORDER 1 (A/B knob): XCD x instead owns the contiguous chunk [x*T/8, (x+1)*T/8) and
// its workgroups walk it 32 tiles at a time, so a bin's record run is split between XCDs 8 times
// in total rather than once per 256 tiles. Returns >= n_tiles when this workgroup is done.
#ifndef RL_TILE_ORDER
#define RL_TILE_ORDER 0
#endif
__device__ inline uint32_t tile_at(uint32_t it, uint32_t n_tiles) {
    if constexpr (RL_TILE_ORDER == 1) {
        if (gridDim.x % 8 == 0) {
            const uint32_t per = gridDim.x / 8, chunk = (n_tiles + 7) / 8;
            const uint32_t k = it * per + blockIdx.x / 8;
            return k < chunk ? (blockIdx.x % 8) * chunk + k : n_tiles;
        }
    }
    return it * gridDim.x + xcd_remap(blockIdx.x, gridDim.x);
}

// Global bin id of element i (pass 0: raw arrays; later passes: records).
template <class Codec, bool RAW>
__device__ inline uint32_t bin_of(const PartArgs& a, uint32_t i, const LimLds& L) {
    uint64_t h;
    uint32_t lim;
    if constexpr (RAW) {
        h = mix64(ld<kNtUp>(a.key + i));
        lim = a.limiter ? a.limiter[i] : 0u;
        if (lim >= a.n_lim) lim = 0;  // invalid: routed to limiter 0's region, rejected there
    } else {
        const typename Codec::Rec* r = (const typename Codec::Rec*)a.rec_in + i;
        h = r->h;
        lim = Codec::limiter_of(*r);
    }
    return (L.base[lim] + region_local(h, a.shard_bits, L.bits[lim])) >> a.bin_shift;
}

// ------------------------------------------------------------------ 1. upsweep
template <class Codec, bool RAW>
__global__ __launch_bounds__(kTileThreads) void k_upsweep(PartArgs a) {
    __shared__ uint32_t hist[1u << kMaxDigitBits];
    __shared__ LimLds L;
    const uint32_t t = threadIdx.x;
    const uint32_t bins = 1u << a.digit_bits;
    load_lim_lds(L, a);
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
        }
    }
    const uint32_t mask = bins - 1;
    for (uint32_t it = 0;; ++it) {
        const uint32_t tile = tile_at(it, a.n_tiles);
        if (tile >= a.n_tiles) break;
        for (uint32_t b = t; b < bins; b += kTileThreads) hist[b] = 0;
        __syncthreads();
#pragma unroll 8
        for (int r = 0; r < kTileItems; ++r) {
            const uint32_t i = tile * (uint32_t)kTile + (uint32_t)r * kTileThreads + t;
            if (i < a.n) {
                const uint32_t g = bin_of<Codec, RAW>(a, i, L);
                atomicAdd(&hist[(g >> a.digit_shift) & mask], 1u);
                if (a.region_count) atomicAdd(&a.region_count[g], 1u);
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
    uint64_t key; int64_t now_ns; int32_t permits; uint32_t lim; uint32_t op;
    __device__ inline void load(const PartArgs& a, uint32_t i) {
        key = ld<kNtScIn>(a.key + i);
        now_ns = ld<kNtScIn>(a.now_ns + i);
        permits = ld<kNtScIn>(a.permits + i);
        lim = a.limiter ? a.limiter[i] : 0u;
        op = a.op ? a.op[i] : 0u;
    }
};

template <class Codec>
struct ScatterIn<Codec, false> {
    typename Codec::Rec rec;
    __device__ inline void load(const PartArgs& a, uint32_t i) {
        rec = ((const typename Codec::Rec*)a.rec_in)[i];
    }
};

#ifndef RL_SCATTER_DEPTH
#define RL_SCATTER_DEPTH 8
#endif
constexpr int kScatterDepth = RL_SCATTER_DEPTH;   // rounds of inputs in flight (divides kTileItems)

template <class Codec, bool RAW>
__global__ __launch_bounds__(kTileThreads) void k_scatter(PartArgs a) {
    using Rec = typename Codec::Rec;
    static_assert(kTileThreads / 64 <= 8, "per-wave counts are packed 8 to a bin");
    __shared__ uint32_t cur[1u << kMaxDigitBits];                    // next slot per bin
    // this round's count of each wave per bin, the waves' bytes packed in one word: a lane
    // sums the earlier waves' counts for its bin with one read and two v_sad_u8
    __shared__ uint64_t cntw[1u << kMaxDigitBits];
    __shared__ LimLds L;
    __shared__ uint64_t s_mm[2][kTileThreads / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t bins = 1u << a.digit_bits, mask = bins - 1;
    load_lim_lds(L, a);
    int64_t base = 0;
    if constexpr (RAW) base = a.ctl->base_ms;
    const uint32_t last = a.n - 1;
    uint64_t mn = ~0ULL, mx = 0;
    bool overflow = false;
    for (uint32_t it = 0;; ++it) {
        const uint32_t tile = tile_at(it, a.n_tiles);
        if (tile >= a.n_tiles) break;
        const uint32_t tile0 = tile * (uint32_t)kTile;
        __syncthreads();     // previous tile's LDS users are done
        for (uint32_t b = t; b < bins; b += kTileThreads) {
            cur[b] = a.bin_base[b] + a.counts[(size_t)b * a.n_tiles + tile];
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
            const bool active = i < a.n;
            Rec rec{};
            uint32_t d = 0;
            if (active) {
                if constexpr (RAW) {
                    uint32_t lim = in.lim, op = in.op;
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
                    d = (((L.base[lim] + region_local(h, a.shard_bits, L.bits[lim])) >> a.bin_shift)
                         >> a.digit_shift) & mask;
                } else {
                    rec = in.rec;
                    const uint32_t lim = Codec::limiter_of(rec);
                    d = (((L.base[lim] + region_local(rec.h, a.shard_bits, L.bits[lim])) >> a.bin_shift)
                         >> a.digit_shift) & mask;
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
            if (abl & (kAblNoMatch | kAblNoBarrier)) pos = min(pos, a.n - 1);
            // inactive lanes write to the padding slot past n (buffers carry spare entries)
            uint32_t wpos = active ? pos : a.n + t;
            if (abl & kAblSeqRecStore) wpos = active ? i : a.n + t;
            if (!(abl & kAblNoRecStore)) st_rec<kNtScRec>((Rec*)a.rec_out + wpos, rec);
            if (!(abl & kAblNoPosStore)) st<kNtScPos>(a.pos_out + (active ? i : a.n + t), pos);
        };
        // Unrolled by the prefetch depth so the input registers rotate without moves (a
        // move would wait on its load). vmcnt retires loads and stores in issue order, so
        // waiting for round r's inputs also waits for the scattered stores issued before
        // them: a deep ring spreads that store-ack latency over kScatterDepth rounds.
        for (int r = 0; r < kTileItems; r += kScatterDepth) {
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

// ------------------------------------------------------------------ 4. regions
// One single-wave workgroup per REGION. The region's 256 slots (8 KB) live in the wave's
// LDS for the whole batch. The wave streams its BIN's records (arrival order, 8
// regions interleaved) 64 at a time, keeps the ones of its region in an LDS ring and
// applies them 64 at a time. The 8 waves of a bin have block ids congruent mod 8 and
// adjacent in dispatch order, i.e. they run together on one XCD, so the bin's stream is
// fetched from HBM once and re-read from that XCD's L2. No barriers anywhere.
__device__ inline void wave_fence() { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); }

// first probe position of a key inside its region (4-slot aligned: probing reads buckets)
__device__ inline uint32_t slot_home(uint64_t h) { return (uint32_t)h & (kRegionSlots - 4); }

struct RegionTable {
    static constexpr bool kCache = false;
    alignas(16) uint64_t tag[kRegionSlots];
    uint64_t sa[kRegionSlots];
    uint64_t sb[kRegionSlots];
    uint64_t sc[kRegionSlots];
    alignas(16) uint32_t occ[kRegionSlots];   // bit0 occupied, bit1 touched by this batch
#ifdef RL_CHAINS
    int64_t xrem[64];                         // wave_apply's per-key chains: results by lane
    double xtok[64];
    uint32_t xalw[64];
#endif
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
    Rec ring[kRing];                  // this region's pending requests (bins of 8 regions)
    uint32_t ring_pos[kRing];         // ... and their result index
};
template <class Codec>
struct RegionLds<Codec, false> : RegionTable {};

#ifndef RL_NO_SPARSE
#define RL_NO_SPARSE 0                    // A/B builds: 1 compiles the sparse-region path out
#endif
constexpr bool kSparseOn = !RL_NO_SPARSE;

// Sparse region (few records): the LDS table starts with every bucket kOccUnloaded and a
// probe that reaches such a bucket faults it in from HBM (128 B, + 32 B of cache words);
// dead slots come in as tombstones. tab == nullptr: the whole image is in LDS.
struct SparseSrc {
    const Slot* tab;
    const uint64_t* xtab;             // local-cache words (nullable)
    int64_t keep;                     // slot_live threshold (keep_from)
    bool long_chain;                  // per lane: a probe went past two used buckets
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

#ifdef RL_CHAINS
// A/B build only (-DRL_CHAINS): measured slower than the rounds on every bench config
// (same-box A/B: tb_uniform region 1.21 -> 1.28 ms, zipf_1b 6.16 -> 6.64, mixed 13.93 -> 14.03).
// The per-key chains of wave_apply: every pending lane's key has its state in S[slot]; the
// lowest pending lane of each key runs that key's pending requests in lane (= arrival) order,
// reading each request's fields from its lane; results go through LDS back to their lanes.
template <class Codec, int ALGO, class LdsT>
__device__ inline void wave_chains(LdsT& S, const DevLimiter& L, uint32_t lane, const Req& q,
                                   const SWGeo& geo, int32_t slot, bool& pending, uint64_t kp,
                                   Applied& r, uint32_t& n_allowed) {
    const bool leader = pending && (kp & ((1ULL << lane) - 1)) == 0;
    uint64_t todo = leader ? kp : 0ULL;
    uint64_t sa = 0, sb = 0, sc = 0;
    if (leader) { sa = S.sa[slot]; sb = S.sb[slot]; sc = S.sc[slot]; }
    while (__any(todo != 0)) {
        const bool act = todo != 0;
        const uint32_t l = act ? (uint32_t)__builtin_ctzll(todo) : lane;
        todo &= todo - 1;
        // every lane takes part in the shuffles (a source lane may be idle)
        const int64_t t_l = __shfl(q.now_ms, (int)l, 64);
        const int32_t p_l = __shfl(q.permits, (int)l, 64);
        const uint32_t op_l = (uint32_t)__shfl((int)q.op, (int)l, 64);
        Outcome o{};
        if constexpr (ALGO == kAlgoTB) {
            if (act) o = tb_step(L, op_l, p_l, t_l, sa, sb, sc);
        } else {
            SWGeo g;
            g.curr_start = __shfl(geo.curr_start, (int)l, 64);
            g.prev_start = __shfl(geo.prev_start, (int)l, 64);
            g.prev_weight = __shfl(geo.prev_weight, (int)l, 64);
            if (act) o = sw_step_g(L, op_l, p_l, t_l, g, sa, sb, sc);
        }
        if (act) {
            S.xrem[l] = o.remaining;
            S.xtok[l] = o.tokens;
            S.xalw[l] = o.allowed ? 1u : 0u;
            if (o.mutate) { sa = o.a; sb = o.b; sc = o.c; }
        }
    }
    if (leader) { S.sa[slot] = sa; S.sb[slot] = sb; S.sc[slot] = sc; }
    wave_fence();
    if (pending) {
        r.alw = S.xalw[lane] != 0;
        r.rem = S.xrem[lane];
        r.tok = S.xtok[lane];
        n_allowed += r.alw ? 1u : 0u;
        pending = false;
    }
    wave_fence();
}
#endif

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
        const uint32_t expect = cand_tomb ? (kOccUsed | kOccTomb) : 0u;
        if (need && cand != kNone && atomicCAS(&S.occ[cand], expect, kOccUsed) == expect) {
            S.tag[cand] = q.h; S.sa[cand] = 0; S.sb[cand] = 0; S.sc[cand] = 0;
            if constexpr (LdsT::kCache) S.sx[cand] = 0;
            slot = (int32_t)cand;
            need = false;
        }
        wave_fence();
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
    const bool one_round = (a.ablate & kAblNoRounds) != 0;
    const uint64_t peers = one_round ? (1ULL << lane)
                                     : wave_match((uint32_t)slot, kRegionBits, slot >= 0);
    bool pending = slot >= 0;
    SWGeo geo{};
    uint64_t same_w = 0, elig_m = 0;        // (A): lanes in my window / acquires
    if constexpr (!tb) {
        if (slot >= 0) geo = sw_geo(q.now_ms, L);
        // window index relative to the wave's first window (2 bits; 3 = "far")
        int64_t wmin = slot >= 0 ? geo.curr_start : INT64_MAX;
        for (int o = 32; o > 0; o >>= 1) {
            const int64_t x = __shfl_xor(wmin, o, 64);
            wmin = x < wmin ? x : wmin;
        }
        int64_t wi = slot >= 0 ? (geo.curr_start - wmin) / L.window_ms : 3;
        if (wi > 3) wi = 3;
        const uint64_t b0 = __ballot(wi & 1), b1 = __ballot(wi & 2);
        same_w = ((wi & 1) ? b0 : ~b0) & ((wi & 2) ? b1 : ~b1);
        elig_m = __ballot(slot >= 0 && wi < 3 && q.op == (uint32_t)kOpAcquire);
    }
    [[maybe_unused]] uint32_t my_rounds = 0;      // -DRL_CHAINS only
    while (__any(pending)) {
        // Chains: after two rounds, if every key still pending has changed state in (nearly)
        // every round so far (runs of TB allows, SW allows across windows) and some key still
        // has >= 4 requests pending, the rounds would go on finalizing one request per key
        // each; the lowest pending lane of every key then applies the key's remaining
        // requests itself, in arrival order (each a full exact step; a deny leaves the state
        // as it is), instead of one wave round per state change.
#ifdef RL_CHAINS
        if (!CACHE && my_rounds >= 2 && !one_round) {
            const uint64_t kp = peers & __ballot(pending);
            const uint32_t fin = (uint32_t)__popcll(peers) - (uint32_t)__popcll(kp);
            if (__all(!pending || fin <= 2u * my_rounds) && __any(pending && __popcll(kp) >= 4)) {
                ++n_rounds;
                wave_chains<Codec, ALGO>(S, L, lane, q, geo, slot, pending, kp, r, n_allowed);
                break;
            }
        }
#endif
        ++my_rounds;
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

template <class Codec, class Res, bool TOK, int BS, class LdsT>
__device__ inline void region_body_t(const RegionArgs& a, uint32_t g, LdsT& S) {
    using Rec = typename Codec::Rec;
    constexpr uint32_t NS = kRegionSlots;
    constexpr uint32_t RPB = 1u << BS;              // regions per bin

    // RPB = 8: block g = 64q + 8r + x  ->  bin 8q + x, region r of that bin (see above)
    const uint32_t bin = RPB == 1 ? g : (g / 64) * 8 + (g % 8);
    const uint32_t rb = RPB == 1 ? 0u : (g / 8) % 8;
    const uint32_t n_bins = a.n_regions / RPB;
    if (bin >= n_bins) return;
    if (a.hot_mark && a.hot_mark[bin] == a.epoch) return;     // owned by hot_chain
    if (a.ablate & kAblNoNormal) return;
    const uint32_t start = a.rstart[bin];
    const uint32_t cnt = a.rend ? a.rend[bin] - start : a.rcount[bin];
    if (cnt == 0) return;
    const uint32_t end = start + cnt;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t region = bin * RPB + rb;
    const DevLimiter L = a.lims[a.region_lim[region]];
    const int64_t base = a.ctl->base_ms;
    const int64_t batch_min = keep_from(a);
    const uint32_t pad = a.n_total + lane;          // padding slot for idle lanes
    const Rec* recs = (const Rec*)a.rec;
    Res* res = (Res*)a.res;

    if (a.ctl->span_overflow != 0) {
        // compact records cannot represent this batch's time span: reject it whole,
        // before any state is touched (the host reports RL_E_INVALID_ARG). Wave rb of
        // the bin writes its region's share.
        for (uint32_t j = start + lane; j < end; j += 64) {
            const Rec r = recs[j];
            if ((region_local(r.h, a.shard_bits, L.region_bits) & (RPB - 1)) == rb) {
                res[j] = (Res)pack_result(false, kRemInvalid);
                if (TOK) a.tok[j] = __builtin_nan("");
            }
        }
        return;
    }
    // kDepth slices of the bin's stream in flight (issued while the region image loads)
    constexpr uint32_t kDepth = 4;
    // unconditional; read once when the bin is the region (streaming), else shared by RPB waves
    auto fetch = [&](uint32_t c) { return ld_rec<kNtRgRec && RPB == 1>(recs + min(c + lane, end - 1)); };
    Rec q0 = fetch(start), q1 = fetch(start + 64), q2 = fetch(start + 128), q3 = fetch(start + 192);

    // ---- load the region, dropping entries no request of this batch can see, and
    // rebuild its open-addressing table (no tombstones ever reach HBM)
    Slot* tab = (Slot*)L.table + (size_t)(region - L.region_base) * NS;
    uint64_t* xtab = nullptr;                       // the slots' local-cache states
    if constexpr (LdsT::kCache)
        if (L.cache_table) xtab = (uint64_t*)L.cache_table + (size_t)(region - L.region_base) * NS;
    // Few records: probe and update single buckets in HBM (128 B read + 32 B written per
    // distinct key) instead of moving the 8 KB image both ways.
    const bool sparse = kSparseOn && RPB == 1 && cnt <= a.sparse_max && !(a.ablate & kAblNoProbe);
    SparseSrc sp{sparse ? tab : nullptr, xtab, batch_min, false};
    // rebuild the LDS table from registers: linear probing from each key's home
    auto rebuild = [&](const Slot (&img)[NS / 64], const uint64_t (&xim)[NS / 64], const bool (&keep)[NS / 64]) {
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) S.occ[lane + 64 * i] = 0;
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
        for (uint32_t i = 0; i < NS / 64; ++i) S.occ[lane + 64 * i] = kOccUnloaded;
        wave_fence();
    } else {
        // load the region, dropping entries no request of this batch can see
        Slot img[NS / 64];
        uint64_t xim[NS / 64];
        bool keep[NS / 64];
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) {
            img[i] = tab[lane + 64 * i];
            xim[i] = xtab ? xtab[lane + 64 * i] : 0;
        }
#pragma unroll
        for (uint32_t i = 0; i < NS / 64; ++i) keep[i] = slot_live(L, img[i], batch_min, xim[i]);
        rebuild(img, xim, keep);
    }

    uint32_t n_allowed = 0, n_invalid = 0, n_caperr = 0, n_rounds = 0, n_hits = 0;
    const uint64_t t_start = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t head = 0, count = 0;                    // ring state (wave-uniform)
    // the whole stream is instantiated once per algorithm (uniform per region), so the
    // compiler hoists nothing of the other algorithm into the hot loop
    auto stream = [&](auto algo, auto spc) {
        constexpr int A = decltype(algo)::value;
        constexpr bool SPX = decltype(spc)::value;
        auto slice = [&](const Rec& r, uint32_t c0) {
            const uint32_t idx = c0 + lane;
            if constexpr (RPB == 1) {
                // the bin is the region: every record is ours, applied straight from registers
                const Applied ap = wave_apply<Codec, A, SPX>(a, S, L, lane, r, idx < end, idx, base, pad,
                                                     n_allowed, n_invalid, n_caperr, n_rounds, n_hits, sp);
                put_res<Res>(a, ap.j, ap.alw, ap.rem);
                if (TOK) a.tok[ap.j] = ap.tok;
            } else {
                const bool mine = idx < end &&
                    (region_local(r.h, a.shard_bits, L.region_bits) & (RPB - 1)) == rb;
                const uint64_t bal = __ballot(mine);
                if (mine) {
                    const uint32_t k = (head + count + popc_below(bal)) % kRing;
                    S.ring[k] = r;
                    S.ring_pos[k] = idx;
                }
                count += (uint32_t)__popcll(bal);
                wave_fence();
                Applied ap;
                ap.j = pad; ap.alw = false; ap.rem = kRemError; ap.tok = 0.0;
                if (count >= 64) {
                    const uint32_t ri = (head + lane) % kRing;
                    ap = wave_apply<Codec, A, SPX>(a, S, L, lane, S.ring[ri], true, S.ring_pos[ri], base, pad,
                                           n_allowed, n_invalid, n_caperr, n_rounds, n_hits, sp);
                    head = (head + 64) % kRing;
                    count -= 64;
                }
                put_res<Res>(a, ap.j, ap.alw, ap.rem);   // exactly one store per slice
                if (TOK) a.tok[ap.j] = ap.tok;
            }
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
        if constexpr (RPB > 1) {
            if (count > 0) {
                const bool v = lane < count;
                const uint32_t ri = (head + (v ? lane : 0u)) % kRing;
                const Applied ap = wave_apply<Codec, A, SPX>(a, S, L, lane, S.ring[ri], v, S.ring_pos[ri], base,
                                                     pad, n_allowed, n_invalid, n_caperr, n_rounds, n_hits, sp);
                put_res<Res>(a, ap.j, ap.alw, ap.rem);
                if (TOK) a.tok[ap.j] = ap.tok;
            }
        }
    };
    using SpOn = std::integral_constant<bool, kSparseOn && RPB == 1>;
    using SpOff = std::integral_constant<bool, false>;
    if (L.algo == kAlgoTB) {
        if (sparse) stream(std::integral_constant<int, kAlgoTB>{}, SpOn{});
        else stream(std::integral_constant<int, kAlgoTB>{}, SpOff{});
    } else {
        if (sparse) stream(std::integral_constant<int, kAlgoSW>{}, SpOn{});
        else stream(std::integral_constant<int, kAlgoSW>{}, SpOff{});
    }
    wave_fence();
    uint32_t touched = 0;
    for (uint32_t s = lane; s < NS; s += 64) touched += (S.occ[s] & kOccTouched) ? 1u : 0u;
    bool whole = !sparse;
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
    // ---- write the region back: every slot (free ones as zeros), or in a sparse region
    // only the slots this batch touched
    uint32_t used = 0;                               // live keys (whole regions only)
    uint32_t moved = 0;                              // table bytes read + written (sparse)
    const uint32_t xw = xtab ? 8u : 0u;              // local-cache word per slot
    for (uint32_t s = lane; s < NS; s += 64) {
        const uint32_t o = S.occ[s];
        used += (whole && (o & kOccUsed) && !(o & kOccTomb)) ? 1u : 0u;
        if (!whole) moved += (!(o & kOccUnloaded) && (s & 3u) == 0 ? 4u * (32u + xw) : 0u) +
                             ((o & kOccTouched) ? 32u + xw : 0u);
        if (!whole && !(o & kOccTouched)) continue;
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
        atomicAdd(st + kStTableBytes, whole ? (unsigned long long)(2u * NS * (32u + xw))
                                            : (unsigned long long)moved);
        if (n_allowed) atomicAdd(st + kStAllowed, (unsigned long long)n_allowed);
        if (n_invalid) atomicAdd(st + kStInvalid, (unsigned long long)n_invalid);
        if (n_caperr) atomicAdd(st + kStCapErr, (unsigned long long)n_caperr);
        atomicAdd(st + kStDistinct, (unsigned long long)touched);
        atomicAdd(st + kStRegions, 1ULL);
        if (n_hits) atomicAdd(st + kStCacheHits, (unsigned long long)n_hits);
        if (a.dbg) {
            uint64_t* d = a.dbg + (size_t)bin * kDbgWords;
            d[0] = t_start; d[1] = __builtin_amdgcn_s_memrealtime(); d[2] = cnt; d[3] = n_rounds;
        }
    }
}

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
// of the region's first 64 records (a hot region is dominated by its hot key).
template <class Codec>
__global__ __launch_bounds__(64) void k_hot_prep(RegionArgs a) {
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t i = blockIdx.x, lane = threadIdx.x;
    if (i >= hc) return;
    const uint32_t bin = a.hot_list[i];
    const uint32_t start = a.rstart[bin];
    const uint32_t end = start + (a.rend ? a.rend[bin] - start : a.rcount[bin]);
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
    if (lane == 0) {
        HotInfo f;
        f.tag = tag; f.bin = bin; f.start = start; f.end = end;
        f.n_chunks = (end - start + kHotChunk - 1) / kHotChunk;
        f.chunk_base = 0;
        f.ok = (key >> 6) >= 2u ? 1u : 0u;
        f.n_groups = (f.n_chunks + 63) / 64;
        f.group_base = 0;
        f.pad[0] = f.pad[1] = 0;
        a.hot_info[i] = f;
    }
}

__global__ __launch_bounds__(1024) void k_hot_scan(RegionArgs a) {
    __shared__ uint32_t tmp[16];
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t t = threadIdx.x;
    const uint32_t v = t < hc ? a.hot_info[t].n_chunks : 0u;
    uint32_t tot, tot2;
    const uint32_t ex = block_exclusive_scan<1024>(v, tmp, &tot);
    const uint32_t v2 = t < hc ? a.hot_info[t].n_groups : 0u;
    const uint32_t ex2 = block_exclusive_scan<1024>(v2, tmp, &tot2);
    if (t < hc) {
        a.hot_info[t].chunk_base = ex;
        a.hot_info[t].group_base = ex2;
    }
    if (t == 0) { a.hot_total[0] = tot; a.hot_total[1] = tot2; }
}

// Phase A2 (one wave per 64 chunks): the same summary over 4096 records, so the chain
// decides the long runs of a hot key's denials 4096 records per test.
__global__ __launch_bounds__(256) void k_hot_summ2(RegionArgs a) {
    __shared__ uint32_t s_base[kHotMax + 1];
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t total = a.hot_total[1];
    for (uint32_t i = threadIdx.x; i < hc; i += 256) s_base[i] = a.hot_info[i].group_base;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t g = blockIdx.x * 4 + wid; g < total; g += gridDim.x * 4) {
        const uint32_t i = hot_region_of(s_base, hc, g);
        const HotInfo f = a.hot_info[i];
        const uint32_t c = (g - s_base[i]) * 64 + lane;
        uint64_t mn = ~0ULL, mx = 0;
        uint32_t w = 0;
        if (c < f.n_chunks) {
            const uint64_t* d = a.hot_summ + (size_t)(f.chunk_base + c) * 4;
            mn = ord_key((int64_t)d[0]);
            mx = ord_key((int64_t)d[1]);
            w = (uint32_t)d[2];
        }
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t x = __shfl_xor(mn, o, 64), y = __shfl_xor(mx, o, 64);
            mn = x < mn ? x : mn;
            mx = y > mx ? y : mx;
        }
        const uint32_t ns = __ballot((w & 0xFFu) != 0) ? 1u : 0u;       // flags, not counts
        const uint32_t nh = __ballot(((w >> 8) & 0xFFu) != 0) ? 1u : 0u;
        const uint32_t ne = __ballot(((w >> 16) & 0xFFu) != 0) ? 1u : 0u;
        const uint32_t no = __ballot(((w >> 24) & 0xFFu) != 0) ? 1u : 0u;
        if (lane == 0) {
            uint64_t* d = a.hot_summ2 + (size_t)g * 4;
            d[0] = mn ^ 0x8000000000000000ULL;
            d[1] = mx ^ 0x8000000000000000ULL;
            d[2] = ns | (nh << 8) | (ne << 16);
            d[3] = (uint64_t)no << 8;                   // other keys: kept through the verdict
        }
    }
}

// Phase A (one wave per 64-record chunk, all CUs): what the chain needs to decide the hot
// key's records of a chunk without reading it: the time range of its plain acquires, and
// how many of its records need the exact path (peek / reset). Summary words: [0] min now,
// [1] max now, [2] n_special | n_hot << 8 | n_early << 16 | n_other << 24, [3] verdict:
// bit 0 = hot records decided by the thresholds (words 0-2 then hold the key's state),
// bit 1 = TB early rejects among them, bits 8-15 = records of other keys.
template <class Codec>
__global__ __launch_bounds__(256) void k_hot_summ(RegionArgs a) {
    __shared__ uint32_t s_base[kHotMax + 1];
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t total = a.hot_total[0];
    for (uint32_t i = threadIdx.x; i < hc; i += 256) s_base[i] = a.hot_info[i].chunk_base;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const typename Codec::Rec* recs = (const typename Codec::Rec*)a.rec;
    const int64_t base = a.ctl->base_ms;
    for (uint32_t g = blockIdx.x * 4 + wid; g < total; g += gridDim.x * 4) {
        const uint32_t i = hot_region_of(s_base, hc, g);
        const HotInfo f = a.hot_info[i];
        const DevLimiter& L = a.lims[a.region_lim[f.bin]];
        const uint32_t j = f.start + (g - s_base[i]) * kHotChunk + lane;
        const bool valid = j < f.end;
        Req q{};
        if (valid) q = Codec::dec(recs[j], base);
        const bool hot = valid && f.ok && !q.invalid && q.h == f.tag;
        const bool acq = q.op == (uint32_t)kOpAcquire;
        const bool early = hot && acq && L.algo == kAlgoTB && (int64_t)q.permits > L.max_permits;
        const bool plain = hot && acq && !early;
        const bool special = hot && !acq;                 // the hot key's peek / reset
        const bool other = valid && !hot;                 // every other key (and invalid)
        uint64_t mn = plain ? ord_key(q.now_ms) : ~0ULL, mx = plain ? ord_key(q.now_ms) : 0ULL;
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t x = __shfl_xor(mn, o, 64), y = __shfl_xor(mx, o, 64);
            mn = x < mn ? x : mn;
            mx = y > mx ? y : mx;
        }
        const uint32_t ns = (uint32_t)__popcll(__ballot(special));
        const uint32_t nh = (uint32_t)__popcll(__ballot(hot));
        const uint32_t ne = (uint32_t)__popcll(__ballot(early));
        const uint32_t no = (uint32_t)__popcll(__ballot(other));
        if (lane == 0) {
            uint64_t* d = a.hot_summ + (size_t)g * 4;
            d[0] = mn == ~0ULL ? (uint64_t)INT64_MAX : (mn ^ 0x8000000000000000ULL);
            d[1] = mx == 0ULL ? (uint64_t)INT64_MIN : (mx ^ 0x8000000000000000ULL);
            d[2] = ns | (nh << 8) | (ne << 16) | (no << 24);
            d[3] = (uint64_t)no << 8;
        }
    }
}

// Phase B (one 2-wave workgroup per listed region, beside k_regions). Wave 0 (pass 1)
// walks the region's summaries in arrival order with the hot key's threshold pair: a
// group of 64 chunks, or a chunk, whose hot-key times all lie in [T0, T1) has its hot
// records decided without being read (verdict + the key's state go back into the summary
// for k_hot_fill); any other chunk has its hot records processed one by one (fast check,
// then the wavefront-per-key sequential run). Wave 1 (pass 2), at the same time, applies
// every other key of the region in arrival order, 64 records at a time through
// wave_apply. The passes touch disjoint slots of the shared LDS table (wave 0 only the
// hot key's state, wave 1 never that slot), so they need no synchronisation.
// Runs as the first kHotMax workgroups of k_regions<..., HOT = true>, so the chains are
// dispatched before the normal regions fill the machine.
template <class Codec, class Res, bool TOK>
__device__ inline void hot_chain(const RegionArgs& a, uint32_t i, RegionLds<Codec, true>& S) {
    using Rec = typename Codec::Rec;
    constexpr uint32_t NS = kRegionSlots;
    __shared__ int32_t s_hslot;
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (i >= hc) return;
    // the passes are sequential critical paths beside thousands of normal-region waves
    __builtin_amdgcn_s_setprio(3);
    const HotInfo f = a.hot_info[i];
    const uint32_t region = f.bin;                    // bin_shift 0: bin == region
    const DevLimiter L = a.lims[a.region_lim[region]];
    const int64_t base = a.ctl->base_ms;
    const int64_t lo = batch_lo(a.ctl);
    const int64_t hi = batch_hi(a.ctl);
    const Rec* recs = (const Rec*)a.rec;
    Res* res = (Res*)a.res;
    const uint32_t pad = a.n_total + lane;
    if (a.ctl->span_overflow != 0) {                  // whole batch rejected (see k_regions)
        for (uint32_t j = f.start + threadIdx.x; j < f.end; j += 128) {
            res[j] = (Res)pack_result(false, kRemInvalid);
            if (TOK) a.tok[j] = __builtin_nan("");
        }
        return;
    }
    const uint64_t t_start = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    Slot* tab = (Slot*)L.table + (size_t)(region - L.region_base) * NS;
    if (wid == 0) {
        // ---- load + rebuild the region (as k_regions), find or insert the hot key's slot
        Slot img[NS / 64];
#pragma unroll
        for (uint32_t k = 0; k < NS / 64; ++k) {
            S.occ[lane + 64 * k] = 0;
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
        int32_t hslot = -1;
        if (f.ok) {
            const uint32_t p0 = slot_home(f.tag);
            for (uint32_t k = 0; k < NS; ++k) {             // linear probing, as the rebuild
                const uint32_t p = (p0 + k) & (NS - 1);
                const uint32_t o = S.occ[p];
                if (!(o & 1u) || S.tag[p] == f.tag) { hslot = (int32_t)p; break; }
            }
            if (hslot >= 0 && !(S.occ[hslot] & 1u) && lane == 0) {
                S.occ[hslot] = 1u; S.tag[hslot] = f.tag; S.sa[hslot] = 0; S.sb[hslot] = 0; S.sc[hslot] = 0;
            }
        }
        if (lane == 0) s_hslot = hslot;
    }
    __syncthreads();
    // hot_ok false (no dominant key, or its region is full): pass 2 takes every record
    const int32_t hslot = s_hslot;
    const bool hot_ok = hslot >= 0;
    const uint32_t hs = hot_ok ? (uint32_t)hslot : 0u;
    const uint64_t tag = f.tag;
    auto is_hot = [&](const Req& q, bool valid) { return hot_ok && valid && !q.invalid && q.h == tag; };
    auto summ_at = [&](uint32_t c) {
        return a.hot_summ + (size_t)(f.chunk_base + (c < f.n_chunks ? c : 0)) * 4;
    };
    auto grp_at = [&](uint32_t g) {
        return a.hot_summ2 + (size_t)(f.group_base + (g < f.n_groups ? g : 0)) * 4;
    };

    uint32_t n_allowed = 0, n_invalid = 0, n_caperr = 0, n_rounds = 0, n_detail = 0, n_other = 0;
    uint32_t n_changed = 0, n_tk = 0, n_fb = 0;       // debug: changes, [T0, T1) updates,
    uint32_t n_late = 0;                              // detailed chunks starting before T0 / ending past T1
    uint64_t cyc_run = 0, cyc_search = 0, cyc_detail = 0, cyc_pass2 = 0;   // debug stamps
    bool any_hot = false;
    auto pass1 = [&](auto algo) {
        constexpr int A = decltype(algo)::value;
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
        int64_t T0 = hot_t0<A>(lo, hi, sa, sb, sc);
        int64_t T1 = t1_of(T0);
        // the hot records of one chunk (lane = arrival order inside the chunk). The next
        // chunk's records are prefetched: undecided chunks come in runs.
        Rec pre = recs[min(f.start + lane, f.end - 1)];
        uint32_t pre_c = 0;
        auto detail = [&](uint32_t c) {
            ++n_detail;
            const uint64_t c_det = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
            const uint32_t j = f.start + c * kHotChunk + lane;
            const bool valid = j < f.end;
            const Rec r = pre_c == c ? pre : recs[valid ? j : f.start];
            pre_c = c + 1;
            pre = recs[min(f.start + pre_c * kHotChunk + lane, f.end - 1)];
            const Req q = Codec::dec(r, base);
            const bool hot = is_hot(q, valid);
            bool oa = false;
            int64_t orem = 0;
            double tk = __builtin_nan("");
            bool pend = hot;
            if (A == kAlgoTB && hot && q.op == (uint32_t)kOpAcquire && (int64_t)q.permits > L.max_permits) {
                orem = kRemUnknown;                       // :110-116, no state access
                pend = false;
            }
            {
                const bool fast = q.op == (uint32_t)kOpAcquire && q.now_ms >= T0 && q.now_ms < T1;
                const uint64_t m = __ballot(pend && !fast);
                const uint32_t first = m ? (uint32_t)__builtin_ctzll(m) : 64u;
                if (pend && lane < first) {               // inside [T0, T1): denied, remaining 0
                    orem = 0;
                    if (TOK && A == kAlgoTB) tk = tb_refill(L, q.now_ms, sa, sb, sc);
                    pend = false;
                }
            }
            bool changed = false;
            bool t_fresh = false;                         // [T0, T1) is for the current state
            const uint64_t c_run = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
            if constexpr (A == kAlgoTB) {
                // token bucket: rounds; each applies the prefix up to the first state change
                // (every earlier pending request is denied and leaves the state alone, Lua
                // :61-67), so a chunk costs 1 + its allows (the balance is a sequential fp64
                // recurrence, Lua :56-63)
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
                            const bool fast = q.op == (uint32_t)kOpAcquire && q.now_ms >= T0 && q.now_ms < T1;
                            const uint64_t m = __ballot(pend && !fast);
                            const uint32_t first = m ? (uint32_t)__builtin_ctzll(m) : 64u;
                            if (pend && lane < first) {
                                oa = false;
                                orem = 0;
                                if (TOK) tk = tb_refill(L, q.now_ms, sa, sb, sc);
                                pend = false;
                            }
                        }
                    }
                }
            } else {
                // sliding window: inside one window W the acquires only INCR the current
                // bucket (:114-116), so with k allows before it a request's estimate is
                // d2l(tv + (C0 + k)), tv = prev * pw at its own time (:174): the request is
                // allowed iff k <= K, its largest such k. One pass computes tv and K per
                // lane; the allows then follow by a greedy scan of integer compares (the
                // k-th allow is the first request after the (k-1)-th with K >= k). Requests
                // the scan cannot take (another window, before the newest bucket, a peek or
                // a reset) run the exact step alone.
                const SWGeo geo = pend ? sw_geo(q.now_ms, L) : SWGeo{};
                const int64_t w = L.window_ms, mx = L.max_permits;
                while (__any(pend)) {
                    const uint32_t f0 = (uint32_t)__builtin_ctzll(__ballot(pend));
                    const int64_t W0 = (int64_t)readlane64((uint64_t)geo.curr_start, f0);
                    const bool scan = pend && q.op == (uint32_t)kOpAcquire && geo.curr_start == W0 &&
                                      (int64_t)sa <= W0 && geo.prev_start != geo.curr_start;
                    const uint64_t und = __ballot(pend && !scan);
                    const uint32_t stop = und ? (uint32_t)__builtin_ctzll(und) : 64u;
                    const bool in = scan && lane < stop;
                    if (__any(in)) {
                        const SW2 s0 = sw_unpack(sa, sb, sc);
                        const int64_t C0 = s0.b1_start == W0 ? (int64_t)s0.b1_cnt : 0;
                        const int64_t P = in ? sw_get(s0, geo.prev_start, q.now_ms, w) : 0;
                        const double tv = (double)P * geo.prev_weight;           // :174, rounded
                        auto est = [&](int64_t k) { return d2l(tv + (double)(C0 + k)); };
                        int64_t K = mx - (int64_t)q.permits - C0 - (int64_t)tv;  // ~ largest k
                        if (K >= 0 && est(K) + q.permits > mx) --K;             // rounding edges
                        if (K >= 0 && est(K) + q.permits > mx) --K;
                        if (est(K + 1) + q.permits <= mx) ++K;
                        if (K < -1) K = -1;
                        // greedy scan: kk = allows before this request inside the chunk
                        int64_t kk = 0, k = 0;
                        bool al = false;
                        uint32_t cur = 0, last = 0;
                        for (;;) {
                            const uint64_t m = __ballot(in && lane >= cur && K >= k);
                            if (in && lane >= cur) kk = k;
                            if (!m) break;
                            const uint32_t fa = (uint32_t)__builtin_ctzll(m);
                            if (lane == fa) al = true;
                            last = fa;
                            ++k;
                            cur = fa + 1;
                        }
                        if (in) {
                            const int64_t e = est(al ? kk + 1 : kk);             // after the request
                            oa = al;
                            orem = mx - e > 0 ? mx - e : 0;
                            n_allowed += al ? 1u : 0u;
                            pend = false;
                        }
                        if (k > 0) {
                            const int64_t t_last = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                                (int)(uint32_t)(q.now_ms >> 32), (int)last) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)q.now_ms, (int)last));
                            SWGeo gl{};
                            gl.curr_start = W0;
                            sw_commit_allows(L, gl, sa, sb, sc, (uint32_t)k, t_last);
                            changed = true;
                        }
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
                T1 = t1_of(T0);
                ++n_tk;
            } else if (T1 < hi && __any(hot && q.op == (uint32_t)kOpAcquire && q.now_ms >= T1)) {
                // no change although requests lay past T1: T1 was only a lower bound of the
                // first allowed time (the guess undershot); without this the chunks up to
                // the real one would all be read and decided one by one. Exact, from T0.
                T1 = wave_first_true(T0, hi, lane,
                                     [&](int64_t t) { return hot_pred_k<A>(L, t, sa, sb, sc, 1); });
                ++n_tk;
            }
            if (a.dbg) {
                const uint64_t c_end = __builtin_amdgcn_s_memtime();
                cyc_run += c_srch - c_run;
                cyc_search += c_end - c_srch;
            }
            if (hot) {
                put_res<Res>(a, j, oa, orem);
                if (TOK) a.tok[j] = tk;
            }
            if (a.dbg) cyc_detail += __builtin_amdgcn_s_memtime() - c_det;
        };
        // level 1: the chunks of one group of 64
        auto walk_group = [&](uint32_t grp) {
            const uint32_t c = grp * 64 + lane;
            const bool has = c < f.n_chunks;
            uint64_t* sm = summ_at(c);
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
                detail(grp * 64 + fst);
            }
        };
        // level 2: 64 groups per test, the next 64 in flight
        ulonglong2 nx01 = *(const ulonglong2*)grp_at(lane);
        uint64_t nx2 = grp_at(lane)[2], nx3 = grp_at(lane)[3];
        for (uint32_t g0 = 0; g0 < f.n_groups; g0 += 64) {
            const uint32_t g = g0 + lane;
            const bool has = g < f.n_groups;
            uint64_t* sg = grp_at(g);
            const ulonglong2 v01 = nx01;
            const uint64_t v2 = nx2, v3 = nx3;
            nx01 = *(const ulonglong2*)grp_at(g + 64);
            nx2 = grp_at(g + 64)[2];
            nx3 = grp_at(g + 64)[3];
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
            if (v) {
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
            return __ballot(g < f.n_groups && (!hot_ok || ((grp_at(g)[3] >> 8) & 1u)));
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
                if (c < f.n_chunks) no = hot_ok ? (uint32_t)(summ_at(c)[3] >> 8) & 0xFFu : 64u;
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
    if (wid == 0) {
        if (hot_ok) {
            if (L.algo == kAlgoTB) pass1(std::integral_constant<int, kAlgoTB>{});
            else pass1(std::integral_constant<int, kAlgoSW>{});
        }
    } else {
        if (L.algo == kAlgoTB) pass2(std::integral_constant<int, kAlgoTB>{});
        else pass2(std::integral_constant<int, kAlgoSW>{});
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
    __shared__ uint64_t s_w1[2];                      // wave 1's debug counters
    if (wid == 1 && lane == 0) { s_w1[0] = n_other; s_w1[1] = cyc_pass2; }
    const bool touched_hot = __syncthreads_or(any_hot);
    if (wid != 0) return;
    if (lane == 0 && hot_ok && touched_hot) S.occ[hs] |= 2u;
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
        }
    }
}

// HOT: 2-wave workgroups; the first kHotMax run the hot regions' chains (hot_chain), the
// rest two normal regions each: one launch, so the chains are dispatched before the
// normal regions fill the machine, at the LDS per wave of the plain kernel.
#ifndef RL_HOT_MIN_WAVES
#define RL_HOT_MIN_WAVES 4
#endif
// Normal regions (one wave each) at >= RL_REGION_MIN_WAVES waves per SIMD (VGPR budget).
#ifndef RL_REGION_MIN_WAVES
#define RL_REGION_MIN_WAVES 4
#endif
template <class Codec, class Res, bool TOK, int BS, bool HOT, bool CACHE = false>
__global__ __launch_bounds__(HOT ? 128 : 64, HOT ? RL_HOT_MIN_WAVES : BS > 0 ? 3 : RL_REGION_MIN_WAVES)
void k_regions(RegionArgs a) {
    if constexpr (CACHE) {                       // some limiter keeps a local cache (BS 0, no hot path)
        __shared__ RegionTableX S;
        region_body_t<Codec, Res, TOK, 0>(a, blockIdx.x, S);
    } else if constexpr (HOT) {
        __shared__ union U { RegionTable two[2]; RegionLds<Codec, true> one; } S;
        if (blockIdx.x < kHotMax) {
            hot_chain<Codec, Res, TOK>(a, blockIdx.x, S.one);
            return;
        }
        region_body_t<Codec, Res, TOK, BS>(a, (blockIdx.x - kHotMax) * 2 + (threadIdx.x >> 6),
                                           S.two[threadIdx.x >> 6]);
    } else {
        __shared__ RegionLds<Codec, (BS > 0)> S;
        region_body_t<Codec, Res, TOK, BS>(a, blockIdx.x, S);
    }
}

// The hot chains alone (2-wave workgroups), launched on a side stream just before the
// normal regions' single-wave launch: no normal region waits for the other region of a
// 2-wave workgroup, and the chains still start first.
template <class Codec, class Res, bool TOK>
__global__ __launch_bounds__(128, RL_HOT_MIN_WAVES) void k_hot_chains(RegionArgs a) {
    __shared__ RegionLds<Codec, true> S;
    hot_chain<Codec, Res, TOK>(a, blockIdx.x, S);
}

// Normal regions, persistent (rl_tune "region_walk"): `walk` waves per CU claim chunks of
// regions from 8 counters (one per eighth of the region range; a wave starts at its own
// and then helps the others), so no wave slot waits for a workgroup launch and a sparse
// region's memory latency overlaps other regions' work on the same SIMD.
template <class Codec, class Res, bool TOK>
__global__ __launch_bounds__(64, RL_REGION_MIN_WAVES) void k_regions_walk(RegionArgs a, uint32_t chunk) {
    __shared__ RegionLds<Codec, false> S;
    constexpr uint32_t K = 8;
    const uint32_t n = a.n_regions, per = (n + K - 1) / K;
    for (uint32_t k = 0; k < K; ++k) {
        const uint32_t c = (blockIdx.x + k) % K;
        const uint32_t lo = c * per, hi = min(n, lo + per);
        for (;;) {
            uint32_t g0 = 0;
            if (threadIdx.x == 0) g0 = atomicAdd(a.work + c * 16, chunk);
            g0 = __builtin_amdgcn_readfirstlane(g0);
            if (g0 >= hi - min(hi, lo)) break;
            const uint32_t end = min(hi, lo + g0 + chunk);
            for (uint32_t g = lo + g0; g < end; ++g) {
                region_body_t<Codec, Res, TOK, 0>(a, g, S);
                wave_fence();
            }
        }
    }
}

// Phase C (one wave per chunk, all CUs): results of the chunks the chain decided.
template <class Codec, class Res, bool TOK>
__global__ __launch_bounds__(256) void k_hot_fill(RegionArgs a) {
    __shared__ uint32_t s_base[kHotMax + 1];
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const uint32_t total = a.hot_total[0];
    for (uint32_t i = threadIdx.x; i < hc; i += 256) s_base[i] = a.hot_info[i].chunk_base;
    __syncthreads();
    if (a.ctl->span_overflow != 0) return;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const typename Codec::Rec* recs = (const typename Codec::Rec*)a.rec;
    const int64_t base = a.ctl->base_ms;
    Res* res = (Res*)a.res;
    for (uint32_t g = blockIdx.x * 4 + wid; g < total; g += gridDim.x * 4) {
        const uint32_t i = hot_region_of(s_base, hc, g);
        const HotInfo f = a.hot_info[i];
        const uint32_t c = g - s_base[i];
        const uint64_t* s1 = a.hot_summ + (size_t)g * 4;
        const uint64_t* s2 = a.hot_summ2 + (size_t)(f.group_base + c / 64) * 4;
        const uint64_t v2 = s2[3], v1 = s1[3];
        // decided as part of its group (state in the group summary), or on its own
        const uint64_t* sm = (v2 & 1u) ? s2 : s1;
        const uint64_t verdict = (v2 & 1u) ? ((v2 & 3u) | (v1 & 0xFF00u)) : v1;
        if (!(verdict & 1u)) continue;
        const uint32_t j = f.start + c * kHotChunk + lane;
        if (j >= f.end) continue;
        // the hot records here are acquires (n_special == 0); TB permits > max (verdict
        // bit 1) are the only ones not (deny, 0); other keys' records (bits 8-15) are
        // k_hot_chain's
        const DevLimiter& L = a.lims[a.region_lim[f.bin]];
        if (!TOK && !(verdict & 0xFF02u)) {
            res[j] = (Res)pack_result(false, 0);
            continue;
        }
        const Req q = Codec::dec(recs[j], base);
        if (q.invalid || q.h != f.tag) continue;          // another key (f.ok holds here)
        const bool early = L.algo == kAlgoTB && (int64_t)q.permits > L.max_permits;
        res[j] = (Res)pack_result(false, early ? kRemUnknown : 0);
        if (TOK) a.tok[j] = (L.algo == kAlgoTB && !early) ? tb_refill(L, q.now_ms, sm[0], sm[1], sm[2])
                                                         : __builtin_nan("");
    }
}

// Hot-region selection, largest first: k_hot_hist counts the bins at or above the
// threshold per power-of-two size class; k_hot_select then raises the threshold to the
// smallest class boundary that admits at most kHotMax bins and lists those bins.
// hot_meta: [0] listed count, [1 .. 33] size-class histogram.
__device__ inline uint32_t bin_records(const uint32_t* rstart, const uint32_t* rcount,
                                       const uint32_t* rend, uint32_t b) {
    return rend ? rend[b] - rstart[b] : rcount[b];
}

__global__ __launch_bounds__(256) void k_hot_hist(const uint32_t* rstart, const uint32_t* rcount,
                                                  const uint32_t* rend, uint32_t n_bins,
                                                  uint32_t threshold, uint32_t* hot_meta) {
    __shared__ uint32_t h[33];
    if (threadIdx.x < 33) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b < n_bins) {
        const uint32_t cnt = bin_records(rstart, rcount, rend, b);
        if (cnt >= threshold && cnt > 0) atomicAdd(&h[31 - __builtin_clz(cnt)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 33 && h[threadIdx.x]) atomicAdd(&hot_meta[1 + threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_hot_select(const uint32_t* rstart, const uint32_t* rcount,
                                                    const uint32_t* rend, uint32_t n_bins,
                                                    uint32_t threshold, uint32_t* hot_list,
                                                    uint32_t* hot_meta, uint32_t* hot_mark,
                                                    uint32_t epoch) {
    __shared__ uint32_t s_thr;
    __shared__ uint32_t s_off[33];                    // list offset of each size class
    if (threadIdx.x == 0) {
        uint32_t above = 0, thr = 0xFFFFFFFFu;
        for (int c = 32; c >= 0; --c) {               // classes from the largest down
            s_off[c] = above;
            above += hot_meta[1 + c];
            if (above > kHotMax) break;
            thr = c == 0 ? 1u : (1u << c);
        }
        s_thr = thr > threshold ? thr : threshold;
    }
    __syncthreads();
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= n_bins) return;
    const uint32_t cnt = bin_records(rstart, rcount, rend, b);
    if (cnt == 0 || cnt < s_thr) return;
    // largest size class first: the chains' workgroups are dispatched in list order, and the
    // longest chains must not be the ones that wait for a slot beside the normal regions
    const uint32_t c = 31u - (uint32_t)__builtin_clz(cnt);
    const uint32_t k = s_off[c] + atomicAdd(&hot_meta[kHotClassCursor + c], 1u);
    atomicAdd(&hot_meta[0], 1u);
    if (k < kHotMax) {                                // (always, by the choice of s_thr)
        hot_list[k] = b;
        hot_mark[b] = epoch;
    }
}

// Bin boundaries of the final record order (two-pass partitions): rstart[b] / rend[b]
// for every bin b < n_bins. The high-digit pass leaves run hi = [hi_base[hi],
// hi_base[hi] + hi_total[hi]) whose records are still in low-digit order (the pass is
// stable over the low-digit pass's output), so each low digit's first record is a
// binary search inside its run: one workgroup per run, ~log2(run) record probes per
// bin instead of reading every record of the batch.
template <class Codec>
__global__ __launch_bounds__(256) void k_bin_bounds(BoundsArgs a) {
    __shared__ uint32_t s_base[256];
    __shared__ uint8_t s_bits[256];
    __shared__ uint32_t s_lb[(1u << kMaxDigitBits) + 1];
    for (uint32_t l = threadIdx.x; l < a.n_lim; l += 256) {
        s_base[l] = a.lims[l].region_base;
        s_bits[l] = (uint8_t)a.lims[l].region_bits;
    }
    __syncthreads();
    const typename Codec::Rec* recs = (const typename Codec::Rec*)a.rec;
    const uint32_t nlo = 1u << a.d0, lo_mask = nlo - 1;
    auto lo_of = [&](uint32_t i) {
        const typename Codec::Rec r = recs[i];
        const uint32_t lim = Codec::limiter_of(r);
        return ((s_base[lim] + region_local(r.h, a.shard_bits, s_bits[lim])) >> a.bin_shift) & lo_mask;
    };
    const uint32_t hi = blockIdx.x;
    const uint32_t beg = a.hi_base[hi], end = beg + a.hi_total[hi];
    for (uint32_t lo = threadIdx.x; lo <= nlo; lo += 256) {
        uint32_t L = beg, R = end;                    // first record with low digit >= lo
        if (lo == nlo) L = end;
        while (L < R) {
            const uint32_t m = L + (R - L) / 2;
            if (lo_of(m) < lo) L = m + 1;
            else R = m;
        }
        s_lb[lo] = L;
    }
    __syncthreads();
    for (uint32_t lo = threadIdx.x; lo < nlo; lo += 256) {
        const uint32_t b = (hi << a.d0) | lo;
        if (b < a.n_bins) {
            a.rstart[b] = s_lb[lo];
            a.rend[b] = s_lb[lo + 1];
        }
    }
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
            for (int k = 0; k < B; ++k) v[k] = res[p[k]];
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
#pragma unroll
            for (int k = 0; k < B; ++k) p[k] = pos1[p[k]];
        }
        if (a.ablate & kAblNoGather) {
#pragma unroll
            for (int k = 0; k < B; ++k) v[k] = (Res)p[k];
        } else {
#pragma unroll
            for (int k = 0; k < B; ++k) v[k] = res[p[k]];
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
        if (a.pos1_final) j = a.pos1_final[j];
        if ((uint64_t)rf[j] == kResEscape) {
          allowed[i] = 0;
          remaining[i] = a.ext[j];
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
template <class Res>
__global__ __launch_bounds__(256) void k_unpermute_mid(const uint32_t* __restrict__ pos1,
                                                       const Res* __restrict__ res,
                                                       Res* __restrict__ mid, uint32_t n) {
    constexpr int B = 8;
    const uint32_t base = blockIdx.x * (256u * B) + threadIdx.x;
    uint32_t p[B];
#pragma unroll
    for (int k = 0; k < B; ++k) {
        const uint32_t j = base + (uint32_t)k * 256u;
        p[k] = pos1[j < n ? j : 0];
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

// ------------------------------------------------------------------ synthetic traces
// Deterministic in (seed, global index). Zipf via rejection-inversion (Hoermann &
// Derflinger 1996, as in Apache Commons RejectionInversionZipfSampler).
__device__ inline uint64_t splitmix(uint64_t x) { return mix64(x + 0x9E3779B97F4A7C15ULL); }
__device__ inline double u01(uint64_t x) { return (double)(splitmix(x) >> 11) * 0x1.0p-53; }
__device__ inline double zh1(double x) { return fabs(x) > 1e-8 ? log1p(x) / x : 1.0 - x * (0.5 - x / 3.0); }
__device__ inline double zh2(double x) { return fabs(x) > 1e-8 ? expm1(x) / x : 1.0 + x * 0.5 * (1.0 + x / 3.0); }
__device__ inline double zH(double x, double s) { const double lx = log(x); return zh2((1.0 - s) * lx) * lx; }
__device__ inline double zh(double x, double s) { return exp(-s * log(x)); }
__device__ inline double zHinv(double x, double s) {
    double t = x * (1.0 - s);
    if (t < -1.0) t = -1.0;
    return exp(zh1(t) * x);
}

__global__ __launch_bounds__(256) void k_synth(SynthArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint64_t gi = a.index_base + i;
    const uint64_t sd = a.seed * 0xD1B54A32D192ED03ULL;
    uint64_t rank;
    if (a.dist == 0) {
        rank = splitmix(sd ^ (gi * 0x9E3779B97F4A7C15ULL)) % a.n_keys;
    } else {
        const double n = (double)a.n_keys;
        uint64_t k = 1;
        for (uint32_t att = 0; att < 64; ++att) {
            const double u = a.hn + u01(sd ^ (gi * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)att << 56)) *
                                        (a.hx1 - a.hn);
            const double x = zHinv(u, a.zs);
            double kd = floor(x + 0.5);
            if (kd < 1.0) kd = 1.0;
            if (kd > n) kd = n;
            k = (uint64_t)kd;
            if (kd - x <= a.sconst || u >= zH(kd + 0.5, a.zs) - zh(kd, a.zs)) break;
        }
        rank = k - 1;
    }
    a.key[i] = mix64(rank ^ (a.seed << 32) ^ 0x5EEDULL);
    const uint64_t r2 = splitmix(sd ^ (gi * 0xA24BAED4963EE407ULL) ^ 0x77ULL);
    a.permits[i] = 1 + (int32_t)(r2 % (uint64_t)a.permits_max);
    a.now_ns[i] = a.t0_ns + (int64_t)((double)gi * (double)a.span_ns / (double)a.n_total);
    if (a.limiter) a.limiter[i] = (uint16_t)(rank % a.n_limiters);
}

// ------------------------------------------------------------------ owner partition
// Stable partition of a batch by owner shard (multi-GPU routing). One block per
// 16K tile computes per-tile counts (upsweep), the host-side scan is done by
// k_scan_rows, and the same tile re-ranks stably (shard_count <= 64).
//
// owner(h) = top log2(G) bits of mix64(h), except for the keys of the hot-key directory
// (rl_set_owner_directory): an open-addressing table of kDirSlots {tag, owner} that places
// the hottest keys explicitly so that one owner does not carry the top Zipf keys together.
__device__ inline uint32_t owner_of_tag(uint64_t t, int sbits, const DirSlot* dir) {
    if (dir) {
        uint32_t p = (uint32_t)t & (kDirSlots - 1);
        for (uint32_t i = 0; i < kDirSlots; ++i) {
            const DirSlot d = dir[p];
            if (d.owner == kDirEmpty) break;
            if (d.tag == t) return d.owner;
            p = (p + 1) & (kDirSlots - 1);
        }
    }
    return sbits ? (uint32_t)(t >> (64 - sbits)) : 0u;
}

__global__ __launch_bounds__(kTileThreads) void k_owner_count(const uint64_t* key, uint32_t n,
                                                              int sbits, uint32_t n_tiles,
                                                              uint32_t* counts, const DirSlot* dir) {
    __shared__ uint32_t hist[64];
    const uint32_t t = threadIdx.x;
    if (t < 64) hist[t] = 0;
    __syncthreads();
    const uint32_t tile = blockIdx.x;
    for (int r = 0; r < kTileItems; ++r) {
        const uint32_t i = tile * (uint32_t)kTile + (uint32_t)r * kTileThreads + t;
        if (i < n) atomicAdd(&hist[owner_of_tag(mix64(key[i]), sbits, dir)], 1u);
    }
    __syncthreads();
    if (t < (1u << sbits)) counts[(size_t)t * n_tiles + tile] = hist[t];
}

__global__ __launch_bounds__(kTileThreads) void k_owner_scatter(const uint64_t* key, uint32_t n,
                                                                int sbits, uint32_t n_tiles,
                                                                const uint32_t* counts,
                                                                const uint32_t* bin_base,
                                                                uint32_t* perm, const DirSlot* dir) {
    __shared__ uint32_t cur[64];
    __shared__ uint8_t cntw[kTileThreads / 64][64];
    const uint32_t t = threadIdx.x, wid = t >> 6;
    const uint32_t tile = blockIdx.x;
    const uint32_t bins = 1u << sbits;
    if (t < bins) {
        cur[t] = bin_base[t] + counts[(size_t)t * n_tiles + tile];
        for (int w = 0; w < kTileThreads / 64; ++w) cntw[w][t] = 0;
    }
    __syncthreads();
    for (int r = 0; r < kTileItems; ++r) {
        const uint32_t i = tile * (uint32_t)kTile + (uint32_t)r * kTileThreads + t;
        const bool active = i < n;
        const uint32_t d = active ? owner_of_tag(mix64(key[i]), sbits, dir) : 0u;
        const uint64_t m = wave_match(d, sbits, active);
        const uint32_t lr = popc_below(m);
        const uint32_t c = (uint32_t)__popcll(m);
        const bool leader = active && lr == 0;
        if (leader) cntw[wid][d] = (uint8_t)c;
        __syncthreads();
        uint32_t pos = 0;
        if (active) {
            pos = cur[d] + lr;
            for (uint32_t w = 0; w < wid; ++w) pos += cntw[w][d];
        }
        __syncthreads();
        if (leader) { atomicAdd(&cur[d], c); cntw[wid][d] = 0; }
        if (active) perm[pos] = i;
    }
}

// ------------------------------------------------------------------ route pack / unpack
// Multi-GPU routing: gather requests into owner order (perm from k_owner_scatter) before
// the all-to-all, and scatter the returned decisions back to arrival order after it.
__global__ __launch_bounds__(256) void k_route_pack(uint32_t n, const uint32_t* __restrict__ perm,
                                                    const uint64_t* __restrict__ key,
                                                    const int32_t* __restrict__ permits,
                                                    const int64_t* __restrict__ now,
                                                    const uint16_t* __restrict__ lim,
                                                    uint64_t* __restrict__ key_o,
                                                    int32_t* __restrict__ permits_o,
                                                    int64_t* __restrict__ now_o,
                                                    uint16_t* __restrict__ lim_o) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = perm[j];
    key_o[j] = key[i];
    permits_o[j] = permits[i];
    now_o[j] = now[i];
    if (lim_o) lim_o[j] = lim ? lim[i] : 0;
}

// decisions travel as one int64 per request: remaining * 2 + allowed
__global__ __launch_bounds__(256) void k_route_fold(uint32_t n, const uint8_t* __restrict__ allowed,
                                                    const int64_t* __restrict__ remaining,
                                                    int64_t* __restrict__ packed) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) packed[j] = (int64_t)((uint64_t)remaining[j] << 1) | (int64_t)(allowed[j] & 1u);
}

__global__ __launch_bounds__(256) void k_route_unpack(uint32_t n, const uint32_t* __restrict__ perm,
                                                      const int64_t* __restrict__ packed,
                                                      uint8_t* __restrict__ allowed,
                                                      int64_t* __restrict__ remaining) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int64_t v = packed[j];
    const uint32_t i = perm[j];
    allowed[i] = (uint8_t)(v & 1);
    remaining[i] = v >> 1;
}

// Compact wire: 16 B per request in owner order. wire[2j] = key hash, wire[2j+1] =
// permits (as u32) << 32 | (now_ms - base_ms). base_ms = floor(now_ns[0] / 1e6) - 2^31 of
// this source's batch, so any batch spanning < 2^31 ms each side of its first request is
// exact; hdr[1] flags a request outside that range (the router then sends this step in
// the wide layout). The engine floors now_ns to ms, so nothing it reads is lost.
__global__ __launch_bounds__(256) void k_route_pack_wire(uint32_t n, const uint32_t* __restrict__ perm,
                                                         const uint64_t* __restrict__ key,
                                                         const int32_t* __restrict__ permits,
                                                         const int64_t* __restrict__ now,
                                                         const uint16_t* __restrict__ lim,
                                                         uint64_t* __restrict__ wire,
                                                         uint16_t* __restrict__ lim_o,
                                                         int64_t* __restrict__ hdr,
                                                         uint64_t* __restrict__ part) {
    // grid-stride (a capped grid): with `part`, block b leaves the ordered-key min / max of
    // its requests' now_ms in part[2b], part[2b+1] (the router's header reduces them; no
    // atomics on one word, which sustains only ~88 adds per us)
    const int64_t base = floor_div_ms(now[0]) - (1LL << 31);
    if (blockIdx.x == 0 && threadIdx.x == 0) hdr[0] = base;
    bool bad = false;
    uint64_t mn = ~0ULL, mx = 0;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const uint32_t i = perm[j];
        const int64_t ms = floor_div_ms(now[i]);
        const int64_t rel = ms - base;
        bad |= rel < 0 || rel > 0xFFFFFFFFLL;
        const uint64_t k = ord_key(ms);
        mn = k < mn ? k : mn;
        mx = k > mx ? k : mx;
        ulonglong2 w;
        w.x = key[i];
        w.y = (uint64_t)(uint32_t)permits[i] << 32 | (uint64_t)(uint32_t)rel;
        *(ulonglong2*)(wire + 2 * (size_t)j) = w;
        if (lim_o) lim_o[j] = lim ? lim[i] : 0;
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr((unsigned long long*)&hdr[1], 1ULL);
    if (part) {
        __shared__ uint64_t s_mm[2][4];
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
        }
        const uint32_t w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) { s_mm[0][w] = mn; s_mm[1][w] = mx; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (uint32_t k = 1; k < blockDim.x / 64; ++k) {
                mn = s_mm[0][k] < mn ? s_mm[0][k] : mn;
                mx = s_mm[1][k] > mx ? s_mm[1][k] : mx;
            }
            part[2 * blockIdx.x] = mn;
            part[2 * blockIdx.x + 1] = mx;
        }
    }
}


struct WireSrc {                 // receiver: source s holds requests [end[s-1], end[s])
    int64_t base[kMaxShards];
    uint32_t end[kMaxShards];
    uint32_t n_src;
};

__global__ __launch_bounds__(256) void k_route_unwire(uint32_t m, const uint64_t* __restrict__ wire,
                                                      WireSrc src, uint64_t* __restrict__ key_o,
                                                      int32_t* __restrict__ permits_o,
                                                      int64_t* __restrict__ now_o) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    uint32_t s = 0;
    while (s + 1 < src.n_src && j >= src.end[s]) ++s;
    const ulonglong2 w = *(const ulonglong2*)(wire + 2 * (size_t)j);
    key_o[j] = w.x;
    permits_o[j] = (int32_t)(uint32_t)(w.y >> 32);
    now_o[j] = (src.base[s] + (int64_t)(uint32_t)w.y) * 1000000LL;
}

// Decisions travel back in the engine's packed-result width W (1 B for max <= 124):
// ((remaining + 3) << 1) | allowed, as pack_result.
template <class W>
__global__ __launch_bounds__(256) void k_route_fold_w(uint32_t n, const uint8_t* __restrict__ allowed,
                                                      const int64_t* __restrict__ remaining,
                                                      W* __restrict__ packed) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) packed[j] = (W)pack_result(allowed[j] & 1u, remaining[j]);
}

template <class W>
__global__ __launch_bounds__(256) void k_route_unpack_w(uint32_t n, const uint32_t* __restrict__ perm,
                                                        const W* __restrict__ packed,
                                                        uint8_t* __restrict__ allowed,
                                                        int64_t* __restrict__ remaining) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t v = (uint64_t)packed[j];
    const uint32_t i = perm[j];
    allowed[i] = (uint8_t)(v & 1u);
    remaining[i] = (int64_t)(v >> 1) - kResBias;
}

// Return trip in segments (router): the decisions for peer s travel as
//   [ round8(count_s * W) bytes of packed results ][ exception block ]
// where the block = {count u64, cap x (position i64, remaining i64)} lists the results
// whose remaining is outside W's range (TB balances below -3 after time regression,
// kResEscape). One all-to-all carries both, with byte splits the host already knows from
// the header exchange; nothing else crosses for the rare exact values.
struct RetLayout {
    uint64_t off[kMaxShards];    // byte offset of segment s
    uint32_t end[kMaxShards];    // requests [end[s-1], end[s]) belong to segment s
    uint32_t n_seg;
    uint32_t cap;                // exception entries per block
};

__device__ inline uint32_t seg_of(const RetLayout& L, uint32_t j) {
    uint32_t s = 0;
    while (s + 1 < L.n_seg && j >= L.end[s]) ++s;
    return s;
}
__device__ inline uint64_t seg_block(const RetLayout& L, uint32_t s, uint32_t W) {
    const uint32_t beg = s ? L.end[s - 1] : 0u;
    return L.off[s] + (((uint64_t)(L.end[s] - beg) * W + 7) & ~7ULL);
}

__global__ __launch_bounds__(64) void k_ret_init(uint8_t* out, RetLayout L, uint32_t W) {
    for (uint32_t s = threadIdx.x; s < L.n_seg; s += 64) *(uint64_t*)(out + seg_block(L, s, W)) = 0;
}

template <class W>
__global__ __launch_bounds__(256) void k_route_fold_ret(uint32_t m, const uint8_t* __restrict__ allowed,
                                                        const int64_t* __restrict__ remaining,
                                                        uint8_t* __restrict__ out, RetLayout L) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t s = seg_of(L, j);
    const uint32_t beg = s ? L.end[s - 1] : 0u;
    const int64_t rem = remaining[j];
    W* seg = (W*)(out + L.off[s]);
    if (res_fits<W>(rem)) {
        seg[j - beg] = (W)pack_result(allowed[j] & 1u, rem);
    } else {
        seg[j - beg] = (W)kResEscape;
        uint64_t* blk = (uint64_t*)(out + seg_block(L, s, sizeof(W)));
        const uint64_t k = atomicAdd((unsigned long long*)blk, 1ULL);
        if (k < L.cap) { blk[1 + 2 * k] = j - beg; blk[2 + 2 * k] = (uint64_t)rem; }
    }
}

template <class W>
__global__ __launch_bounds__(256) void k_route_unpack_ret(uint32_t n, const uint32_t* __restrict__ perm,
                                                          const uint8_t* __restrict__ in, RetLayout L,
                                                          uint8_t* __restrict__ allowed,
                                                          int64_t* __restrict__ remaining,
                                                          uint32_t* __restrict__ lost) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t s = seg_of(L, j);
    const uint32_t beg = s ? L.end[s - 1] : 0u;
    const uint64_t v = (uint64_t)((const W*)(in + L.off[s]))[j - beg];
    const uint32_t i = perm[j];
    if (v != kResEscape) {
        allowed[i] = (uint8_t)(v & 1u);
        remaining[i] = (int64_t)(v >> 1) - kResBias;
        return;
    }
    const uint64_t* blk = (const uint64_t*)(in + seg_block(L, s, sizeof(W)));
    const uint64_t cnt = blk[0] < L.cap ? blk[0] : L.cap;
    int64_t r = kRemError;                       // not found: the block overflowed
    bool found = false;
    for (uint64_t k = 0; k < cnt; ++k)
        if (blk[1 + 2 * k] == j - beg) { r = (int64_t)blk[2 + 2 * k]; found = true; break; }
    if (!found) atomicAdd(lost, 1u);
    allowed[i] = 0;
    remaining[i] = r;
}

hipError_t launch_route_fold_ret(uint32_t m, const uint8_t* allowed, const int64_t* remaining,
                                 void* out, int width, uint32_t n_seg, const uint64_t* counts,
                                 uint32_t cap, hipStream_t s) {
    if (n_seg == 0 || n_seg > (uint32_t)kMaxShards) return hipErrorInvalidValue;
    RetLayout L{};
    ret_layout(counts, n_seg, width, cap, L.off, L.end);
    L.n_seg = n_seg;
    L.cap = cap;
    hipLaunchKernelGGL(k_ret_init, dim3(1), dim3(64), 0, s, (uint8_t*)out, L, (uint32_t)width);
    if (m == 0) return hipGetLastError();
    const dim3 g((m + 255) / 256), b(256);
    uint8_t* o = (uint8_t*)out;
    switch (width) {
    case 1: hipLaunchKernelGGL(k_route_fold_ret<uint8_t>, g, b, 0, s, m, allowed, remaining, o, L); break;
    case 2: hipLaunchKernelGGL(k_route_fold_ret<uint16_t>, g, b, 0, s, m, allowed, remaining, o, L); break;
    case 4: hipLaunchKernelGGL(k_route_fold_ret<uint32_t>, g, b, 0, s, m, allowed, remaining, o, L); break;
    case 8: hipLaunchKernelGGL(k_route_fold_ret<uint64_t>, g, b, 0, s, m, allowed, remaining, o, L); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_route_unpack_ret(uint32_t n, const uint32_t* perm, const void* in, int width,
                                   uint32_t n_seg, const uint64_t* counts, uint32_t cap,
                                   uint8_t* allowed, int64_t* remaining, uint32_t* lost,
                                   hipStream_t s) {
    if (n_seg == 0 || n_seg > (uint32_t)kMaxShards) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    RetLayout L{};
    ret_layout(counts, n_seg, width, cap, L.off, L.end);
    L.n_seg = n_seg;
    L.cap = cap;
    const dim3 g((n + 255) / 256), b(256);
    const uint8_t* x = (const uint8_t*)in;
    switch (width) {
    case 1: hipLaunchKernelGGL(k_route_unpack_ret<uint8_t>, g, b, 0, s, n, perm, x, L, allowed, remaining, lost); break;
    case 2: hipLaunchKernelGGL(k_route_unpack_ret<uint16_t>, g, b, 0, s, n, perm, x, L, allowed, remaining, lost); break;
    case 4: hipLaunchKernelGGL(k_route_unpack_ret<uint32_t>, g, b, 0, s, n, perm, x, L, allowed, remaining, lost); break;
    case 8: hipLaunchKernelGGL(k_route_unpack_ret<uint64_t>, g, b, 0, s, n, perm, x, L, allowed, remaining, lost); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Owner partition with the per-owner counts left on the device as int64 (column 0 of the
// router's G x 3 header, `stride` int64 apart): no host round-trip before the header
// exchange.
__global__ void k_counts_to_header(const uint32_t* counts, uint32_t g, int64_t* hdr, uint32_t stride) {
    const uint32_t t = threadIdx.x;
    if (t < g) hdr[(size_t)t * stride] = counts[t];
}

// Router header rows (kHdrWords int64 each): {count (already there), base_ms, overflow,
// published status, capacity, min now_ms, max now_ms, 0}; min / max folded from
// k_route_pack_wire's per-block partials (nparts = 0: an empty batch, min > max).
__global__ __launch_bounds__(256) void k_fill_header(int64_t* hdr, const int64_t* base_ovf,
                                                     int64_t status, int64_t cap, uint32_t g,
                                                     const uint64_t* part, uint32_t nparts) {
    __shared__ uint64_t s_mm[2][4];
    const uint32_t t = threadIdx.x;
    uint64_t mn = ~0ULL, mx = 0;
    for (uint32_t b = t; b < nparts; b += 256) {
        mn = part[2 * b] < mn ? part[2 * b] : mn;
        mx = part[2 * b + 1] > mx ? part[2 * b + 1] : mx;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    if ((t & 63) == 0) { s_mm[0][t >> 6] = mn; s_mm[1][t >> 6] = mx; }
    __syncthreads();
    for (int k = 0; k < 4; ++k) {
        mn = s_mm[0][k] < mn ? s_mm[0][k] : mn;
        mx = s_mm[1][k] > mx ? s_mm[1][k] : mx;
    }
    if (t < g) {
        int64_t* row = hdr + (size_t)t * kHdrWords;
        row[1] = base_ovf[0];
        row[2] = base_ovf[1];
        row[3] = status;
        row[4] = cap;
        row[5] = mn == ~0ULL ? INT64_MAX : (int64_t)(mn ^ 0x8000000000000000ULL);
        row[6] = mx == 0ULL ? INT64_MIN : (int64_t)(mx ^ 0x8000000000000000ULL);
        row[7] = 0;
    }
}

hipError_t launch_fill_header(int64_t* hdr, const int64_t* base_ovf, int64_t status, int64_t cap,
                              uint32_t g, const uint64_t* part, uint32_t nparts, hipStream_t s) {
    hipLaunchKernelGGL(k_fill_header, dim3(1), dim3(256), 0, s, hdr, base_ovf, status, cap, g, part,
                       nparts);
    return hipGetLastError();
}

// Requests not decided (a router step whose engine call failed): allowed 0, remaining `rem`.
__global__ void k_fill_value(uint8_t* allowed, int64_t* remaining, uint32_t n, int64_t rem) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { allowed[i] = 0; remaining[i] = rem; }
}

hipError_t launch_fill_value(uint8_t* allowed, int64_t* remaining, uint32_t n, int64_t rem,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill_value, dim3((n + 255) / 256), dim3(256), 0, s, allowed, remaining, n, rem);
    return hipGetLastError();
}

hipError_t launch_counts_to_header(const uint32_t* counts, uint32_t g, int64_t* hdr, uint32_t stride,
                                   hipStream_t s) {
    hipLaunchKernelGGL(k_counts_to_header, dim3(1), dim3(64), 0, s, counts, g, hdr, stride);
    return hipGetLastError();
}

// ------------------------------------------------------------------ state export / import
// Export: one thread per slot of one limiter's table; every bucket live at `now` becomes one
// Redis-layout entry (SW: "rl:<key>:<W>" counters, deadline last INCR + w; TB: "tb:<key>",
// deadline last_refill + 2w), compacted through one counter. The host sorts the entries.
__global__ __launch_bounds__(256) void k_export(const Slot* __restrict__ tab, uint64_t n_slots,
                                                DevLimiter L, uint16_t lim, int64_t now,
                                                StateRec* __restrict__ out, uint32_t cap,
                                                uint32_t* count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_slots) return;
    const Slot v = tab[i];
    StateRec r[2];
    int m = 0;
    const uint64_t key = unmix64(v.tag);
    if (L.algo == kAlgoTB) {
        if ((v.c & 1u) && !(now > (int64_t)v.b + L.ttl_ms)) {
            StateRec& e = r[m++];
            e = StateRec{};
            e.key_hash = key; e.limiter = lim; e.kind = 1;
            e.tokens = __longlong_as_double((long long)v.a);
            e.last_refill_ms = (int64_t)v.b;
            e.expire_at_ms = (int64_t)v.b + L.ttl_ms;
        }
    } else {
        const SW2 q = sw_unpack(v.a, v.b, v.c);
        const int64_t w = L.window_ms;
        const int64_t d1 = q.b1_start + q.b1_off + w, d0 = q.b1_start + q.b0_off;
        if (q.b0_cnt != 0 && !(now > d0)) {          // bucket b1_start - w (sorted first)
            StateRec& e = r[m++];
            e = StateRec{};
            e.key_hash = key; e.limiter = lim; e.kind = 0;
            e.window_start_ms = q.b1_start - w; e.count = q.b0_cnt; e.expire_at_ms = d0;
        }
        if (q.b1_cnt != 0 && !(now > d1)) {
            StateRec& e = r[m++];
            e = StateRec{};
            e.key_hash = key; e.limiter = lim; e.kind = 0;
            e.window_start_ms = q.b1_start; e.count = q.b1_cnt; e.expire_at_ms = d1;
        }
    }
    if (m == 0) return;
    const uint32_t k = atomicAdd(count, (uint32_t)m);
    for (int j = 0; j < m; ++j)
        if (k + (uint32_t)j < cap) out[k + j] = r[j];
}

// Whole-region rewrite shared by the state import and the TTL sweep: one wave stages the
// region's 256 slots, keeps those `keep` accepts, rebuilds the probe chains in LDS
// (linear probing from each key's home, as a batch's region load does) and later writes
// every slot back, so the HBM slot invariant (rl_device.hpp, slot_free) holds afterwards.
struct RegionStage {
    alignas(16) uint64_t tag[kRegionSlots];
    uint64_t sa[kRegionSlots], sb[kRegionSlots], sc[kRegionSlots], sx[kRegionSlots];
    uint32_t occ[kRegionSlots];
};

template <class Keep>
__device__ inline uint32_t stage_region(RegionStage& S, const Slot* tab, const uint64_t* xt,
                                        uint32_t lane, Keep keep) {
    constexpr uint32_t NS = kRegionSlots;
    Slot img[NS / 64];
    uint64_t xim[NS / 64];
    bool kp[NS / 64];
    uint32_t dropped = 0;
#pragma unroll
    for (uint32_t i = 0; i < NS / 64; ++i) {
        img[i] = tab[lane + 64 * i];
        xim[i] = xt ? xt[lane + 64 * i] : 0;
        kp[i] = !slot_free(img[i], xim[i]) && keep(img[i], xim[i]);
        dropped += (!slot_free(img[i], xim[i]) && !kp[i]) ? 1u : 0u;
        S.occ[lane + 64 * i] = 0;
    }
    wave_fence();
#pragma unroll
    for (uint32_t i = 0; i < NS / 64; ++i) {
        if (!kp[i]) continue;
        uint32_t p = slot_home(img[i].tag);
        while (atomicCAS(&S.occ[p], 0u, 1u) != 0u) p = (p + 1) & (NS - 1);
        S.tag[p] = img[i].tag; S.sa[p] = img[i].a; S.sb[p] = img[i].b; S.sc[p] = img[i].c;
        S.sx[p] = xim[i];
    }
    wave_fence();
    return dropped;
}

__device__ inline void write_region(const RegionStage& S, Slot* tab, uint64_t* xt, uint32_t lane) {
    for (uint32_t k = lane; k < kRegionSlots; k += 64) {
        Slot v{0, 0, 0, 0};
        uint64_t x = 0;
        if (S.occ[k] & kOccUsed) {
            x = S.sx[k];
            v = slot_used(Slot{S.tag[k], S.sa[k], S.sb[k], S.sc[k]}, x);
        }
        tab[k] = v;
        if (xt) xt[k] = x;
    }
}

// Import: one wave per region that receives entries. The region's present slots are
// staged and rebuilt, then its keys are applied in order: replace the slot holding the
// key's tag, else claim the first free slot of the key's probe sequence.
__global__ __launch_bounds__(64) void k_import(ImportArgs a) {
    __shared__ RegionStage S;
    constexpr uint32_t NS = kRegionSlots;
    const uint32_t g = blockIdx.x, lane = threadIdx.x;
    if (g >= a.n_groups) return;
    Slot* tab = (Slot*)(uintptr_t)a.region_addr[g];
    const int algo = a.group_algo[g];
    uint64_t* xt = (uint64_t*)(uintptr_t)a.xregion_addr[g];
    stage_region(S, tab, xt, lane,
                 [&](const Slot& v, uint64_t x) { return x != 0 || state_present(algo, v.b, v.c); });
    for (uint32_t j = a.group_off[g]; j < a.group_off[g + 1]; ++j) {
        const Slot im = a.img[j];
        const uint32_t home = slot_home(im.tag);
        int32_t p = -1;
        for (uint32_t b = 0; b < NS / 64 && p < 0; ++b) {    // probe order = (b, lane)
            const uint32_t s = (home + b * 64 + lane) & (NS - 1);
            const bool used = (S.occ[s] & kOccUsed) != 0;
            const uint64_t fre = __ballot(!used);
            const uint64_t hit = __ballot(used && S.tag[s] == im.tag);
            const uint64_t before = fre ? ((fre & (0 - fre)) - 1) | (fre & (0 - fre)) : ~0ULL;
            const uint64_t h = hit & before;                  // a hit before the first free slot
            if (h) p = (int32_t)((home + b * 64 + (uint32_t)__builtin_ctzll(h)) & (NS - 1));
            else if (fre) p = (int32_t)((home + b * 64 + (uint32_t)__builtin_ctzll(fre)) & (NS - 1));
        }
        if (p < 0) {
            if (lane == 0) atomicAdd(a.fail, 1u);
        } else if (lane == 0) {
            S.occ[p] = kOccUsed;
            S.tag[p] = im.tag; S.sa[p] = im.a; S.sb[p] = im.b; S.sc[p] = im.c; S.sx[p] = 0;
        }
        wave_fence();
    }
    write_region(S, tab, xt, lane);
}

// Table growth (rl_grow_limiter): old region r of a limiter with 2^(k_new-1) regions splits
// into new regions 2r and 2r+1 by the next tag bit (region_local with one more bit); every
// slot holding state keeps its words and is re-inserted from its home in its new region.
// One wave per old region; each new region is written whole (free slots as zeros).
__global__ __launch_bounds__(64) void k_grow(const Slot* __restrict__ old_tab, const uint64_t* old_x,
                                             Slot* __restrict__ new_tab, uint64_t* new_x,
                                             uint64_t n_old, int shard_bits, int k_new, int algo) {
    __shared__ RegionStage S[2];
    constexpr uint32_t NS = kRegionSlots;
    const uint32_t lane = threadIdx.x;
    const uint64_t r = blockIdx.x;
    if (r >= n_old) return;
    Slot img[NS / 64];
    uint64_t xim[NS / 64];
    bool kp[NS / 64];
#pragma unroll
    for (uint32_t i = 0; i < NS / 64; ++i) {
        img[i] = old_tab[r * NS + lane + 64 * i];
        xim[i] = old_x ? old_x[r * NS + lane + 64 * i] : 0;
        kp[i] = !slot_free(img[i], xim[i]) && (xim[i] != 0 || state_present(algo, img[i].b, img[i].c));
        S[0].occ[lane + 64 * i] = 0;
        S[1].occ[lane + 64 * i] = 0;
    }
    wave_fence();
#pragma unroll
    for (uint32_t i = 0; i < NS / 64; ++i) {
        if (!kp[i]) continue;
        RegionStage& T = S[region_local(img[i].tag, shard_bits, k_new) & 1u];
        uint32_t p = slot_home(img[i].tag);
        while (atomicCAS(&T.occ[p], 0u, 1u) != 0u) p = (p + 1) & (NS - 1);
        T.tag[p] = img[i].tag; T.sa[p] = img[i].a; T.sb[p] = img[i].b; T.sc[p] = img[i].c;
        T.sx[p] = xim[i];
    }
    wave_fence();
    write_region(S[0], new_tab + (2 * r) * NS, new_x ? new_x + (2 * r) * NS : nullptr, lane);
    write_region(S[1], new_tab + (2 * r + 1) * NS, new_x ? new_x + (2 * r + 1) * NS : nullptr, lane);
}

hipError_t launch_grow(const Slot* old_tab, const uint64_t* old_x, Slot* new_tab, uint64_t* new_x,
                       uint64_t n_old_regions, int shard_bits, int k_new, int algo, hipStream_t s) {
    if (n_old_regions == 0) return hipSuccess;
    hipLaunchKernelGGL(k_grow, dim3((uint32_t)n_old_regions), dim3(64), 0, s, old_tab, old_x, new_tab,
                       new_x, n_old_regions, shard_bits, k_new, algo);
    return hipGetLastError();
}

// TTL sweep: one wave per region; every used slot none of whose buckets is live at `now`
// (slot_live, the criterion a batch's region load applies) is dropped and the region is
// rebuilt (no tombstone survives a sweep). One counter atomic per wave.
__global__ __launch_bounds__(64) void k_sweep(Slot* __restrict__ tab0, uint64_t n_regions,
                                              DevLimiter L, int64_t now, uint32_t* count) {
    __shared__ RegionStage S;
    const uint32_t lane = threadIdx.x;
    const uint64_t r = blockIdx.x;
    if (r >= n_regions) return;
    Slot* tab = tab0 + r * kRegionSlots;
    uint64_t* xt = L.cache_table ? (uint64_t*)L.cache_table + r * kRegionSlots : nullptr;
    uint32_t dead = stage_region(S, tab, xt, lane,
                                 [&](const Slot& v, uint64_t x) { return slot_live(L, v, now, x); });
    write_region(S, tab, xt, lane);
    for (int o = 32; o > 0; o >>= 1) dead += __shfl_xor(dead, o, 64);
    if (lane == 0 && dead) atomicAdd(count, dead);
}

hipError_t launch_sweep(Slot* table, uint64_t n_slots, const DevLimiter& L, int64_t now_ms,
                        uint32_t* count, hipStream_t s) {
    const uint64_t regions = n_slots / kRegionSlots;
    if (regions == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sweep, dim3((uint32_t)regions), dim3(64), 0, s, table, regions, L, now_ms,
                       count);
    return hipGetLastError();
}

hipError_t launch_export(const Slot* table, uint64_t n_slots, const DevLimiter& L, uint16_t lim,
                         int64_t now_ms, StateRec* out, uint32_t cap, uint32_t* count,
                         hipStream_t s) {
    const uint64_t blocks = (n_slots + 255) / 256;
    hipLaunchKernelGGL(k_export, dim3((uint32_t)blocks), dim3(256), 0, s, table, n_slots, L, lim,
                       now_ms, out, cap, count);
    return hipGetLastError();
}

hipError_t launch_import(const ImportArgs& a, hipStream_t s) {
    if (a.n_groups == 0) return hipSuccess;
    hipLaunchKernelGGL(k_import, dim3(a.n_groups), dim3(64), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------ launchers
static inline uint32_t tiles_for(uint32_t n) { return (n + kTile - 1) / kTile; }

static uint32_t persistent_grid(uint32_t n_tiles, uint32_t per_cu) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return std::max<uint32_t>(1u, std::min<uint32_t>(n_tiles, (uint32_t)cus * per_cu));
}

hipError_t launch_upsweep(const PartArgs& a, bool raw, bool wide, hipStream_t s) {
    dim3 grid(persistent_grid(a.n_tiles, a.up_per_cu ? a.up_per_cu : 4)), block(kTileThreads);
    if (raw) {
        if (wide) hipLaunchKernelGGL((k_upsweep<CodecW, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_upsweep<CodecC, true>), grid, block, 0, s, a);
    } else {
        if (wide) hipLaunchKernelGGL((k_upsweep<CodecW, false>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_upsweep<CodecC, false>), grid, block, 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_scatter(const PartArgs& a, bool raw, bool wide, hipStream_t s) {
    dim3 grid(persistent_grid(a.n_tiles, a.sc_per_cu ? a.sc_per_cu : 1)), block(kTileThreads);
    if (raw) {
        if (wide) hipLaunchKernelGGL((k_scatter<CodecW, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_scatter<CodecC, true>), grid, block, 0, s, a);
    } else {
        if (wide) hipLaunchKernelGGL((k_scatter<CodecW, false>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_scatter<CodecC, false>), grid, block, 0, s, a);
    }
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

template <class Codec, class Res>
static void region_launch(const RegionArgs& a, hipStream_t s, hipStream_t hs, hipEvent_t e0,
                          hipEvent_t e1) {
    const dim3 b(64);
    if (a.bin_shift == 0 && a.hot_mark && hs) {          // hot chains beside normal regions
        (void)hipEventRecord(e0, s);
        (void)hipStreamWaitEvent(hs, e0, 0);
        if (a.tok) hipLaunchKernelGGL((k_hot_chains<Codec, Res, true>), dim3(kHotMax), dim3(128), 0, hs, a);
        else hipLaunchKernelGGL((k_hot_chains<Codec, Res, false>), dim3(kHotMax), dim3(128), 0, hs, a);
        if (a.walk && a.work) {
            const uint32_t grid = persistent_grid(a.n_regions, a.walk);
            const uint32_t chunk = std::max<uint32_t>(1u, a.n_regions / (grid * 32u));
            (void)hipMemsetAsync(a.work, 0, 8 * 64, s);
            if (a.tok) hipLaunchKernelGGL((k_regions_walk<Codec, Res, true>), dim3(grid), b, 0, s, a, chunk);
            else hipLaunchKernelGGL((k_regions_walk<Codec, Res, false>), dim3(grid), b, 0, s, a, chunk);
        } else {
            const dim3 g(a.n_regions);
            if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 0, false>), g, b, 0, s, a);
            else hipLaunchKernelGGL((k_regions<Codec, Res, false, 0, false>), g, b, 0, s, a);
        }
        (void)hipEventRecord(e1, hs);
        (void)hipStreamWaitEvent(s, e1, 0);
    } else if (a.bin_shift == 0 && a.hot_mark) {         // hot chains + normal regions
        const dim3 g(kHotMax + (a.n_regions + 1) / 2), b2(128);
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 0, true>), g, b2, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false, 0, true>), g, b2, 0, s, a);
    } else if (a.bin_shift == 0 && a.cache) {
        const dim3 g(a.n_regions);
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 0, false, true>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false, 0, false, true>), g, b, 0, s, a);
    } else if (a.bin_shift == 0) {
        const dim3 g(a.n_regions);
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 0, false>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false, 0, false>), g, b, 0, s, a);
    } else {
        const uint32_t n_bins = a.n_regions / kRegionsPerBin;
        const dim3 g((n_bins + 7) / 8 * 64);
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 3, false>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false, 3, false>), g, b, 0, s, a);
    }
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

hipError_t launch_region(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s,
                         hipStream_t hs, hipEvent_t e0, hipEvent_t e1) {
    if (wide) region_launch<CodecW, uint64_t>(a, s, hs, e0, e1);
    else if (res_bytes == 1) region_launch<CodecC, uint8_t>(a, s, hs, e0, e1);
    else if (res_bytes == 2) region_launch<CodecC, uint16_t>(a, s, hs, e0, e1);
    else region_launch<CodecC, uint32_t>(a, s, hs, e0, e1);
    return hipGetLastError();
}

hipError_t launch_hot_prepare(const RegionArgs& a, bool wide, hipStream_t s) {
    const dim3 gp(persistent_grid(1u << 30, 4));
    if (wide) hipLaunchKernelGGL(k_hot_prep<CodecW>, dim3(kHotMax), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(k_hot_prep<CodecC>, dim3(kHotMax), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_hot_scan, dim3(1), dim3(1024), 0, s, a);
    if (wide) hipLaunchKernelGGL(k_hot_summ<CodecW>, gp, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_hot_summ<CodecC>, gp, dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hot_summ2, gp, dim3(256), 0, s, a);
    return hipGetLastError();
}

template <class Codec, class Res>
static void hot_fill_launch(const RegionArgs& a, hipStream_t s) {
    const dim3 gp(persistent_grid(1u << 30, 4));
    if (a.tok) hipLaunchKernelGGL((k_hot_fill<Codec, Res, true>), gp, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_hot_fill<Codec, Res, false>), gp, dim3(256), 0, s, a);
}

hipError_t launch_hot_fill(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s) {
    if (wide) hot_fill_launch<CodecW, uint64_t>(a, s);
    else if (res_bytes == 1) hot_fill_launch<CodecC, uint8_t>(a, s);
    else if (res_bytes == 2) hot_fill_launch<CodecC, uint16_t>(a, s);
    else hot_fill_launch<CodecC, uint32_t>(a, s);
    return hipGetLastError();
}

hipError_t launch_hot_select(const uint32_t* rstart, const uint32_t* rcount, const uint32_t* rend,
                             uint32_t n_bins, uint32_t threshold, uint32_t* hot_list,
                             uint32_t* hot_count, uint32_t* hot_mark, uint32_t epoch,
                             hipStream_t s) {
    const dim3 g((n_bins + 255) / 256), b(256);
    hipLaunchKernelGGL(k_hot_hist, g, b, 0, s, rstart, rcount, rend, n_bins, threshold, hot_count);
    hipLaunchKernelGGL(k_hot_select, g, b, 0, s, rstart, rcount, rend, n_bins, threshold, hot_list,
                       hot_count, hot_mark, epoch);
    return hipGetLastError();
}

hipError_t launch_bin_bounds(const BoundsArgs& a, bool wide, hipStream_t s) {
    if (a.n_bins == 0 || a.d0 > kMaxDigitBits || a.d1 > kMaxDigitBits || a.d0 < 1)
        return hipErrorInvalidValue;
    const dim3 g(1u << a.d1), b(256);
    if (wide) hipLaunchKernelGGL(k_bin_bounds<CodecW>, g, b, 0, s, a);
    else hipLaunchKernelGGL(k_bin_bounds<CodecC>, g, b, 0, s, a);
    return hipGetLastError();
}

template <class Res>
static void unpermute_mid(const UnpermArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_unpermute_mid<Res>, dim3((a.n + 2047) / 2048), dim3(256), 0, s, a.pos1,
                       (const Res*)a.res, (Res*)a.mid, a.n);
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
        a.res = a.mid;
        a.pos1 = nullptr;
    }
    dim3 g(persistent_grid(a.n_tiles, a.per_cu ? a.per_cu : 1)), b(kTileThreads);
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

hipError_t launch_synth(const SynthArgs& a, hipStream_t s) {
    const uint64_t blocks = (a.n + 255) / 256;
    hipLaunchKernelGGL(k_synth, dim3((uint32_t)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_owner_partition(const uint64_t* key, uint32_t n, uint32_t shard_count,
                                  uint32_t* perm, uint32_t* counts_dev, uint32_t* scratch,
                                  const DirSlot* dir, hipStream_t s) {
    int sbits = 0;
    while ((1u << sbits) < shard_count) ++sbits;
    const uint32_t nt = tiles_for(n);
    uint32_t* counts = scratch;                       // [shards][tiles]
    uint32_t* base = scratch + (size_t)shard_count * nt;
    hipLaunchKernelGGL(k_owner_count, dim3(nt), dim3(kTileThreads), 0, s, key, n, sbits, nt, counts, dir);
    hipLaunchKernelGGL(k_scan_rows, dim3(shard_count), dim3(256), 0, s, counts, counts, nt, counts_dev);
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, s, counts_dev, base, shard_count);
    hipLaunchKernelGGL(k_owner_scatter, dim3(nt), dim3(kTileThreads), 0, s, key, n, sbits, nt,
                       counts, base, perm, dir);
    return hipGetLastError();
}

hipError_t launch_route_pack(uint32_t n, const uint32_t* perm, const uint64_t* key,
                             const int32_t* permits, const int64_t* now, const uint16_t* lim,
                             uint64_t* key_o, int32_t* permits_o, int64_t* now_o, uint16_t* lim_o,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_route_pack, dim3((n + 255) / 256), dim3(256), 0, s, n, perm, key, permits,
                       now, lim, key_o, permits_o, now_o, lim_o);
    return hipGetLastError();
}

hipError_t launch_route_fold(uint32_t n, const uint8_t* allowed, const int64_t* remaining,
                             int64_t* packed, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_route_fold, dim3((n + 255) / 256), dim3(256), 0, s, n, allowed, remaining, packed);
    return hipGetLastError();
}

hipError_t launch_route_unpack(uint32_t n, const uint32_t* perm, const int64_t* packed,
                               uint8_t* allowed, int64_t* remaining, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_route_unpack, dim3((n + 255) / 256), dim3(256), 0, s, n, perm, packed,
                       allowed, remaining);
    return hipGetLastError();
}


hipError_t launch_route_pack_wire(uint32_t n, const uint32_t* perm, const uint64_t* key,
                                  const int32_t* permits, const int64_t* now, const uint16_t* lim,
                                  uint64_t* wire, uint16_t* lim_o, int64_t* hdr, hipStream_t s,
                                  uint64_t* part, uint32_t* nparts) {
    if (nparts) *nparts = 0;
    hipError_t e = hipMemsetAsync(hdr, 0, 2 * sizeof(int64_t), s);
    if (e != hipSuccess || n == 0) return e;
    const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, kWireBlocksMax);
    if (nparts) *nparts = blocks;
    hipLaunchKernelGGL(k_route_pack_wire, dim3(blocks), dim3(256), 0, s, n, perm, key,
                       permits, now, lim, wire, lim_o, hdr, part);
    return hipGetLastError();
}

hipError_t launch_route_unwire(uint32_t m, const uint64_t* wire, uint32_t n_src, const int64_t* base,
                               const uint32_t* end, uint64_t* key_o, int32_t* permits_o,
                               int64_t* now_o, hipStream_t s) {
    if (m == 0) return hipSuccess;
    if (n_src == 0 || n_src > (uint32_t)kMaxShards) return hipErrorInvalidValue;
    WireSrc src{};
    for (uint32_t i = 0; i < n_src; ++i) { src.base[i] = base[i]; src.end[i] = end[i]; }
    src.n_src = n_src;
    hipLaunchKernelGGL(k_route_unwire, dim3((m + 255) / 256), dim3(256), 0, s, m, wire, src, key_o,
                       permits_o, now_o);
    return hipGetLastError();
}

hipError_t launch_route_fold_w(uint32_t n, const uint8_t* allowed, const int64_t* remaining,
                               void* packed, int width, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const dim3 g((n + 255) / 256), b(256);
    switch (width) {
    case 1: hipLaunchKernelGGL(k_route_fold_w<uint8_t>, g, b, 0, s, n, allowed, remaining, (uint8_t*)packed); break;
    case 2: hipLaunchKernelGGL(k_route_fold_w<uint16_t>, g, b, 0, s, n, allowed, remaining, (uint16_t*)packed); break;
    case 4: hipLaunchKernelGGL(k_route_fold_w<uint32_t>, g, b, 0, s, n, allowed, remaining, (uint32_t*)packed); break;
    case 8: hipLaunchKernelGGL(k_route_fold_w<uint64_t>, g, b, 0, s, n, allowed, remaining, (uint64_t*)packed); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_route_unpack_w(uint32_t n, const uint32_t* perm, const void* packed, int width,
                                 uint8_t* allowed, int64_t* remaining, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const dim3 g((n + 255) / 256), b(256);
    switch (width) {
    case 1: hipLaunchKernelGGL(k_route_unpack_w<uint8_t>, g, b, 0, s, n, perm, (const uint8_t*)packed, allowed, remaining); break;
    case 2: hipLaunchKernelGGL(k_route_unpack_w<uint16_t>, g, b, 0, s, n, perm, (const uint16_t*)packed, allowed, remaining); break;
    case 4: hipLaunchKernelGGL(k_route_unpack_w<uint32_t>, g, b, 0, s, n, perm, (const uint32_t*)packed, allowed, remaining); break;
    case 8: hipLaunchKernelGGL(k_route_unpack_w<uint64_t>, g, b, 0, s, n, perm, (const uint64_t*)packed, allowed, remaining); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rl
