// rl_kcommon.hpp — device helpers shared by the kernel translation units.
//
// The batched rate-limit decision pipeline for gfx950 (MI355X): rl_partition.hip,
// rl_region.hip, rl_hot.hip, rl_misc.hip share this header.
//
// One batch = requests in arrival order. The pipeline groups every request with
// the other requests of its (limiter, key) WITHOUT a full sort:
//
//   1. k_upsweep  : per 64K-request tile, histogram of the partition digit of each
//                   request's BIN (one state-table region; region = top bits of
//                   mix64(key) below the shard bits).
//   2. k_scan_rows/k_scan_small : exclusive scan of the [bin][tile] histogram.
//   3. k_scatter  : stable partition (wave ballot-match ranking) of the requests
//                   into bin order, packed into 16-byte records.
//   (more than 8192 regions: pass 0 partitions by the region's high digit and k_group
//    then groups each pass-0 bin by region locally.)
//   4. k_regions  : one single-wave workgroup per REGION. The wave loads its region's
//                   256 state slots (8 KB) into LDS once (or faults in single buckets of
//                   a sparse region), streams the region's records in arrival order and
//                   applies the reference semantics per key in order, 64 at a time (SW:
//                   a greedy scan per key; TB: 1 + (#state changes of its busiest key)
//                   rounds, deny never mutates); the region is written back once. Hot
//                   regions run as chains beside it (rl_hot.hpp).
//   5. k_unpermute: results back to the caller's order (allowed u8, remaining i64).
//
// Partition and unpermute grids are persistent and walk tiles XCD-aware: at any
// time the 32 CUs of an XCD work on 32 consecutive tiles, so the per-bin record runs
// they write (and the result runs they gather) share lines in that XCD's L2.
#pragma once
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

// A pointer read from memory (the state tables in DevLimiter) is a generic one: its loads and
// stores become flat instructions, which count against both vmcnt and lgkmcnt, so every wait
// around them — LDS waits included — turns into a full drain. Table accesses go through
// global-address-space pointers instead.
#ifdef __HIP_DEVICE_COMPILE__
#define RL_GLOBAL __attribute__((address_space(1)))
#else
#define RL_GLOBAL                       // (the host pass parses device code only)
#endif
template <class T>
__device__ inline RL_GLOBAL T* as_global(T* p) { return (RL_GLOBAL T*)p; }

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

__device__ inline int64_t shfl64(int64_t v, int src) {
    return (int64_t)(((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uint64_t)v >> 32), src, 64) << 32) |
                     (uint32_t)__shfl((int)(uint32_t)v, src, 64));
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
// streaming partial-line store goes to memory on its own (scatter 1.5 -> 3.3 ms); the
// upsweep's key reads too (streaming them measured no faster, rounds 3-4).
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
constexpr bool kNtScIn = true;
constexpr bool kNtScRec = false;
constexpr bool kNtScPos = true;
constexpr bool kNtUp = false;
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
constexpr bool kNtRgRec = true;
constexpr bool kNtUn = true;

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
// workgroups of one XCD (blocks b, b+8, ...) take consecutive tiles. (Giving each XCD one
// contiguous eighth of the tiles instead measured no faster, round 4.) Returns >= n_tiles when
// this workgroup is done.
__device__ inline uint32_t tile_at(uint32_t it, uint32_t n_tiles) {
    (void)n_tiles;
    return it * gridDim.x + xcd_remap(blockIdx.x, gridDim.x);
}

// A pass-0 tile's cursor base for bin b (added to the row prefix counts[b][tile]).
__device__ inline uint32_t cursor_base(const PartArgs& a, uint32_t b, uint32_t tile) {
    return a.seg_adj ? a.seg_adj[b * a.n_segs + tile / a.seg_tiles] : a.bin_base[b];
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
    return L.base[lim] + region_local(h, a.shard_bits, L.bits[lim]);
}

// Routed regions (pass 0): the route table (kRouteSlots region ids) in LDS; a region is
// routed iff it sits at one of its two slots (route_slots), and that slot is its bin.
struct RouteLds {
    uint32_t key[kRouteSlots];
    uint16_t idx[kRouteSlots];               // dense routed bin of the slot (lo_bins + idx)
};
__device__ inline void route_load(RouteLds& R, const uint32_t* table) {
    for (uint32_t s = threadIdx.x; s < kRouteSlots; s += blockDim.x) {
        R.key[s] = table[s];
        R.idx[s] = (uint16_t)table[kRouteSlots + s];
    }
    __syncthreads();
}
__device__ inline uint32_t route_find(const RouteLds& R, uint32_t b) {
    uint32_t s1, s2;
    route_slots(b, s1, s2);
    const uint32_t k1 = R.key[s1], k2 = R.key[s2];         // independent reads
    return k1 == b ? s1 : k2 == b ? s2 : kNone;
}
// Partition digit of global bin g (a region id) in pass 0: routed region -> lo_bins + its dense index,
// else its high digit g >> digit_shift (two-pass batches: k_group then groups each of
// those bins by region; one-pass batches: digit_shift 0, the region itself).
__device__ inline uint32_t pass_digit(const PartArgs& a, uint32_t g, const RouteLds& R) {
    if (a.route_list) {
        const uint32_t rs = route_find(R, g);
        return rs != kNone ? a.lo_bins + R.idx[rs] : (g >> a.digit_shift);
    }
    return (g >> a.digit_shift) & ((1u << a.digit_bits) - 1);
}

// first probe position of a key inside its region (4-slot aligned: probing reads buckets)
__device__ inline uint32_t slot_home(uint64_t h) { return (uint32_t)h & (kRegionSlots - 4); }
// Wave-wide min / max with every lane active: DPP inside each 16-lane row (xor 1, xor 2, half
// mirror, mirror: each an ALU op reading a neighbour's register), then the four rows' results
// by readlane; uniform result. (__shfl_xor lowers to ds_bpermute: six dependent LDS round
// trips per reduction, twelve for 64 bits.)
template <int C>
__device__ inline uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, C, 0xF, 0xF, false);
}
template <int C>
__device__ inline uint64_t dpp64(uint64_t v) {
    return (uint64_t)dpp32<C>((uint32_t)v) | ((uint64_t)dpp32<C>((uint32_t)(v >> 32)) << 32);
}
template <class T, class Op>
__device__ inline T wave_reduce_dpp(T v, Op op) {
    if constexpr (sizeof(T) == 8) {
        v = op(v, (T)dpp64<0xB1>((uint64_t)v));      // quad_perm(1,0,3,2): lane ^ 1
        v = op(v, (T)dpp64<0x4E>((uint64_t)v));      // quad_perm(2,3,0,1): lane ^ 2
        v = op(v, (T)dpp64<0x141>((uint64_t)v));     // row_half_mirror: 8-lane groups
        v = op(v, (T)dpp64<0x140>((uint64_t)v));     // row_mirror: 16-lane rows
        const uint64_t u = (uint64_t)v;
        auto rl = [&](int l) {
            return (T)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l) << 32));
        };
        return op(op(rl(0), rl(16)), op(rl(32), rl(48)));
    } else {
        v = op(v, (T)dpp32<0xB1>((uint32_t)v));
        v = op(v, (T)dpp32<0x4E>((uint32_t)v));
        v = op(v, (T)dpp32<0x141>((uint32_t)v));
        v = op(v, (T)dpp32<0x140>((uint32_t)v));
        auto rl = [&](int l) { return (T)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l); };
        return op(op(rl(0), rl(16)), op(rl(32), rl(48)));
    }
}
template <class T> __device__ inline T wave_min_dpp(T v) {
    return wave_reduce_dpp(v, [](T x, T y) { return y < x ? y : x; });
}
template <class T> __device__ inline T wave_max_dpp(T v) {
    return wave_reduce_dpp(v, [](T x, T y) { return y > x ? y : x; });
}

__device__ inline void wave_fence() { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); }

static inline uint32_t tiles_for(uint32_t n) { return (n + kTile - 1) / kTile; }

static inline uint32_t persistent_grid(uint32_t n_tiles, uint32_t per_cu) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return std::max<uint32_t>(1u, std::min<uint32_t>(n_tiles, (uint32_t)cus * per_cu));
}

}  // namespace rl
