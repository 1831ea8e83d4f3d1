// rl_hot.hip — 4b. hot regions: the untemplated kernels (chunk scan, group summaries,
// selection) and the launchers of the hot and region stages, which dispatch to the
// per-width instantiations in rl_rt_*.hip.
#include "rl_hot.hpp"

#pragma clang fp contract(off)

namespace rl {

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
    // listed regions whose key could be walked (walk_table_on without the table): the host
    // allocates the walk tables only once a batch has one (tb_uniform never does)
    const int64_t lo = batch_lo(a.ctl), hi = batch_hi(a.ctl);
    const bool wants = t < hc && t < walk_regions(lo, hi) &&
                       walk_dense(a.hot_info[t], a.lims[a.region_lim[a.hot_info[t].bin]], lo, hi, a.walk_min);
    const uint32_t nw = (uint32_t)__syncthreads_count(wants);
    if (t == 0) a.ctl->n_walk = nw;
}

// Hot-region selection, largest first: k_hot_hist counts the bins at or above the
// threshold per power-of-two size class; k_hot_select then raises the threshold to the
// smallest class boundary that admits at most kHotMax bins and lists those bins.
// hot_meta: [0] listed count, [1 .. 33] size-class histogram.
__device__ inline uint32_t bin_records(const uint32_t* rstart, const uint32_t* rcount,
                                       const uint32_t* rend, uint32_t b) {
    return rend ? rend[b] - rstart[b] : rcount[b];
}
// The hot path assumes that a denial never changes state; with the local cache a denial
// puts the estimate (SlidingWindowRateLimiter.java:106-108). Regions of such limiters stay
// with the region waves (and k_solo); every other limiter of the engine keeps its chains.
// lims == nullptr: no limiter has the cache.
__device__ inline bool hot_eligible(const DevLimiter* lims, const uint8_t* region_lim, uint32_t b) {
    return !lims || lims[region_lim[b]].cache_ttl_ms <= 0;
}

__global__ __launch_bounds__(256) void k_hot_hist(const uint32_t* rstart, const uint32_t* rcount,
                                                  const uint32_t* rend, uint32_t n_bins,
                                                  uint32_t threshold, uint32_t* hot_meta,
                                                  const DevLimiter* lims, const uint8_t* region_lim) {
    __shared__ uint32_t h[33];
    if (threadIdx.x < 33) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b < n_bins && hot_eligible(lims, region_lim, b)) {
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
                                                    uint32_t epoch, const DevLimiter* lims,
                                                    const uint8_t* region_lim) {
    __shared__ uint32_t s_thr;
    __shared__ uint32_t s_off[33];                    // list offset of each size class
    // routed regions (k_hot_route_list) hold the first entries of the list
    const uint32_t routed = hot_meta[kHotRoutedOff];
    if (threadIdx.x == 0) {
        uint32_t above = 0, thr = 0xFFFFFFFFu;
        for (int c = 32; c >= 0; --c) {               // classes from the largest down
            s_off[c] = above;
            above += hot_meta[1 + c];
            if (above > kHotMax - routed) break;
            thr = c == 0 ? 1u : (1u << c);
        }
        s_thr = thr > threshold ? thr : threshold;
    }
    __syncthreads();
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= n_bins || !hot_eligible(lims, region_lim, b)) return;
    const uint32_t cnt = bin_records(rstart, rcount, rend, b);
    if (cnt == 0 || cnt < s_thr) return;
    // largest size class first: the chains' workgroups are dispatched in list order, and the
    // longest chains must not be the ones that wait for a slot beside the normal regions
    const uint32_t c = 31u - (uint32_t)__builtin_clz(cnt);
    const uint32_t k = routed + s_off[c] + atomicAdd(&hot_meta[kHotClassCursor + c], 1u);
    atomicAdd(&hot_meta[0], 1u);
    if (k < kHotMax) {                                // (always, by the choice of s_thr)
        hot_list[k] = b;
        hot_mark[b] = epoch;
    }
}


// Routed regions first in the hot list, every slot that received records (nothing else sees
// them: their records skipped the normal partition), largest first (a size-class counting
// sort: the longest chains are dispatched first). hot_meta[0] and [kHotRoutedOff] = count.
__global__ __launch_bounds__(1024) void k_hot_route_list(const uint32_t* __restrict__ route_list,
                                                         const uint32_t* __restrict__ route_cnt,
                                                         uint32_t* hot_list, uint32_t* hot_meta) {
    __shared__ uint32_t s_cls[33], s_base[33];
    static_assert(kRouteSlots == 2 * 1024, "two slots per thread");
    const uint32_t t = threadIdx.x;
    if (t < 33) s_cls[t] = 0;
    __syncthreads();
    uint32_t cls[2], k[2];
    bool has[2];
    for (int u = 0; u < 2; ++u) {
        const uint32_t sl = t + 1024u * u;
        const uint32_t c = route_cnt[sl];
        has[u] = route_list[sl] != kNone && c > 0;
        cls[u] = has[u] ? 31u - (uint32_t)__builtin_clz(c) : 0u;
        k[u] = has[u] ? atomicAdd(&s_cls[cls[u]], 1u) : 0u;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t above = 0;
        for (int c = 32; c >= 0; --c) { s_base[c] = above; above += s_cls[c]; }
        hot_meta[0] = above;
        hot_meta[kHotRoutedOff] = above;
    }
    __syncthreads();
    for (int u = 0; u < 2; ++u)
        if (has[u]) hot_list[s_base[cls[u]] + k[u]] = kHotRoutedBit | (t + 1024u * u);
}

// The next batch's route table: this batch's listed hot regions with >= threshold records,
// in list order (largest size class first), each placed at a free one of its two slots
// (route_slots), 128 entries at a time so that larger regions win the slots; at most
// kRouteMax. A region whose slots are both taken stays unrouted (it is then partitioned
// normally and found by the hot selection).
__global__ __launch_bounds__(1024) void k_route_next(const HotInfo* __restrict__ info,
                                                     const uint32_t* __restrict__ hot_count,
                                                     uint32_t threshold, uint32_t* route_list) {
    __shared__ uint32_t s_tab[kRouteSlots];
    __shared__ uint32_t s_placed;
    const uint32_t hc = min(hot_count[0], kHotMax);
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < kRouteSlots; i += blockDim.x) s_tab[i] = kNone;
    if (t == 0) s_placed = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < hc; b0 += 128) {
        const uint32_t i = b0 + t;
        if (t < 128 && i < hc && info[i].end - info[i].start >= threshold) {
            const uint32_t b = info[i].bin;
            uint32_t s1, s2;
            route_slots(b, s1, s2);
            if (atomicCAS(&s_tab[s1], kNone, b) == kNone || atomicCAS(&s_tab[s2], kNone, b) == kNone)
                atomicAdd(&s_placed, 1u);
        }
        __syncthreads();
        if (s_placed >= kRouteMax) break;              // (block-uniform)
    }
    __syncthreads();
    // the slots' dense indices (pass-0 bin lo_bins + idx): occupied slots before each slot
    __shared__ uint32_t s_tmp[16];
    static_assert(kRouteSlots == 2 * 1024, "two slots per thread");
    const uint32_t occ = (s_tab[2 * t] != kNone ? 1u : 0u) + (s_tab[2 * t + 1] != kNone ? 1u : 0u);
    const uint32_t ex = block_exclusive_scan<1024>(occ, s_tmp, nullptr);
    route_list[kRouteSlots + 2 * t] = ex;
    route_list[kRouteSlots + 2 * t + 1] = ex + (s_tab[2 * t] != kNone ? 1u : 0u);
    for (uint32_t i = t; i < kRouteSlots; i += blockDim.x) route_list[i] = s_tab[i];
}

// Region dispatch order (launch_region_order): class c = floor(log2(records)) for non-empty
// regions; classes are laid out largest first. meta[c] counts, meta[34 + c] cursors.
__global__ __launch_bounds__(256) void k_order_count(const uint32_t* rstart, const uint32_t* rcount,
                                                     const uint32_t* rend, uint32_t n_bins,
                                                     uint32_t* meta) {
    __shared__ uint32_t h[33];
    if (threadIdx.x < 33) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b < n_bins) {
        const uint32_t cnt = bin_records(rstart, rcount, rend, b);
        if (cnt > 0) atomicAdd(&h[31 - __builtin_clz(cnt)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 33 && h[threadIdx.x]) atomicAdd(&meta[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_order_place(const uint32_t* rstart, const uint32_t* rcount,
                                                     const uint32_t* rend, uint32_t n_bins,
                                                     uint32_t* meta, uint32_t* order) {
    __shared__ uint32_t s_base[33], s_cnt[33], s_blk[33];
    const uint32_t t = threadIdx.x;
    if (t == 0) {
        uint32_t above = 0;
        for (int c = 32; c >= 0; --c) { s_base[c] = above; above += meta[c]; }
        if (blockIdx.x == 0) order[n_bins] = above;
    }
    if (t < 33) s_cnt[t] = 0;
    __syncthreads();
    const uint32_t b = blockIdx.x * 256 + t;
    const uint32_t cnt = b < n_bins ? bin_records(rstart, rcount, rend, b) : 0u;
    const uint32_t c = cnt ? 31u - (uint32_t)__builtin_clz(cnt) : 0u;
    const uint32_t k = cnt ? atomicAdd(&s_cnt[c], 1u) : 0u;
    __syncthreads();
    if (t < 33 && s_cnt[t]) s_blk[t] = atomicAdd(&meta[34 + t], s_cnt[t]);   // one per class per block
    __syncthreads();
    if (cnt) order[s_base[c] + s_blk[c] + k] = b;
}

hipError_t launch_region_order(const uint32_t* rstart, const uint32_t* rcount, const uint32_t* rend,
                               uint32_t n_bins, uint32_t* meta, uint32_t* order, hipStream_t s) {
    hipError_t e = hipMemsetAsync(meta, 0, kOrderMeta * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const dim3 g((n_bins + 255) / 256), b(256);
    hipLaunchKernelGGL(k_order_count, g, b, 0, s, rstart, rcount, rend, n_bins, meta);
    hipLaunchKernelGGL(k_order_place, g, b, 0, s, rstart, rcount, rend, n_bins, meta, order);
    return hipGetLastError();
}

hipError_t launch_hot_route_list(const uint32_t* route_list, const uint32_t* route_cnt,
                                 uint32_t* hot_list, uint32_t* hot_meta, hipStream_t s) {
    hipLaunchKernelGGL(k_hot_route_list, dim3(1), dim3(1024), 0, s, route_list, route_cnt, hot_list,
                       hot_meta);
    return hipGetLastError();
}

hipError_t launch_route_next(const HotInfo* hot_info, const uint32_t* hot_count, uint32_t threshold,
                             uint32_t* route_list, hipStream_t s) {
    hipLaunchKernelGGL(k_route_next, dim3(1), dim3(1024), 0, s, hot_info, hot_count, threshold,
                       route_list);
    return hipGetLastError();
}

// Allow-walk tables of this batch's walk keys (slots 2 i + k, i < walk_regions listed
// regions, each walk_stride entries): every entry "none" before k_hot_summ merges the firsts in.
__global__ __launch_bounds__(256) void k_walk_init(RegionArgs a) {
    const uint32_t hc = min(a.hot_count[0], kHotMax);
    const int64_t lo = batch_lo(a.ctl), hi = batch_hi(a.ctl);
    const uint32_t nreg = min(hc, walk_regions(lo, hi));
    const uint32_t per_reg = walk_stride(lo, hi);    // uint4 per region: 2 tables of stride entries
    const uint32_t parts = (per_reg + 4095) / 4096;  // (work units of 4096 uint4)
    const uint4 none = make_uint4(kWalkNone, kWalkNone, kWalkNone, kWalkNone);
    for (uint32_t u = blockIdx.x; u < nreg * parts; u += gridDim.x) {
        const uint32_t i = u / parts, p = u % parts;  // listed region: tables of walked keys only
        const HotInfo& f = a.hot_info[i];
        if (!walk_dense(f, a.lims[a.region_lim[f.bin]], lo, hi, a.walk_min)) continue;
        uint4* t = (uint4*)a.walk_tab + (size_t)i * per_reg;
        const uint32_t e = min(per_reg, (p + 1) * 4096);
        for (uint32_t k = p * 4096 + threadIdx.x; k < e; k += 256) t[k] = none;
    }
}

hipError_t launch_hot_prepare(const RegionArgs& a, bool wide, hipStream_t s) {
    const dim3 gp(persistent_grid(1u << 30, 4));
    if (wide) hipLaunchKernelGGL(k_hot_prep<CodecW>, dim3(kHotMax), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(k_hot_prep<CodecC>, dim3(kHotMax), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_hot_scan, dim3(1), dim3(1024), 0, s, a);
    if (a.walk_tab) hipLaunchKernelGGL(k_walk_init, dim3(2048), dim3(256), 0, s, a);
    if (wide) hipLaunchKernelGGL(k_hot_summ<CodecW>, gp, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_hot_summ<CodecC>, gp, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_hot_select(const uint32_t* rstart, const uint32_t* rcount, const uint32_t* rend,
                             uint32_t n_bins, uint32_t threshold, uint32_t* hot_list,
                             uint32_t* hot_count, uint32_t* hot_mark, uint32_t epoch,
                             const DevLimiter* lims, const uint8_t* region_lim, hipStream_t s) {
    const dim3 g((n_bins + 255) / 256), b(256);
    hipLaunchKernelGGL(k_hot_hist, g, b, 0, s, rstart, rcount, rend, n_bins, threshold, hot_count,
                       lims, region_lim);
    hipLaunchKernelGGL(k_hot_select, g, b, 0, s, rstart, rcount, rend, n_bins, threshold, hot_list,
                       hot_count, hot_mark, epoch, lims, region_lim);
    return hipGetLastError();
}

// ---- per-width dispatch (the kernels are instantiated in rl_rt_{u8,u16,u32,w}.hip)
#define RL_BY_WIDTH(F, ...)                                              \
    (wide ? F<CodecW, uint64_t>(__VA_ARGS__)                             \
          : res_bytes == 1 ? F<CodecC, uint8_t>(__VA_ARGS__)             \
          : res_bytes == 2 ? F<CodecC, uint16_t>(__VA_ARGS__)            \
                           : F<CodecC, uint32_t>(__VA_ARGS__))

hipError_t launch_chains(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s,
                         hipStream_t hs, hipEvent_t e0) {
    return RL_BY_WIDTH(chains_launch_t, a, s, hs, e0);
}
hipError_t launch_region(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s,
                         hipStream_t hs, hipEvent_t e1) {
    return RL_BY_WIDTH(region_launch_t, a, s, hs, e1);
}
hipError_t launch_hot_fill(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s) {
    return RL_BY_WIDTH(hot_fill_t, a, s);
}

}  // namespace rl
