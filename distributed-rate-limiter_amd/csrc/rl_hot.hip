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

// ---- per-width dispatch (the kernels are instantiated in rl_rt_{u8,u16,u32,w}.hip)
#define RL_BY_WIDTH(F, ...)                                              \
    (wide ? F<CodecW, uint64_t>(__VA_ARGS__)                             \
          : res_bytes == 1 ? F<CodecC, uint8_t>(__VA_ARGS__)             \
          : res_bytes == 2 ? F<CodecC, uint16_t>(__VA_ARGS__)            \
                           : F<CodecC, uint32_t>(__VA_ARGS__))

hipError_t launch_region(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s,
                         hipStream_t hs, hipEvent_t e0, hipEvent_t e1) {
    return RL_BY_WIDTH(region_launch_t, a, s, hs, e0, e1);
}
hipError_t launch_hot_chains(const RegionArgs& a, bool wide, int res_bytes, hipStream_t hs) {
    return RL_BY_WIDTH(hot_chains_t, a, hs);
}
hipError_t launch_regions_combined(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s) {
    return RL_BY_WIDTH(regions_combined_t, a, s);
}
hipError_t launch_hot_fill(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s) {
    return RL_BY_WIDTH(hot_fill_t, a, s);
}

}  // namespace rl
