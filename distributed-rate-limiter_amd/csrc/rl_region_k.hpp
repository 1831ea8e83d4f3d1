// rl_region_k.hpp — the normal-region kernels and their launch (templates, instantiated per
// result width in rl_rt_*.hip).
#pragma once
#include "rl_region.hpp"

#pragma clang fp contract(off)

namespace rl {

template <class Codec, class Res, bool TOK, bool CACHE = false>
__global__ __launch_bounds__(64, CACHE ? 3 : kRegionMinWaves) void k_regions(RegionArgs a) {
    if constexpr (CACHE) {                       // some limiter keeps a local cache
        __shared__ RegionTableX S;
        region_body_t<Codec, Res, TOK>(a, blockIdx.x, S);
    } else {
        __shared__ RegionTable S;
        region_body_t<Codec, Res, TOK>(a, blockIdx.x, S);
    }
}

// The region stage: the hot chains (a side stream of the device's highest priority, forked
// from and joined to the engine stream by events) beside one single-wave workgroup per
// normal region.
template <class Codec, class Res>
hipError_t chains_launch_t(const RegionArgs& a, hipStream_t s, hipStream_t hs, hipEvent_t e0) {
    (void)hipEventRecord(e0, s);
    (void)hipStreamWaitEvent(hs, e0, 0);
    (void)hot_chains_t<Codec, Res>(a, hs);
    return hipGetLastError();
}
template <class Codec, class Res>
hipError_t region_launch_t(const RegionArgs& a, hipStream_t s, hipStream_t hs, hipEvent_t e1) {
    const dim3 b(64), g(a.n_regions);
    if (a.hot_mark && hs) {                          // (the chains are running on hs)
        // (a cache-on limiter beside hot ones: its regions run in the cache variant)
        if (a.cache && a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, true>), g, b, 0, s, a);
        else if (a.cache) hipLaunchKernelGGL((k_regions<Codec, Res, false, true>), g, b, 0, s, a);
        else if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false>), g, b, 0, s, a);
        (void)hipEventRecord(e1, hs);
        (void)hipStreamWaitEvent(s, e1, 0);
    } else if (a.cache) {
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, true>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false, true>), g, b, 0, s, a);
    } else {
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false>), g, b, 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace rl
