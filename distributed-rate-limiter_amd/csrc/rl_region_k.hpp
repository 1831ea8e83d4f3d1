// rl_region_k.hpp — the normal-region kernels and their launch (templates, instantiated per
// result width in rl_rt_*.hip).
#pragma once
#include "rl_region.hpp"

#pragma clang fp contract(off)

namespace rl {

template <class Codec, class Res, bool TOK, int BS, bool CACHE = false>
__global__ __launch_bounds__(64, BS > 0 ? 3 : RL_REGION_MIN_WAVES)
void k_regions(RegionArgs a) {
    if constexpr (CACHE) {                       // some limiter keeps a local cache (BS 0, no hot path)
        __shared__ RegionTableX S;
        region_body_t<Codec, Res, TOK, 0>(a, blockIdx.x, S);
    } else {
        __shared__ RegionLds<Codec, (BS > 0)> S;
        region_body_t<Codec, Res, TOK, BS>(a, blockIdx.x, S);
    }
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

template <class Codec, class Res>
hipError_t region_launch_t(const RegionArgs& a, hipStream_t s, hipStream_t hs, hipEvent_t e0,
                           hipEvent_t e1, hipStream_t hs2, hipEvent_t e2) {
    const dim3 b(64);
    if (a.bin_shift == 0 && a.hot_mark && hs && hs2) {          // hot chains beside normal regions
        (void)hipEventRecord(e0, s);
        (void)hipStreamWaitEvent(hs, e0, 0);
        (void)hipStreamWaitEvent(hs2, e0, 0);
        (void)hot_chains_t<Codec, Res>(a, hs, hs2);
        if (a.walk && a.work) {
            const uint32_t grid = persistent_grid(a.n_regions, a.walk);
            const uint32_t chunk = std::max<uint32_t>(1u, a.n_regions / (grid * 32u));
            (void)hipMemsetAsync(a.work, 0, 8 * 64, s);
            if (a.tok) hipLaunchKernelGGL((k_regions_walk<Codec, Res, true>), dim3(grid), b, 0, s, a, chunk);
            else hipLaunchKernelGGL((k_regions_walk<Codec, Res, false>), dim3(grid), b, 0, s, a, chunk);
        } else {
            const dim3 g(a.n_regions);
            if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 0>), g, b, 0, s, a);
            else hipLaunchKernelGGL((k_regions<Codec, Res, false, 0>), g, b, 0, s, a);
        }
        (void)hipEventRecord(e1, hs);
        (void)hipEventRecord(e2, hs2);
        (void)hipStreamWaitEvent(s, e1, 0);
        (void)hipStreamWaitEvent(s, e2, 0);
    } else if (a.bin_shift == 0 && a.hot_mark) {         // hot chains + normal regions
        (void)regions_combined_t<Codec, Res>(a, s);
    } else if (a.bin_shift == 0 && a.cache) {
        const dim3 g(a.n_regions);
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 0, true>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false, 0, true>), g, b, 0, s, a);
    } else if (a.bin_shift == 0) {
        const dim3 g(a.n_regions);
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 0>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false, 0>), g, b, 0, s, a);
    } else {
        const uint32_t n_bins = a.n_regions / kRegionsPerBin;
        const dim3 g((n_bins + 7) / 8 * 64);
        if (a.tok) hipLaunchKernelGGL((k_regions<Codec, Res, true, 3>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_regions<Codec, Res, false, 3>), g, b, 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace rl
