// rl_misc.hip — synthetic traces, multi-GPU routing kernels, state export / import /
// growth / TTL sweep.
#include "rl_kcommon.hpp"

#pragma clang fp contract(off)

namespace rl {

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
// published status, capacity, min now_ms, max now_ms, receive capacity} and then this
// source's count for every owner (column 0 of every row); min / max folded from
// k_route_pack_wire's per-block partials (nparts = 0: an empty batch, min > max).
__global__ __launch_bounds__(256) void k_fill_header(int64_t* hdr, const int64_t* base_ovf,
                                                     int64_t status, int64_t cap, int64_t rcap,
                                                     uint32_t g, const uint64_t* part,
                                                     uint32_t nparts) {
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
        row[7] = rcap;
        for (uint32_t q = 0; q < g; ++q) row[kHdrFixed + q] = hdr[(size_t)q * kHdrWords];
    }
}

hipError_t launch_fill_header(int64_t* hdr, const int64_t* base_ovf, int64_t status, int64_t cap,
                              int64_t rcap, uint32_t g, const uint64_t* part, uint32_t nparts,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_fill_header, dim3(1), dim3(256), 0, s, hdr, base_ovf, status, cap, rcap, g,
                       part, nparts);
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

// Router split rounds: fold one engine batch's status flags and growth bits into a
// router-owned accumulator (kStatusAccWords), so the rounds of a step need no host read.
// ctl == nullptr: the engine call enqueued no batch (nothing received, or a status set on the
// host), whose flags come in `flags` alone.
__global__ void k_status_accum(const BatchCtl* ctl, unsigned long long flags, unsigned long long* acc) {
    if (threadIdx.x != 0) return;
    if (ctl) {
        flags |= (ctl->invalid ? 1ULL : 0ULL) | (ctl->cap_err ? 2ULL : 0ULL) |
                 (ctl->span_overflow ? 4ULL : 0ULL) | (ctl->internal_err ? 8ULL : 0ULL);
        for (int i = 0; i < 4; ++i) acc[1 + i] |= ctl->grow[i];
    }
    acc[0] |= flags;
}

hipError_t launch_status_accum(const BatchCtl* ctl, unsigned long long flags, unsigned long long* acc,
                               hipStream_t s) {
    hipLaunchKernelGGL(k_status_accum, dim3(1), dim3(64), 0, s, ctl, flags, acc);
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
    hipError_t e = launch_scan_rows(counts, counts, shard_count, nt, counts_dev, s);
    if (e == hipSuccess) e = launch_scan_small(counts_dev, base, shard_count, s);
    if (e != hipSuccess) return e;
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
