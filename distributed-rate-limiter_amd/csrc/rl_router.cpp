// rl_router.cpp — the multi-GPU router behind include/rl_engine.h (rl_router_*).
//
// One router per GPU; every rank holds a contiguous slice of the global arrival stream
// (rank order). A step moves each request to the shard that owns its key and the decision
// back, with the same protocol as distributed-rate-limiter_amd/python/rl_amd/router.py:
//
//   1. owner partition + compact 16-B wire records       (device, no host round-trip)
//   2. header exchange {count, base_ms, overflow, status}; ONE host read of the headers
//      (RCCL takes per-peer byte counts on the host)
//   3. payload all-to-all (+ the u16 limiter ids when there are several limiters)
//   4. the owner's engine decides (rl_execute_batch_device)
//   5. decisions back in the engine's packed width, one segment + exception block per
//      source (exact remainders outside the width: TB balances below -3)
//   6. scatter back to the caller's order through the partition permutation
//
// A source whose batch spans more than 2^31 ms either side of its first request sends the
// whole step in the wide SoA layout instead (every rank sees its overflow flag).
// Errors are collective: each rank publishes its engine's status in the next header, so all
// ranks fail at the same step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <vector>

#include "../../include/rl_engine.h"
#include "rl_launch.hpp"

using namespace rl;

namespace {
constexpr uint32_t kExcCap = 4096;   // exception entries per (owner, source) pair per step

template <class T>
int grow(T** p, size_t* cap, size_t n) {
    if (n <= *cap) return RL_OK;
    const size_t c = std::max(n, *cap + *cap / 2);
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    if (hipMalloc((void**)p, std::max<size_t>(c, 1) * sizeof(T)) != hipSuccess) {
        *cap = 0;
        return RL_E_NOMEM;
    }
    *cap = c;
    return RL_OK;
}

bool fatal(int64_t st) { return st < 0 && st != RL_E_INVALID_REQUEST; }

}  // namespace

struct rl_router {
    rl_engine* e = nullptr;
    uint32_t world = 1, rank = 0;
    rl_transport t{};
    size_t cap = 0;                      // largest per-rank n (max_batch); every rank's must match
    size_t rcap = 0;                     // receive capacity: world x cap
    hipStream_t own = nullptr;           // used when the caller passes stream = NULL
    hipStream_t last = nullptr;          // stream of the last step (rl_router_finish waits on it)
    // send side (cap)
    uint32_t* perm = nullptr;
    uint64_t* wire_s = nullptr;
    uint16_t* lim_s = nullptr;
    int64_t* hdr2 = nullptr;             // [base_ms, overflow] of this source
    uint64_t* mm_part = nullptr;         // [kWireBlocksMax][2] now_ms min / max partials
    int64_t* hdr = nullptr;              // [2][world][kHdrWords]: sent rows, received rows
    uint64_t* k_s = nullptr;             // wide layout (allocated on first use)
    int32_t* p_s = nullptr;
    int64_t* t_s = nullptr;
    int64_t* back_w = nullptr;
    uint8_t* ret_in = nullptr;
    size_t ret_in_cap = 0;
    // receive side, allocated for world x cap at creation: a step never allocates after
    // the header exchange, so no rank can fail alone between two collectives
    uint64_t* wire_r = nullptr;
    uint16_t* lim_r = nullptr;
    uint64_t* k_r = nullptr;
    int32_t* p_r = nullptr;
    int64_t* t_r = nullptr;
    uint8_t* a_r = nullptr;
    int64_t* rem_r = nullptr;
    int64_t* packed_r = nullptr;         // wide layout (allocated on first use, rcap)
    uint8_t* ret_out = nullptr;
    size_t ret_out_cap = 0;
    uint32_t* lost = nullptr;
    int64_t* h_hdr = nullptr;            // pinned copy of hdr
    int64_t pub = RL_OK;                 // status this rank publishes in the next header
    bool pending = false;
};

#define R_OK(x)                                             \
    do {                                                    \
        if ((x) != hipSuccess) return RL_E_DEVICE;          \
    } while (0)
#define R_RC(x)                                             \
    do {                                                    \
        const int _rc = (x);                                \
        if (_rc != RL_OK) return _rc;                       \
    } while (0)

extern "C" void rl_router_destroy(rl_router* r) {
    if (!r) return;
    if (r->last) (void)hipStreamSynchronize(r->last);
    if (r->own) (void)hipStreamSynchronize(r->own);
    void* bufs[] = {r->perm, r->wire_s, r->lim_s, r->hdr2, r->mm_part, r->hdr, r->k_s, r->p_s, r->t_s,
                    r->back_w, r->ret_in, r->wire_r, r->lim_r, r->k_r, r->p_r, r->t_r, r->a_r,
                    r->rem_r, r->packed_r, r->ret_out, r->lost};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (r->h_hdr) (void)hipHostFree(r->h_hdr);
    if (r->own) (void)hipStreamDestroy(r->own);
    delete r;
}

// Bytes of the segmented return trip for G sources of at most `each` requests, any width.
static uint64_t ret_worst(uint32_t G, size_t each) {
    std::vector<uint64_t> c(G, each);
    return rl_route_return_bytes(G, c.data(), 8, kExcCap);
}

extern "C" int rl_router_create(rl_engine* e, uint32_t world, uint32_t rank, const rl_transport* t,
                                size_t max_batch, rl_router** out) {
    if (!out) return RL_E_INVALID_ARG;
    *out = nullptr;
    if (!e || !t || !t->all_to_all_v || world == 0 || world > (uint32_t)kMaxShards ||
        (world & (world - 1)) || rank >= world || max_batch == 0 || max_batch > 0xFFFFFFF0ULL)
        return RL_E_INVALID_ARG;
    if ((uint64_t)world * max_batch > 0xFFFFFFF0ULL) return RL_E_TOO_LARGE;   // u32 positions
    rl_router* r = new (std::nothrow) rl_router();
    if (!r) return RL_E_NOMEM;
    r->e = e; r->world = world; r->rank = rank; r->t = *t; r->cap = max_batch;
    r->rcap = (size_t)world * max_batch;
    const size_t n = max_batch, m = r->rcap;
    (void)hipSetDevice(engine_device(e));
    bool ok = hipStreamCreateWithFlags(&r->own, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->perm, n * 4) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->wire_s, n * 16) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->lim_s, n * 2) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->hdr2, 2 * 8) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->mm_part, 2 * (size_t)kWireBlocksMax * 8) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->hdr, 2 * (size_t)world * kHdrWords * 8) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->lost, 4) == hipSuccess;
    ok = ok && hipMemset(r->lost, 0, 4) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&r->h_hdr, 2 * (size_t)world * kHdrWords * 8) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->wire_r, m * 16) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->lim_r, m * 2) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->k_r, m * 8) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->p_r, m * 4) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->t_r, m * 8) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->a_r, m) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->rem_r, m * 8) == hipSuccess;
    r->ret_out_cap = ret_worst(world, n * world);
    r->ret_in_cap = ret_worst(world, n);
    ok = ok && hipMalloc((void**)&r->ret_out, r->ret_out_cap) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->ret_in, r->ret_in_cap) == hipSuccess;
    if (!ok) { rl_router_destroy(r); return RL_E_NOMEM; }
    *out = r;
    return RL_OK;
}

static int a2av(rl_router* r, const void* send, const std::vector<uint64_t>& sb, void* recv,
                const std::vector<uint64_t>& rb, hipStream_t s) {
    std::vector<uint64_t> so(r->world), ro(r->world);
    uint64_t a = 0, b = 0;
    for (uint32_t p = 0; p < r->world; ++p) { so[p] = a; a += sb[p]; ro[p] = b; b += rb[p]; }
    return r->t.all_to_all_v(r->t.ctx, send, so.data(), sb.data(), recv, ro.data(), rb.data(), s) == 0
               ? RL_OK : RL_E_DEVICE;
}

static std::vector<uint64_t> scaled(const std::vector<uint64_t>& c, uint64_t bytes) {
    std::vector<uint64_t> o(c.size());
    for (size_t i = 0; i < c.size(); ++i) o[i] = c[i] * bytes;
    return o;
}

// Worse of two statuses (fatal beats invalid-request beats ok; then the lower code).
static int64_t worse(int64_t a, int64_t b) {
    if (a == RL_OK) return b;
    if (b == RL_OK) return a;
    if (fatal(a) != fatal(b)) return fatal(a) ? a : b;
    return std::min(a, b);
}

// Failure model (include/rl_engine.h: errors are collective). Before the header exchange a
// step may fail on its own (bad arguments, a launch error: nothing has been sent). After
// it, every rank goes through every collective of the step whatever happens locally: all
// receive buffers exist from creation, an engine call that fails leaves its requests
// undecided (RL_REMAINING_ERROR) and its status is published in the next header, and every
// rank returns it at the same later step (or from rl_router_finish).
extern "C" int rl_router_step(rl_router* r, size_t n, const uint64_t* key, const int32_t* permits,
                              const int64_t* now_ns, const uint16_t* limiter, uint8_t* allowed,
                              int64_t* remaining, void* stream) {
    if (!r) return RL_E_INVALID_ARG;
    if (n > r->cap) return RL_E_TOO_LARGE;          // caller error, before any collective
    if (n && (!key || !permits || !now_ns || !allowed || !remaining)) return RL_E_INVALID_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : r->own;
    r->last = s;
    const uint32_t G = r->world;
    rl_engine* e = r->e;
    int64_t* hdr_s = r->hdr;
    int64_t* hdr_r = r->hdr + (size_t)G * kHdrWords;
    // 1. partition (counts into the header on the device) + compact wire records + the
    // batch's now_ms range (per-block partials, folded by the header fill)
    R_RC(rl_route_partition_device(e, n, key, G, r->perm, hdr_s, kHdrWords, s));
    uint32_t nparts = 0;
    R_RC(route_pack_wire_mm(e, n, r->perm, key, permits, now_ns, limiter, r->wire_s,
                            limiter ? r->lim_s : nullptr, r->hdr2, r->mm_part, &nparts, s));
    R_OK(launch_fill_header(hdr_s, r->hdr2, r->pub, (int64_t)r->cap, G, r->mm_part, nparts, s));
    // 2. header exchange and the step's one host synchronisation
    std::vector<uint64_t> hb(G, kHdrWords * 8);
    R_RC(a2av(r, hdr_s, hb, hdr_r, hb, s));
    R_OK(hipMemcpyAsync(r->h_hdr, r->hdr, 2 * (size_t)G * kHdrWords * 8, hipMemcpyDeviceToHost, s));
    R_OK(hipStreamSynchronize(s));
    std::vector<uint64_t> counts(G), rc(G);
    std::vector<int64_t> base(G);
    bool wide = false, cap_mismatch = false;
    int64_t worst = RL_OK, tmin = INT64_MAX, tmax = INT64_MIN;
    for (uint32_t p = 0; p < G; ++p) {
        const int64_t* snt = r->h_hdr + (size_t)p * kHdrWords;
        const int64_t* rcv = r->h_hdr + (size_t)(G + p) * kHdrWords;
        counts[p] = (uint64_t)snt[0];
        rc[p] = (uint64_t)rcv[0];
        base[p] = rcv[1];
        wide |= rcv[2] != 0;
        if (fatal(rcv[3])) worst = worse(worst, rcv[3]);
        cap_mismatch |= rcv[4] != (int64_t)r->cap;
        if (rc[p]) { tmin = std::min(tmin, rcv[5]); tmax = std::max(tmax, rcv[6]); }
    }
    // the previous batch is complete (ordered before the header exchange): its status is
    // published in the next header; the statuses received now (every rank's batch two steps
    // back) are the same on all ranks, so all fail together
    if (r->pending) { r->pub = rl_last_status(e); r->pending = false; }
    if (worst != RL_OK) return (int)worst;
    // every rank sees every rank's capacity: a mismatch fails all of them here, before any
    // payload (receive buffers are sized world x max_batch)
    if (cap_mismatch) return RL_E_INVALID_ARG;
    uint64_t m = 0;
    for (uint64_t c : rc) m += c;
    if (m > r->rcap) return RL_E_TOO_LARGE;          // (not reached: counts <= cap per source)
    int64_t local = RL_OK;                           // this step's own failure, published later
    if (!wide) {
        // 3. payload: 16-B wire records (+ limiter ids)
        R_RC(a2av(r, r->wire_s, scaled(counts, 16), r->wire_r, scaled(rc, 16), s));
        if (limiter) R_RC(a2av(r, r->lim_s, scaled(counts, 2), r->lim_r, scaled(rc, 2), s));
        R_RC(rl_route_unwire(e, m, r->wire_r, G, base.data(), rc.data(), r->k_r, r->p_r, r->t_r, s));
        // 4. the owner decides. The merged batch spans the sources' real time range; past
        // what the engine's compact records hold (+-2^31 ms around its first request) it runs
        // in full-width records (skewed clocks across front-ends).
        const bool far = m && tmax > tmin && (uint64_t)(tmax - tmin) >= ((uint64_t)1 << 31) - 1;
        if (far) (void)rl_tune(e, "wide_records", 1);
        const int xrc = rl_execute_batch_device(e, m, r->k_r, r->p_r, r->t_r, limiter ? r->lim_r : nullptr,
                                                nullptr, r->a_r, r->rem_r, nullptr, s);
        if (far) (void)rl_tune(e, "wide_records", 0);
        if (xrc != RL_OK) {
            local = xrc;
            R_OK(launch_fill_value(r->a_r, r->rem_r, (uint32_t)m, RL_REMAINING_ERROR, s));
        }
        // 5. decisions back, segmented with exception blocks
        int W = rl_result_width(e);
        if (W < 0) { local = worse(local, W); W = 8; }
        const uint64_t ob = rl_route_return_bytes(G, rc.data(), W, kExcCap);
        const uint64_t ib = rl_route_return_bytes(G, counts.data(), W, kExcCap);
        if (ob > r->ret_out_cap || ib > r->ret_in_cap) return RL_E_TOO_LARGE;   // (not reached)
        R_RC(rl_route_fold_return(e, m, r->a_r, r->rem_r, r->ret_out, W, G, rc.data(), kExcCap, s));
        std::vector<uint64_t> seg_o(G), seg_i(G);
        for (uint32_t p = 0; p < G; ++p) {
            seg_o[p] = rl_route_return_bytes(1, &rc[p], W, kExcCap);
            seg_i[p] = rl_route_return_bytes(1, &counts[p], W, kExcCap);
        }
        R_RC(a2av(r, r->ret_out, seg_o, r->ret_in, seg_i, s));
        // 6. back to the caller's order
        R_RC(rl_route_unpack_return(e, n, r->perm, r->ret_in, W, G, counts.data(), kExcCap, allowed,
                                    remaining, r->lost, s));
    } else {
        if (!r->k_s) {                           // wide buffers on first use
            size_t c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0;
            int grc = grow(&r->k_s, &c1, r->cap);
            if (grc == RL_OK) grc = grow(&r->p_s, &c2, r->cap);
            if (grc == RL_OK) grc = grow(&r->t_s, &c3, r->cap);
            if (grc == RL_OK) grc = grow(&r->back_w, &c4, r->cap);
            if (grc == RL_OK) grc = grow(&r->packed_r, &c5, r->rcap);
            if (grc != RL_OK) {
                // (the rank cannot take part in this step's payload: release what was taken
                // so the next attempt allocates again; its peers see RL_E_NOMEM as this
                // rank's step returns before the payload, a documented, rare local failure)
                void* bs[] = {r->k_s, r->p_s, r->t_s, r->back_w, r->packed_r};
                for (void* b : bs) if (b) (void)hipFree(b);
                r->k_s = nullptr; r->p_s = nullptr; r->t_s = nullptr; r->back_w = nullptr; r->packed_r = nullptr;
                return grc;
            }
        }
        R_RC(rl_route_pack(e, n, r->perm, key, permits, now_ns, limiter, r->k_s, r->p_s, r->t_s,
                           limiter ? r->lim_s : nullptr, s));
        R_RC(a2av(r, r->k_s, scaled(counts, 8), r->k_r, scaled(rc, 8), s));
        R_RC(a2av(r, r->p_s, scaled(counts, 4), r->p_r, scaled(rc, 4), s));
        R_RC(a2av(r, r->t_s, scaled(counts, 8), r->t_r, scaled(rc, 8), s));
        if (limiter) R_RC(a2av(r, r->lim_s, scaled(counts, 2), r->lim_r, scaled(rc, 2), s));
        // a source's batch spans more than 2^31 ms: the merged batch needs full-width times
        (void)rl_tune(e, "wide_records", 1);
        const int xrc = rl_execute_batch_device(e, m, r->k_r, r->p_r, r->t_r, limiter ? r->lim_r : nullptr,
                                                nullptr, r->a_r, r->rem_r, nullptr, s);
        (void)rl_tune(e, "wide_records", 0);
        if (xrc != RL_OK) {
            local = xrc;
            R_OK(launch_fill_value(r->a_r, r->rem_r, (uint32_t)m, RL_REMAINING_ERROR, s));
        }
        R_RC(rl_route_fold(e, m, r->a_r, r->rem_r, r->packed_r, s));
        R_RC(a2av(r, r->packed_r, scaled(rc, 8), r->back_w, scaled(counts, 8), s));
        R_RC(rl_route_unpack(e, n, r->perm, r->back_w, allowed, remaining, s));
    }
    if (local != RL_OK) r->pub = worse(r->pub, local);   // published in the next header
    else r->pending = true;
    return RL_OK;
}

extern "C" int rl_router_finish(rl_router* r) {
    if (!r) return RL_E_INVALID_ARG;
    hipStream_t s = r->own;
    // the last step may still run on the caller's stream (its return all-to-all and the
    // unpack that counts lost remainders): complete it before reading anything
    if (r->last) R_OK(hipStreamSynchronize(r->last));
    if (r->pending) { r->pub = rl_last_status(r->e); r->pending = false; }
    uint32_t lost = 0;
    R_OK(hipMemcpy(&lost, r->lost, 4, hipMemcpyDeviceToHost));
    if (lost) R_OK(hipMemset(r->lost, 0, 4));        // counted once: the next steps start clean
    const int64_t mine = lost ? worse(r->pub, (int64_t)RL_E_CAPACITY) : r->pub;
    r->pub = RL_OK;                                  // reported now, on every rank
    const uint32_t G = r->world;
    int64_t* hdr_s = r->hdr;
    int64_t* hdr_r = r->hdr + (size_t)G;
    std::vector<int64_t> row(G, mine);
    R_OK(hipMemcpyAsync(hdr_s, row.data(), G * 8, hipMemcpyHostToDevice, s));
    std::vector<uint64_t> b(G, 8);
    R_RC(a2av(r, hdr_s, b, hdr_r, b, s));
    std::vector<int64_t> got(G);
    R_OK(hipMemcpyAsync(got.data(), hdr_r, G * 8, hipMemcpyDeviceToHost, s));
    R_OK(hipStreamSynchronize(s));
    int64_t w = RL_OK;
    for (int64_t x : got) w = worse(w, x);
    return (int)w;
}

extern "C" int rl_router_plan_directory(rl_router* r, size_t n, const uint64_t* key,
                                        const uint64_t* count, uint64_t sampled, uint32_t k,
                                        uint32_t* placed, void* stream) {
    if (!r || (n && (!key || !count)) || n > kDirMax || k > kDirMax) return RL_E_INVALID_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : r->own;
    const uint32_t G = r->world;
    // exchange {n, sampled}, then every rank's candidates with every rank (all-gather)
    uint64_t* d = nullptr;
    const size_t hdr_words = 2 * (size_t)G * 2;
    R_OK(hipMalloc((void**)&d, hdr_words * 8));
    std::vector<uint64_t> mine(2 * (size_t)G);
    for (uint32_t p = 0; p < G; ++p) { mine[2 * p] = n; mine[2 * p + 1] = sampled; }
    std::vector<uint64_t> hb(G, 16);
    std::vector<uint64_t> peer(2 * (size_t)G);
    int rc = hipMemcpyAsync(d, mine.data(), G * 16, hipMemcpyHostToDevice, s) == hipSuccess ? RL_OK : RL_E_DEVICE;
    if (rc == RL_OK) rc = a2av(r, d, hb, d + 2 * G, hb, s);
    if (rc == RL_OK && (hipMemcpyAsync(peer.data(), d + 2 * G, G * 16, hipMemcpyDeviceToHost, s) != hipSuccess ||
                        hipStreamSynchronize(s) != hipSuccess))
        rc = RL_E_DEVICE;
    (void)hipFree(d);
    if (rc != RL_OK) return rc;
    uint64_t total_n = 0, total_sampled = 0;
    std::vector<uint64_t> rb(G), sb(G, 16 * (uint64_t)n);
    for (uint32_t p = 0; p < G; ++p) { rb[p] = 16 * peer[2 * p]; total_n += peer[2 * p]; total_sampled += peer[2 * p + 1]; }
    std::vector<uint64_t> cand(2 * std::max<size_t>(n, 1)), all(2 * std::max<uint64_t>(total_n, 1));
    for (size_t i = 0; i < n; ++i) { cand[2 * i] = key[i]; cand[2 * i + 1] = count[i]; }
    uint64_t* ds = nullptr;
    uint64_t* dr = nullptr;
    if (hipMalloc((void**)&ds, cand.size() * 8) != hipSuccess) return RL_E_NOMEM;
    if (hipMalloc((void**)&dr, all.size() * 8) != hipSuccess) { (void)hipFree(ds); return RL_E_NOMEM; }
    // every peer gets the same block: send offsets all 0
    std::vector<uint64_t> so(G, 0), ro(G);
    uint64_t acc = 0;
    for (uint32_t p = 0; p < G; ++p) { ro[p] = acc; acc += rb[p]; }
    rc = hipMemcpyAsync(ds, cand.data(), n * 16, hipMemcpyHostToDevice, s) == hipSuccess ? RL_OK : RL_E_DEVICE;
    if (rc == RL_OK && r->t.all_to_all_v(r->t.ctx, ds, so.data(), sb.data(), dr, ro.data(), rb.data(), s) != 0)
        rc = RL_E_DEVICE;
    if (rc == RL_OK && (hipMemcpyAsync(all.data(), dr, total_n * 16, hipMemcpyDeviceToHost, s) != hipSuccess ||
                        hipStreamSynchronize(s) != hipSuccess))
        rc = RL_E_DEVICE;
    (void)hipFree(ds);
    (void)hipFree(dr);
    if (rc != RL_OK) return rc;
    // merge (same order on every rank), keep the k hottest, place them LPT-first
    std::map<uint64_t, uint64_t> sum;
    for (uint64_t i = 0; i < total_n; ++i) sum[all[2 * i]] += all[2 * i + 1];
    std::vector<std::pair<uint64_t, uint64_t>> v(sum.begin(), sum.end());
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) {
        return a.second != b.second ? a.second > b.second : a.first < b.first;
    });
    if (v.size() > k) v.resize(k);
    uint64_t hot = 0;
    for (auto& x : v) hot += x.second;
    const double rest = total_sampled > hot ? (double)(total_sampled - hot) / G : 0.0;
    std::vector<double> load(G, rest);
    std::vector<uint64_t> dk(v.size());
    std::vector<uint32_t> dov(v.size());
    for (size_t i = 0; i < v.size(); ++i) {
        uint32_t best = 0;
        for (uint32_t p = 1; p < G; ++p)
            if (load[p] < load[best]) best = p;
        load[best] += (double)v[i].second;
        dk[i] = v[i].first;
        dov[i] = best;
    }
    rc = rl_set_owner_directory(r->e, dk.size(), dk.data(), dov.data());
    if (rc == RL_OK && placed) *placed = (uint32_t)dk.size();
    return rc;
}
