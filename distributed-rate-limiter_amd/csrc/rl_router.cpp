// rl_router.cpp — the multi-GPU router behind include/rl_engine.h (rl_router_*).
//
// One router per GPU; every rank holds a contiguous slice of the global arrival stream
// (rank order). A step moves each request to the shard that owns its key and the decision
// back, with the same protocol as distributed-rate-limiter_amd/python/rl_amd/router.py:
//
//   1. owner partition + compact 16-B wire records       (device, no host round-trip)
//   2. header exchange {count, base_ms, overflow, status, capacities, now range, and the
//      source's count for every owner}; ONE host read of the headers (RCCL takes per-peer
//      byte counts on the host). Every rank then knows the whole count matrix, so all of
//      them derive the same exchange plan: one round, or — when some owner would receive
//      more than its receive capacity — several rounds, each moving the next piece of every
//      owner's incoming stream (sources in rank order, so per-key arrival order holds)
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
#include <chrono>
#include <cstring>
#include <map>
#include <vector>

#include "../../include/rl_engine.h"
#include "rl_launch.hpp"

using namespace rl;

namespace {
constexpr uint32_t kExcCap = 4096;   // exception entries per (owner, source) pair per step

bool fatal(int64_t st) { return st < 0 && st != RL_E_INVALID_REQUEST; }

// Bytes of a segmented return trip of `total` requests over G segments, any width and split.
uint64_t ret_bound(uint32_t G, uint64_t total) {
    return total * 8 + (uint64_t)G * (8 + ret_block_bytes(kExcCap));
}
// Words of the directory exchange: {n, sampled} rows both ways, this rank's candidates, and
// every rank's candidates.
size_t dir_words(uint32_t G) { return 4 * (size_t)G + 2 * (size_t)kDirMax * (1 + (size_t)G); }

}  // namespace

struct rl_router {
    rl_engine* e = nullptr;
    uint32_t world = 1, rank = 0;
    rl_transport t{};
    size_t cap = 0;                      // largest per-rank n (max_batch); every rank's must match
    size_t rcap = 0;                     // requests an owner decides per exchange round
    hipStream_t own = nullptr;           // used when the caller passes stream = NULL
    hipEvent_t done = nullptr;           // recorded at the end of every step on its stream
    bool stepped = false;                // `done` has been recorded
    // send side (cap); everything below is allocated by rl_router_create, so a step never
    // allocates and no rank can fail alone between two collectives
    uint32_t* perm = nullptr;
    uint64_t* wire_s = nullptr;
    uint16_t* lim_s = nullptr;
    int64_t* hdr2 = nullptr;             // [base_ms, overflow] of this source
    uint64_t* mm_part = nullptr;         // [kWireBlocksMax][2] now_ms min / max partials
    int64_t* hdr = nullptr;              // [2][world][kHdrWords]: sent rows, received rows
    uint64_t* k_s = nullptr;             // wide layout (SoA in owner order)
    int32_t* p_s = nullptr;
    int64_t* t_s = nullptr;
    int64_t* back_w = nullptr;           // 8-B decisions back (wide layout / split steps)
    uint8_t* ret_in = nullptr;
    uint64_t ret_in_cap = 0;
    uint64_t* dir = nullptr;             // directory exchange (dir_words)
    // receive side (rcap)
    uint64_t* wire_r = nullptr;
    uint16_t* lim_r = nullptr;
    uint64_t* k_r = nullptr;
    int32_t* p_r = nullptr;
    int64_t* t_r = nullptr;
    uint8_t* a_r = nullptr;
    int64_t* rem_r = nullptr;
    int64_t* packed_r = nullptr;
    uint8_t* ret_out = nullptr;
    uint64_t ret_out_cap = 0;
    uint32_t* lost = nullptr;
    int64_t* h_hdr = nullptr;            // pinned copy of hdr
    unsigned long long* acc = nullptr;   // split rounds: the rounds' engine statuses, folded on
                                         // device (kStatusAccWords), settled at the next step
    int64_t pub = RL_OK;                 // status this rank publishes in the next header
    bool pending = false;                // the last engine batch's status is still to collect
    bool acc_pending = false;            // acc holds a split step's statuses to settle
    rl_router_stats st{};
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
    // the last step's work (on the caller's stream, which may be gone by now: wait on our
    // own event instead)
    if (r->done && r->stepped) (void)hipEventSynchronize(r->done);
    if (r->own) (void)hipStreamSynchronize(r->own);
    void* bufs[] = {r->perm, r->wire_s, r->lim_s, r->hdr2, r->mm_part, r->hdr, r->k_s, r->p_s, r->t_s,
                    r->back_w, r->ret_in, r->dir, r->wire_r, r->lim_r, r->k_r, r->p_r, r->t_r, r->a_r,
                    r->rem_r, r->packed_r, r->ret_out, r->lost, r->acc};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (r->h_hdr) (void)hipHostFree(r->h_hdr);
    if (r->done) (void)hipEventDestroy(r->done);
    if (r->own) (void)hipStreamDestroy(r->own);
    delete r;
}

extern "C" int rl_router_create_ex(rl_engine* e, uint32_t world, uint32_t rank, const rl_transport* t,
                                   const rl_router_opts* opts, rl_router** out) {
    if (!out) return RL_E_INVALID_ARG;
    *out = nullptr;
    if (!e || !t || !t->all_to_all_v || !opts || world == 0 || world > (uint32_t)kMaxShards ||
        (world & (world - 1)) || rank >= world || opts->max_batch == 0 ||
        opts->max_batch > 0xFFFFFFF0ULL)
        return RL_E_INVALID_ARG;
    const size_t n = opts->max_batch;
    size_t m = opts->recv_cap ? opts->recv_cap : std::min<size_t>(world, 2) * n;
    m = std::min(m, engine_max_batch(e));           // the owner's engine decides <= m at once
    if (m == 0) return RL_E_INVALID_ARG;
    rl_router* r = new (std::nothrow) rl_router();
    if (!r) return RL_E_NOMEM;
    r->e = e; r->world = world; r->rank = rank; r->t = *t; r->cap = n; r->rcap = m;
    (void)hipSetDevice(engine_device(e));
    uint64_t bytes = 0;
    auto take = [&](auto** p, size_t b) {
        bytes += b;
        return hipMalloc((void**)p, std::max<size_t>(b, 8)) == hipSuccess;
    };
    r->ret_out_cap = ret_bound(world, m);
    r->ret_in_cap = ret_bound(world, n);
    bool ok = hipStreamCreateWithFlags(&r->own, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&r->done, hipEventDisableTiming) == hipSuccess;
    ok = ok && take(&r->perm, n * 4) && take(&r->wire_s, n * 16) && take(&r->lim_s, n * 2);
    ok = ok && take(&r->k_s, n * 8) && take(&r->p_s, n * 4) && take(&r->t_s, n * 8);
    ok = ok && take(&r->back_w, n * 8) && take(&r->ret_in, r->ret_in_cap);
    ok = ok && take(&r->hdr2, 2 * 8) && take(&r->mm_part, 2 * (size_t)kWireBlocksMax * 8);
    ok = ok && take(&r->hdr, 2 * (size_t)world * kHdrWords * 8) && take(&r->lost, 4);
    ok = ok && take(&r->dir, dir_words(world) * 8);
    ok = ok && take(&r->wire_r, m * 16) && take(&r->lim_r, m * 2) && take(&r->k_r, m * 8);
    ok = ok && take(&r->p_r, m * 4) && take(&r->t_r, m * 8) && take(&r->a_r, m);
    ok = ok && take(&r->rem_r, m * 8) && take(&r->packed_r, m * 8) && take(&r->ret_out, r->ret_out_cap);
    ok = ok && take(&r->acc, kStatusAccWords * 8);
    ok = ok && hipMemset(r->lost, 0, 4) == hipSuccess;
    ok = ok && hipMemset(r->acc, 0, kStatusAccWords * 8) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&r->h_hdr, 2 * (size_t)world * kHdrWords * 8) == hipSuccess;
    if (!ok) { rl_router_destroy(r); return RL_E_NOMEM; }
    r->st.recv_cap = m;
    r->st.reserved_bytes = bytes;
    *out = r;
    return RL_OK;
}

extern "C" int rl_router_create(rl_engine* e, uint32_t world, uint32_t rank, const rl_transport* t,
                                size_t max_batch, rl_router** out) {
    rl_router_opts o{};
    o.max_batch = max_batch;
    return rl_router_create_ex(e, world, rank, t, &o, out);
}

extern "C" int rl_router_stats_get(rl_router* r, rl_router_stats* out) {
    if (!r || !out) return RL_E_INVALID_ARG;
    *out = r->st;
    return RL_OK;
}

// all-to-all with explicit element offsets / counts (host arrays of `world` entries)
static int a2av_at(rl_router* r, const void* send, const uint64_t* so, const uint64_t* sc,
                   void* recv, const uint64_t* ro, const uint64_t* rc, uint64_t bytes, hipStream_t s) {
    const uint32_t G = r->world;
    std::vector<uint64_t> sob(G), scb(G), rob(G), rcb(G);
    for (uint32_t p = 0; p < G; ++p) {
        sob[p] = so[p] * bytes; scb[p] = sc[p] * bytes; rob[p] = ro[p] * bytes; rcb[p] = rc[p] * bytes;
    }
    return r->t.all_to_all_v(r->t.ctx, send, sob.data(), scb.data(), recv, rob.data(), rcb.data(), s) == 0
               ? RL_OK : RL_E_DEVICE;
}

// contiguous segments: offsets are the running sums of the counts
static std::vector<uint64_t> offsets(const std::vector<uint64_t>& c) {
    std::vector<uint64_t> o(c.size());
    uint64_t a = 0;
    for (size_t i = 0; i < c.size(); ++i) { o[i] = a; a += c[i]; }
    return o;
}

static int a2av(rl_router* r, const void* send, const std::vector<uint64_t>& sc, void* recv,
                const std::vector<uint64_t>& rc, uint64_t bytes, hipStream_t s) {
    const std::vector<uint64_t> so = offsets(sc), ro = offsets(rc);
    return a2av_at(r, send, so.data(), sc.data(), recv, ro.data(), rc.data(), bytes, s);
}

// Worse of two statuses (fatal beats invalid-request beats ok; then the lower code).
static int64_t worse(int64_t a, int64_t b) {
    if (a == RL_OK) return b;
    if (b == RL_OK) return a;
    if (fatal(a) != fatal(b)) return fatal(a) ? a : b;
    return std::min(a, b);
}

// The status of this rank's last step's engine batches (the previous step is complete:
// everything before the caller's header exchange or finish). One batch: the engine's own
// collection; a split step: the rounds' statuses folded on device. Either applies the table
// growth the batches asked for, here at the step boundary and never between two rounds.
static int64_t settle_pending(rl_router* r) {
    int64_t st = RL_OK;
    if (r->pending) { st = worse(st, rl_last_status(r->e)); r->pending = false; }
    if (r->acc_pending) {
        unsigned long long h[kStatusAccWords];
        if (r->stepped && hipEventSynchronize(r->done) != hipSuccess) return RL_E_DEVICE;
        if (hipMemcpy(h, r->acc, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemset(r->acc, 0, sizeof(h)) != hipSuccess)
            return RL_E_DEVICE;
        st = worse(st, engine_status_settle(r->e, h));
        r->acc_pending = false;
    }
    return st;
}

static uint64_t clampu(int64_t x, uint64_t hi) {
    return x <= 0 ? 0 : ((uint64_t)x > hi ? hi : (uint64_t)x);
}

// Failure model (include/rl_engine.h: errors are collective). Before the header exchange a
// step may fail on its own (bad arguments, a launch error: nothing has been sent). After
// it, every rank goes through every collective of the step whatever happens locally: all
// buffers exist from creation, an engine call that fails leaves its requests undecided
// (RL_REMAINING_ERROR) and its status is published in the next header, and every rank
// returns it at the same later step (or from rl_router_finish). Every rank derives the
// step's exchange plan (rounds, per-pair ranges) from the same header rows.
extern "C" int rl_router_step(rl_router* r, size_t n, const uint64_t* key, const int32_t* permits,
                              const int64_t* now_ns, const uint16_t* limiter, uint8_t* allowed,
                              int64_t* remaining, void* stream) {
    if (!r) return RL_E_INVALID_ARG;
    if (n > r->cap) return RL_E_TOO_LARGE;          // caller error, before any collective
    if (n && (!key || !permits || !now_ns || !allowed || !remaining)) return RL_E_INVALID_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : r->own;
    const uint32_t G = r->world, me = r->rank;
    rl_engine* e = r->e;
    int64_t* hdr_s = r->hdr;
    int64_t* hdr_r = r->hdr + (size_t)G * kHdrWords;
    // 1. partition (counts into the header on the device) + compact wire records + the
    // batch's now_ms range (per-block partials, folded by the header fill)
    R_RC(rl_route_partition_device(e, n, key, G, r->perm, hdr_s, kHdrWords, s));
    uint32_t nparts = 0;
    R_RC(route_pack_wire_mm(e, n, r->perm, key, permits, now_ns, limiter, r->wire_s,
                            limiter ? r->lim_s : nullptr, r->hdr2, r->mm_part, &nparts, s));
    R_OK(launch_fill_header(hdr_s, r->hdr2, r->pub, (int64_t)r->cap, (int64_t)r->rcap, G, r->mm_part,
                            nparts, s));
    // 2. header exchange and the step's one host synchronisation
    const std::vector<uint64_t> hw(G, kHdrWords);
    R_RC(a2av(r, hdr_s, hw, hdr_r, hw, 8, s));
    R_OK(hipMemcpyAsync(r->h_hdr, r->hdr, 2 * (size_t)G * kHdrWords * 8, hipMemcpyDeviceToHost, s));
    const auto c0 = std::chrono::steady_clock::now();
    R_OK(hipStreamSynchronize(s));
    const auto c1 = std::chrono::steady_clock::now();
    r->st.header_sync_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(c1 - c0).count();
    ++r->st.steps;
    // count matrix C[src][owner] from every source's row (the same on every rank)
    std::vector<uint64_t> C((size_t)G * G);
    std::vector<int64_t> base(G);
    bool wide = false, cap_mismatch = false;
    int64_t worst = RL_OK, tmin = INT64_MAX, tmax = INT64_MIN;
    for (uint32_t p = 0; p < G; ++p) {
        const int64_t* rcv = r->h_hdr + (size_t)(G + p) * kHdrWords;
        for (uint32_t o = 0; o < G; ++o) C[(size_t)p * G + o] = (uint64_t)rcv[kHdrFixed + o];
        base[p] = rcv[1];
        wide |= rcv[2] != 0;
        if (fatal(rcv[3])) worst = worse(worst, rcv[3]);
        cap_mismatch |= rcv[4] != (int64_t)r->cap || rcv[7] != (int64_t)r->rcap;
        if (rcv[0]) { tmin = std::min(tmin, rcv[5]); tmax = std::max(tmax, rcv[6]); }
    }
    std::vector<uint64_t> counts(G), rc(G);         // mine to each owner, each source's to me
    for (uint32_t p = 0; p < G; ++p) { counts[p] = C[(size_t)me * G + p]; rc[p] = C[(size_t)p * G + me]; }
    // the previous batch is complete (ordered before the header exchange): its status is
    // published in the next header; the statuses received now (every rank's batch two steps
    // back) are the same on all ranks, so all fail together
    if (fatal(r->pub)) r->pub = RL_OK;              // delivered: every rank returns it now, once
    r->pub = worse(r->pub, settle_pending(r));
    // every rank sees every rank's capacities: a mismatch fails all of them here, before
    // any payload (all ranks must derive the same exchange plan)
    if (worst != RL_OK || cap_mismatch) {
        // this step's own requests are not decided: say so in its outputs, so that a caller
        // that goes on does not read the previous step's decisions as this one's
        R_OK(launch_fill_value(allowed, remaining, (uint32_t)n, RL_REMAINING_ERROR, s));
        R_OK(hipEventRecord(r->done, s));
        r->stepped = true;
        return worst != RL_OK ? (int)worst : RL_E_INVALID_ARG;
    }
    // rounds: each owner's incoming stream (sources in rank order = global arrival order)
    // is cut into pieces of at most rcap requests; round k moves piece k of every owner
    uint64_t rounds = 1, m = 0;
    for (uint32_t o = 0; o < G; ++o) {
        uint64_t mo = 0;
        for (uint32_t p = 0; p < G; ++p) mo += C[(size_t)p * G + o];
        rounds = std::max<uint64_t>(rounds, (mo + r->rcap - 1) / r->rcap);
        if (o == me) m = mo;
    }
    r->st.max_recv = std::max<uint64_t>(r->st.max_recv, m);
    r->st.rounds += rounds;
    int64_t local = RL_OK;                           // this step's own failure, published later
    const bool far = m && tmax > tmin && (uint64_t)(tmax - tmin) >= ((uint64_t)1 << 31) - 1;
    if (!wide && rounds == 1) {
        // 3. payload: 16-B wire records (+ limiter ids)
        R_RC(a2av(r, r->wire_s, counts, r->wire_r, rc, 16, s));
        if (limiter) R_RC(a2av(r, r->lim_s, counts, r->lim_r, rc, 2, s));
        R_RC(rl_route_unwire(e, m, r->wire_r, G, base.data(), rc.data(), r->k_r, r->p_r, r->t_r, s));
        // 4. the owner decides. The merged batch spans the sources' real time range; past
        // what the engine's compact records hold (+-2^31 ms around its first request) it runs
        // in full-width records (skewed clocks across front-ends).
        if (far) (void)rl_tune(e, "wide_records", 1);
        const int xrc = rl_execute_batch_device(e, m, r->k_r, r->p_r, r->t_r, limiter ? r->lim_r : nullptr,
                                                nullptr, r->a_r, r->rem_r, nullptr, s);
        if (far) (void)rl_tune(e, "wide_records", 0);
        if (xrc != RL_OK) {
            local = xrc;
            R_OK(launch_fill_value(r->a_r, r->rem_r, (uint32_t)m, RL_REMAINING_ERROR, s));
        } else {
            r->pending = true;
        }
        // 5. decisions back, segmented with exception blocks
        int W = rl_result_width(e);
        if (W < 0) { local = worse(local, W); W = 8; }
        R_RC(rl_route_fold_return(e, m, r->a_r, r->rem_r, r->ret_out, W, G, rc.data(), kExcCap, s));
        std::vector<uint64_t> seg_o(G), seg_i(G);
        for (uint32_t p = 0; p < G; ++p) {
            seg_o[p] = rl_route_return_bytes(1, &rc[p], W, kExcCap);
            seg_i[p] = rl_route_return_bytes(1, &counts[p], W, kExcCap);
        }
        R_RC(a2av(r, r->ret_out, seg_o, r->ret_in, seg_i, 1, s));
        // 6. back to the caller's order
        R_RC(rl_route_unpack_return(e, n, r->perm, r->ret_in, W, G, counts.data(), kExcCap, allowed,
                                    remaining, r->lost, s));
    } else {
        // Wide layout (a source's batch spans more than 2^31 ms: SoA payload) and/or several
        // rounds (some owner receives more than rcap requests): 8-B decisions back into
        // back_w at each request's owner-order position, one unpack at the end.
        if (wide) R_RC(rl_route_pack(e, n, r->perm, key, permits, now_ns, limiter, r->k_s, r->p_s,
                                     r->t_s, limiter ? r->lim_s : nullptr, s));
        if (rounds > 1) ++r->st.split_steps;
        const std::vector<uint64_t> seg = offsets(counts);
        std::vector<uint64_t> Pm(G, 0), Q(G, 0);      // my start in each owner's stream; sources' in mine
        for (uint32_t o = 0; o < G; ++o)
            for (uint32_t p = 0; p < me; ++p) Pm[o] += C[(size_t)p * G + o];
        for (uint32_t p = 1; p < G; ++p) Q[p] = Q[p - 1] + rc[p - 1];
        for (uint64_t k = 0; k < rounds; ++k) {
            const int64_t lo_w = (int64_t)(k * r->rcap), hi_w = (int64_t)((k + 1) * r->rcap);
            std::vector<uint64_t> so(G), sc(G), rr(G);
            for (uint32_t o = 0; o < G; ++o) {
                const uint64_t lo = clampu(lo_w - (int64_t)Pm[o], counts[o]);
                const uint64_t hi = clampu(hi_w - (int64_t)Pm[o], counts[o]);
                so[o] = seg[o] + lo;
                sc[o] = hi - lo;
            }
            uint64_t mk = 0;
            for (uint32_t p = 0; p < G; ++p) {
                rr[p] = clampu(hi_w - (int64_t)Q[p], rc[p]) - clampu(lo_w - (int64_t)Q[p], rc[p]);
                mk += rr[p];
            }
            const std::vector<uint64_t> ro = offsets(rr);
            if (!wide) {
                R_RC(a2av_at(r, r->wire_s, so.data(), sc.data(), r->wire_r, ro.data(), rr.data(), 16, s));
                if (limiter)
                    R_RC(a2av_at(r, r->lim_s, so.data(), sc.data(), r->lim_r, ro.data(), rr.data(), 2, s));
                R_RC(rl_route_unwire(e, mk, r->wire_r, G, base.data(), rr.data(), r->k_r, r->p_r, r->t_r, s));
            } else {
                R_RC(a2av_at(r, r->k_s, so.data(), sc.data(), r->k_r, ro.data(), rr.data(), 8, s));
                R_RC(a2av_at(r, r->p_s, so.data(), sc.data(), r->p_r, ro.data(), rr.data(), 4, s));
                R_RC(a2av_at(r, r->t_s, so.data(), sc.data(), r->t_r, ro.data(), rr.data(), 8, s));
                if (limiter)
                    R_RC(a2av_at(r, r->lim_s, so.data(), sc.data(), r->lim_r, ro.data(), rr.data(), 2, s));
            }
            const bool w = wide || far;
            if (w) (void)rl_tune(e, "wide_records", 1);
            const int xrc = rl_execute_batch_device(e, mk, r->k_r, r->p_r, r->t_r,
                                                    limiter ? r->lim_r : nullptr, nullptr, r->a_r,
                                                    r->rem_r, nullptr, s);
            if (w) (void)rl_tune(e, "wide_records", 0);
            if (xrc != RL_OK) {
                local = worse(local, xrc);
                R_OK(launch_fill_value(r->a_r, r->rem_r, (uint32_t)mk, RL_REMAINING_ERROR, s));
            } else {
                // the round's data-dependent status is folded on device (the next round's
                // batch replaces the engine's own) and settled at the next step: no host
                // synchronisation and no table growth between the rounds' collectives
                R_RC(engine_status_accum(e, r->acc, s));
                r->acc_pending = true;
            }
            R_RC(rl_route_fold(e, mk, r->a_r, r->rem_r, r->packed_r, s));
            R_RC(a2av_at(r, r->packed_r, ro.data(), rr.data(), r->back_w, so.data(), sc.data(), 8, s));
        }
        R_RC(rl_route_unpack(e, n, r->perm, r->back_w, allowed, remaining, s));
    }
    if (local != RL_OK) r->pub = worse(r->pub, local);   // published in the next header
    R_OK(hipEventRecord(r->done, s));
    r->stepped = true;
    return RL_OK;
}

extern "C" int rl_router_finish(rl_router* r) {
    if (!r) return RL_E_INVALID_ARG;
    hipStream_t s = r->own;
    // the last step may still run on the caller's stream (its return all-to-all and the
    // unpack that counts lost remainders): complete it before reading anything
    if (r->stepped) R_OK(hipEventSynchronize(r->done));
    r->pub = worse(r->pub, settle_pending(r));
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
    const std::vector<uint64_t> one(G, 1);
    R_RC(a2av(r, hdr_s, one, hdr_r, one, 8, s));
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
    // exchange {n, sampled}, then every rank's candidates with every rank (all-gather), in
    // the buffer reserved at creation (no allocation between the two collectives)
    uint64_t* d = r->dir;                          // [2G] sent rows, [2G] received rows
    uint64_t* ds = d + 4 * (size_t)G;              // [2 kDirMax] my candidates
    uint64_t* dr = ds + 2 * (size_t)kDirMax;       // [2 kDirMax G] everyone's
    std::vector<uint64_t> mine(2 * (size_t)G);
    for (uint32_t p = 0; p < G; ++p) { mine[2 * p] = n; mine[2 * p + 1] = sampled; }
    const std::vector<uint64_t> two(G, 2);
    std::vector<uint64_t> peer(2 * (size_t)G);
    R_OK(hipMemcpyAsync(d, mine.data(), G * 16, hipMemcpyHostToDevice, s));
    R_RC(a2av(r, d, two, d + 2 * G, two, 8, s));
    R_OK(hipMemcpyAsync(peer.data(), d + 2 * G, G * 16, hipMemcpyDeviceToHost, s));
    R_OK(hipStreamSynchronize(s));
    uint64_t total_n = 0, total_sampled = 0;
    std::vector<uint64_t> rb(G), sb(G, 2 * (uint64_t)n), so(G, 0), ro(G);
    for (uint32_t p = 0; p < G; ++p) {
        rb[p] = 2 * peer[2 * p];
        total_n += peer[2 * p];
        total_sampled += peer[2 * p + 1];
    }
    uint64_t acc = 0;
    for (uint32_t p = 0; p < G; ++p) { ro[p] = acc; acc += rb[p]; }
    std::vector<uint64_t> cand(2 * std::max<size_t>(n, 1)), all(2 * std::max<uint64_t>(total_n, 1));
    for (size_t i = 0; i < n; ++i) { cand[2 * i] = key[i]; cand[2 * i + 1] = count[i]; }
    R_OK(hipMemcpyAsync(ds, cand.data(), n * 16, hipMemcpyHostToDevice, s));
    // every peer gets the same block: send offsets all 0
    R_RC(a2av_at(r, ds, so.data(), sb.data(), dr, ro.data(), rb.data(), 8, s));
    R_OK(hipMemcpyAsync(all.data(), dr, total_n * 16, hipMemcpyDeviceToHost, s));
    R_OK(hipStreamSynchronize(s));
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
    const int rc = rl_set_owner_directory(r->e, dk.size(), dk.data(), dov.data());
    if (rc == RL_OK && placed) *placed = (uint32_t)dk.size();
    return rc;
}
