// rl_engine.cpp — host runtime behind include/rl_engine.h.
//
// Owns, per GPU: the HBM state table (one region array per limiter), the
// limiter table, the batch scratch and one HIP stream. A batch is a fixed chain
// of kernel launches on that stream (see csrc/rl_*.hip); nothing in the chain
// synchronises with the host, so the device entry point is fully asynchronous.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <utility>
#include <vector>

#include "../../include/rl_engine.h"
#include "rl_launch.hpp"

using namespace rl;

namespace {

// Stage timing: events bracket every kernel of a batch; a ring of per-batch event
// sets is averaged when rl_stage_times is called (no host sync inside a batch).
constexpr int kMarks = 12;   // marks 0..11 on the engine stream
constexpr int kStages = 11;
// (two-pass batches: "group" is k_group; "scan1" / "scatter1" are empty since round 6, when
// k_group replaced the global second pass)
const char* kStageNames[kStages] = {"upsweep0", "scan0", "scatter0", "group", "scan1",
                                    "scatter1", "region_offsets", "region", "unpermute", "total",
                                    "hot_fill"};
const int kStagePairs[kStages][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {5, 6},
                                     {6, 7}, {7, 8}, {8, 9}, {0, 9}, {10, 11}};
constexpr int kEvRing = 64;

struct HostLimiter {
    rl_limiter_config cfg;
    DevLimiter dev;
    void* table = nullptr;
    size_t table_bytes = 0;
    void* cache_table = nullptr;            // SW local cache: u64 per slot
};

inline int ceil_log2(uint64_t x) {
    int b = 0;
    while ((1ULL << b) < x) ++b;
    return b;
}

}  // namespace

// Per-batch scratch: the partition's records/positions, the [bin][tile] counts, the packed
// results and the batch control block. Two sets, so that with RL_OPT_PIPELINE the partition
// of batch k+1 (its own stream) can run while batch k's region stage still reads its set.
struct BatchScratch {
    size_t cap_n = 0;
    bool cap_wide = false;
    void* rec0 = nullptr;
    void* rec1 = nullptr;
    uint32_t* pos0 = nullptr;
    uint32_t* pos1 = nullptr;
    uint16_t* digit = nullptr;              // routing: pass-0 digit per request
    void* res = nullptr;
    int64_t* ext = nullptr;                 // escaped remainders (kResEscape), like res
    double* tok = nullptr;
    uint32_t* counts = nullptr;             // [bins][tiles]
    size_t counts_cap = 0;
    uint32_t* bin_total = nullptr;          // [2^kMaxDigitBits]
    uint32_t* bin_base = nullptr;           // [2^kMaxDigitBits]
    uint32_t* region_count = nullptr;       // [P padded]
    uint32_t* region_start = nullptr;
    size_t region_cap = 0;
    uint32_t* gtile = nullptr;              // k_group*: tile_base, tile_bin, per-tile counts
    size_t gtile_cap = 0;
    uint32_t* seg = nullptr;                // segmented pass 0: seg_adj, seg_start, seg_cnt
    size_t seg_cap = 0;
    BatchCtl* d_ctl = nullptr;
    hipEvent_t parted = nullptr;            // pipeline: partition done (partition stream)
    hipEvent_t freed = nullptr;             // pipeline: last reader of the set done (engine stream)
    bool used = false;                      // `freed` has been recorded
};

struct rl_engine {
    int device = 0;
    rl_opts opts{};
    int shard_bits = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;                          // one batch in flight per engine handle

    std::vector<HostLimiter> lims;
    uint32_t n_regions = 0;
    DevLimiter* d_lims = nullptr;
    uint8_t* d_region_lim = nullptr;
    size_t region_lim_cap = 0;

    // per-batch scratch (sized for opts.max_batch); sc[0] unless pipelined
    BatchScratch sc[2];
    int next_set = 0;
    bool pipeline = false;                  // RL_OPT_PIPELINE
    hipStream_t pstream = nullptr;          // partition stream (pipeline)
    hipEvent_t in_ev = nullptr;             // pipeline: inputs ready on e->stream
    hipStream_t hstream = nullptr;          // hot chains beside the normal regions
    hipEvent_t hot_ev[2] = {};              // fork, join of hstream
    // hot regions
    uint32_t* hot_list = nullptr;           // [kHotListWords]: list, k_hot_select's meta, totals
    HotInfo* hot_info = nullptr;            // [kHotMax]
    uint64_t* hot_summ = nullptr;           // [hot_summ_cap][8]
    size_t hot_summ_cap = 0, hot_summ_l1 = 0;
    uint2* walk_tab = nullptr;              // [kWalkTabEntries] allow-walk tables (hot chains)
    bool walk = true;                       // rl_tune("walk"): allow walks in the hot chains
    uint32_t walk_hint = 0;                 // listed regions that wanted a walk in the last batch
                                            // seen complete (walk_tab is allocated once it is > 0)
    uint32_t walk_min = kWalkMinAllows;     // rl_tune("walk_min"): fewest expected allows walked
    bool chain_split = true;                // rl_tune("chain_split"): two-wave hot chains
    uint32_t* hot_mark = nullptr;           // [hot_mark_cap] epoch marks per bin
    size_t hot_mark_cap = 0;
    uint32_t epoch = 0;
    uint32_t hot_threshold = 16384;         // rl_tune("hot_threshold"); 0 disables
    bool hot_thr_auto = true;               // until set: max(hot_threshold, n / 4096) per batch
    // Hot-region routing (two-pass batches): the previous batch's hot regions get pass-0 bins
    // of their own and skip pass 1. route_list holds region ids (kNone = unused); it is built
    // on device at the end of each batch's hot preparation and cleared when region ids change.
    bool route = true;                      // rl_tune("route")
    bool region_order = true;               // rl_tune("region_order"): largest regions dispatched first
    uint32_t order_prefix = 4096;           // rl_tune("order_prefix"): ... after this many of the smallest
    uint32_t tile_items = 0;                // rl_tune("tile_items"): partition tile rounds (0: auto)
    uint32_t segments = 1;                  // rl_tune("segments"): two-pass batches' pass-0 output
                                            // in that many tile segments ([segment][bin])
    uint32_t group_bits = 12;               // rl_tune("group_bits"): two-pass batches' pass-0
                                            // high digit (2^12 bins + the routed ones)
    uint32_t* order = nullptr;              // [order_cap + 1]
    size_t order_cap = 0;
    uint32_t* order_meta = nullptr;         // [kOrderMeta]
    // One table per scratch set: with RL_OPT_PIPELINE batch k+1's partition runs while batch
    // k's region stage still reads its routed ranges and writes the next table, so batch k uses
    // set k % 2's table, written by batch k - 2 (set 0 only without the option: batch k - 1).
    uint32_t* route_list = nullptr;         // [2][kRouteWords] region ids (kNone = empty), dense indices
    uint32_t* route_start = nullptr;        // [2][kRouteSlots] this batch's routed bins
    uint32_t* route_cnt = nullptr;          // [2][kRouteSlots]
    uint32_t solo_threshold = 4096;         // rl_tune("solo_threshold"): records per cache-on SW
                                            // region for the single-key allow-run pass (0: off)
    uint32_t* solo_list = nullptr;          // [kSoloMax + 1]: the listed regions, then their count
    uint32_t sparse_max = 96;               // rl_tune("sparse_max"): records per region up to
                                            // which a region probes single buckets; 0 = never
    uint64_t* dbg = nullptr;                // rl_tune("debug_regions"): per-bin stamps
    size_t dbg_cap = 0;
    bool debug_regions = false;
    unsigned long long* d_stats = nullptr;  // [kStatSlots][kStWords] sharded counters (zeroed)
    BatchCtl* h_ctl = nullptr;              // pinned copy of the last batch's ctl

    // host-API staging (device copies of caller buffers)
    size_t stage_cap = 0;
    uint64_t* s_key = nullptr;
    int32_t* s_permits = nullptr;
    int64_t* s_now = nullptr;
    uint16_t* s_lim = nullptr;
    uint8_t* s_op = nullptr;
    uint8_t* s_allowed = nullptr;
    int64_t* s_remaining = nullptr;
    double* s_tokens = nullptr;
    std::vector<std::pair<void*, size_t>> pinned;   // caller buffers registered by rl_pin_host

    // routing scratch
    uint32_t* route_scratch = nullptr;
    size_t route_cap = 0;
    uint32_t* route_counts = nullptr;
    DirSlot* d_dir = nullptr;               // hot-key owner directory (nullptr: hash owners)
    std::vector<DirSlot> h_dir;             // host copy (rl_owner_of_engine)

    hipEvent_t ev[kEvRing][kMarks] = {};
    int ring_used = 0;                      // batches recorded since the last query
    int ring_next = 0;
    bool timing = false;
    bool last_wide = false;
    bool pending_status = false;
    bool enqueued = false;                  // the last engine call enqueued a batch (d_ctl is its)
    uint32_t hot_hint = 0xFFFFFFFFu;        // hot regions of the last batch seen complete
    int last_status = RL_OK;
    uint64_t last_n = 0;
    uint32_t ablate = 0;                    // rl_tune("ablate"), measurement only
    uint32_t up_per_cu = 0, sc_per_cu = 0, un_per_cu = 0;   // rl_tune("*_per_cu"), 0 = default
    uint32_t sc_split = 1;                  // rl_tune("scatter_split"): k_scatter_split
    uint32_t un_split = 2;                  // rl_tune("unpermute_split"): k_unpermute_split
    uint32_t mid_xcd = 0;                   // rl_tune("mid_xcd"): k_unpermute_mid blocks XCD-aware (measured slower)
                                            // 0 off, 1 on, 2 two-pass batches (measured faster there)
    bool force_wide = false;                // rl_tune("wide_records"): 32-B records (any time span)
    bool auto_grow = true;                  // !RL_OPT_FIXED_CAPACITY
    uint32_t inject_fail = 0;               // rl_tune("fail_batches"): tests of callers' error paths
    uint64_t grows = 0;                     // region-count doublings done (rl_batch_stats)
};

#define HIP_OK(x)                                                      \
    do {                                                               \
        hipError_t _e = (x);                                           \
        if (_e != hipSuccess) {                                        \
            std::fprintf(stderr, "rl_engine: %s failed: %s (%s:%d)\n", #x, \
                         hipGetErrorString(_e), __FILE__, __LINE__);   \
            return RL_E_DEVICE;                                        \
        }                                                              \
    } while (0)

static void ensure_events(rl_engine* e) {
    if (e->ev[0][0]) return;
    for (int r = 0; r < kEvRing; ++r)
        for (int i = 0; i < kMarks; ++i) (void)hipEventCreate(&e->ev[r][i]);
}

static void dfree(void*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}
template <class T>
static void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

static int dalloc(void** p, size_t bytes) {
    if (hipMalloc(p, bytes ? bytes : 16) != hipSuccess) {
        *p = nullptr;
        return RL_E_NOMEM;
    }
    return RL_OK;
}
template <class T>
static int dalloc(T** p, size_t count) {
    return dalloc((void**)p, count * sizeof(T));
}

extern "C" int rl_abi_version(void) { return RL_ABI_VERSION; }

extern "C" const char* rl_strerror(int s) {
    switch (s) {
        case RL_OK: return "ok";
        case RL_E_INVALID_ARG: return "invalid argument";
        case RL_E_INVALID_REQUEST: return "invalid request(s) in batch (permits <= 0 or unknown limiter)";
        case RL_E_CAPACITY: return "state-table region full";
        case RL_E_DEVICE: return "HIP device error";
        case RL_E_NOMEM: return "out of memory";
        case RL_E_TOO_LARGE: return "batch larger than max_batch";
        case RL_E_LIMITERS: return "too many limiters";
        case RL_E_INTERNAL: return "internal error (engine logic)";
        default: return "unknown status";
    }
}

extern "C" uint32_t rl_owner_of(uint64_t key_hash, uint16_t, uint32_t shard_count) {
    if (shard_count <= 1) return 0;
    const int s = ceil_log2(shard_count);
    return (uint32_t)(mix64(key_hash) >> (64 - s));
}

extern "C" int rl_create(const rl_opts* opts, rl_engine** out) {
    if (!out) return RL_E_INVALID_ARG;
    *out = nullptr;
    rl_opts o{};
    if (opts) o = *opts;
    if (o.max_batch == 0) o.max_batch = 1u << 22;
    if (o.max_batch > 0xFFFFFFF0ULL) return RL_E_INVALID_ARG;   // u32 positions
    if (o.default_capacity == 0) o.default_capacity = 1u << 20;
    if (o.shard_count == 0) o.shard_count = 1;
    if ((o.shard_count & (o.shard_count - 1)) != 0 || o.shard_count > 64) return RL_E_INVALID_ARG;
    if (o.shard_index >= o.shard_count) return RL_E_INVALID_ARG;
    if (o.max_skew_ms < 0) return RL_E_INVALID_ARG;
    rl_engine* e = new (std::nothrow) rl_engine();
    if (!e) return RL_E_NOMEM;
    e->opts = o;
    e->shard_bits = ceil_log2(o.shard_count);
    if (o.device >= 0) {
        if (hipSetDevice(o.device) != hipSuccess) { delete e; return RL_E_DEVICE; }
        e->device = o.device;
    } else {
        (void)hipGetDevice(&e->device);
    }
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        rl_destroy(e);
        return RL_E_DEVICE;
    }
    // The hot chains' stream has the device's highest priority: their workgroups are a few
    // long sequential critical paths launched beside ~10^5-10^6 short normal-region waves,
    // and at equal priority the dispatcher interleaved the two launches, so some chains
    // only started once normal regions had drained (sw_zipf: up to 2.5 ms late).
    int prio_least = 0, prio_greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) prio_greatest = 0;
    if (hipStreamCreateWithPriority(&e->hstream, hipStreamNonBlocking, prio_greatest) != hipSuccess ||
        hipEventCreateWithFlags(&e->hot_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->hot_ev[1], hipEventDisableTiming) != hipSuccess) {
        rl_destroy(e);
        return RL_E_DEVICE;
    }
    e->timing = (o.flags & RL_OPT_STAGE_TIMING) != 0;
    if (e->timing) ensure_events(e);
    e->pipeline = (o.flags & RL_OPT_PIPELINE) != 0;
    e->auto_grow = (o.flags & RL_OPT_FIXED_CAPACITY) == 0;
    if (e->pipeline && hipStreamCreateWithFlags(&e->pstream, hipStreamNonBlocking) != hipSuccess) {
        rl_destroy(e);
        return RL_E_DEVICE;
    }
    int rc = RL_OK;
    if (e->pipeline && hipEventCreateWithFlags(&e->in_ev, hipEventDisableTiming) != hipSuccess)
        rc = RL_E_DEVICE;
    for (int k = 0; k < (e->pipeline ? 2 : 1); ++k) {
        BatchScratch& B = e->sc[k];
        if (rc == RL_OK) rc = dalloc(&B.d_ctl, 1);
        if (rc == RL_OK) rc = dalloc(&B.bin_total, 1u << kMaxDigitBits);
        if (rc == RL_OK) rc = dalloc(&B.bin_base, 1u << kMaxDigitBits);
        if (rc == RL_OK && e->pipeline &&
            (hipEventCreateWithFlags(&B.parted, hipEventDisableTiming) != hipSuccess ||
             hipEventCreateWithFlags(&B.freed, hipEventDisableTiming) != hipSuccess))
            rc = RL_E_DEVICE;
    }
    if (rc == RL_OK) rc = dalloc(&e->d_stats, (size_t)kStatSlots * kStWords);
    if (rc == RL_OK && hipMemset(e->d_stats, 0, (size_t)kStatSlots * kStWords * 8) != hipSuccess)
        rc = RL_E_DEVICE;
    if (rc == RL_OK && hipHostMalloc((void**)&e->h_ctl, sizeof(BatchCtl)) != hipSuccess) rc = RL_E_NOMEM;
    if (rc == RL_OK) rc = dalloc(&e->d_lims, RL_MAX_LIMITERS);
    if (rc == RL_OK) rc = dalloc(&e->hot_list, kHotListWords);
    if (rc == RL_OK) rc = dalloc(&e->hot_info, kHotMax);
    if (rc == RL_OK) rc = dalloc(&e->route_list, 2 * kRouteWords);
    if (rc == RL_OK) rc = dalloc(&e->route_start, 2 * kRouteSlots);
    if (rc == RL_OK) rc = dalloc(&e->route_cnt, 2 * kRouteSlots);
    if (rc == RL_OK) rc = dalloc(&e->order_meta, kOrderMeta);
    if (rc == RL_OK) rc = dalloc(&e->solo_list, kSoloMax + 1);
    if (rc == RL_OK && hipMemset(e->route_list, 0xFF, 2 * kRouteWords * sizeof(uint32_t)) != hipSuccess)
        rc = RL_E_DEVICE;
    if (rc != RL_OK) { rl_destroy(e); return rc; }
    std::memset(e->h_ctl, 0, sizeof(BatchCtl));
    *out = e;
    return RL_OK;
}

extern "C" void rl_destroy(rl_engine* e) {
    if (!e) return;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->pstream) (void)hipStreamSynchronize(e->pstream);
    if (e->hstream) (void)hipStreamSynchronize(e->hstream);
    for (auto& l : e->lims) { dfree(l.table); dfree(l.cache_table); }
    dfree(e->d_lims); dfree(e->d_region_lim);
    for (BatchScratch& B : e->sc) {
        dfree(B.rec0); dfree(B.rec1); dfree(B.pos0); dfree(B.pos1); dfree(B.res); dfree(B.tok);
        dfree(B.ext); dfree(B.digit);
        dfree(B.counts); dfree(B.bin_total); dfree(B.bin_base);
        dfree(B.region_count); dfree(B.region_start); dfree(B.gtile); dfree(B.seg);
        dfree(B.d_ctl);
        if (B.parted) (void)hipEventDestroy(B.parted);
        if (B.freed) (void)hipEventDestroy(B.freed);
    }
    dfree(e->hot_list); dfree(e->hot_mark); dfree(e->dbg); dfree(e->hot_info); dfree(e->hot_summ);
    dfree(e->walk_tab);
    dfree(e->route_list); dfree(e->route_start); dfree(e->route_cnt);
    dfree(e->order); dfree(e->order_meta); dfree(e->solo_list);
    dfree(e->d_stats);
    dfree(e->s_key); dfree(e->s_permits); dfree(e->s_now); dfree(e->s_lim); dfree(e->s_op);
    dfree(e->s_allowed); dfree(e->s_remaining); dfree(e->s_tokens);
    dfree(e->route_scratch); dfree(e->route_counts); dfree(e->d_dir);
    if (e->h_ctl) (void)hipHostFree(e->h_ctl);
    for (auto& pb : e->pinned) (void)hipHostUnregister(pb.first);
    for (int r = 0; r < kEvRing; ++r)
        for (int i = 0; i < kMarks; ++i) if (e->ev[r][i]) (void)hipEventDestroy(e->ev[r][i]);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->pstream) (void)hipStreamDestroy(e->pstream);
    if (e->in_ev) (void)hipEventDestroy(e->in_ev);
    if (e->hstream) (void)hipStreamDestroy(e->hstream);
    for (hipEvent_t ev : e->hot_ev) if (ev) (void)hipEventDestroy(ev);
    delete e;
}

static int upload_limiters(rl_engine* e) {
    std::vector<DevLimiter> dv;
    for (auto& l : e->lims) dv.push_back(l.dev);
    HIP_OK(hipMemcpy(e->d_lims, dv.data(), dv.size() * sizeof(DevLimiter), hipMemcpyHostToDevice));
    std::vector<uint8_t> map(e->n_regions);
    for (size_t li = 0; li < e->lims.size(); ++li) {
        const auto& d = e->lims[li].dev;
        std::fill(map.begin() + d.region_base, map.begin() + d.region_base + (1u << d.region_bits),
                  (uint8_t)li);
    }
    if (e->region_lim_cap < map.size()) {
        dfree(e->d_region_lim);
        if (dalloc(&e->d_region_lim, map.size()) != RL_OK) return RL_E_NOMEM;
        e->region_lim_cap = map.size();
    }
    HIP_OK(hipMemcpy(e->d_region_lim, map.data(), map.size(), hipMemcpyHostToDevice));
    return RL_OK;
}

// kLfPctMul / kLfPctFma (rl_device.hpp): checked for every remainder of windows up to 2^22 ms.
static uint32_t pct_flags(int64_t w, double inv) {
    if (w > (int64_t(1) << 22)) return 0;
    const double dw = (double)w;
    bool mul = true, fma = true;
    for (int64_t r = 1; r < w && (mul || fma); ++r) {
        const double dr = (double)r, exact = dr / dw, q = dr * inv;
        if (q != exact) mul = false;
        if (std::fma(std::fma(-q, dw, dr), inv, q) != exact) fma = false;
    }
    return mul ? kLfPctMul : fma ? kLfPctFma : 0u;
}

extern "C" int rl_add_limiter_ex(rl_engine* e, const rl_limiter_config* c, uint16_t* id) {
    if (!e || !c) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    // RateLimitConfig.validate() (RateLimitConfig.java:46-56)
    if (c->max_permits <= 0 || c->window_ms <= 0 || !(c->refill_per_s >= 0.0)) return RL_E_INVALID_ARG;
    if ((c->flags & ~RL_LIM_LOCAL_CACHE) != 0 || c->local_cache_ttl_ms < 0) return RL_E_INVALID_ARG;
    if (c->algo == RL_ALGO_TOKEN_BUCKET && !(c->refill_per_s > 0.0)) return RL_E_INVALID_ARG;  // TB ctor :77-79
    if (c->algo != RL_ALGO_TOKEN_BUCKET && c->algo != RL_ALGO_SLIDING_WINDOW) return RL_E_INVALID_ARG;
    if (c->window_ms > RL_MAX_WINDOW_MS) return RL_E_INVALID_ARG;
    if (c->algo == RL_ALGO_SLIDING_WINDOW && c->max_permits > RL_SW_MAX_PERMITS_LIMIT) return RL_E_INVALID_ARG;
    if (c->algo == RL_ALGO_TOKEN_BUCKET && c->max_permits > RL_TB_MAX_PERMITS_LIMIT) return RL_E_INVALID_ARG;
    if (e->lims.size() >= RL_MAX_LIMITERS) return RL_E_LIMITERS;
    (void)hipSetDevice(e->device);
    HostLimiter h;
    h.cfg = *c;
    uint64_t cap = c->capacity ? c->capacity : e->opts.default_capacity;
    uint64_t per_shard = (cap + e->opts.shard_count - 1) / e->opts.shard_count;
    uint64_t slots = std::max<uint64_t>(per_shard * 2, kRegionSlots);   // load <= 0.5
    uint64_t regions = (slots + kRegionSlots - 1) / kRegionSlots;
    int k = std::max(ceil_log2(regions), kBinShift);     // whole bins of kRegionsPerBin regions
    if (k + e->shard_bits > 40) return RL_E_INVALID_ARG;
    if ((uint64_t)e->n_regions + (1ULL << k) > (1ULL << 24)) return RL_E_LIMITERS;
    DevLimiter& d = h.dev;
    std::memset(&d, 0, sizeof(d));
    d.algo = c->algo;
    d.region_bits = k;
    d.region_base = e->n_regions;
    d.max_permits = c->max_permits;
    d.window_ms = c->window_ms;
    d.ttl_ms = c->algo == RL_ALGO_TOKEN_BUCKET ? c->window_ms * 2 : c->window_ms;
    d.rate_per_ms = c->refill_per_s / 1000.0;        // TokenBucketRateLimiter.java:85
    d.inv_rate = d.rate_per_ms > 0.0 ? 1.0 / d.rate_per_ms : 0.0;
    d.inv_window = 1.0 / (double)c->window_ms;
    d.lflags = pct_flags(c->window_ms, d.inv_window);
    d.capacity = (double)c->max_permits;
    h.table_bytes = (size_t)(1ULL << k) * kRegionSlots * sizeof(Slot);
    if (dalloc(&h.table, h.table_bytes) != RL_OK) return RL_E_NOMEM;
    if (hipMemset(h.table, 0, h.table_bytes) != hipSuccess) { dfree(h.table); return RL_E_DEVICE; }
    d.table = (uint64_t)(uintptr_t)h.table;
    if (c->algo == RL_ALGO_SLIDING_WINDOW && (c->flags & RL_LIM_LOCAL_CACHE) && c->local_cache_ttl_ms > 0) {
        const size_t xb = (size_t)(1ULL << k) * kRegionSlots * sizeof(uint64_t);
        if (dalloc(&h.cache_table, xb) != RL_OK) { dfree(h.table); return RL_E_NOMEM; }
        if (hipMemset(h.cache_table, 0, xb) != hipSuccess) { dfree(h.table); dfree(h.cache_table); return RL_E_DEVICE; }
        d.cache_table = (uint64_t)(uintptr_t)h.cache_table;
        d.cache_ttl_ms = c->local_cache_ttl_ms;
    }
    e->lims.push_back(h);
    e->n_regions += 1u << k;
    int rc = upload_limiters(e);
    if (rc != RL_OK) return rc;
    if (id) *id = (uint16_t)(e->lims.size() - 1);
    return RL_OK;
}

extern "C" int rl_add_limiter(rl_engine* e, int algo, int64_t max_permits, int64_t window_ms,
                              double refill_per_s, uint16_t* id) {
    rl_limiter_config c{};
    c.algo = algo;
    c.max_permits = max_permits;
    c.window_ms = window_ms;
    c.refill_per_s = refill_per_s;
    c.capacity = 0;                                  // local cache off: the parity-mode default
    return rl_add_limiter_ex(e, &c, id);
}

// Double limiter li's region count (k -> k + 1 region bits): new table, every old region
// split in two by k_grow, old table freed, region ids of the later limiters shifted.
// Synchronous; nothing may be in flight on the engine's streams.
static int grow_once(rl_engine* e, size_t li) {
    HostLimiter& h = e->lims[li];
    DevLimiter& d = h.dev;
    const int k = d.region_bits;
    if (k + 1 + e->shard_bits > 40 || (uint64_t)e->n_regions + (1ULL << k) > (1ULL << 24))
        return RL_E_LIMITERS;
    HIP_OK(hipStreamSynchronize(e->stream));
    if (e->pstream) HIP_OK(hipStreamSynchronize(e->pstream));
    const size_t nb = h.table_bytes * 2;
    void* nt = nullptr;
    void* nx = nullptr;
    if (dalloc(&nt, nb) != RL_OK) return RL_E_NOMEM;
    if (h.cache_table && dalloc(&nx, nb / sizeof(Slot) * sizeof(uint64_t)) != RL_OK) {
        dfree(nt);
        return RL_E_NOMEM;
    }
    if (launch_grow((const Slot*)h.table, (const uint64_t*)h.cache_table, (Slot*)nt, (uint64_t*)nx,
                    1ULL << k, e->shard_bits, k + 1, d.algo, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess) {
        dfree(nt); dfree(nx);
        return RL_E_DEVICE;
    }
    dfree(h.table); dfree(h.cache_table);
    h.table = nt; h.cache_table = nx; h.table_bytes = nb;
    d.table = (uint64_t)(uintptr_t)nt;
    d.cache_table = (uint64_t)(uintptr_t)nx;
    d.region_bits = k + 1;
    uint32_t base = 0;
    for (auto& l : e->lims) { l.dev.region_base = base; base += 1u << l.dev.region_bits; }
    e->n_regions = base;
    ++e->grows;
    // region ids changed: the next batch routes nothing (its hot preparation lists anew)
    HIP_OK(hipMemset(e->route_list, 0xFF, 2 * kRouteWords * sizeof(uint32_t)));
    return upload_limiters(e);
}

static int grow_to(rl_engine* e, size_t li, uint64_t min_keys) {
    const uint64_t per_shard = (min_keys + e->opts.shard_count - 1) / e->opts.shard_count;
    while ((e->lims[li].table_bytes / sizeof(Slot)) < per_shard * 2) {   // load <= 0.5
        const int rc = grow_once(e, li);
        if (rc != RL_OK) return rc;
    }
    return RL_OK;
}

extern "C" int rl_grow_limiter(rl_engine* e, uint16_t limiter, uint64_t min_keys) {
    if (!e) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    if (limiter >= e->lims.size()) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    return grow_to(e, limiter, min_keys);
}

extern "C" int rl_limiter_slots(rl_engine* e, uint16_t limiter, uint64_t* slots) {
    if (!e || !slots) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    if (limiter >= e->lims.size()) return RL_E_INVALID_ARG;
    *slots = e->lims[limiter].table_bytes / sizeof(Slot);
    return RL_OK;
}

static int ensure_scratch(rl_engine* e, BatchScratch& B, size_t n, bool wide, uint32_t bins, uint32_t n_tiles) {
    if (n > B.cap_n || (wide && !B.cap_wide)) {
        // sized for this batch (+1/8 headroom), not max_batch: a router's engine accepts up
        // to its receive capacity but usually sees about its per-rank share
        size_t cap = std::max<size_t>(n, std::min<size_t>(e->opts.max_batch,
                                                          std::max<size_t>(n + n / 8, 1u << 20)));
        const size_t rb = wide ? sizeof(RecW) : sizeof(RecC);
        const size_t padn = cap + kTileThreads;   // kernels write inactive lanes past n
        dfree(B.rec0); dfree(B.rec1); dfree(B.pos0); dfree(B.pos1); dfree(B.res); dfree(B.tok);
        dfree(B.ext); dfree(B.digit);
        int rc = dalloc(&B.rec0, padn * rb);
        if (rc == RL_OK) rc = dalloc(&B.digit, padn);
        if (rc == RL_OK) rc = dalloc(&B.rec1, padn * rb);
        if (rc == RL_OK) rc = dalloc(&B.pos0, padn);
        if (rc == RL_OK) rc = dalloc(&B.pos1, padn);
        if (rc == RL_OK) rc = dalloc(&B.res, padn * sizeof(uint64_t));
        if (rc == RL_OK) rc = dalloc(&B.tok, padn);
        if (rc == RL_OK) rc = dalloc(&B.ext, padn);
        if (rc != RL_OK) { B.cap_n = 0; return rc; }
        B.cap_n = cap;
        B.cap_wide = wide;
    }
    const size_t need_counts = (size_t)bins * n_tiles;
    if (need_counts > B.counts_cap) {
        dfree(B.counts);
        size_t c = std::max(need_counts, (size_t)(1u << kMaxDigitBits) *
                                              ((std::max<size_t>(n, B.cap_n) + kTile - 1) / kTile));
        if (dalloc(&B.counts, c) != RL_OK) return RL_E_NOMEM;
        B.counts_cap = c;
    }
    return RL_OK;
}

// rstart / rend per region for two-pass partitions (k_group).
static int ensure_regions(BatchScratch& B, size_t bins) {
    if (bins <= B.region_cap) return RL_OK;
    dfree(B.region_count); dfree(B.region_start);
    int rc = dalloc(&B.region_count, bins);
    if (rc == RL_OK) rc = dalloc(&B.region_start, bins);
    if (rc != RL_OK) { B.region_cap = 0; return rc; }
    B.region_cap = bins;
    return RL_OK;
}

// chunk summaries [l1] then group summaries [l1 / 64 + kHotMax + 1], 64 B each (two keys)
static int ensure_hot_summ(rl_engine* e, size_t n) {
    const size_t l1 = n / kHotChunk + kHotMax + 1;
    const size_t need = l1 + l1 / 64 + kHotMax + 1;
    if (need <= e->hot_summ_cap) return RL_OK;
    dfree(e->hot_summ);
    if (dalloc(&e->hot_summ, need * 8) != RL_OK) { e->hot_summ_cap = 0; return RL_E_NOMEM; }
    e->hot_summ_cap = need;
    e->hot_summ_l1 = l1;
    return RL_OK;
}

static int ensure_hot_mark(rl_engine* e, size_t bins) {
    if (bins <= e->hot_mark_cap) return RL_OK;
    dfree(e->hot_mark);
    if (dalloc(&e->hot_mark, bins) != RL_OK) { e->hot_mark_cap = 0; return RL_E_NOMEM; }
    HIP_OK(hipMemset(e->hot_mark, 0, bins * sizeof(uint32_t)));
    e->hot_mark_cap = bins;
    e->epoch = 0;
    return RL_OK;
}

static inline void mark_on(rl_engine* e, hipStream_t st, int i) {
    if (e->timing) (void)hipEventRecord(e->ev[e->ring_next][i], st);
}
static inline void mark(rl_engine* e, int i) { mark_on(e, e->stream, i); }

// The pipeline on device buffers, enqueued on e->stream. Returns an immediate status
// (argument/launch errors); the data-dependent status is read back by rl_last_status.
static int run_batch_device(rl_engine* e, size_t n, const uint64_t* key, const int32_t* permits,
                            const int64_t* now_ns, const uint16_t* limiter, const uint8_t* op,
                            uint8_t* allowed, int64_t* remaining, double* tokens_after,
                            bool overlap = false) {
    if (n > e->opts.max_batch) return RL_E_TOO_LARGE;
    e->last_n = n;
    e->pending_status = false;
    e->enqueued = false;
    e->last_status = RL_OK;
    if (n == 0) return RL_OK;
    if (!key || !permits || !now_ns || !allowed || !remaining) return RL_E_INVALID_ARG;
    if (e->inject_fail) { --e->inject_fail; return RL_E_DEVICE; }   // nothing enqueued
    hipStream_t s = e->stream;
    if (e->lims.empty()) {
        HIP_OK(launch_fill_invalid(allowed, remaining, tokens_after, (uint32_t)n, s));
        e->last_status = RL_E_INVALID_REQUEST;
        return RL_OK;
    }
    bool wide = e->force_wide;
    int64_t max_any = 0;
    for (auto& l : e->lims) {
        wide |= l.cfg.max_permits > kCompactMaxPermits;
        max_any = std::max<int64_t>(max_any, l.cfg.max_permits);
    }
    const int res_bytes = res_bytes_for(max_any, wide);
    // partition tiles of 128K requests for large batches (half the [bin][tile] counts to write
    // and scan: sw_zipf's 2^28-request batches, scan0 0.16 -> 0.06 ms, upsweep0 0.89 -> 0.75 ms),
    // 64K below (tb_uniform's 2^26 needs the 1024 tiles to keep every CU busy; the unpermute keeps
    // 64K tiles: run_r06o.sh)
    const uint32_t titems = e->tile_items ? e->tile_items
                                          : (n >= ((size_t)3 << 26) ? 2u * kTileItems : (uint32_t)kTileItems);
    const size_t tile_n = (size_t)titems * kTileThreads;
    const uint32_t nt = (uint32_t)((n + tile_n - 1) / tile_n);
    const uint32_t nt_un = (uint32_t)((n + kTile - 1) / kTile);
    bool cache = false;
    for (auto& l : e->lims) cache |= l.dev.cache_ttl_ms > 0;
    const uint32_t n_bins = e->n_regions;            // one partition bin per region
    const int bitsP = std::max(1, ceil_log2(n_bins));
    const int passes = bitsP <= kMaxDigitBits ? 1 : 2;
    if (bitsP > 2 * kMaxDigitBits) return RL_E_LIMITERS;
    // Two passes: pass 0 partitions by the high dh bits of the region id (2^dh bins of 2^s0
    // consecutive regions), then k_group groups each bin by region locally (rl_partition.hip)
    const int dh = passes == 1 ? bitsP
                               : std::max(bitsP - kMaxDigitBits, std::min<int>((int)e->group_bits, kMaxDigitBits));
    const int s0 = bitsP - dh;
    // hot-region routing: pass 0 gets kRouteBins dense bins beyond the 2^dh high-digit ones. The
    // hot path is gated per limiter: regions of a limiter with the local cache are never
    // listed hot (k_hot_select), so they are never routed either; the other limiters keep it.
    const bool hot_on = e->hot_threshold > 0;
    const bool route = hot_on && e->route && passes == 2 &&
                       (1u << dh) + kRouteBins <= (1u << kMaxDigitBits);
    const uint32_t nb0 = route ? (1u << dh) + kRouteBins : 1u << dh;
    // segmented pass-0 output (two passes): n_segs runs of seg_tiles tiles
    const uint32_t seg_tiles = passes == 2 && e->segments > 1 ? (nt + e->segments - 1) / e->segments : nt;
    const uint32_t n_segs = (nt + seg_tiles - 1) / seg_tiles;
    // Scratch set and partition stream. With RL_OPT_PIPELINE the partition (stages 1-3)
    // runs on e->pstream into one of two scratch sets, so batch k+1's partition overlaps
    // batch k's region stage; the region stage and the unpermute stay on e->stream (state
    // updates in batch order). `overlap`: the caller guarantees the inputs are complete
    // (device call with no stream); otherwise the partition first waits for everything
    // enqueued on e->stream (inputs copied or produced there, or the caller's stream).
    const int set = e->pipeline ? e->next_set : 0;
    BatchScratch& B = e->sc[set];
    uint32_t* r_list = e->route_list + (size_t)set * kRouteWords;
    uint32_t* r_start = e->route_start + (size_t)set * kRouteSlots;
    uint32_t* r_cnt = e->route_cnt + (size_t)set * kRouteSlots;
    hipStream_t ps = e->pipeline ? e->pstream : s;
    const size_t need_counts = (size_t)nb0 * nt;
    if (e->pipeline && (n > B.cap_n || (wide && !B.cap_wide) || need_counts > B.counts_cap ||
                        (passes == 2 && n_bins > B.region_cap))) {
        // growing a set frees its old buffers: nothing may still be using them
        HIP_OK(hipStreamSynchronize(s));
        HIP_OK(hipStreamSynchronize(ps));
    }
    int rc = ensure_scratch(e, B, n, wide, nb0, nt);
    if (rc != RL_OK) return rc;
    if (passes == 2) {
        rc = ensure_regions(B, n_bins);
        if (rc != RL_OK) return rc;
    }
    if (e->pipeline) {
        if (B.used) HIP_OK(hipStreamWaitEvent(ps, B.freed, 0));    // the set's last batch is done
        if (!overlap) {
            HIP_OK(hipEventRecord(e->in_ev, s));
            HIP_OK(hipStreamWaitEvent(ps, e->in_ev, 0));
        }
    }
    const bool hot = hot_on;
    // records per region for the hot path: scaled with the batch by default (measured per
    // config: sw_zipf best at 65536 for 2^28 requests, zipf_1b at 32768 for 2^27)
    const uint32_t hot_thr = e->hot_thr_auto ? std::max<uint32_t>(e->hot_threshold, (uint32_t)(n >> 12))
                                             : e->hot_threshold;
    if (hot) {
        rc = ensure_hot_mark(e, n_bins);
        if (rc == RL_OK) rc = ensure_hot_summ(e, n);
        if (rc != RL_OK) return rc;
        // Allow-walk tables (512 MiB): only once a batch had a key dense enough to walk
        // (k_hot_scan's count; a workload that never walks, such as tb_uniform, holds none).
        // The walk is optional and decides identically: a failed allocation turns it off.
        if (e->walk && !e->walk_tab && e->walk_hint > 0 && dalloc(&e->walk_tab, kWalkTabEntries) != RL_OK) {
            std::fprintf(stderr, "rl_engine: no device memory for the allow-walk tables; walks off\n");
            e->walk = false;
        }
        if (++e->epoch == 0) {                       // marks hold epochs: restart after wrap
            HIP_OK(hipMemsetAsync(e->hot_mark, 0, e->hot_mark_cap * sizeof(uint32_t), s));
            e->epoch = 1;
        }
    }
    e->last_wide = wide;

    mark_on(e, ps, 0);
    PartArgs pa{};
    pa.key = key; pa.permits = permits; pa.now_ns = now_ns; pa.limiter = limiter; pa.op = op;
    pa.n = (uint32_t)n; pa.n_tiles = nt; pa.tile_items = titems; pa.n_lim = (uint32_t)e->lims.size();
    pa.shard_bits = e->shard_bits; pa.lims = e->d_lims; pa.ctl = B.d_ctl;
    pa.counts = B.counts; pa.bin_base = B.bin_base; pa.ablate = e->ablate;
    // (128K-request tiles: one upsweep tile per workgroup, 8 per CU: upsweep0 0.76 -> 0.73 ms on
    // sw_zipf over 6 runs, run_r06ab.sh)
    pa.up_per_cu = e->up_per_cu ? e->up_per_cu : (titems > (uint32_t)kTileItems ? 8u : 0u);
    pa.sc_per_cu = e->sc_per_cu; pa.sc_split = e->sc_split;
    // ---- pass 0 (the high digit: region >> s0) from the caller's arrays; routed hot
    // regions get bins 2^dh + slot and their records go straight to the final array (rec1)
    pa.digit_shift = s0; pa.digit_bits = route ? ceil_log2(nb0) : dh;
    pa.n_bins_pass = nb0;
    pa.rec_out = passes == 2 ? B.rec0 : B.rec1; pa.pos_out = B.pos0;
    if (route) {
        pa.route_list = r_list; pa.lo_bins = 1u << dh; pa.rec_out_route = B.rec1;
        pa.digit = B.digit;
    }
    HIP_OK(launch_upsweep(pa, true, wide, ps));
    mark_on(e, ps, 1);
    HIP_OK(launch_scan_rows(B.counts, B.counts, nb0, nt, B.bin_total, ps));
    HIP_OK(launch_scan_small(B.bin_total, B.bin_base, nb0, ps));
    if (n_segs > 1) {
        const size_t words = (size_t)3 * nb0 * n_segs;
        if (words > B.seg_cap) {
            if (e->pipeline) { HIP_OK(hipStreamSynchronize(s)); HIP_OK(hipStreamSynchronize(ps)); }
            dfree(B.seg);
            if (dalloc(&B.seg, words) != RL_OK) { B.seg_cap = 0; return RL_E_NOMEM; }
            B.seg_cap = words;
        }
        const size_t m = (size_t)nb0 * n_segs;
        HIP_OK(launch_seg_base(B.counts, B.bin_total, B.bin_base, nb0, 1u << dh, nt, seg_tiles, n_segs,
                               B.seg, B.seg + m, B.seg + 2 * m, ps));
        pa.seg_adj = B.seg; pa.n_segs = n_segs; pa.seg_tiles = seg_tiles;
    }
    mark_on(e, ps, 2);
    HIP_OK(launch_scatter(pa, true, wide, ps));
    if (route)
        HIP_OK(launch_route_ranges(r_list, B.bin_base, B.bin_total, 1u << dh, r_start, r_cnt,
                                   B.d_ctl, ps));
    mark_on(e, ps, 3);
    const void* rec_final = B.rec1;
    const uint32_t* rstart = B.bin_base;
    const uint32_t* rcount = B.bin_total;
    const uint32_t* rend = nullptr;
    if (passes == 2) {
        // ---- each normal pass-0 bin grouped by region in its own range of the final array
        // (stable: arrival order inside each region); the regions' bounds and the pass-0 ->
        // final positions (pos1) come with it. Routed records stay where pass 0 put them.
        GroupArgs ga{};
        ga.rec_in = B.rec0; ga.rec_out = B.rec1; ga.pos_out = B.pos1;
        ga.bin_base = B.bin_base; ga.bin_total = B.bin_total;
        ga.rstart = B.region_start; ga.rend = B.region_count;
        ga.lims = e->d_lims; ga.n_lim = (uint32_t)e->lims.size(); ga.shard_bits = e->shard_bits;
        ga.n_bins0 = 1u << dh; ga.sub_bits = (uint32_t)s0; ga.n_regions = n_bins;
        ga.tile_recs = group_tile_recs((uint32_t)s0);
        ga.pad = (uint32_t)n;
        ga.ablate = e->ablate;
        ga.max_tiles = (uint32_t)((n + ga.tile_recs - 1) / ga.tile_recs) + ga.n_bins0 * n_segs;
        const size_t words = (size_t)ga.n_bins0 + 1 + (size_t)ga.max_tiles * (1 + ((size_t)1 << s0)) +
                             (n_segs > 1 ? (size_t)2 * ga.max_tiles : 0);
        if (words > B.gtile_cap) {
            if (e->pipeline) { HIP_OK(hipStreamSynchronize(s)); HIP_OK(hipStreamSynchronize(ps)); }
            dfree(B.gtile);
            if (dalloc(&B.gtile, words) != RL_OK) { B.gtile_cap = 0; return RL_E_NOMEM; }
            B.gtile_cap = words;
        }
        ga.tile_base = B.gtile;
        ga.tile_bin = B.gtile + ga.n_bins0 + 1;
        ga.tcount = ga.tile_bin + ga.max_tiles;
        if (n_segs > 1) {
            const size_t m = (size_t)nb0 * n_segs;
            ga.seg_start = B.seg + m; ga.seg_cnt = B.seg + 2 * m; ga.n_segs = n_segs;
            ga.tile_beg = ga.tcount + (size_t)ga.max_tiles * ((size_t)1 << s0);
            ga.tile_end = ga.tile_beg + ga.max_tiles;
        }
        HIP_OK(launch_group(ga, wide, ps));
        rstart = B.region_start;
        rcount = nullptr;
        rend = B.region_count;
    }
    mark_on(e, ps, 4);
    mark_on(e, ps, 5);
    mark_on(e, ps, 6);
    if (e->pipeline) {
        HIP_OK(hipEventRecord(B.parted, ps));
        HIP_OK(hipStreamWaitEvent(s, B.parted, 0));
    }
    RegionArgs ra{};
    ra.rec = rec_final; ra.rstart = rstart; ra.rcount = rcount; ra.rend = rend;
    ra.region_lim = e->d_region_lim;
    ra.lims = e->d_lims; ra.res = B.res; ra.ext = B.ext; ra.tok = tokens_after ? B.tok : nullptr;
    ra.ctl = B.d_ctl; ra.n_regions = e->n_regions; ra.n_total = (uint32_t)n; ra.ablate = e->ablate;
    ra.shard_bits = e->shard_bits;
    ra.skew_ms = e->opts.max_skew_ms;
    ra.stats = e->d_stats;
    ra.cache = cache ? 1u : 0u;
    ra.sparse_max = e->sparse_max;
    // chain launch size: twice the hot count of the last batch the host saw complete (a
    // hint only: the chains loop over the hot list with the grid's stride), the whole
    // kHotMax before any batch has completed
    ra.chain_split = e->chain_split ? 1u : 0u;
    if (e->hot_hint != 0xFFFFFFFFu) {
        const uint32_t nh = e->hot_hint;
        ra.chain_grid = nh ? std::min<uint32_t>(kHotMax, std::max<uint32_t>(256u, 2u * nh)) : 64u;
    }
    if (e->debug_regions) {
        if (e->dbg_cap < (size_t)n_bins * kDbgWords) {
            dfree(e->dbg);
            if (dalloc(&e->dbg, (size_t)n_bins * kDbgWords) != RL_OK) { e->dbg_cap = 0; return RL_E_NOMEM; }
            e->dbg_cap = (size_t)n_bins * kDbgWords;
        }
        HIP_OK(hipMemsetAsync(e->dbg, 0, e->dbg_cap * sizeof(uint64_t), s));
        ra.dbg = e->dbg;
    }
    if (hot) {
        uint32_t* hot_count = e->hot_list + kHotMax;
        HIP_OK(hipMemsetAsync(hot_count, 0, kHotMetaWords * sizeof(uint32_t), s));
        if (route) HIP_OK(launch_hot_route_list(r_list, r_cnt, e->hot_list, hot_count, s));
        HIP_OK(launch_hot_select(rstart, rcount, rend, n_bins, hot_thr, e->hot_list,
                                 hot_count, e->hot_mark, e->epoch, cache ? e->d_lims : nullptr,
                                 e->d_region_lim, s));
        ra.hot_list = e->hot_list; ra.hot_count = hot_count; ra.hot_mark = e->hot_mark;
        ra.epoch = e->epoch;
        ra.hot_info = e->hot_info; ra.hot_summ = e->hot_summ;
        ra.hot_summ2 = e->hot_summ + e->hot_summ_l1 * 8; ra.hot_total = e->hot_list + kHotMax + kHotTotalOff;
        ra.route_list = r_list; ra.route_start = r_start; ra.route_cnt = r_cnt;
        ra.walk_tab = e->walk ? e->walk_tab : nullptr;
        ra.walk_min = e->walk_min;
        HIP_OK(launch_hot_prepare(ra, wide, s));          // dominant keys, chunk summaries
        HIP_OK(launch_chains(ra, wide, res_bytes, s, e->hstream, e->hot_ev[0]));
        // the chains' decided chunks filled on the side stream as soon as the chains end,
        // beside the normal regions' tail (sw_zipf: chains ~2.8 ms, normal drain ~3.3 ms)
        HIP_OK(launch_hot_fill(ra, wide, res_bytes, e->hstream));
    }
    if (e->region_order) {
        if (e->order_cap < n_bins) {
            dfree(e->order);
            if (dalloc(&e->order, (size_t)n_bins + 1) != RL_OK) { e->order_cap = 0; return RL_E_NOMEM; }
            e->order_cap = n_bins;
        }
        HIP_OK(launch_region_order(rstart, rcount, rend, n_bins, e->order_meta, e->order, s));
        ra.order = e->order;
        ra.order_prefix = e->order_prefix;
    }
    if (cache && e->solo_threshold) {
        // cache-on sliding windows have no hot path: a key's leading allow run in a large
        // region is decided by a whole workgroup, the rest by its region wave (rl_solo.hip).
        // (k_solo_select lists cache-on regions only, which k_hot_select never lists.)
        uint32_t* cnt = e->solo_list + kSoloMax;
        HIP_OK(hipMemsetAsync(cnt, 0, sizeof(uint32_t), s));
        HIP_OK(launch_solo_select(rstart, rcount, rend, n_bins, e->solo_threshold, e->d_lims,
                                  e->d_region_lim, e->solo_list, cnt, s));
        HIP_OK(launch_solo(ra, wide, res_bytes, (uint32_t*)rstart, (uint32_t*)rcount, e->solo_list, cnt, s));
    }
    mark(e, 7);
    // the regions (the hot chains run on the side stream since launch_chains)
    HIP_OK(launch_region(ra, wide, res_bytes, s, hot ? e->hstream : nullptr, e->hot_ev[1]));
    mark(e, 10);
    // (hot: the fill ran on the side stream, joined by launch_region)
    // the next batch's routed regions: this batch's largest hot regions (two-pass tables)
    if (hot && e->route && passes == 2)
        HIP_OK(launch_route_next(e->hot_info, e->hot_list + kHotMax, hot_thr, r_list, s));
    HIP_OK(launch_stats_reduce(e->d_stats, B.d_ctl, s));
    mark(e, 11);
    mark(e, 8);
    UnpermArgs ua{};
    ua.pos0 = B.pos0; ua.pos1 = passes == 2 ? B.pos1 : nullptr; ua.res = B.res;
    ua.mid = B.rec0;                                    // pass-0 records are dead by now
    ua.tok = tokens_after ? B.tok : nullptr;
    ua.ext = B.ext; ua.ctl = B.d_ctl;
    ua.allowed = allowed; ua.remaining = remaining; ua.tokens_out = tokens_after;
    ua.n = (uint32_t)n; ua.n_tiles = nt_un; ua.ablate = e->ablate; ua.per_cu = e->un_per_cu;
    ua.split = e->un_split == 1 || (e->un_split == 2 && passes == 2);
    ua.mid_xcd = e->mid_xcd;
    HIP_OK(launch_unpermute(ua, res_bytes, s));
    mark(e, 9);
    if (e->timing) {
        e->ring_next = (e->ring_next + 1) % kEvRing;
        e->ring_used = std::min(e->ring_used + 1, kEvRing);
    }
    HIP_OK(hipMemcpyAsync(e->h_ctl, B.d_ctl, sizeof(BatchCtl), hipMemcpyDeviceToHost, s));
    if (e->pipeline) {
        HIP_OK(hipEventRecord(B.freed, s));
        B.used = true;
        e->next_set ^= 1;
    }
    e->pending_status = true;
    e->enqueued = true;
    return RL_OK;
}

// on-demand growth: a limiter whose regions are filling up (or overflowed: then twice)
// gets twice (four times) the regions before the next batch
static void apply_growth(rl_engine* e, const unsigned long long (&grow)[4], bool overflowed) {
    if (!e->auto_grow || !(grow[0] | grow[1] | grow[2] | grow[3])) return;
    for (size_t li = 0; li < e->lims.size(); ++li) {
        if (!((grow[li >> 6] >> (li & 63)) & 1ULL)) continue;
        for (int t = 0; t < (overflowed ? 2 : 1); ++t)
            if (grow_once(e, li) != RL_OK) break;          // at the table-size limit: stay
    }
}

static int status_of(bool invalid, bool cap_err, bool span_overflow, bool internal) {
    int st = RL_OK;
    if (invalid) st = RL_E_INVALID_REQUEST;
    if (cap_err) st = RL_E_CAPACITY;
    if (span_overflow) st = RL_E_INVALID_ARG;
    if (internal) st = RL_E_INTERNAL;
    return st;
}

static int collect_status(rl_engine* e) {
    HIP_OK(hipStreamSynchronize(e->stream));
    if (e->pstream) HIP_OK(hipStreamSynchronize(e->pstream));
    if (!e->pending_status) return e->last_status;
    e->pending_status = false;
    BatchCtl& c = *e->h_ctl;
    e->hot_hint = c.n_hot;
    e->walk_hint = c.n_walk;
    const int st = status_of(c.invalid != 0, c.cap_err != 0, c.span_overflow != 0, c.internal_err != 0);
    e->last_status = st;
    apply_growth(e, c.grow, c.cap_err != 0);
    c.grow[0] = c.grow[1] = c.grow[2] = c.grow[3] = 0;
    return st;
}

namespace rl {
int engine_status_accum(rl_engine* e, unsigned long long* acc, void* stream) {
    if (!e || !acc) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    const BatchScratch& B = e->sc[e->pipeline ? e->next_set ^ 1 : 0];   // the last batch's set
    // A call that enqueued no batch (nothing received in this round, or a status set on the
    // host) leaves d_ctl holding an earlier batch whose status and growth were already
    // applied: fold only the host-side status then.
    const unsigned long long host = e->last_status == RL_E_INVALID_REQUEST ? 1ULL : 0ULL;
    HIP_OK(launch_status_accum(e->enqueued ? B.d_ctl : nullptr, e->enqueued ? 0ULL : host, acc,
                               stream ? (hipStream_t)stream : e->stream));
    return RL_OK;
}

int engine_status_settle(rl_engine* e, const unsigned long long* acc) {
    if (!e || !acc) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_OK(hipStreamSynchronize(e->stream));
    if (e->pstream) HIP_OK(hipStreamSynchronize(e->pstream));
    // the last batch's own status is part of acc: it must not be collected (grown) again
    e->pending_status = false;
    if (e->enqueued) { e->hot_hint = e->h_ctl->n_hot; e->walk_hint = e->h_ctl->n_walk; }
    const int st = status_of(acc[0] & 1u, acc[0] & 2u, acc[0] & 4u, acc[0] & 8u);
    e->last_status = st;
    const unsigned long long grow[4] = {acc[1], acc[2], acc[3], acc[4]};
    apply_growth(e, grow, (acc[0] & 2u) != 0);
    return st;
}
}  // namespace rl

extern "C" int rl_execute_batch_device(rl_engine* e, size_t n, const uint64_t* key,
                                       const int32_t* permits, const int64_t* now_ns,
                                       const uint16_t* limiter, const uint8_t* op,
                                       uint8_t* allowed, int64_t* remaining, double* tokens_after,
                                       void* stream) {
    if (!e) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipSetDevice(e->device);
    hipStream_t user = (hipStream_t)stream;
    if (user && user != e->stream) {
        // order the engine stream after the caller's work, and the caller's after ours
        hipEvent_t ev;
        HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_OK(hipEventRecord(ev, user));
        HIP_OK(hipStreamWaitEvent(e->stream, ev, 0));
        int rc = run_batch_device(e, n, key, permits, now_ns, limiter, op, allowed, remaining,
                                  tokens_after);
        HIP_OK(hipEventRecord(ev, e->stream));
        HIP_OK(hipStreamWaitEvent(user, ev, 0));
        (void)hipEventDestroy(ev);
        return rc;
    }
    return run_batch_device(e, n, key, permits, now_ns, limiter, op, allowed, remaining,
                            tokens_after, /*overlap=*/user == nullptr);
}

extern "C" int rl_last_status(rl_engine* e) {
    if (!e) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    return collect_status(e);
}

static int ensure_staging(rl_engine* e, size_t n) {
    if (n <= e->stage_cap) return RL_OK;
    dfree(e->s_key); dfree(e->s_permits); dfree(e->s_now); dfree(e->s_lim); dfree(e->s_op);
    dfree(e->s_allowed); dfree(e->s_remaining); dfree(e->s_tokens);
    int rc = dalloc(&e->s_key, n);
    if (rc == RL_OK) rc = dalloc(&e->s_permits, n);
    if (rc == RL_OK) rc = dalloc(&e->s_now, n);
    if (rc == RL_OK) rc = dalloc(&e->s_lim, n);
    if (rc == RL_OK) rc = dalloc(&e->s_op, n);
    if (rc == RL_OK) rc = dalloc(&e->s_allowed, n);
    if (rc == RL_OK) rc = dalloc(&e->s_remaining, n);
    if (rc == RL_OK) rc = dalloc(&e->s_tokens, n);
    if (rc != RL_OK) { e->stage_cap = 0; return rc; }
    e->stage_cap = n;
    return RL_OK;
}

extern "C" int rl_execute_batch(rl_engine* e, size_t n, const uint64_t* key,
                                const int32_t* permits, const int64_t* now_ns,
                                const uint16_t* limiter, const uint8_t* op, uint8_t* allowed,
                                int64_t* remaining, double* tokens_after) {
    if (!e) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    if (n > e->opts.max_batch) return RL_E_TOO_LARGE;
    if (n == 0) return RL_OK;
    if (!key || !permits || !now_ns || !allowed || !remaining) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    int rc = ensure_staging(e, n);
    if (rc != RL_OK) return rc;
    hipStream_t s = e->stream;
    HIP_OK(hipMemcpyAsync(e->s_key, key, n * 8, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(e->s_permits, permits, n * 4, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(e->s_now, now_ns, n * 8, hipMemcpyHostToDevice, s));
    if (limiter) HIP_OK(hipMemcpyAsync(e->s_lim, limiter, n * 2, hipMemcpyHostToDevice, s));
    if (op) HIP_OK(hipMemcpyAsync(e->s_op, op, n, hipMemcpyHostToDevice, s));
    rc = run_batch_device(e, n, e->s_key, e->s_permits, e->s_now, limiter ? e->s_lim : nullptr,
                          op ? e->s_op : nullptr, e->s_allowed, e->s_remaining,
                          tokens_after ? e->s_tokens : nullptr);
    if (rc != RL_OK) { (void)hipStreamSynchronize(s); return rc; }
    rc = collect_status(e);
    if (rc == RL_E_INVALID_ARG && e->h_ctl->span_overflow && !e->force_wide) {
        // the batch spans more than the compact record's 2^32 ms: it was rejected before any
        // state was touched, so run it again in 32-B records (full now_ms)
        e->force_wide = true;
        rc = run_batch_device(e, n, e->s_key, e->s_permits, e->s_now, limiter ? e->s_lim : nullptr,
                              op ? e->s_op : nullptr, e->s_allowed, e->s_remaining,
                              tokens_after ? e->s_tokens : nullptr);
        e->force_wide = false;
        if (rc != RL_OK) { (void)hipStreamSynchronize(s); return rc; }
        rc = collect_status(e);
    }
    HIP_OK(hipMemcpyAsync(allowed, e->s_allowed, n, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(remaining, e->s_remaining, n * 8, hipMemcpyDeviceToHost, s));
    if (tokens_after) HIP_OK(hipMemcpyAsync(tokens_after, e->s_tokens, n * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return rc;
}

// Page-lock a caller's host buffer so the host-buffer entry points DMA it directly instead
// of staging it through the runtime's bounce buffers (pageable memory). Registering an
// already page-locked range (hipHostMalloc, another registration) is a no-op.
extern "C" int rl_pin_host(rl_engine* e, void* ptr, size_t bytes) {
    if (!e || !ptr || bytes == 0) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    for (auto& pb : e->pinned)
        if (pb.first == ptr) return pb.second >= bytes ? RL_OK : RL_E_INVALID_ARG;
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, ptr) == hipSuccess && at.type == hipMemoryTypeHost) {
        (void)hipGetLastError();
        return RL_OK;                               // already page-locked by its owner
    }
    (void)hipGetLastError();
    if (hipHostRegister(ptr, bytes, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();
        return RL_E_DEVICE;
    }
    e->pinned.emplace_back(ptr, bytes);
    return RL_OK;
}

// Undo rl_pin_host; must be called before the caller frees the buffer. Unknown pointers
// (never pinned by this engine) return RL_E_INVALID_ARG.
extern "C" int rl_unpin_host(rl_engine* e, void* ptr) {
    if (!e || !ptr) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    for (size_t i = 0; i < e->pinned.size(); ++i) {
        if (e->pinned[i].first != ptr) continue;
        (void)hipStreamSynchronize(e->stream);     // no copy of it in flight
        const hipError_t r = hipHostUnregister(ptr);
        e->pinned.erase(e->pinned.begin() + (long)i);
        return r == hipSuccess ? RL_OK : RL_E_DEVICE;
    }
    return RL_E_INVALID_ARG;
}

extern "C" int rl_try_acquire_batch(rl_engine* e, size_t n, const uint64_t* key_hash,
                                    const int32_t* permits, const int64_t* now_ns,
                                    const uint16_t* limiter, uint8_t* allowed, int64_t* remaining,
                                    double* tokens_after) {
    return rl_execute_batch(e, n, key_hash, permits, now_ns, limiter, nullptr, allowed, remaining,
                            tokens_after);
}

static int admin_op(rl_engine* e, uint16_t limiter, size_t n, const uint64_t* key,
                    const int64_t* now_ns, uint8_t opcode, int64_t* out) {
    if (!e || (n && (!key || !now_ns))) return RL_E_INVALID_ARG;
    if (limiter >= e->lims.size()) return RL_E_INVALID_ARG;
    if (n == 0) return RL_OK;
    std::vector<int32_t> p(n, 1);
    std::vector<uint16_t> l(n, limiter);
    std::vector<uint8_t> o(n, opcode), a(n);
    std::vector<int64_t> r(n);
    int rc = rl_execute_batch(e, n, key, p.data(), now_ns, l.data(), o.data(), a.data(), r.data(),
                              nullptr);
    if (out) std::memcpy(out, r.data(), n * sizeof(int64_t));
    return rc;
}

extern "C" int rl_available(rl_engine* e, uint16_t limiter, size_t n, const uint64_t* key_hash,
                            const int64_t* now_ns, int64_t* available) {
    if (!available && n) return RL_E_INVALID_ARG;
    return admin_op(e, limiter, n, key_hash, now_ns, RL_OP_PEEK, available);
}

extern "C" int rl_reset(rl_engine* e, uint16_t limiter, size_t n, const uint64_t* key_hash,
                        const int64_t* now_ns) {
    return admin_op(e, limiter, n, key_hash, now_ns, RL_OP_RESET, nullptr);
}

extern "C" int rl_batch_stats_get(rl_engine* e, rl_batch_stats* out) {
    if (!e || !out) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    collect_status(e);
    const BatchCtl& c = *e->h_ctl;
    out->n = e->last_n;
    out->allowed = c.allowed;
    out->distinct_keys = c.distinct;
    out->invalid = c.invalid;
    out->capacity_errors = c.cap_err;
    out->regions_touched = c.regions;
    out->table_bytes = c.table_bytes;
    out->cache_hits = c.cache_hits;
    out->table_grows = e->grows;
    out->hot_regions = c.n_hot;
    out->routed = e->last_n >= c.n_normal ? e->last_n - c.n_normal : 0;
    return RL_OK;
}

// Average per-stage milliseconds over the batches enqueued since the previous call
// (at most the last 64). Stages a batch did not run (second pass) read 0.
extern "C" int rl_stage_times(rl_engine* e, const char** names, float* ms, int cap) {
    if (!e) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    collect_status(e);
    const int k = std::min(cap, kStages);
    const int nb = e->ring_used;
    for (int i = 0; i < k; ++i) {
        double acc = 0.0;
        for (int b = 0; b < nb; ++b) {
            const int r = (e->ring_next - 1 - b + kEvRing) % kEvRing;
            float x = 0.f;
            if (hipEventElapsedTime(&x, e->ev[r][kStagePairs[i][0]], e->ev[r][kStagePairs[i][1]]) != hipSuccess)
                x = 0.f;
            acc += x;
        }
        if (names) names[i] = kStageNames[i];
        if (ms) ms[i] = (e->timing && nb) ? (float)(acc / nb) : -1.f;
    }
    e->ring_used = 0;
    return k;
}

extern "C" int rl_tune(rl_engine* e, const char* key, int64_t value) {
    if (!e || !key) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    if (std::strcmp(key, "ablate") == 0) { e->ablate = (uint32_t)value; return RL_OK; }
    if (std::strcmp(key, "upsweep_per_cu") == 0) { e->up_per_cu = (uint32_t)value; return RL_OK; }
    if (std::strcmp(key, "scatter_per_cu") == 0) { e->sc_per_cu = (uint32_t)value; return RL_OK; }
    if (std::strcmp(key, "scatter_split") == 0) { e->sc_split = value != 0; return RL_OK; }
    if (std::strcmp(key, "unpermute_split") == 0) { e->un_split = (uint32_t)value; return RL_OK; }
    if (std::strcmp(key, "mid_xcd") == 0) { e->mid_xcd = value ? 1u : 0u; return RL_OK; }
    if (std::strcmp(key, "unpermute_per_cu") == 0) { e->un_per_cu = (uint32_t)value; return RL_OK; }
    if (std::strcmp(key, "debug_regions") == 0) { e->debug_regions = value != 0; return RL_OK; }
    if (std::strcmp(key, "wide_records") == 0) { e->force_wide = value != 0; return RL_OK; }
    if (std::strcmp(key, "stage_timing") == 0) {     // hipEvents around every stage on/off
        if (value) ensure_events(e);
        e->timing = value != 0;
        e->ring_used = 0;
        return RL_OK;
    }
    if (std::strcmp(key, "hot_threshold") == 0) {      // records per region; 0 = no hot path
        if (value < 0 || value > 0xFFFFFFFFLL) return RL_E_INVALID_ARG;
        e->hot_threshold = (uint32_t)value;
        e->hot_thr_auto = false;
        return RL_OK;
    }
    if (std::strcmp(key, "solo_threshold") == 0) {     // records per region; 0 = off
        if (value < 0 || value > 0xFFFFFFFFLL) return RL_E_INVALID_ARG;
        e->solo_threshold = (uint32_t)value;
        return RL_OK;
    }
    if (std::strcmp(key, "sparse_max") == 0) {         // records per region; 0 = image mode only
        if (value < 0 || value > 0xFFFFFFFFLL) return RL_E_INVALID_ARG;
        e->sparse_max = (uint32_t)value;
        return RL_OK;
    }
    if (std::strcmp(key, "region_order") == 0) {
        e->region_order = value != 0;
        return RL_OK;
    }
    if (std::strcmp(key, "order_prefix") == 0) {
        if (value < 0) return RL_E_INVALID_ARG;
        e->order_prefix = (uint32_t)value;
        return RL_OK;
    }
    if (std::strcmp(key, "route") == 0) {             // hot-region routing in pass 0
        e->route = value != 0;
        return RL_OK;
    }
    if (std::strcmp(key, "tile_items") == 0) {        // partition tile = value x 512 requests
        if (value != 0 && (value < 8 || value > 1024 || value % 8 != 0)) return RL_E_INVALID_ARG;
        e->tile_items = (uint32_t)value;
        return RL_OK;
    }
    if (std::strcmp(key, "segments") == 0) {          // two-pass batches: pass-0 output segments
        if (value < 1 || value > 64) return RL_E_INVALID_ARG;
        e->segments = (uint32_t)value;
        return RL_OK;
    }
    if (std::strcmp(key, "group_bits") == 0) {        // two-pass batches: pass-0 high-digit bits
        if (value < 1 || value > kMaxDigitBits) return RL_E_INVALID_ARG;
        e->group_bits = (uint32_t)value;
        return RL_OK;
    }
    if (std::strcmp(key, "walk") == 0) {              // allow walks of the hot chains
        e->walk = value != 0;
        if (!e->walk && e->walk_tab) {                 // (hipFree waits for the batches in flight)
            HIP_OK(hipStreamSynchronize(e->stream));
            if (e->hstream) HIP_OK(hipStreamSynchronize(e->hstream));
            dfree(e->walk_tab);
        }
        return RL_OK;
    }
    if (std::strcmp(key, "chain_split") == 0) {       // a hot region's other keys on a second wave
        e->chain_split = value != 0;
        return RL_OK;
    }
    if (std::strcmp(key, "walk_min") == 0) {          // keys walked: at least this many allows expected
        if (value < 0 || value > 0xFFFFFFFFLL) return RL_E_INVALID_ARG;
        e->walk_min = (uint32_t)value;
        return RL_OK;
    }
    if (std::strcmp(key, "fail_batches") == 0) {      // the next `value` batches fail (RL_E_DEVICE)
        if (value < 0 || value > 0xFFFFFFFFLL) return RL_E_INVALID_ARG;
        e->inject_fail = (uint32_t)value;
        return RL_OK;
    }
    return RL_E_INVALID_ARG;
}

extern "C" int rl_sync(rl_engine* e) {
    if (!e) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_OK(hipStreamSynchronize(e->stream));
    if (e->pstream) HIP_OK(hipStreamSynchronize(e->pstream));
    if (e->pending_status) {                                 // the last batch is complete
        e->hot_hint = e->h_ctl->n_hot;
        e->walk_hint = e->h_ctl->n_walk;
    }
    return RL_OK;
}

extern "C" int rl_route_partition(rl_engine* e, size_t n, const uint64_t* key_hash,
                                  const uint16_t*, uint32_t shard_count, uint32_t* perm,
                                  uint64_t* counts_host, void* stream) {
    if (!e || !key_hash || !perm || !counts_host) return RL_E_INVALID_ARG;
    if (shard_count == 0 || shard_count > 64 || (shard_count & (shard_count - 1))) return RL_E_INVALID_ARG;
    if (n > 0xFFFFFFF0ULL) return RL_E_TOO_LARGE;
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    const size_t nt = (n + kTile - 1) / kTile;
    const size_t need = (size_t)shard_count * nt + 64;
    if (need > e->route_cap) {
        dfree(e->route_scratch);
        if (dalloc(&e->route_scratch, need) != RL_OK) return RL_E_NOMEM;
        e->route_cap = need;
    }
    if (!e->route_counts && dalloc(&e->route_counts, 64) != RL_OK) return RL_E_NOMEM;
    if (n == 0) {
        for (uint32_t i = 0; i < shard_count; ++i) counts_host[i] = 0;
        return RL_OK;
    }
    HIP_OK(launch_owner_partition(key_hash, (uint32_t)n, shard_count, perm, e->route_counts,
                                  e->route_scratch, e->d_dir, s));
    uint32_t c[64];
    HIP_OK(hipMemcpyAsync(c, e->route_counts, shard_count * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    for (uint32_t i = 0; i < shard_count; ++i) counts_host[i] = c[i];
    return RL_OK;
}

// Hot-key owner directory: key_hash[i] is owned by owner[i] instead of its hash owner.
// Every rank of a router must install the same directory, before any state exists for
// those keys (or after moving it with rl_export_state / rl_import_state).
extern "C" int rl_set_owner_directory(rl_engine* e, size_t n, const uint64_t* key_hash,
                                      const uint32_t* owner) {
    if (!e || (n && (!key_hash || !owner)) || n > kDirMax) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    for (size_t i = 0; i < n; ++i)
        if (owner[i] >= e->opts.shard_count) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    if (n == 0) {
        dfree(e->d_dir);
        e->h_dir.clear();
        return RL_OK;
    }
    std::vector<DirSlot> t(kDirSlots, DirSlot{0, kDirEmpty, 0});
    for (size_t i = 0; i < n; ++i) {
        const uint64_t tag = mix64(key_hash[i]);
        uint32_t p = (uint32_t)tag & (kDirSlots - 1);
        while (t[p].owner != kDirEmpty && t[p].tag != tag) p = (p + 1) & (kDirSlots - 1);
        t[p].tag = tag;
        t[p].owner = owner[i];
    }
    if (!e->d_dir && dalloc(&e->d_dir, kDirSlots) != RL_OK) return RL_E_NOMEM;
    HIP_OK(hipMemcpy(e->d_dir, t.data(), kDirSlots * sizeof(DirSlot), hipMemcpyHostToDevice));
    e->h_dir.swap(t);
    return RL_OK;
}

extern "C" uint32_t rl_owner_of_engine(rl_engine* e, uint64_t key_hash) {
    if (!e) return 0;
    const uint64_t tag = mix64(key_hash);
    if (!e->h_dir.empty()) {
        uint32_t p = (uint32_t)tag & (kDirSlots - 1);
        for (uint32_t i = 0; i < kDirSlots && e->h_dir[p].owner != kDirEmpty; ++i) {
            if (e->h_dir[p].tag == tag) return e->h_dir[p].owner;
            p = (p + 1) & (kDirSlots - 1);
        }
    }
    return e->opts.shard_count <= 1 ? 0u : (uint32_t)(tag >> (64 - e->shard_bits));
}

extern "C" int rl_route_pack(rl_engine* e, size_t n, const uint32_t* perm, const uint64_t* key,
                             const int32_t* permits, const int64_t* now_ns, const uint16_t* limiter,
                             uint64_t* key_out, int32_t* permits_out, int64_t* now_out,
                             uint16_t* limiter_out, void* stream) {
    if (!e || (n && (!perm || !key || !permits || !now_ns || !key_out || !permits_out || !now_out)))
        return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_pack((uint32_t)n, perm, key, permits, now_ns, limiter, key_out, permits_out,
                             now_out, limiter_out, s));
    return RL_OK;
}

extern "C" int rl_route_fold(rl_engine* e, size_t n, const uint8_t* allowed, const int64_t* remaining,
                             int64_t* packed, void* stream) {
    if (!e || (n && (!allowed || !remaining || !packed))) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_fold((uint32_t)n, allowed, remaining, packed, s));
    return RL_OK;
}

extern "C" int rl_route_unpack(rl_engine* e, size_t n, const uint32_t* perm, const int64_t* packed,
                               uint8_t* allowed, int64_t* remaining, void* stream) {
    if (!e || (n && (!perm || !packed || !allowed || !remaining))) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_unpack((uint32_t)n, perm, packed, allowed, remaining, s));
    return RL_OK;
}

extern "C" int rl_route_pack_wire(rl_engine* e, size_t n, const uint32_t* perm, const uint64_t* key,
                                  const int32_t* permits, const int64_t* now_ns,
                                  const uint16_t* limiter, uint64_t* wire_out,
                                  uint16_t* limiter_out, int64_t* hdr, void* stream) {
    if (!e || !hdr || (n && (!perm || !key || !permits || !now_ns || !wire_out))) return RL_E_INVALID_ARG;
    if (n > 0xFFFFFFF0ULL) return RL_E_TOO_LARGE;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_pack_wire((uint32_t)n, perm, key, permits, now_ns, limiter, wire_out,
                                  limiter_out, hdr, s));
    return RL_OK;
}

namespace rl {
// rl_route_pack_wire plus the per-block now_ms min / max partials of the router's header
// (internal: rl_router.cpp).
int route_pack_wire_mm(rl_engine* e, size_t n, const uint32_t* perm, const uint64_t* key,
                       const int32_t* permits, const int64_t* now_ns, const uint16_t* limiter,
                       uint64_t* wire_out, uint16_t* limiter_out, int64_t* hdr, uint64_t* part,
                       uint32_t* nparts, void* stream) {
    if (!e || !hdr || !part || !nparts || (n && (!perm || !key || !permits || !now_ns || !wire_out)))
        return RL_E_INVALID_ARG;
    if (n > 0xFFFFFFF0ULL) return RL_E_TOO_LARGE;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_pack_wire((uint32_t)n, perm, key, permits, now_ns, limiter, wire_out,
                                  limiter_out, hdr, s, part, nparts));
    return RL_OK;
}
int engine_device(rl_engine* e) { return e ? e->device : 0; }
size_t engine_max_batch(rl_engine* e) { return e ? (size_t)e->opts.max_batch : 0; }
}  // namespace rl

extern "C" int rl_route_unwire(rl_engine* e, size_t m, const uint64_t* wire, uint32_t n_src,
                               const int64_t* src_base, const uint64_t* src_count,
                               uint64_t* key_out, int32_t* permits_out, int64_t* now_out,
                               void* stream) {
    if (!e || !src_base || !src_count || n_src == 0 || n_src > (uint32_t)kMaxShards)
        return RL_E_INVALID_ARG;
    if (m && (!wire || !key_out || !permits_out || !now_out)) return RL_E_INVALID_ARG;
    if (m > 0xFFFFFFF0ULL) return RL_E_TOO_LARGE;
    uint32_t end[kMaxShards];
    uint64_t run = 0;
    for (uint32_t i = 0; i < n_src; ++i) { run += src_count[i]; end[i] = (uint32_t)run; }
    if (run != m) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_unwire((uint32_t)m, wire, n_src, src_base, end, key_out, permits_out,
                               now_out, s));
    return RL_OK;
}

extern "C" int rl_result_width(rl_engine* e) {
    if (!e) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    bool wide = false;
    int64_t max_any = 0;
    for (auto& l : e->lims) {
        wide |= l.cfg.max_permits > kCompactMaxPermits;
        max_any = std::max<int64_t>(max_any, l.cfg.max_permits);
    }
    return res_bytes_for(max_any, wide);
}

extern "C" int rl_route_fold_packed(rl_engine* e, size_t n, const uint8_t* allowed,
                                    const int64_t* remaining, void* packed, int width,
                                    void* stream) {
    if (!e || (n && (!allowed || !remaining || !packed))) return RL_E_INVALID_ARG;
    if (width != 1 && width != 2 && width != 4 && width != 8) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_fold_w((uint32_t)n, allowed, remaining, packed, width, s));
    return RL_OK;
}

extern "C" int rl_route_unpack_packed(rl_engine* e, size_t n, const uint32_t* perm,
                                      const void* packed, int width, uint8_t* allowed,
                                      int64_t* remaining, void* stream) {
    if (!e || (n && (!perm || !packed || !allowed || !remaining))) return RL_E_INVALID_ARG;
    if (width != 1 && width != 2 && width != 4 && width != 8) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_unpack_w((uint32_t)n, perm, packed, width, allowed, remaining, s));
    return RL_OK;
}

extern "C" uint64_t rl_route_return_bytes(uint32_t n_seg, const uint64_t* seg_counts, int width,
                                          uint32_t exc_cap) {
    if (!seg_counts || n_seg == 0 || n_seg > (uint32_t)kMaxShards) return 0;
    if (width != 1 && width != 2 && width != 4 && width != 8) return 0;
    return ret_layout(seg_counts, n_seg, width, exc_cap, nullptr, nullptr);
}

extern "C" int rl_route_fold_return(rl_engine* e, size_t m, const uint8_t* allowed,
                                    const int64_t* remaining, void* out, int width, uint32_t n_seg,
                                    const uint64_t* seg_counts, uint32_t exc_cap, void* stream) {
    if (!e || !out || !seg_counts || (m && (!allowed || !remaining))) return RL_E_INVALID_ARG;
    if (width != 1 && width != 2 && width != 4 && width != 8) return RL_E_INVALID_ARG;
    if (n_seg == 0 || n_seg > (uint32_t)kMaxShards || m > 0xFFFFFFF0ULL) return RL_E_INVALID_ARG;
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n_seg; ++i) tot += seg_counts[i];
    if (tot != m) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_fold_ret((uint32_t)m, allowed, remaining, out, width, n_seg, seg_counts,
                                 exc_cap, s));
    return RL_OK;
}

extern "C" int rl_route_unpack_return(rl_engine* e, size_t n, const uint32_t* perm, const void* in,
                                      int width, uint32_t n_seg, const uint64_t* seg_counts,
                                      uint32_t exc_cap, uint8_t* allowed, int64_t* remaining,
                                      uint32_t* lost, void* stream) {
    if (!e || !seg_counts || !lost || (n && (!perm || !in || !allowed || !remaining)))
        return RL_E_INVALID_ARG;
    if (width != 1 && width != 2 && width != 4 && width != 8) return RL_E_INVALID_ARG;
    if (n_seg == 0 || n_seg > (uint32_t)kMaxShards || n > 0xFFFFFFF0ULL) return RL_E_INVALID_ARG;
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n_seg; ++i) tot += seg_counts[i];
    if (tot != n) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_route_unpack_ret((uint32_t)n, perm, in, width, n_seg, seg_counts, exc_cap, allowed,
                                   remaining, lost, s));
    return RL_OK;
}

extern "C" int rl_route_partition_device(rl_engine* e, size_t n, const uint64_t* key_hash,
                                         uint32_t shard_count, uint32_t* perm, int64_t* counts_dev,
                                         size_t counts_stride, void* stream) {
    if (!e || !key_hash || !perm || !counts_dev || counts_stride == 0) return RL_E_INVALID_ARG;
    if (shard_count == 0 || shard_count > 64 || (shard_count & (shard_count - 1))) return RL_E_INVALID_ARG;
    if (n > 0xFFFFFFF0ULL) return RL_E_TOO_LARGE;
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    const size_t nt = (n + kTile - 1) / kTile;
    const size_t need = (size_t)shard_count * std::max<size_t>(nt, 1) + 64;
    if (need > e->route_cap) {
        dfree(e->route_scratch);
        if (dalloc(&e->route_scratch, need) != RL_OK) return RL_E_NOMEM;
        e->route_cap = need;
    }
    if (!e->route_counts && dalloc(&e->route_counts, 64) != RL_OK) return RL_E_NOMEM;
    if (n == 0) {
        HIP_OK(hipMemsetAsync(e->route_counts, 0, 64 * sizeof(uint32_t), s));
    } else {
        HIP_OK(launch_owner_partition(key_hash, (uint32_t)n, shard_count, perm, e->route_counts,
                                      e->route_scratch, e->d_dir, s));
    }
    HIP_OK(launch_counts_to_header(e->route_counts, shard_count, counts_dev, (uint32_t)counts_stride, s));
    return RL_OK;
}

extern "C" int rl_synth_trace_device(rl_engine* e, const rl_trace_spec* sp, size_t n,
                                     uint64_t* key_hash, int32_t* permits, int64_t* now_ns,
                                     uint16_t* limiter, void* stream) {
    if (!e || !sp || !key_hash || !permits || !now_ns) return RL_E_INVALID_ARG;
    if (sp->n_keys == 0 || sp->permits_max <= 0 || sp->n_total == 0) return RL_E_INVALID_ARG;
    (void)hipSetDevice(e->device);
    SynthArgs a{};
    a.seed = sp->seed; a.n_keys = sp->n_keys; a.dist = sp->dist; a.permits_max = sp->permits_max;
    a.t0_ns = sp->t0_ns; a.span_ns = sp->span_ns; a.index_base = sp->index_base;
    a.n_total = sp->n_total; a.n_limiters = sp->n_limiters ? sp->n_limiters : 1;
    a.key = key_hash; a.permits = permits; a.now_ns = now_ns; a.limiter = limiter; a.n = n;
    if (sp->dist == RL_DIST_ZIPF) {
        const double s = sp->zipf_s;
        if (!(s > 0.0) || s == 1.0) return RL_E_INVALID_ARG;
        auto h1 = [](double x) { return std::fabs(x) > 1e-8 ? std::log1p(x) / x : 1.0 - x * (0.5 - x / 3.0); };
        auto h2 = [](double x) { return std::fabs(x) > 1e-8 ? std::expm1(x) / x : 1.0 + x * 0.5 * (1.0 + x / 3.0); };
        auto H = [&](double x) { double lx = std::log(x); return h2((1.0 - s) * lx) * lx; };
        auto hh = [&](double x) { return std::exp(-s * std::log(x)); };
        auto Hinv = [&](double x) { double t = x * (1.0 - s); if (t < -1.0) t = -1.0; return std::exp(h1(t) * x); };
        a.zs = s;
        a.hx1 = H(1.5) - 1.0;
        a.hn = H((double)sp->n_keys + 0.5);
        a.sconst = 2.0 - Hinv(H(2.5) - hh(2.0));
    }
    hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    HIP_OK(launch_synth(a, st));
    return RL_OK;
}

extern "C" int rl_debug_fetch(rl_engine* e, const char* what, void* out, size_t bytes) {
    if (!e || !what || (!out && bytes)) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    if (std::strcmp(what, "region_times") == 0) {
        if (!e->dbg) return RL_E_INVALID_ARG;
        HIP_OK(hipStreamSynchronize(e->stream));
        const size_t nb = std::min(bytes, e->dbg_cap * sizeof(uint64_t));
        HIP_OK(hipMemcpy(out, e->dbg, nb, hipMemcpyDeviceToHost));
        return (int)(nb / (kDbgWords * sizeof(uint64_t)));
    }
    if (std::strcmp(what, "bin_totals") == 0) {      // the last batch's pass-0 bin sizes
        const BatchScratch& B = e->sc[e->pipeline ? e->next_set ^ 1 : 0];
        HIP_OK(hipStreamSynchronize(e->stream));
        const size_t nb = std::min(bytes, ((size_t)1 << kMaxDigitBits) * sizeof(uint32_t));
        HIP_OK(hipMemcpy(out, B.bin_total, nb, hipMemcpyDeviceToHost));
        return (int)(nb / sizeof(uint32_t));
    }
    return RL_E_INVALID_ARG;
}

// ---------------------------------------------------------------- state export / import
// the engine's state in the reference's Redis keyspace layout
// (SlidingWindowRateLimiter.java:185-188 + RedisRateLimitStorage.java:38-49;
// TokenBucketRateLimiter.java:46-48,63-64).
static_assert(sizeof(StateRec) == sizeof(rl_state_entry), "StateRec layout");
static_assert(offsetof(StateRec, expire_at_ms) == offsetof(rl_state_entry, expire_at_ms), "StateRec layout");

extern "C" int rl_export_state(rl_engine* e, int64_t now_ns, rl_state_entry* out, size_t cap,
                               size_t* n_out) {
    if (!e || !n_out || (cap && !out)) return RL_E_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipSetDevice(e->device);
    const int64_t now = floor_div_ms(now_ns);
    const uint32_t dcap = (uint32_t)std::min<size_t>(cap, 0xFFFFFFF0u);
    StateRec* d_out = nullptr;
    uint32_t* d_count = nullptr;
    if (dalloc(&d_out, std::max<uint32_t>(dcap, 1u)) != RL_OK) return RL_E_NOMEM;
    if (dalloc(&d_count, e->lims.size() + 1) != RL_OK) { dfree(d_out); return RL_E_NOMEM; }
    int rc = RL_OK;
    uint32_t total = 0;
    if (hipMemsetAsync(d_count, 0, sizeof(uint32_t), e->stream) != hipSuccess) rc = RL_E_DEVICE;
    for (size_t li = 0; rc == RL_OK && li < e->lims.size(); ++li) {
        const HostLimiter& h = e->lims[li];
        if (launch_export((const Slot*)h.table, h.table_bytes / sizeof(Slot), h.dev, (uint16_t)li,
                          now, d_out, dcap, d_count, e->stream) != hipSuccess)
            rc = RL_E_DEVICE;
    }
    if (rc == RL_OK && (hipMemcpyAsync(&total, d_count, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                       e->stream) != hipSuccess ||
                        hipStreamSynchronize(e->stream) != hipSuccess))
        rc = RL_E_DEVICE;
    if (rc == RL_OK) {
        *n_out = total;
        if (total > cap) {
            rc = RL_E_TOO_LARGE;
        } else if (total) {
            if (hipMemcpy(out, d_out, (size_t)total * sizeof(StateRec), hipMemcpyDeviceToHost) != hipSuccess) {
                rc = RL_E_DEVICE;
            } else {
                std::sort(out, out + total, [](const rl_state_entry& x, const rl_state_entry& y) {
                    if (x.limiter != y.limiter) return x.limiter < y.limiter;
                    if (x.key_hash != y.key_hash) return x.key_hash < y.key_hash;
                    return x.window_start_ms < y.window_start_ms;
                });
            }
        }
    }
    dfree(d_out);
    dfree(d_count);
    return rc;
}

extern "C" int rl_import_state(rl_engine* e, const rl_state_entry* in, size_t n, size_t* n_imported) {
    if (!e || (n && !in)) return RL_E_INVALID_ARG;
    if (n_imported) *n_imported = 0;
    if (n == 0) return RL_OK;
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipSetDevice(e->device);
    std::vector<const rl_state_entry*> v(n);
    for (size_t i = 0; i < n; ++i) {
        const rl_state_entry& x = in[i];
        if (x.limiter >= e->lims.size()) return RL_E_INVALID_ARG;
        const DevLimiter& L = e->lims[x.limiter].dev;
        if (x.kind != (L.algo == kAlgoTB ? RL_STATE_TB_BUCKET : RL_STATE_SW_BUCKET)) return RL_E_INVALID_ARG;
        if (L.algo == kAlgoTB) {
            if (x.expire_at_ms != x.last_refill_ms + L.ttl_ms) return RL_E_INVALID_ARG;
        } else {
            const int64_t w = L.window_ms;
            if (x.count < 1 || x.count > 0xFFFFFFFFLL || x.window_start_ms % w != 0) return RL_E_INVALID_ARG;
            const int64_t off = x.expire_at_ms - w - x.window_start_ms;   // last INCR - W
            if (off < 0 || off >= w) return RL_E_INVALID_ARG;
        }
        v[i] = &x;
    }
    // (limiter, key) groups, newest bucket first
    std::sort(v.begin(), v.end(), [](const rl_state_entry* x, const rl_state_entry* y) {
        if (x->limiter != y->limiter) return x->limiter < y->limiter;
        if (x->key_hash != y->key_hash) return x->key_hash < y->key_hash;
        return x->window_start_ms > y->window_start_ms;
    });
    struct Img { uint64_t addr, xaddr; uint8_t algo; Slot s; };
    std::vector<Img> imgs;
    size_t taken = 0;
    for (size_t i = 0; i < n;) {
        size_t j = i + 1;
        while (j < n && v[j]->limiter == v[i]->limiter && v[j]->key_hash == v[i]->key_hash) ++j;
        const rl_state_entry& x = *v[i];
        const HostLimiter& h = e->lims[x.limiter];
        const DevLimiter& L = h.dev;
        const uint64_t tag = mix64(x.key_hash);
        const bool mine = e->opts.shard_count <= 1 ||
                          (uint32_t)(tag >> (64 - e->shard_bits)) == e->opts.shard_index;
        if (mine) {
            Img im{};
            im.algo = (uint8_t)L.algo;
            im.s.tag = tag;
            if (L.algo == kAlgoTB) {                   // one hash per key: the first one wins
                uint64_t bits;
                std::memcpy(&bits, &x.tokens, 8);
                im.s.a = bits; im.s.b = (uint64_t)x.last_refill_ms; im.s.c = 1;
                taken += 1;
            } else {
                const int64_t w = L.window_ms;
                int64_t b1 = x.window_start_ms;
                uint64_t c1 = (uint64_t)x.count, c0 = 0;
                int64_t o1 = x.expire_at_ms - w - b1, o0 = 0;
                taken += 1;
                if (j > i + 1 && v[i + 1]->window_start_ms == b1 - w) {
                    c0 = (uint64_t)v[i + 1]->count;
                    o0 = v[i + 1]->expire_at_ms - w - (b1 - w);
                    taken += 1;
                }
                im.s.a = (uint64_t)b1;
                im.s.b = c1 | (c0 << 32);
                im.s.c = (uint64_t)(uint32_t)o1 | ((uint64_t)(uint32_t)o0 << 32);
            }
            const uint32_t region = region_local(tag, e->shard_bits, L.region_bits);
            im.addr = (uint64_t)(uintptr_t)h.table + (uint64_t)region * kRegionSlots * sizeof(Slot);
            im.xaddr = h.cache_table ? (uint64_t)(uintptr_t)h.cache_table +
                                           (uint64_t)region * kRegionSlots * sizeof(uint64_t) : 0;
            imgs.push_back(im);
        }
        i = j;
    }
    if (imgs.empty()) return RL_OK;
    std::stable_sort(imgs.begin(), imgs.end(), [](const Img& x, const Img& y) { return x.addr < y.addr; });
    std::vector<uint32_t> off;
    std::vector<uint64_t> addr, xaddr;
    std::vector<uint8_t> algo;
    std::vector<Slot> slots(imgs.size());
    for (size_t k = 0; k < imgs.size(); ++k) {
        if (k == 0 || imgs[k].addr != imgs[k - 1].addr) {
            off.push_back((uint32_t)k);
            addr.push_back(imgs[k].addr);
            xaddr.push_back(imgs[k].xaddr);
            algo.push_back(imgs[k].algo);
        }
        slots[k] = imgs[k].s;
    }
    off.push_back((uint32_t)imgs.size());
    const size_t G = addr.size();
    const size_t bytes = slots.size() * sizeof(Slot) + G * 16 + (G + 1) * 4 + G + 16;
    uint8_t* d = nullptr;
    if (dalloc(&d, bytes) != RL_OK) return RL_E_NOMEM;
    Slot* d_img = (Slot*)d;
    uint64_t* d_addr = (uint64_t*)(d + slots.size() * sizeof(Slot));
    uint64_t* d_xaddr = d_addr + G;
    uint32_t* d_off = (uint32_t*)(d_xaddr + G);
    uint32_t* d_fail = d_off + G + 1;
    uint8_t* d_algo = (uint8_t*)(d_fail + 1);
    int rc = RL_OK;
    uint32_t fail = 0;
    if (hipMemcpyAsync(d_img, slots.data(), slots.size() * sizeof(Slot), hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        hipMemcpyAsync(d_addr, addr.data(), G * 8, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        hipMemcpyAsync(d_xaddr, xaddr.data(), G * 8, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        hipMemcpyAsync(d_off, off.data(), (G + 1) * 4, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        hipMemcpyAsync(d_algo, algo.data(), G, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        hipMemsetAsync(d_fail, 0, 4, e->stream) != hipSuccess)
        rc = RL_E_DEVICE;
    if (rc == RL_OK) {
        ImportArgs a{};
        a.n_groups = (uint32_t)G; a.group_off = d_off; a.region_addr = d_addr; a.xregion_addr = d_xaddr;
        a.group_algo = d_algo;
        a.img = d_img; a.fail = d_fail;
        if (launch_import(a, e->stream) != hipSuccess ||
            hipMemcpyAsync(&fail, d_fail, 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess)
            rc = RL_E_DEVICE;
    }
    (void)hipFree(d);
    if (rc != RL_OK) return rc;
    if (n_imported) *n_imported = taken;
    return fail ? RL_E_CAPACITY : RL_OK;
}

extern "C" int rl_sweep_expired(rl_engine* e, int64_t now_ns, uint64_t* reclaimed) {
    if (!e) return RL_E_INVALID_ARG;
    if (reclaimed) *reclaimed = 0;
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipSetDevice(e->device);
    const int64_t now = floor_div_ms(now_ns);
    uint32_t* d_count = nullptr;
    if (dalloc(&d_count, e->lims.size() + 1) != RL_OK) return RL_E_NOMEM;
    std::vector<uint32_t> h(e->lims.size() + 1, 0);
    int rc = RL_OK;
    if (hipMemsetAsync(d_count, 0, h.size() * sizeof(uint32_t), e->stream) != hipSuccess) rc = RL_E_DEVICE;
    for (size_t li = 0; rc == RL_OK && li < e->lims.size(); ++li) {
        HostLimiter& hl = e->lims[li];
        if (launch_sweep((Slot*)hl.table, hl.table_bytes / sizeof(Slot), hl.dev, now, d_count + li,
                         e->stream) != hipSuccess)
            rc = RL_E_DEVICE;
    }
    if (rc == RL_OK && (hipMemcpyAsync(h.data(), d_count, h.size() * sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
                        hipStreamSynchronize(e->stream) != hipSuccess))
        rc = RL_E_DEVICE;
    dfree(d_count);
    if (rc == RL_OK && reclaimed)
        for (uint32_t c : h) *reclaimed += c;
    return rc;
}
