// rl_launch.hpp — host-side launchers for the kernels in csrc/rl_*.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_device.hpp"

struct rl_engine;   // include/rl_engine.h

namespace rl {

// Ablation bits (rl_tune "ablate"): timing experiments only; results are wrong when set.
enum : uint32_t {
    kAblNoRecStore = 1u << 0,    // scatter: skip the record store
    kAblSeqRecStore = 1u << 1,   // scatter: store records at their input index (coalesced)
    kAblNoMatch = 1u << 2,       // scatter: skip the ballot match (rank 0 for every lane)
    kAblNoPosStore = 1u << 3,    // scatter: skip pos_out
    kAblNoBarrier = 1u << 4,     // scatter: skip the two per-round barriers
    kAblGroupSeq = 1u << 5,      // k_gplace: store records at their pass-0 index (coalesced)
    kAblNoStep = 1u << 8,        // region: skip the per-request semantics
    kAblNoProbe = 1u << 9,       // region: slot = home (no lookup / insert)
    kAblNoRounds = 1u << 10,     // region: one round, no peer match
    kAblNoNormal = 1u << 11,     // region: skip every non-hot region (hot chains run alone)
    kAblNoChainStores = 1u << 12,// hot chains: skip the result stores (measures their waits)
    kAblNoGather = 1u << 16,     // unpermute: skip the res gather
};

// Per-batch device control block (written by kernels, read by later kernels/host).
struct BatchCtl {
    int64_t base_ms;           // compact records: now_ms = base_ms + now_rel
    uint64_t min_now_key;      // ordered-unsigned encoding of min now_ms
    uint64_t max_now_key;
    uint32_t span_overflow;    // compact: some valid request's now_ms outside [base, base + 2^32)
    uint32_t n_esc;            // results stored through kResEscape (exact value in `ext`)
    unsigned long long allowed;
    unsigned long long distinct;
    unsigned long long invalid;
    unsigned long long cap_err;
    unsigned long long regions;
    unsigned long long cache_hits; // SW local-cache rejections (ratelimiter.cache.hits)
    unsigned long long grow[4];    // limiter bit set: one of its regions is filling up
    unsigned long long table_bytes;// state-table bytes read + written by the region stage
    uint32_t n_normal;         // records in the normal partition: pass 0 routes the previous
                               // batch's hot regions to bins of their own (k_route_ranges)
    uint32_t n_hot;            // hot regions of the batch (k_hot_prep): the next batches'
                               // chain-launch size hint (RegionArgs::chain_grid)
    uint32_t internal_err;     // a kernel met a state its logic excludes (RL_E_INTERNAL)
    uint32_t n_walk;           // listed hot regions with a key dense enough for an allow walk
                               // (k_hot_scan): the host allocates the walk tables once it is > 0
};
// A region holding more than kGrowUsed live keys after a batch (or one that overflowed)
// flags its limiter for growth (rl_engine doubles its region count at the next status
// collection): Redis grows its keyspace on demand (RedisRateLimitStorage.java:38-49).
// 208 of 256: at the design load (0.5, 128 keys per region on average) the fullest of 8192
// regions holds ~128 + 4.5 sigma ~ 180 keys, so a table at its configured capacity does not
// grow; at ~0.62 average load it does, well before the fullest region (~217) overflows.
constexpr uint32_t kGrowUsed = 208;

struct PartArgs {
    // pass 0 reads the caller's SoA request arrays
    const uint64_t* key;
    const int32_t* permits;
    const int64_t* now_ns;
    const uint16_t* limiter;   // nullable
    const uint8_t* op;         // nullable
    // later passes read records
    const void* rec_in;
    void* rec_out;
    uint32_t* pos_out;         // pos_out[i] = destination of element i
    uint32_t n;
    uint32_t n_tiles;
    uint32_t tile_items;       // rounds of kTileThreads requests per tile (kTileItems, or twice
                               // it for large batches: fewer [bin][tile] counts to write and scan)
    uint32_t n_lim;
    int32_t shard_bits;
    const DevLimiter* lims;
    int32_t digit_shift;
    int32_t digit_bits;
    uint32_t up_per_cu;        // persistent-grid workgroups per CU (0: default)
    uint32_t sc_per_cu;
    uint32_t sc_split;         // rl_tune("scatter_split"): loads and stores in separate waves
    uint32_t* counts;          // [bins][n_tiles]: per-tile histogram, then exclusive row scan
    const uint32_t* bin_base;  // [bins]
    // Segmented output (two-pass batches, rl_tune "segments" > 1; nullable): the tiles cut into
    // n_segs runs of seg_tiles, the normal bins laid out [segment][bin] so that the write
    // fronts of all bins stay inside one segment's part of the array at a time; a tile's
    // cursor base is seg_adj[bin * n_segs + tile / seg_tiles] instead of bin_base[bin]
    const uint32_t* seg_adj;
    uint32_t n_segs, seg_tiles;
    BatchCtl* ctl;
    uint32_t ablate;           // rl_tune("ablate"): measurement-only variants (0 = product)
    uint32_t n_bins_pass;      // bins of this pass (0: 1 << digit_bits)
    // Hot-region routing (pass 0 of a two-pass batch): route_list is a kRouteSlots-entry
    // table of region ids (kNone = empty; the previous batch's largest hot regions, each at
    // one of its two hash slots, route_slots) followed by the slots' dense indices. A routed
    // region's requests get bin lo_bins + idx[slot], every other request its high digit; the upsweep stores each request's
    // digit in `digit`, the scatter reads it back, and routed records go straight to
    // rec_out_route (the final record array) at their pass-0 position, skipping pass 1.
    const uint32_t* route_list;
    uint32_t lo_bins;
    void* rec_out_route;
    uint16_t* digit;           // [n]: pass-0 digit per request (routing only)
    const uint32_t* n_dev;     // pass 1: records to partition, on device (the normal ones)
};

struct HotInfo;

struct RegionArgs {
    const void* rec;           // records in region order
    const uint32_t* rstart;    // [bins] first record of each bin
    const uint32_t* rcount;    // [bins]
    const uint8_t* region_lim; // [P]
    const DevLimiter* lims;
    void* res;                 // packed results in region order (u32 compact, u64 wide)
    int64_t* ext;              // remaining of results stored as kResEscape (same positions)
    double* tok;               // nullable: TB fp64 balances in region order
    BatchCtl* ctl;
    uint32_t n_regions;        // one workgroup per region (= partition bin)
    uint32_t n_total;          // batch size: res/tok carry 64 padding entries past it
    int32_t shard_bits;
    uint32_t ablate;
    int64_t skew_ms;           // rl_opts.max_skew_ms: slots kept until dead at batch min - skew
    unsigned long long* stats; // [kStatSlots][8] sharded batch counters (k_stats_reduce)
    uint32_t cache;            // some limiter keeps a local cache (k_regions<..., CACHE>)
    uint32_t sparse_max;       // one region per bin: a region with <= this many records
                               // probes single buckets in HBM instead of loading its image
    const uint32_t* rend;      // nullable: bin b holds records [rstart[b], rend[b]) (2 passes)
    // hot regions: k_hot_select lists the largest bins (>= hot_threshold
    // records, at most kHotMax); the k_hot_* kernels own them (hot_mark[bin] == epoch),
    // k_regions skips them.
    const uint32_t* hot_list;  // [kHotMax]
    const uint32_t* hot_count; // [0]: number listed
    const uint32_t* hot_mark;  // [bins] nullable
    uint32_t epoch;
    HotInfo* hot_info;         // [kHotMax]
    uint64_t* hot_summ;        // [chunks][8]: k_hot_summ's summary, then the chains' verdicts
                               // (words 0-3 the dominant key, 4-7 the second key)
    uint64_t* hot_summ2;       // [groups][8]: the same over 64 chunks (4096 records)
    uint32_t* hot_total;       // [0] chunks, [1] groups over the listed regions
    uint64_t* dbg;             // nullable (rl_tune "debug_regions"): per bin kDbgWords words
                               // {t_start, t_end, records, rounds, 4 x cycle counters}
    // nullable: dispatch order of the normal regions, largest size class first (block g runs
    // region order[g]; order[n_regions] = number of non-empty regions listed)
    const uint32_t* order;
    uint32_t order_prefix;     // that many of the smallest regions are dispatched first
    uint32_t chain_split;      // chains as two-wave workgroups (pass 2 beside pass 1; default)
    uint32_t chain_grid;       // workgroups of the chain launch (each loops over the hot list
                               // with that stride): sized on the host from an earlier batch's
                               // hot count, so a batch with no hot region launches few idle ones
    // routed hot regions (hot_list entries with kHotRoutedBit): region, first record, count
    const uint32_t* route_list;
    const uint32_t* route_start;
    const uint32_t* route_cnt;
    // Allow walks (nullable): per key of the first walk_regions() listed regions
    // (slot 2 * i + key), per ms of the batch's span, the first record (relative to the
    // region's start) of the key's plain acquires of 1 permit (.x) and of at most 2 (.y) in
    // that ms; kWalkNone = none. Built by k_hot_summ, read by the chains (hot_chain, walk).
    uint2* walk_tab;
    uint32_t walk_min;         // walked keys expect at least this many allows (walk_dense)
};
constexpr int kMaxShards = 64;              // routing: shards per router
// Hot-key owner directory (rl_set_owner_directory): at most kDirMax keys in kDirSlots slots.
constexpr uint32_t kDirSlots = 8192;
constexpr uint32_t kDirMax = 4096;
constexpr uint32_t kDirEmpty = 0xFFFFFFFFu;
struct DirSlot { uint64_t tag; uint32_t owner; uint32_t pad; };
constexpr uint32_t kHotMax = 1024;       // hot regions per batch (<= one k_hot_scan block)
// Allow walks: one table per key of the listed hot regions (slot 2 i + key), each over the
// batch's time span (at most kWalkSpan ms) rounded up to 64 entries: 512 MiB hold 256 regions'
// tables at the longest span, all 1024 at a span up to 32 s.
constexpr uint32_t kWalkSpan = 1u << 17;
constexpr uint32_t kWalkNone = 0xFFFFFFFFu;
// A chain's allows are a dependent sequence (~4K cycles each on the chunk path): below a few
// thousand of them the chain ends before the normal regions drain and a walk only adds its
// table build and verdict fills (sw_zipf: 1000/min keys, ~1-3K allows, +0.3 ms/step walked).
constexpr uint32_t kWalkMinAllows = 4000;
constexpr size_t kWalkTabEntries = (size_t)1 << 26;
__host__ __device__ inline uint32_t walk_stride(int64_t lo, int64_t hi) {
    return (uint32_t)((hi - lo + 64) & ~(int64_t)63);
}
// listed regions with tables (the first ones of the hot list)
__host__ __device__ inline uint32_t walk_regions(int64_t lo, int64_t hi) {
    if (hi < lo || (uint64_t)(hi - lo) >= kWalkSpan) return 0;
    const size_t r = kWalkTabEntries / (2 * (size_t)walk_stride(lo, hi));
    return r < kHotMax ? (uint32_t)r : kHotMax;
}
// hot_list layout: [kHotMax] list, then the selection's meta words: [0] listed count,
// [1 .. 33] size-class histogram, [kHotClassCursor ..+33] per-class list cursors, then
// [kHotTotalOff .. +2] chunk / group totals (k_hot_scan), [kHotRoutedOff] routed entries
// listed first (k_hot_route_list).
constexpr uint32_t kHotClassCursor = 34;
constexpr uint32_t kHotTotalOff = 68;
constexpr uint32_t kHotRoutedOff = 70;
constexpr uint32_t kHotMetaWords = 71;   // zeroed before every batch
constexpr uint32_t kHotListWords = kHotMax + 72;
// A hot_list entry with this bit names route slot (entry & ~bit), not a normal bin.
constexpr uint32_t kHotRoutedBit = 0x80000000u;
// Hot-region routing: at most kRouteMax regions (the previous batch's largest hot regions)
// get pass-0 bins of their own, one per slot of a kRouteSlots-entry table in which a region
// sits at one of its two hash slots (route_slots): a lookup is two independent reads.
constexpr uint32_t kRouteMax = 512;
constexpr uint32_t kRouteSlots = 2048;
// Routed regions get DENSE pass-0 bins: slot s's region goes to bin lo_bins + idx[s] (idx =
// the number of occupied slots before s, written by k_route_next after the ids, at
// route_list + kRouteSlots), so pass 0 has 2^dh + kRouteBins bins instead of 2^dh + the
// 2048 slots (k_route_next places at most kRouteMax + 127 regions).
constexpr uint32_t kRouteBins = 1024;
static_assert(kRouteMax + 128 <= kRouteBins, "k_route_next places up to kRouteMax + 127");
constexpr uint32_t kRouteWords = 2 * kRouteSlots;   // a route table: ids, then dense indices
__host__ __device__ inline void route_slots(uint32_t region, uint32_t& s1, uint32_t& s2) {
    s1 = (region * 0x9E3779B1u) >> 21;
    s2 = ((region ^ 0x5BD1E995u) * 0x85EBCA6Bu) >> 21;
}
constexpr uint32_t kHotChunk = 64;       // records per summary chunk (one wave)
constexpr uint32_t kDbgWords = 28;       // debug words per bin
// Batch counters are sharded: one device-scope atomic word sustains only ~88 adds per us
// (MI355X_MICROARCH.md, rows 'dequeue' / 'fanin'), and every region wave adds to them, so a
// 1.3M-region batch on ONE set of words serialises for >10 ms. Region waves add to slot
// (block id mod kStatSlots), one 64-B line per slot; k_stats_reduce folds them into BatchCtl.
constexpr uint32_t kStatSlots = 1024;
enum : uint32_t { kStAllowed = 0, kStInvalid, kStCapErr, kStDistinct, kStRegions, kStCacheHits,
                  kStTableBytes, kStCount, kStWords = 8 };

struct HotInfo {             // one listed hot region
    uint64_t tag;            // its dominant key (mix64 of the key hash)
    uint32_t bin;
    uint32_t start, end;     // records [start, end) in bin order
    uint32_t n_chunks;       // ceil((end - start) / kHotChunk)
    uint32_t chunk_base;     // index of its first chunk summary
    uint32_t ok;             // bit 0: dominant key seen at least twice in the sample;
                             // bit 1: a second key heavy enough for a chain of its own
    uint32_t n_groups;       // ceil(n_chunks / 64)
    uint32_t group_base;     // index of its first group summary
    uint64_t tag2;           // a second dominant key (ok bit 1): its own chain wave
};

// Two-pass batches, after pass 0 (which partitions by the high digit of the region id):
// k_gtiles / k_gcount / k_gscan / k_gplace group each normal pass-0 bin's records by region
// inside the bin's own range of the final record array (rstart / rend per region, pos_out
// per pass-0 position). A bin is cut into tiles of tile_recs records, one wave each.
struct GroupArgs {
    const void* rec_in;        // pass-0 records (bin-major, arrival order inside each bin)
    void* rec_out;             // the final record array (region-major)
    uint32_t* pos_out;         // [n_normal]: final position of pass-0 position j
    const uint32_t* bin_base;  // [n_bins0] pass-0 scan: first record of each normal bin
    const uint32_t* bin_total; // [n_bins0]
    uint32_t* rstart;          // [n_regions] first record of each region (final order)
    uint32_t* rend;            // [n_regions]
    const DevLimiter* lims;
    uint32_t n_lim;
    int32_t shard_bits;
    uint32_t n_bins0;          // normal pass-0 bins (2^dh)
    uint32_t sub_bits;         // s0: regions per pass-0 bin = 2^s0 (region id = bin << s0 | sub)
    uint32_t n_regions;
    uint32_t tile_recs;        // records per tile (one wave counts, then places, a tile)
    uint32_t max_tiles;        // tiles the scratch holds (ceil(n / tile_recs) + n_bins0)
    uint32_t* tile_base;       // [n_bins0 + 1] first tile of each bin; [n_bins0] = tiles
    uint32_t* tile_bin;        // [max_tiles] bin of each tile
    uint32_t* tcount;          // [max_tiles][2^s0] per-tile region counts, then cursors
    // segmented pass 0 (nullable): bin b's records in n_segs runs, [seg_start, + seg_cnt)
    // (b * n_segs + s); tiles then never cross a run: tile_beg / tile_end [max_tiles]
    const uint32_t* seg_start;
    const uint32_t* seg_cnt;
    uint32_t n_segs;
    uint32_t* tile_beg;
    uint32_t* tile_end;
    uint32_t pad;              // the batch size: rec_out / pos_out hold 64 padding entries past it
    uint32_t ablate;           // rl_tune("ablate") (measurement only)
};
// records per tile of the grouping: 8192, or 32 per region of a bin when bins are wide
__host__ __device__ inline uint32_t group_tile_recs(uint32_t sub_bits) {
    const uint32_t t = 32u << sub_bits;
    return t > 8192u ? t : 8192u;
}

struct UnpermArgs {
    const uint32_t* pos0;
    const uint32_t* pos1;      // nullable
    const void* res;
    const void* res_hi;        // (set by launch_unpermute) two-pass: results at positions >=
                               // ctl->n_normal (routed records), read in place
    const double* tok;         // nullable
    void* mid;                 // nullable: n results of scratch (two-pass batches)
    const int64_t* ext;        // escaped remainders, indexed like res (before `mid`)
    const BatchCtl* ctl;       // n_esc > 0: fix the escaped results up after the gather
    const void* res_final;     // (set by launch_unpermute) res and pos1 as the region stage
    const uint32_t* pos1_final;//  left them, for the escape fix-up
    uint8_t* allowed;
    int64_t* remaining;
    double* tokens_out;        // nullable
    uint32_t n;
    uint32_t n_tiles;
    uint32_t ablate;
    uint32_t per_cu;           // persistent-grid workgroups per CU (0: default)
    uint32_t split;            // rl_tune("unpermute_split"): gathers and stores in separate waves
    uint32_t mid_xcd;          // rl_tune("mid_xcd"): k_unpermute_mid's blocks XCD-aware
};

struct SynthArgs {
    uint64_t seed;
    uint64_t n_keys;
    int32_t dist;
    int32_t permits_max;
    int64_t t0_ns;
    int64_t span_ns;
    uint64_t index_base;
    uint64_t n_total;
    uint32_t n_limiters;
    // Zipf rejection-inversion constants (host-computed)
    double zs, hx1, hn, sconst;
    uint64_t* key;
    int32_t* permits;
    int64_t* now_ns;
    uint16_t* limiter;
    uint64_t n;
};

// State export / import (rl_export_state / rl_import_state). StateRec has the layout of
// rl_state_entry (include/rl_engine.h; static_assert in rl_engine.cpp).
struct StateRec {
    uint64_t key_hash;
    uint16_t limiter;
    uint8_t kind;
    uint8_t reserved[5];
    int64_t window_start_ms, count;
    double tokens;
    int64_t last_refill_ms, expire_at_ms;
};
struct ImportArgs {
    uint32_t n_groups;
    const uint32_t* group_off;     // [n_groups + 1] into img
    const uint64_t* region_addr;   // [n_groups] device address of the region's 256 slots
    const uint64_t* xregion_addr;  // [n_groups] its local-cache words (0: none)
    const uint8_t* group_algo;     // [n_groups]
    const Slot* img;               // slot images, grouped by region
    uint32_t* fail;                // keys that found no free slot
};

hipError_t launch_export(const Slot* table, uint64_t n_slots, const DevLimiter& L, uint16_t lim,
                         int64_t now_ms, StateRec* out, uint32_t cap, uint32_t* count,
                         hipStream_t s);
hipError_t launch_import(const ImportArgs& a, hipStream_t s);
hipError_t launch_grow(const Slot* old_tab, const uint64_t* old_x, Slot* new_tab, uint64_t* new_x,
                       uint64_t n_old_regions, int shard_bits, int k_new, int algo, hipStream_t s);
hipError_t launch_sweep(Slot* table, uint64_t n_slots, const DevLimiter& L, int64_t now_ms,
                        uint32_t* count, hipStream_t s);

hipError_t launch_upsweep(const PartArgs& a, bool raw, bool wide, hipStream_t s);
hipError_t launch_scatter(const PartArgs& a, bool raw, bool wide, hipStream_t s);
hipError_t launch_scan_rows(const uint32_t* in, uint32_t* out, uint32_t rows, uint32_t cols,
                            uint32_t* totals, hipStream_t s);
hipError_t launch_scan_small(const uint32_t* in, uint32_t* out, uint32_t len, hipStream_t s);
hipError_t launch_add_rows(const uint32_t* row_base, uint32_t* data, uint32_t rows,
                           uint32_t cols, hipStream_t s);
// The hot chains (k_hot_chains) on the side stream hs after event e0 on s, launched before
// the region-order and solo kernels so that their single waves (one SIMD's registers each)
// are dispatched ahead of the normal regions' ~10^6 waves; launch_region then runs the
// normal regions on s and (hs non-null) joins hs by event e1.
hipError_t launch_chains(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s,
                         hipStream_t hs, hipEvent_t e0);
hipError_t launch_region(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s,
                         hipStream_t hs = nullptr, hipEvent_t e1 = nullptr);
// per record codec / packed result width (instantiated in csrc/rl_rt_*.hip)
template <class Codec, class Res>
hipError_t chains_launch_t(const RegionArgs& a, hipStream_t s, hipStream_t hs, hipEvent_t e0);
template <class Codec, class Res>
hipError_t region_launch_t(const RegionArgs& a, hipStream_t s, hipStream_t hs, hipEvent_t e1);
template <class Codec, class Res> hipError_t hot_chains_t(const RegionArgs& a, hipStream_t hs);
template <class Codec, class Res> hipError_t hot_fill_t(const RegionArgs& a, hipStream_t s);
hipError_t launch_stats_reduce(unsigned long long* stats, BatchCtl* ctl, hipStream_t s);
// Single-key allow runs of cache-on sliding-window regions (rl_solo.hip): regions with >= thr
// records are listed (at most kSoloMax), then k_solo decides each one's leading allow run and
// moves its start (rstart / rcount) past it, before the region stage.
constexpr uint32_t kSoloMax = 4096;
constexpr uint32_t kSoloGrid = 256;
hipError_t launch_solo_select(const uint32_t* rstart, const uint32_t* rcount, const uint32_t* rend,
                              uint32_t n_bins, uint32_t thr, const DevLimiter* lims,
                              const uint8_t* region_lim, uint32_t* list, uint32_t* count,
                              hipStream_t s);
hipError_t launch_solo(const RegionArgs& a, bool wide, int res_bytes, uint32_t* rstart, uint32_t* rcount,
                       const uint32_t* list, const uint32_t* count, hipStream_t s);
hipError_t launch_hot_prepare(const RegionArgs& a, bool wide, hipStream_t s);   // prep, scan, summaries
hipError_t launch_hot_fill(const RegionArgs& a, bool wide, int res_bytes, hipStream_t s);
hipError_t launch_hot_select(const uint32_t* rstart, const uint32_t* rcount, const uint32_t* rend,
                             uint32_t n_bins, uint32_t threshold, uint32_t* hot_list,
                             uint32_t* hot_count, uint32_t* hot_mark, uint32_t epoch,
                             const DevLimiter* lims, const uint8_t* region_lim, hipStream_t s);
hipError_t launch_group(const GroupArgs& a, bool wide, hipStream_t s);
// Routing: after the pass-0 scan, copy the routed bins' ranges (before pass 1 reuses the scan
// arrays) and set ctl->n_normal; after the hot selection, list the routed regions first; after
// the batch's hot preparation, the next batch's route list (largest listed regions >= thr).
// Segmented pass 0: from the row-scanned counts, each (bin, segment)'s start in the
// pass-0 array (normal bins segment-major, routed bins bin-major as before) and count.
hipError_t launch_seg_base(const uint32_t* counts, const uint32_t* bin_total,
                           const uint32_t* bin_base, uint32_t bins, uint32_t lo_bins,
                           uint32_t n_tiles, uint32_t seg_tiles, uint32_t n_segs,
                           uint32_t* seg_adj, uint32_t* seg_start, uint32_t* seg_cnt, hipStream_t s);
hipError_t launch_route_ranges(const uint32_t* route_list, const uint32_t* bin_base,
                               const uint32_t* bin_total, uint32_t lo_bins, uint32_t* route_start,
                               uint32_t* route_cnt, BatchCtl* ctl, hipStream_t s);
hipError_t launch_hot_route_list(const uint32_t* route_list, const uint32_t* route_cnt,
                                 uint32_t* hot_list, uint32_t* hot_meta, hipStream_t s);
// Normal-region dispatch order, largest power-of-two size class first (regions are
// independent; a big region dispatched last would set the stage's tail). meta: kOrderMeta
// words, zeroed by the launcher; order: [n_bins + 1].
constexpr uint32_t kOrderMeta = 72;
hipError_t launch_region_order(const uint32_t* rstart, const uint32_t* rcount, const uint32_t* rend,
                               uint32_t n_bins, uint32_t* meta, uint32_t* order, hipStream_t s);
hipError_t launch_route_next(const HotInfo* hot_info, const uint32_t* hot_count, uint32_t threshold,
                             uint32_t* route_list, hipStream_t s);
hipError_t launch_unpermute(const UnpermArgs& a, int res_bytes, hipStream_t s);
hipError_t launch_fill_invalid(uint8_t* allowed, int64_t* remaining, double* tok, uint32_t n,
                               hipStream_t s);
hipError_t launch_synth(const SynthArgs& a, hipStream_t s);
hipError_t launch_owner_partition(const uint64_t* key, uint32_t n, uint32_t shard_count,
                                  uint32_t* perm, uint32_t* counts_dev, uint32_t* scratch,
                                  const DirSlot* dir, hipStream_t s);

hipError_t launch_route_pack(uint32_t n, const uint32_t* perm, const uint64_t* key,
                             const int32_t* permits, const int64_t* now, const uint16_t* lim,
                             uint64_t* key_o, int32_t* permits_o, int64_t* now_o, uint16_t* lim_o,
                             hipStream_t s);
hipError_t launch_route_fold(uint32_t n, const uint8_t* allowed, const int64_t* remaining,
                             int64_t* packed, hipStream_t s);
hipError_t launch_route_unpack(uint32_t n, const uint32_t* perm, const int64_t* packed,
                               uint8_t* allowed, int64_t* remaining, hipStream_t s);
// part (nullable, >= 2 * kWireBlocksMax u64): per-block now_ms min / max partials for the
// router header; *nparts (nullable) = blocks launched.
constexpr uint32_t kWireBlocksMax = 2048;
hipError_t launch_route_pack_wire(uint32_t n, const uint32_t* perm, const uint64_t* key,
                                  const int32_t* permits, const int64_t* now, const uint16_t* lim,
                                  uint64_t* wire, uint16_t* lim_o, int64_t* hdr, hipStream_t s,
                                  uint64_t* part = nullptr, uint32_t* nparts = nullptr);
hipError_t launch_route_unwire(uint32_t m, const uint64_t* wire, uint32_t n_src, const int64_t* base,
                               const uint32_t* end, uint64_t* key_o, int32_t* permits_o,
                               int64_t* now_o, hipStream_t s);
hipError_t launch_route_fold_w(uint32_t n, const uint8_t* allowed, const int64_t* remaining,
                               void* packed, int width, hipStream_t s);
hipError_t launch_route_unpack_w(uint32_t n, const uint32_t* perm, const void* packed, int width,
                                 uint8_t* allowed, int64_t* remaining, hipStream_t s);
// Segmented return trip (rl_route_fold_return / rl_route_unpack_return).
inline uint64_t ret_block_bytes(uint32_t cap) { return 8 + 16 * (uint64_t)cap; }
// off[s] / end[s] of segment s for counts[0..n_seg) requests of `width` bytes; returns the
// total bytes (every segment: its packed results padded to 8 B, then its exception block).
inline uint64_t ret_layout(const uint64_t* counts, uint32_t n_seg, int width, uint32_t cap,
                           uint64_t* off, uint32_t* end) {
    uint64_t o = 0, e = 0;
    for (uint32_t s = 0; s < n_seg; ++s) {
        if (off) off[s] = o;
        e += counts[s];
        if (end) end[s] = (uint32_t)e;
        o += ((counts[s] * (uint64_t)width + 7) & ~7ULL) + ret_block_bytes(cap);
    }
    return o;
}
hipError_t launch_route_fold_ret(uint32_t m, const uint8_t* allowed, const int64_t* remaining,
                                 void* out, int width, uint32_t n_seg, const uint64_t* counts,
                                 uint32_t cap, hipStream_t s);
hipError_t launch_route_unpack_ret(uint32_t n, const uint32_t* perm, const void* in, int width,
                                   uint32_t n_seg, const uint64_t* counts, uint32_t cap,
                                   uint8_t* allowed, int64_t* remaining, uint32_t* lost,
                                   hipStream_t s);
hipError_t launch_counts_to_header(const uint32_t* counts, uint32_t g, int64_t* hdr, uint32_t stride,
                                   hipStream_t s);
// Router header: kHdrWords int64 per peer row: kHdrFixed fixed words, then the source's
// request count for every owner (so every rank knows the whole count matrix).
constexpr uint32_t kHdrFixed = 8;
constexpr uint32_t kHdrWords = kHdrFixed + kMaxShards;
hipError_t launch_fill_header(int64_t* hdr, const int64_t* base_ovf, int64_t status, int64_t cap,
                              int64_t rcap, uint32_t g, const uint64_t* part, uint32_t nparts,
                              hipStream_t s);
hipError_t launch_fill_value(uint8_t* allowed, int64_t* remaining, uint32_t n, int64_t rem,
                             hipStream_t s);
// acc[0] |= status flags (1 invalid, 2 capacity, 4 span overflow, 8 internal) of ctl (nullable)
// and `flags`; acc[1..4] |= ctl->grow
constexpr uint32_t kStatusAccWords = 5;
hipError_t launch_status_accum(const BatchCtl* ctl, unsigned long long flags, unsigned long long* acc,
                               hipStream_t s);

// internal helpers of rl_engine.cpp for rl_router.cpp (not part of the C-ABI)
int route_pack_wire_mm(rl_engine* e, size_t n, const uint32_t* perm, const uint64_t* key,
                       const int32_t* permits, const int64_t* now_ns, const uint16_t* limiter,
                       uint64_t* wire_out, uint16_t* limiter_out, int64_t* hdr, uint64_t* part,
                       uint32_t* nparts, void* stream);
int engine_device(rl_engine* e);
size_t engine_max_batch(rl_engine* e);
// Split router rounds: fold the engine's last batch status into acc on `stream` (after that
// batch), and later settle the folded status of several batches at a step boundary: the
// status those batches return together, with the table growth they asked for applied once.
int engine_status_accum(rl_engine* e, unsigned long long* acc, void* stream);
int engine_status_settle(rl_engine* e, const unsigned long long* acc_host);

}  // namespace rl
