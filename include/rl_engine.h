/*
 * rl_engine.h — C-ABI of the MI355X batched rate-limit decision engine.
 *
 * This is the drop-in boundary that replaces the reference's
 * algorithm + storage pair beneath its unchanged Java `RateLimiter` interface:
 *
 *   reference interface                                  replaced by
 *   ---------------------------------------------------  -----------------------------
 *   RateLimiter.tryAcquire(String)                        rl_try_acquire_batch (permits=1)
 *     core/RateLimiter.java:16
 *   RateLimiter.tryAcquire(String,int)                    rl_try_acquire_batch
 *     core/RateLimiter.java:26
 *     algorithms/SlidingWindowRateLimiter.java:85-131
 *     algorithms/TokenBucketRateLimiter.java:105-143 (+ Lua :38-68)
 *   RateLimiter.getAvailablePermits(String)               rl_available
 *     core/RateLimiter.java:35, SlidingWindowRateLimiter.java:133-137,
 *     TokenBucketRateLimiter.java:145-151
 *   RateLimiter.reset(String)                             rl_reset
 *     core/RateLimiter.java:43, SlidingWindowRateLimiter.java:139-153,
 *     TokenBucketRateLimiter.java:153-158
 *   new SlidingWindowRateLimiter(storage, config, reg)    rl_add_limiter(RL_ALGO_SLIDING_WINDOW, ...)
 *     SlidingWindowRateLimiter.java:46-78
 *   new TokenBucketRateLimiter(storage, config, reg)      rl_add_limiter(RL_ALGO_TOKEN_BUCKET, ...)
 *     TokenBucketRateLimiter.java:70-97
 *   RateLimitConfig.validate()                            rl_add_limiter argument checks
 *     core/RateLimitConfig.java:46-56
 *   RedisRateLimitStorage (JedisPool, Redis keyspace)     rl_create / rl_destroy (HBM state table)
 *     storage/RedisRateLimitStorage.java:22-35
 *
 * Everything is plain C: pointers + sizes, no C++ types, no exceptions. Every
 * entry point returns an int status (RL_OK = 0, < 0 on error). The JNI / FFM
 * bindings that a Java maintainer adds on top are shown in INTEGRATION.md.
 *
 * Semantics (bit-exact with the reference):
 *  - key_hash is the caller's 64-bit hash of the String key (hashing happens on
 *    the JVM side). State is kept per (limiter id, key_hash).
 *  - now_ns is converted to milliseconds as floorDiv(now_ns, 1e6); the reference
 *    reads System.currentTimeMillis().
 *  - Requests of one batch are applied in array (arrival) order per key.
 *    Sliding-window state requires per-key non-decreasing now_ms (in-order
 *    replay of a wall-clock trace); token-bucket state has no such requirement.
 *  - A denied request never changes state (SlidingWindowRateLimiter.java:104-111,
 *    TokenBucketRateLimiter.java:61-67,110-116).
 */
#ifndef RL_ENGINE_H
#define RL_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RL_ABI_VERSION 3

/* ---- status codes -------------------------------------------------------- */
#define RL_OK                   0
#define RL_E_INVALID_ARG      (-1)  /* bad argument to an entry point; IllegalArgumentException on the Java side */
#define RL_E_INVALID_REQUEST  (-2)  /* >=1 request had permits <= 0 or an unknown limiter id (others were applied) */
#define RL_E_CAPACITY         (-3)  /* a state-table region overflowed; affected requests report RL_REMAINING_ERROR */
#define RL_E_DEVICE           (-4)  /* HIP runtime / device failure; StorageException on the Java side */
#define RL_E_NOMEM            (-5)  /* device or host allocation failed */
#define RL_E_TOO_LARGE        (-6)  /* batch larger than rl_opts.max_batch */
#define RL_E_LIMITERS         (-7)  /* too many limiters / table space exhausted */
#define RL_E_INTERNAL         (-8)  /* a kernel met a state its logic excludes (an engine bug,
                                       not a capacity or input problem): the hot chains' allow
                                       walk found an allow in a chunk it had already decided, or
                                       exceeded its step bound. The batch's results for the keys
                                       involved are suspect; report it as a defect. */

/* ---- algorithms ---------------------------------------------------------- */
#define RL_ALGO_SLIDING_WINDOW 0    /* algorithms/SlidingWindowRateLimiter.java */
#define RL_ALGO_TOKEN_BUCKET   1    /* algorithms/TokenBucketRateLimiter.java   */

/* ---- per-request operation (rl_execute_batch) ----------------------------- */
#define RL_OP_ACQUIRE 0             /* tryAcquire(key, permits)     */
#define RL_OP_PEEK    1             /* getAvailablePermits(key)     */
#define RL_OP_RESET   2             /* reset(key)                   */

/* ---- sentinel values of `remaining` --------------------------------------- */
#define RL_REMAINING_UNKNOWN  (-1)  /* TB permits > maxPermits: "unable to determine" (RateLimiter.java:33) */
#define RL_REMAINING_INVALID  (-2)  /* permits <= 0 or unknown limiter (IllegalArgumentException in Java)   */
#define RL_REMAINING_ERROR    (-3)  /* request not applied: state-table region full (RL_E_CAPACITY)         */

/* ---- limits of this implementation (checked by rl_add_limiter) ------------ */
#define RL_MAX_LIMITERS         255
#define RL_SW_MAX_PERMITS_LIMIT 2147483646LL        /* SW counts kept as u32 */
#define RL_TB_MAX_PERMITS_LIMIT 9007199254740992LL  /* 2^53: Lua numbers are IEEE doubles */
#define RL_MAX_WINDOW_MS        1073741823LL        /* ~12.4 days; bucket offsets kept as i32 */

typedef struct rl_engine rl_engine;

typedef struct rl_opts {
    int32_t  device;            /* HIP device ordinal (-1: current device)                  */
    uint32_t flags;             /* RL_OPT_* bits                                            */
    uint64_t max_batch;         /* largest n accepted by the batch entry points             */
    uint64_t default_capacity;  /* expected live keys per limiter when rl_add_limiter is used */
    uint32_t shard_index;       /* multi-GPU: this engine owns keys with owner(h) == shard   */
    uint32_t shard_count;       /* multi-GPU: number of shards (power of two, 1 = no sharding) */
    int64_t  max_skew_ms;       /* how far a request may lag behind the earliest request of an
                                   EARLIER batch (front-ends with skewed clocks); state is kept
                                   until it is dead that long before a batch's earliest now.
                                   0: batches arrive in global time order */
} rl_opts;

#define RL_OPT_STAGE_TIMING 0x1u  /* record hipEvents around every stage (rl_stage_times) */
/* Pipelined device batches: the partition of a batch (stages 1-3) runs on a second engine
 * stream into one of two scratch sets, so it overlaps the previous batch's decision stage;
 * decisions are still applied in submission order. It applies to rl_execute_batch_device
 * calls with stream == NULL, whose inputs must then be complete when the call is made
 * (results are complete when rl_sync / rl_last_status return). Calls with a stream and the
 * host-buffer calls are ordered as without the option. Scratch memory doubles. */
#define RL_OPT_PIPELINE     0x2u
/* Fixed-size state tables. By default a limiter's table grows on demand, as the Redis
 * keyspace does (RedisRateLimitStorage.java:38-49): when a batch leaves one of its regions
 * more than 62.5 % full (or overflows one: those requests report RL_REMAINING_ERROR and the
 * batch RL_E_CAPACITY), the region count doubles (twice after an overflow) when the batch's
 * status is collected (rl_last_status, the host-buffer calls). */
#define RL_OPT_FIXED_CAPACITY 0x4u

#define RL_LIM_LOCAL_CACHE 0x1u  /* RateLimitConfig.enableLocalCache (RateLimitConfig.java:37-38) */

typedef struct rl_limiter_config {
    int32_t  algo;              /* RL_ALGO_*                                                  */
    uint32_t flags;             /* RL_LIM_* bits                                              */
    int64_t  max_permits;       /* RateLimitConfig.maxPermits (RateLimitConfig.java:19)       */
    int64_t  window_ms;         /* RateLimitConfig.window.toMillis() (RateLimitConfig.java:24) */
    double   refill_per_s;      /* RateLimitConfig.refillRate (RateLimitConfig.java:31); TB only */
    uint64_t capacity;          /* expected live keys (table sizing); 0 = rl_opts.default_capacity */
    int64_t  local_cache_ttl_ms;/* RateLimitConfig.localCacheTtl (RateLimitConfig.java:43-44);
                                   with RL_LIM_LOCAL_CACHE on a sliding window the engine
                                   emulates SlidingWindowRateLimiter's Caffeine cache
                                   (:57-64,93-121,148-150) deterministically in trace time:
                                   expireAfterWrite(ttl) at ms resolution, no size eviction
                                   (exact while <= 10k keys are cached, maximumSize(10000)).
                                   Token buckets have no cache (TokenBucketRateLimiter). */
} rl_limiter_config;

typedef struct rl_batch_stats {
    uint64_t n;                 /* requests in the last batch                                 */
    uint64_t allowed;           /* requests allowed                                           */
    uint64_t distinct_keys;     /* U: distinct (limiter, key) touched (for the roofline)      */
    uint64_t invalid;           /* requests rejected as invalid                               */
    uint64_t capacity_errors;   /* requests not applied because a region was full            */
    uint64_t regions_touched;   /* state-table regions loaded + written back                  */
    uint64_t table_bytes;       /* state-table bytes read + written by the batch (whole 8 KB
                                   region images both ways; sparse regions: the 128-B buckets
                                   faulted in + the 32-B slots written back)                  */
    uint64_t cache_hits;        /* SW local-cache rejections (ratelimiter.cache.hits,
                                   SlidingWindowRateLimiter.java:75-77,96)                  */
    uint64_t table_grows;       /* region-count doublings so far (on-demand table growth)   */
    uint64_t hot_regions;       /* regions decided by the hot-key chains in the last batch   */
    uint64_t routed;            /* requests of the last batch routed straight to their final
                                   partition in pass 0 (the previous batch's hot regions)    */
} rl_batch_stats;

/* Create / destroy an engine on one GPU. Replaces the JedisPool + Redis keyspace
 * (RedisRateLimitStorage.java:22-35). */
int  rl_create(const rl_opts* opts, rl_engine** out);
void rl_destroy(rl_engine* e);

/* Register a limiter; mirrors the constructors SlidingWindowRateLimiter.java:46-78 /
 * TokenBucketRateLimiter.java:70-97 (config.validate() + refillRate > 0 for TB).
 * The id is the `limiter` value used in the batch calls. */
int  rl_add_limiter(rl_engine* e, int algo, int64_t max_permits, int64_t window_ms,
                    double refill_per_s, uint16_t* id);
int  rl_add_limiter_ex(rl_engine* e, const rl_limiter_config* cfg, uint16_t* id);

/* Grow a limiter's state table (doubling its regions, live state kept) until it holds
 * min_keys keys at load <= 0.5; rl_limiter_slots reports its current slot count. */
int  rl_grow_limiter(rl_engine* e, uint16_t limiter, uint64_t min_keys);
int  rl_limiter_slots(rl_engine* e, uint16_t limiter, uint64_t* slots);

/* tryAcquire over a batch of HOST buffers (pageable or pinned).
 *   allowed[i]      1 if request i acquired its permits
 *   remaining[i]    SW: max(0, max - estimate) at now_i after applying request i
 *                   TB: (long) token balance returned by the Lua script, -1 if permits > max
 *   tokens_after[i] TB: the fp64 balance returned by the script (NaN otherwise); may be NULL
 * `limiter` may be NULL (all requests use limiter 0). Returns RL_E_INVALID_REQUEST if
 * any request was invalid (those report RL_REMAINING_INVALID; the rest are applied). */
int  rl_try_acquire_batch(rl_engine* e, size_t n,
                          const uint64_t* key_hash, const int32_t* permits,
                          const int64_t* now_ns, const uint16_t* limiter,
                          uint8_t* allowed, int64_t* remaining, double* tokens_after);

/* Page-lock (hipHostRegister) a caller-owned host buffer that is reused across batches,
 * so the host-buffer entry points above and below DMA it directly instead of staging it
 * through pageable bounce buffers (the JNI side pins its direct ByteBuffers once, see
 * INTEGRATION.md). Already page-locked memory is accepted as is. rl_unpin_host must be
 * called before the buffer is freed; rl_destroy unpins whatever is left. */
int  rl_pin_host(rl_engine* e, void* ptr, size_t bytes);
int  rl_unpin_host(rl_engine* e, void* ptr);

/* Mixed operations (RL_OP_*) over host buffers; `op` may be NULL (all ACQUIRE). */
int  rl_execute_batch(rl_engine* e, size_t n,
                      const uint64_t* key_hash, const int32_t* permits,
                      const int64_t* now_ns, const uint16_t* limiter, const uint8_t* op,
                      uint8_t* allowed, int64_t* remaining, double* tokens_after);

/* Same as rl_execute_batch on DEVICE-resident buffers, enqueued on `stream`
 * (a hipStream_t; NULL = the engine's stream). Asynchronous: results are ready
 * when the stream completes; the status of the batch is then available from
 * rl_last_status(). Used by bench.py and the multi-GPU router (HBM-resident data). */
int  rl_execute_batch_device(rl_engine* e, size_t n,
                             const uint64_t* key_hash, const int32_t* permits,
                             const int64_t* now_ns, const uint16_t* limiter, const uint8_t* op,
                             uint8_t* allowed, int64_t* remaining, double* tokens_after,
                             void* stream);
int  rl_last_status(rl_engine* e);     /* synchronises the engine stream */

/* getAvailablePermits for n keys at now_ns[i] (host buffers). SW: max(0, max - estimate).
 * TB: (long) min(cap, tokens + elapsed*rate) without consuming (the reference's TB
 * getAvailablePermits is broken). */
int  rl_available(rl_engine* e, uint16_t limiter, size_t n, const uint64_t* key_hash,
                  const int64_t* now_ns, int64_t* available);

/* reset(key) for n keys at now_ns[i]: SW deletes the current and previous window
 * buckets; TB deletes the bucket. */
int  rl_reset(rl_engine* e, uint16_t limiter, size_t n, const uint64_t* key_hash,
              const int64_t* now_ns);

/* Observability. */
int  rl_batch_stats_get(rl_engine* e, rl_batch_stats* out);
/* Milliseconds of each pipeline stage of the last batch (needs RL_OPT_STAGE_TIMING);
 * names[i] are static strings. Returns the number of stages written (<= cap). */
int  rl_stage_times(rl_engine* e, const char** names, float* ms, int cap);
int  rl_sync(rl_engine* e);
/* Tuning / measurement knobs (not needed by callers): "ablate" = bit set of
 * measurement-only kernel variants whose results are NOT valid (0 = product path);
 * "hot_threshold" (records per region for the hot-key chains, 0 = off), "route" (two-pass
 * tables: the previous batch's hot regions skip the second partition pass, default 1),
 * "region_order" (largest regions dispatched first, default 1), "walk" (the hot chains' allow
 * walk, default 1), "walk_min" (keys walked: at least this many allows expected per batch,
 * default 4000), "chain_split" (hot chains as two-wave workgroups, default 1), "group_bits"
 * (two-pass batches: bits of the pass-0 digit, default 12; the local grouping resolves the
 * rest), "segments" (two-pass batches: pass-0 output in that many tile segments, default 1),
 * "tile_items" (partition tile = value x 512 requests; 0 = by batch size), "sparse_max",
 * "stage_timing", "debug_regions" and the "*_per_cu" grid sizes.
 * Every setting gives the same decisions. "fail_batches" = k makes the next k batch
 * calls fail with RL_E_DEVICE before enqueuing anything (tests of callers' error paths). */
int  rl_tune(rl_engine* e, const char* key, int64_t value);
/* Diagnostics (not needed by callers). "region_times": after a batch run with
 * rl_tune("debug_regions", 1), copies per-bin {t_start, t_end, records, rounds, cycle
 * counters} (uint64 x28 per bin; s_memrealtime ticks; rounds bit 63 = a hot region).
 * Returns the number of bins copied (>= 0) or a status < 0. */
int  rl_debug_fetch(rl_engine* e, const char* what, void* out, size_t bytes);
const char* rl_strerror(int status);
int  rl_abi_version(void);

/* ---- state export / import in the Redis keyspace layout ----
 * The reference keeps all limiter state in Redis; these two calls move the engine's
 * state in and out in that same layout (checkpoint / migration / hybrid deploys).
 * One entry per live Redis key:
 *   RL_STATE_SW_BUCKET  "rl:<key>:<window_start>" counter
 *                       (SlidingWindowRateLimiter.java:185-188; INCR + PEXPIRE w,
 *                        RedisRateLimitStorage.java:38-49)
 *   RL_STATE_TB_BUCKET  "tb:<key>" hash {tokens, last_refill}
 *                       (TokenBucketRateLimiter.java:46-48,63-64; HMSET + PEXPIRE 2w)
 * expire_at_ms is the PEXPIRE deadline: the key is gone once now > expire_at_ms
 * (SW: last INCR + w; TB: last_refill + 2w). */
#define RL_STATE_SW_BUCKET 0
#define RL_STATE_TB_BUCKET 1
typedef struct rl_state_entry {
    uint64_t key_hash;
    uint16_t limiter;
    uint8_t  kind;              /* RL_STATE_*                                          */
    uint8_t  reserved[5];
    int64_t  window_start_ms;   /* SW: bucket start W (a multiple of w); TB: 0         */
    int64_t  count;             /* SW: counter value (>= 1); TB: 0                     */
    double   tokens;            /* TB: balance, the exact fp64 the Lua script stored   */
    int64_t  last_refill_ms;    /* TB: last_refill; SW: 0                              */
    int64_t  expire_at_ms;      /* PEXPIRE deadline                                    */
} rl_state_entry;               /* 56 bytes */

/* Every key live at now_ns (floorDiv to ms, as the batch calls), sorted by
 * (limiter, key_hash, window_start_ms). *n_out = number of live entries; when it
 * exceeds cap nothing is written and RL_E_TOO_LARGE is returned (retry with a larger
 * buffer). `out` is a host buffer. Only this engine's shard is exported. */
int  rl_export_state(rl_engine* e, int64_t now_ns, rl_state_entry* out, size_t cap,
                     size_t* n_out);
/* Load entries (host buffer) into the state table, replacing the state of every key
 * they name. A key's SW buckets are its newest bucket W and, if present, W - w (older
 * ones can never be read again and are dropped). Entries owned by another shard are
 * skipped; *n_imported (nullable) = entries taken. RL_E_INVALID_ARG: unknown limiter,
 * kind not matching the limiter's algorithm, or a deadline the reference could not
 * have set (TB: expire_at != last_refill + 2w; SW: outside [W + w, W + 2w)).
 * RL_E_CAPACITY: a region had no free slot (the other keys are imported). */
int  rl_import_state(rl_engine* e, const rl_state_entry* in, size_t n, size_t* n_imported);

/* Background TTL sweep (Redis active expiry of the PEXPIRE deadlines set at
 * RedisRateLimitStorage.java:41-44 and Lua :64): frees every slot none of whose buckets is live at
 * now_ns, so table memory tracks live keys even for regions no batch touches. (Batches already
 * drop dead slots of the regions they load.) now_ns must not exceed the now of any later request,
 * as with Redis's own clock. *reclaimed (nullable) = slots freed. */
int  rl_sweep_expired(rl_engine* e, int64_t now_ns, uint64_t* reclaimed);

/* ---- multi-GPU routing helpers (device buffers, engine stream) ------------
 * owner(key_hash) is the shard that holds the key's state. rl_route_partition
 * stably partitions a batch by owner: perm[j] = source index of the j-th request
 * in owner order, counts[s] = requests for shard s (host array of shard_count). */
uint32_t rl_owner_of(uint64_t key_hash, uint16_t limiter, uint32_t shard_count);
int  rl_route_partition(rl_engine* e, size_t n, const uint64_t* key_hash,
                        const uint16_t* limiter, uint32_t shard_count,
                        uint32_t* perm, uint64_t* counts_host, void* stream);
/* out[j] = in[perm[j]] for the four request arrays (limiter / limiter_out nullable). */
int  rl_route_pack(rl_engine* e, size_t n, const uint32_t* perm, const uint64_t* key_hash,
                   const int32_t* permits, const int64_t* now_ns, const uint16_t* limiter,
                   uint64_t* key_out, int32_t* permits_out, int64_t* now_out,
                   uint16_t* limiter_out, void* stream);
/* packed[j] = remaining[j] * 2 + allowed[j] (one int64 per decision for the return trip). */
int  rl_route_fold(rl_engine* e, size_t n, const uint8_t* allowed, const int64_t* remaining,
                   int64_t* packed, void* stream);
/* allowed[perm[j]], remaining[perm[j]] = unfold(packed[j]). */
int  rl_route_unpack(rl_engine* e, size_t n, const uint32_t* perm, const int64_t* packed,
                     uint8_t* allowed, int64_t* remaining, void* stream);

/* Compact wire (16 B per request, the default router layout): out in owner order,
 * wire_out[2j] = key_hash, wire_out[2j+1] = (uint32)permits << 32 | (now_ms - base_ms),
 * limiter_out[j] (nullable) = limiter id. hdr (device int64[2]) receives base_ms =
 * floorDiv(now_ns[0], 1e6) - 2^31 and an overflow flag (1: some now_ms outside
 * [base_ms, base_ms + 2^32); the router then sends that step in the wide layout). */
int  rl_route_pack_wire(rl_engine* e, size_t n, const uint32_t* perm, const uint64_t* key_hash,
                        const int32_t* permits, const int64_t* now_ns, const uint16_t* limiter,
                        uint64_t* wire_out, uint16_t* limiter_out, int64_t* hdr, void* stream);
/* Receiver side: m wire records from n_src sources (host arrays: each source's base_ms
 * and request count, in source order, summing to m) -> request SoA for the engine
 * (now_out = now_ms * 1e6; the engine reads now at ms resolution). */
int  rl_route_unwire(rl_engine* e, size_t m, const uint64_t* wire, uint32_t n_src,
                     const int64_t* src_base, const uint64_t* src_count, uint64_t* key_out,
                     int32_t* permits_out, int64_t* now_out, void* stream);
/* Width in bytes (1, 2, 4 or 8) of the engine's packed decision ((remaining + 3) << 1 |
 * allowed) for its current limiter set: 1 B for every maxPermits <= 124. */
int  rl_result_width(rl_engine* e);
/* packed[j] = (remaining[j] + 3) << 1 | allowed[j] in `width` bytes (return trip), and
 * its inverse scattered through perm: allowed[perm[j]], remaining[perm[j]]. */
int  rl_route_fold_packed(rl_engine* e, size_t n, const uint8_t* allowed, const int64_t* remaining,
                          void* packed, int width, void* stream);
int  rl_route_unpack_packed(rl_engine* e, size_t n, const uint32_t* perm, const void* packed,
                            int width, uint8_t* allowed, int64_t* remaining, void* stream);

/* Segmented return trip (the router's default): the decisions for peer s travel as
 *   [ packed results, seg_counts[s] x width bytes, padded to 8 B ][ exception block ]
 * with exception block = { u64 count, exc_cap x (i64 position, i64 remaining) } listing the
 * results whose remaining does not fit the width (token-bucket balances below -3 after
 * time regression, Lua :56-58). Segment s covers requests [sum(seg_counts[<s]), +seg_counts[s]).
 * rl_route_return_bytes = total bytes of that layout (0 on bad arguments).
 * rl_route_unpack_return scatters through perm like rl_route_unpack_packed and adds to
 * *lost (device u32) the escaped results whose block overflowed (they read
 * RL_REMAINING_ERROR). */
uint64_t rl_route_return_bytes(uint32_t n_seg, const uint64_t* seg_counts, int width,
                               uint32_t exc_cap);
int  rl_route_fold_return(rl_engine* e, size_t m, const uint8_t* allowed, const int64_t* remaining,
                          void* out, int width, uint32_t n_seg, const uint64_t* seg_counts,
                          uint32_t exc_cap, void* stream);
int  rl_route_unpack_return(rl_engine* e, size_t n, const uint32_t* perm, const void* in, int width,
                            uint32_t n_seg, const uint64_t* seg_counts, uint32_t exc_cap,
                            uint8_t* allowed, int64_t* remaining, uint32_t* lost, void* stream);
/* Hot-key owner directory (at most 4096 keys): key_hash[i] is owned by shard owner[i]
 * instead of its hash owner, in rl_route_partition(_device) and rl_owner_of_engine. With
 * Zipf traffic the hash owner of the top keys carries a multiple of the mean load (the top
 * key alone draws ~11% of all requests at s = 1.1); listing the hottest keys with owners
 * chosen to even the loads out removes that imbalance. Every rank must
 * install the same directory before any state exists for the listed keys. n = 0 clears. */
int  rl_set_owner_directory(rl_engine* e, size_t n, const uint64_t* key_hash,
                            const uint32_t* owner);
uint32_t rl_owner_of_engine(rl_engine* e, uint64_t key_hash);
/* rl_route_partition without a host round-trip: counts[s] (int64) land in DEVICE memory at
 * counts_dev[s * counts_stride] (the router's header column), on `stream`. */
int  rl_route_partition_device(rl_engine* e, size_t n, const uint64_t* key_hash,
                               uint32_t shard_count, uint32_t* perm, int64_t* counts_dev,
                               size_t counts_stride, void* stream);

/* ---- multi-GPU router ----------------------------------------
 * The reference's "distribution" is many app instances sharing one Redis
 * (README.md:266-269); here each GPU owns a hash shard of the keyspace and one router per
 * GPU moves every request to its owner and the decision back. A router wraps an engine
 * created with rl_opts.shard_index = rank, shard_count = world (power of two <= 64).
 *
 * Transport: how a router reaches its peers; all buffers are device pointers and every
 * call is enqueued on `stream` (collective: every rank makes the same calls in the same
 * order). all_to_all_v sends send[send_off[p] .. +send_bytes[p]) to peer p and receives
 * peer p's bytes at recv + recv_off[p]; byte counts are host arrays of `world` entries.
 * The RCCL transport (librl_rccl.so, rl_transport_rccl_create) is the product one; tests
 * supply an in-process loopback. Return 0 on success. */
typedef struct rl_transport {
    void* ctx;
    int (*all_to_all_v)(void* ctx, const void* send, const uint64_t* send_off,
                        const uint64_t* send_bytes, void* recv, const uint64_t* recv_off,
                        const uint64_t* recv_bytes, void* stream);
} rl_transport;

typedef struct rl_router rl_router;
typedef struct rl_router_opts {
    size_t max_batch;           /* the largest per-rank n of rl_router_step                    */
    size_t recv_cap;            /* requests an owner decides per exchange round; 0 = min(world,
                                   2) x max_batch; clamped to the engine's rl_opts.max_batch. A
                                   step in which some owner receives more runs in several
                                   rounds (every rank derives the same plan from the header)   */
} rl_router_opts;
/* Every device buffer a step uses is reserved here (send side ~50 B x max_batch, receive
 * side ~56 B x recv_cap, the return trip, the directory exchange), so a step never
 * allocates between two collectives. rl_router_create = _ex with recv_cap 0. */
int  rl_router_create_ex(rl_engine* e, uint32_t world, uint32_t rank, const rl_transport* t,
                         const rl_router_opts* opts, rl_router** out);
int  rl_router_create(rl_engine* e, uint32_t world, uint32_t rank, const rl_transport* t,
                      size_t max_batch, rl_router** out);
typedef struct rl_router_stats {
    uint64_t steps;             /* rl_router_step calls that reached the header exchange       */
    uint64_t rounds;            /* exchange rounds (== steps unless a step was split)          */
    uint64_t split_steps;       /* steps in which some owner received more than recv_cap       */
    uint64_t max_recv;          /* most requests this rank's engine received in one step       */
    uint64_t header_sync_ns;    /* host time blocked on the per-step header read, summed (it
                                   also waits for this rank's previous step to drain)          */
    uint64_t recv_cap;
    uint64_t reserved_bytes;    /* device bytes reserved by rl_router_create_ex                */
} rl_router_stats;
int  rl_router_stats_get(rl_router* r, rl_router_stats* out);
/* tryAcquire over this rank's slice of the global arrival stream (device buffers; the
 * ranks' slices are ordered by rank). Same results as one engine on the concatenated
 * stream. One host synchronisation per step (the header exchange: RCCL takes its
 * per-peer counts on the host). Errors are collective: a fatal engine error on any rank is
 * returned, once, by EVERY rank's step — the NEXT step for a failure known when the engine
 * call returns (a launch error, an allocation failure), TWO steps later for a batch's
 * data-dependent status (collected at the next step's header exchange, published in the
 * header after it) — or by rl_router_finish. The failed batch's requests read
 * RL_REMAINING_ERROR. The step that returns a fatal error does not process its own batch:
 * all n of its outputs read allowed = 0, remaining = RL_REMAINING_ERROR, so a caller that
 * goes on never mistakes stale decisions for this batch's. The router then goes on.
 * Non-fatal statuses (RL_E_INVALID_REQUEST) are not returned by a step: rl_router_finish
 * reports the worst of them since the previous finish. */
int  rl_router_step(rl_router* r, size_t n, const uint64_t* key_hash, const int32_t* permits,
                    const int64_t* now_ns, const uint16_t* limiter, uint8_t* allowed,
                    int64_t* remaining, void* stream);
/* Collective: the worst status of every rank's last batches (all ranks get the same). */
int  rl_router_finish(rl_router* r);
/* Hot-key directory for the whole router (collective, before any state exists for the
 * chosen keys): each rank passes its n candidates with their request counts (e.g. the top
 * keys of a sample of its traffic) and the total it sampled; the router merges them, keeps
 * the k hottest and places them on owners by longest-processing-time-first over the
 * owners' expected loads (rl_set_owner_directory on every rank). *placed = keys listed. */
int  rl_router_plan_directory(rl_router* r, size_t n, const uint64_t* key_hash,
                              const uint64_t* count, uint64_t sampled, uint32_t k,
                              uint32_t* placed, void* stream);
void rl_router_destroy(rl_router* r);

/* ---- synthetic traces (bench / tests; deterministic in (seed, index)) ------ */
#define RL_DIST_UNIFORM 0
#define RL_DIST_ZIPF    1
typedef struct rl_trace_spec {
    uint64_t seed;
    uint64_t n_keys;            /* key population                                */
    int32_t  dist;              /* RL_DIST_*                                      */
    int32_t  permits_max;       /* permits uniform in [1, permits_max]            */
    double   zipf_s;            /* Zipf exponent (dist = RL_DIST_ZIPF)            */
    int64_t  t0_ns;             /* first arrival                                  */
    int64_t  span_ns;           /* arrivals evenly spaced over [t0, t0 + span)    */
    uint64_t index_base;        /* global index of element 0 (sharded traces)     */
    uint64_t n_total;           /* total length of the global trace (time axis)  */
    uint16_t n_limiters;        /* limiter ids assigned round-robin by key rank   */
    uint16_t reserved[3];
} rl_trace_spec;
int  rl_synth_trace_device(rl_engine* e, const rl_trace_spec* spec, size_t n,
                           uint64_t* key_hash, int32_t* permits, int64_t* now_ns,
                           uint16_t* limiter, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RL_ENGINE_H */
