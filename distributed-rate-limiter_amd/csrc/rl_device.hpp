// rl_device.hpp — device-side layout, record codecs and the exact per-request
// semantics of the two reference algorithms, for gfx950 (MI355X).
//
// Everything here is compiled with -ffp-contract=off (see Makefile) and also
// carries `#pragma clang fp contract(off)`: Java (SlidingWindowRateLimiter.java:174)
// and Lua (TokenBucketRateLimiter.java:56-58) round every multiply and every add
// separately; hipcc would otherwise fuse `a + b*c` into v_fmac_f64 and flip
// decisions at thresholds (tests/golden "fmaFlip*").
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rl {

// ---------------------------------------------------------------- constants
constexpr int kAlgoSW = 0;
constexpr int kAlgoTB = 1;
constexpr int kOpAcquire = 0;
constexpr int kOpPeek = 1;
constexpr int kOpReset = 2;

constexpr int64_t kRemUnknown = -1;   // TB permits > max
constexpr int64_t kRemInvalid = -2;   // permits <= 0 / unknown limiter
constexpr int64_t kRemError = -3;     // state-table region full

// State table: a limiter's keys live in 2^k regions of kRegionSlots slots. One
// wavefront owns a region for a whole batch (its 8 KB image lives in that wave's
// LDS), so a region needs no atomics in HBM. The batch is partitioned by BIN =
// kRegionsPerBin consecutive regions; one 8-wave workgroup owns a bin and each wave
// picks its region's requests out of the bin's arrival-ordered stream in LDS. Fewer,
// larger bins keep the partition's open write lines (bins x tiles in flight x 128 B)
// inside each XCD's 4 MB L2.
constexpr int kRegionSlots = 256;                 // slots per region (load <= ~0.5)
constexpr int kRegionBits = 8;
constexpr int kRegionsPerBin = 8;                 // every limiter has >= 8 regions ...
constexpr int kBinShift = 3;                      // ... (2^kBinShift)
constexpr int kRing = 128;                        // per-wave pending ring (< 64 + 64 entries)
constexpr uint32_t kNone = 0xFFFFFFFFu;

// Partition tiles (upsweep / scatter / unpermute all share this tiling). 64K
// requests per tile; grids are persistent (one workgroup per CU) and walk the tiles
// so that the 32 workgroups of an XCD work on 32 consecutive tiles at a time.
// 8 waves per tile (2 per SIMD): the scatter is latency-bound at one wave per SIMD, and
// more workgroups per CU would put more tiles' partial record lines in flight per L2
// (same-box A/B, tb_uniform: 3.60 -> 3.24 ms/step vs 4 waves per tile).
constexpr int kTileThreads = 512;
constexpr int kTileItems = 128;                    // per-thread items per tile
constexpr int kTile = kTileThreads * kTileItems;  // 65536 requests per tile (default)
constexpr int kMaxDigitBits = 13;                 // <= 8192 bins per pass

// Compact record field limits.
constexpr uint32_t kPermitBits = 22;
constexpr uint32_t kPermitMask = (1u << kPermitBits) - 1;   // 0 = invalid marker
constexpr int64_t kCompactMaxPermits = (int64_t)kPermitMask - 1;  // clamp is exact below this

// ---------------------------------------------------------------- limiter table
struct DevLimiter {          // 96 B, read-only during a batch
    int32_t algo;
    int32_t region_bits;     // k: the limiter has 2^k regions
    uint32_t region_base;    // first global region id
    uint32_t lflags;         // kLf* (host-derived properties of this limiter's arithmetic)
    int64_t max_permits;
    int64_t window_ms;       // w
    int64_t ttl_ms;          // SW: w (PEXPIRE on INCR); TB: 2w (Lua PEXPIRE)
    double rate_per_ms;      // TB: refillRate / 1000.0 (TokenBucketRateLimiter.java:85)
    double capacity;         // TB: (double)maxPermits (Lua tonumber(ARGV[1]))
    uint64_t table;          // device address of this limiter's region array
    double inv_window;       // 1.0 / w: first guess of Java's now / w (jdiv corrects it)
    uint64_t cache_table;    // SW local cache: one u64 per slot (block-until ms), or 0
    int64_t cache_ttl_ms;    // localCacheTtl (0: no local cache, the parity-mode default)
    double inv_rate;         // TB: 1 / rate_per_ms (first guesses only, never a decision)
};

// DevLimiter::lflags. The window fraction of :170-171, (double)(now % w) / w, is an IEEE
// division; for windows up to 2^22 ms the host checks every remainder r in [0, w) and sets
// kLfPctMul when r * (1/w) rounds to the same double (one multiply), else kLfPctFma when one
// fma correction of that product does (exact by exhaustion, not by a theorem); otherwise the
// kernels divide. Negative remainders (now < 0) follow by symmetry of both roundings.
constexpr uint32_t kLfPctMul = 1u;
constexpr uint32_t kLfPctFma = 2u;

// One 32-byte slot of a region (HBM and the LDS image).
//   TB: a = tokens (f64 bits), b = last_refill ms (i64), c = bit0 "bucket exists"
//   SW: a = start of the newest bucket b1 (i64)
//       b = b1_count (u32) | b0_count (u32) << 32        (b0 = bucket at b1_start - w)
//       c = b1_last_off (i32) | b0_last_off (i32) << 32  (last INCR time - bucket start)
// A slot whose state is absent (TB c == 0, SW both counts 0) is free.
struct Slot {
    uint64_t tag;            // mix64(key_hash)
    uint64_t a, b, c;
};

// HBM slot invariant (open addressing, linear probing from a key's 4-aligned home):
// a slot is FREE iff its four words (and its local-cache word) are all zero; a key is
// always found before the first free slot of its probe sequence. A slot whose state is
// dead (no bucket live) but whose words are not all zero is a TOMBSTONE: it keeps the
// probe chain intact and may be reused by an insert. Writers that load a whole region (a
// region loaded as an LDS image, the TTL sweep, state import) drop dead slots (written as
// zeros) and relink or rebuild the chain; sparse region waves (few records) touch single
// buckets and never create a hole. The only key whose dead state could be all-zero (tag 0 = mix64(0) with
// a deleted token bucket) is written with c = kDeadMark instead, which no live state has
// (TB: c bit 0 clear = absent bucket; SW: both counts zero).
constexpr uint64_t kDeadMark = 2;
__host__ __device__ inline bool slot_free(const Slot& v, uint64_t x = 0) {
    return (v.tag | v.a | v.b | v.c | x) == 0;
}
// A used slot as written to HBM: never all-zero (see kDeadMark).
__host__ __device__ inline Slot slot_used(Slot v, uint64_t x = 0) {
    if (slot_free(v, x)) v.c = kDeadMark;
    return v;
}

// LDS occupancy word of a region slot (k_regions)
constexpr uint32_t kOccUsed = 1u;       // holds a key (live, or a tombstone with kOccTomb)
constexpr uint32_t kOccTouched = 2u;    // read or written by this batch
constexpr uint32_t kOccUnloaded = 4u;   // sparse region: bucket not fetched from HBM yet
constexpr uint32_t kOccTomb = 8u;       // sparse region: dead slot (claimable by an insert)
constexpr uint32_t kOccDirty = 16u;     // image region: changed by the load (dropped, moved)

// ---------------------------------------------------------------- hashing
// splitmix64 finaliser: a bijection on u64, so tags identify keys exactly.
__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
}

// Inverse of mix64 (state export recovers key_hash from a slot's tag).
__host__ __device__ inline uint64_t unmix64(uint64_t x) {
    x ^= (x >> 31) ^ (x >> 62);
    x *= 0x319642b2d24d8ec3ULL;          // 0x94d049bb133111eb^-1 mod 2^64
    x ^= (x >> 27) ^ (x >> 54);
    x *= 0x96de1b173f119089ULL;          // 0xbf58476d1ce4e5b9^-1 mod 2^64
    x ^= (x >> 30) ^ (x >> 60);
    return x;
}

// owner shard = top s bits of h; region = next k bits.
__host__ __device__ inline uint32_t region_local(uint64_t h, int shard_bits, int k) {
    if (k == 0) return 0;
    return (uint32_t)((h << shard_bits) >> (64 - k));
}

__host__ __device__ inline int64_t floor_div_ms(int64_t ns) {
    int64_t q = ns / 1000000;
    if ((ns % 1000000) != 0 && ns < 0) q -= 1;
    return q;
}

// ---------------------------------------------------------------- records
// Compact (16 B): {h, now_ms - base (u32), permits:22 | op:2 | limiter:8}.
// Valid when every limiter has max_permits <= kCompactMaxPermits (so clamping the
// permits field is decision-exact: SW est >= 0, TB early-rejects p > max) and the
// batch's now_ms lies within +-2^31 ms of the first request's.
struct RecC { uint64_t h; uint32_t now_rel; uint32_t pl; };
// Wide (32 B): no limits beyond the engine's.
struct RecW { uint64_t h; int64_t now_ms; int32_t permits; uint16_t limiter; uint8_t op;
              uint8_t invalid; uint64_t pad; };

struct Req {                 // decoded request
    uint64_t h;
    int64_t now_ms;
    int32_t permits;         // >= 1 when valid (compact: clamped)
    uint32_t limiter;
    uint32_t op;
    bool invalid;
};

struct CodecC {
    using Rec = RecC;
    using Res = uint32_t;
    __device__ static inline Rec enc(uint64_t h, int64_t now_ms, int64_t base, int32_t permits,
                                     uint32_t op, uint32_t lim, bool invalid) {
        Rec r;
        r.h = h;
        r.now_rel = (uint32_t)(now_ms - base);
        uint32_t p = 0;
        if (!invalid) {
            if (op != (uint32_t)kOpAcquire) p = 1;
            else p = (uint32_t)permits > kPermitMask ? kPermitMask : (uint32_t)permits;
        }
        r.pl = p | (op << kPermitBits) | (lim << 24);
        return r;
    }
    __device__ static inline Req dec(const Rec& r, int64_t base) {
        Req q;
        q.h = r.h;
        q.now_ms = base + (int64_t)r.now_rel;
        q.permits = (int32_t)(r.pl & kPermitMask);
        q.op = (r.pl >> kPermitBits) & 3u;
        q.limiter = r.pl >> 24;
        q.invalid = q.permits == 0;
        return q;
    }
    __device__ static inline uint32_t limiter_of(const Rec& r) { return r.pl >> 24; }
};

struct CodecW {
    using Rec = RecW;
    using Res = uint64_t;
    __device__ static inline Rec enc(uint64_t h, int64_t now_ms, int64_t, int32_t permits,
                                     uint32_t op, uint32_t lim, bool invalid) {
        Rec r;
        r.h = h; r.now_ms = now_ms; r.permits = permits; r.limiter = (uint16_t)lim;
        r.op = (uint8_t)op; r.invalid = invalid ? 1 : 0; r.pad = 0;
        return r;
    }
    __device__ static inline Req dec(const Rec& r, int64_t) {
        Req q;
        q.h = r.h; q.now_ms = r.now_ms; q.permits = r.permits; q.op = r.op;
        q.limiter = r.limiter; q.invalid = r.invalid != 0;
        return q;
    }
    __device__ static inline uint32_t limiter_of(const Rec& r) { return r.limiter; }
};

// ---------------------------------------------------------------- results
// Packed result in partition order: (remaining + 3) << 1 | allowed (remaining >= -3).
// The width is the narrowest that holds every limiter's max_permits: u8 (max <= 124),
// u16 (max <= 32764), u32 (compact records), u64 (wide records). Rate limits are
// usually small, so the result array is 1-2 bytes per request and stays in the
// 256 MiB Infinity Cache for the unpermute gather.
constexpr int64_t kResBias = 3;
__device__ inline uint64_t pack_result(bool allowed, int64_t remaining) {
    return ((uint64_t)(remaining + kResBias) << 1) | (allowed ? 1u : 0u);
}
// A token-bucket balance goes below -3 only after time regression (elapsed < 0 is not
// clamped, Lua :56-58), and its reply integer can be any negative value. `remaining = -3`
// is never allowed, so the packed code 1 (= pack_result(true, -3)) is free: it marks a
// remaining outside the width's range, kept exactly in an int64 side array (`ext`) at the
// same position and restored by the unpermute.
constexpr uint64_t kResEscape = 1;
template <class Res>
__device__ inline bool res_fits(int64_t remaining) {
    constexpr int64_t hi = (int64_t)((uint64_t)(Res)~(Res)0 >> 1) - kResBias;
    return remaining >= -kResBias && remaining <= hi;
}
__host__ __device__ inline int res_bytes_for(int64_t max_permits, bool wide) {
    if (wide) return 8;
    if ((max_permits + kResBias) * 2 + 1 < 256) return 1;
    if ((max_permits + kResBias) * 2 + 1 < 65536) return 2;
    return 4;
}

// Java (long) narrowing of a double (JLS 5.1.3) / Redis (long long) of a Lua number.
__device__ inline int64_t d2l(double d) {
    if (__builtin_expect(__builtin_fabs(d) < 2147483648.0, 1)) return (int64_t)(int32_t)d;  // one cvt
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

struct Outcome {
    bool mutate;             // the request changes the key's state
    bool allowed;
    int64_t remaining;
    double tokens;           // TB fp64 balance (NaN otherwise)
    uint64_t a, b, c;        // new state when mutate
    int64_t cval;            // SW: the count the reference would put in its local cache
    uint64_t x;              // SW local cache: block-until ms after the request (0: none)
};

// ---------------------------------------------------------------- token bucket
// Lua :46-58: the balance after refill at `now` (absent or expired bucket: full).
// `last` is the ms timestamp stored by HMSET; the bucket exists iff written and
// now <= last + 2w. Non-decreasing in `now` for a fixed state (the hot-key fast
// path relies on that, k_regions_hot).
__device__ inline double tb_refill(const DevLimiter& L, int64_t now, uint64_t a, uint64_t b,
                                   uint64_t c) {
    const int64_t last = (int64_t)b;
    const bool exists = (c & 1u) && !(now > last + L.ttl_ms);
    const double capacity = L.capacity;
    // absent or expired: tokens = capacity, last_refill = now, so elapsed = 0 and the balance
    // is min(capacity, capacity + 0 * rate) = capacity exactly
    if (!exists) return capacity;
    // Lua :56: now - last_refill on doubles is exact (both are integers below 2^53 and so is
    // their difference), i.e. the same as converting the integer difference once
    const double elapsed = (double)(now - last);
    const double tokens_to_add = elapsed * L.rate_per_ms;    // Lua :57
    const double x = __longlong_as_double((long long)a) + tokens_to_add;   // Lua :58
    return x < capacity ? x : capacity;                      // math.min(capacity, x)
}

// TokenBucketRateLimiter.tryAcquire (:105-143) + Lua (:38-68).
__device__ inline Outcome tb_step(const DevLimiter& L, uint32_t op, int32_t permits,
                                  int64_t now, uint64_t a, uint64_t b, uint64_t c) {
    Outcome o;
    o.mutate = false; o.allowed = false; o.remaining = 0; o.tokens = __builtin_nan("");
    o.cval = 0; o.x = 0;
    o.a = a; o.b = b; o.c = c;
    if (op == (uint32_t)kOpReset) {                  // DEL tb:key (:153-158)
        o.mutate = true; o.a = 0; o.b = 0; o.c = 0;
        return o;
    }
    if (op == (uint32_t)kOpAcquire && (int64_t)permits > L.max_permits) {  // :110-116
        o.remaining = kRemUnknown;
        return o;
    }
    double tokens = tb_refill(L, now, a, b, c);
    if (op == (uint32_t)kOpPeek) {
        o.remaining = d2l(tokens);
        o.tokens = tokens;
        return o;
    }
    const double requested = (double)permits;
    if (tokens >= requested) {                               // Lua :61-65
        tokens = tokens - requested;
        o.mutate = true; o.allowed = true;
        o.a = (uint64_t)__double_as_longlong(tokens);
        o.b = (uint64_t)now;
        o.c = 1;
    }
    o.remaining = d2l(tokens);                               // {allowed, tokens} reply
    o.tokens = tokens;
    return o;
}

// ---------------------------------------------------------------- sliding window
struct SW2 {                 // the two most recent buckets of a key
    int64_t b1_start;
    uint32_t b1_cnt, b0_cnt;
    int32_t b1_off, b0_off;
};

__device__ inline SW2 sw_unpack(uint64_t a, uint64_t b, uint64_t c) {
    SW2 s;
    s.b1_start = (int64_t)a;
    s.b1_cnt = (uint32_t)b; s.b0_cnt = (uint32_t)(b >> 32);
    s.b1_off = (int32_t)(uint32_t)c; s.b0_off = (int32_t)(uint32_t)(c >> 32);
    return s;
}

// RedisRateLimitStorage.get (:52-59) of bucket `start` at `now`: 0 if missing or
// expired (PEXPIRE w on every INCR; expired iff now > lastIncr + w).
__device__ inline int64_t sw_get(const SW2& s, int64_t start, int64_t now, int64_t w) {
    if (s.b1_cnt != 0 && s.b1_start == start && !(now > s.b1_start + s.b1_off + w))
        return s.b1_cnt;
    const int64_t b0_start = s.b1_start - w;
    if (s.b0_cnt != 0 && b0_start == start && !(now > b0_start + s.b0_off + w))
        return s.b0_cnt;
    return 0;
}

// Java long division / remainder (truncating) by 0 < w < 2^31, exact for |a| < 2^53:
// a correctly rounded fp64 quotient is within 1 of the true one; fix it up in integers.
__device__ inline int64_t jdiv(int64_t a, int64_t w, double inv_w, int64_t* rem) {
    int64_t q = (int64_t)((double)a * inv_w);              // within 1 of the quotient
    int64_t r = a - q * w;
    if (r < 0 && a >= 0) { q -= 1; r += w; }
    else if (r >= w) { q += 1; r -= w; }
    else if (r > 0 && a < 0) { q += 1; r -= w; }
    else if (r <= -w) { q -= 1; r += w; }
    *rem = r;
    return q;
}

// (double)r / w for |r| < w < 2^31 (:170-171), bit-exact (see kLfPctMul).
__device__ inline double sw_pct(int64_t r, const DevLimiter& L) {
    const double dr = (double)(int32_t)r;
    if (L.lflags & kLfPctMul) return dr * L.inv_window;
    if (L.lflags & kLfPctFma) {
        const double q = dr * L.inv_window;
        return __builtin_fma(__builtin_fma(-q, (double)L.window_ms, dr), L.inv_window, q);
    }
    return dr / (double)L.window_ms;
}

// Window geometry of a request (getWindowKey :185-188 for now and now - w).
struct SWGeo {
    int64_t curr_start, prev_start;
    double prev_weight;      // 1.0 - (double)(now % w) / w   (:170-171)
};

// One true division (the IEEE quotient Java computes, :170); the window starts come from
// a reciprocal multiply corrected in integers.
__device__ inline SWGeo sw_geo(int64_t now, const DevLimiter& L) {
    const int64_t w = L.window_ms;
    SWGeo g;
    int64_t r, r2;
    const int64_t q = jdiv(now, w, L.inv_window, &r);
    g.curr_start = q * w;
    // (now - w) / w == now / w - 1 under truncation iff now >= w (near the epoch it differs)
    g.prev_start = now >= w ? g.curr_start - w : jdiv(now - w, w, L.inv_window, &r2) * w;
    g.prev_weight = 1.0 - sw_pct(r, L);
    return g;
}

// sw_geo for a request of a wave whose window starts near `wref` (wave-uniform: the start of
// a window of this batch, >= 0, or -1): a request in that window or the next one takes its
// start and remainder from one subtraction instead of a division.
__device__ inline SWGeo sw_geo_ref(int64_t now, const DevLimiter& L, int64_t wref) {
    const int64_t w = L.window_ms;
    if (wref >= 0 && now >= wref && now - wref < 2 * w && now >= w) {
        const int64_t d = now - wref;
        const bool nx = d >= w;
        SWGeo g;
        g.curr_start = nx ? wref + w : wref;
        g.prev_start = g.curr_start - w;              // (now >= w: truncation agrees, see sw_geo)
        g.prev_weight = 1.0 - sw_pct(nx ? d - w : d, L);
        return g;
    }
    return sw_geo(now, L);
}

// getCurrentCount (SlidingWindowRateLimiter.java:158-180).
__device__ inline int64_t sw_estimate(const SW2& s, const SWGeo& g, int64_t now, int64_t w) {
    const int64_t curr = sw_get(s, g.curr_start, now, w);
    const int64_t prev = sw_get(s, g.prev_start, now, w);
    const double t = (double)prev * g.prev_weight;            // :174, rounded
    const double sum = t + (double)curr;                      //       rounded separately
    return d2l(sum);
}

// sw_step with the request's window geometry precomputed (it depends only on now, w).
__device__ inline Outcome sw_step_g(const DevLimiter& L, uint32_t op, int32_t permits,
                                    int64_t now, const SWGeo& geo, uint64_t a, uint64_t b,
                                    uint64_t c) {
    Outcome o;
    o.mutate = false; o.allowed = false; o.remaining = 0; o.tokens = __builtin_nan("");
    o.cval = 0; o.x = 0;
    o.a = a; o.b = b; o.c = c;
    const int64_t w = L.window_ms;
    SW2 s = sw_unpack(a, b, c);
    const int64_t curr_start = geo.curr_start;
    if (op == (uint32_t)kOpReset) {                  // reset (:139-153): DEL curr and prev
        const int64_t prev_start = geo.prev_start;
        if (s.b1_start == curr_start || s.b1_start == prev_start) s.b1_cnt = 0;
        const int64_t b0_start = s.b1_start - w;
        if (b0_start == curr_start || b0_start == prev_start) s.b0_cnt = 0;
        o.mutate = true;
        o.b = (uint64_t)s.b1_cnt | ((uint64_t)s.b0_cnt << 32);
        return o;
    }
    const int64_t est = sw_estimate(s, geo, now, w);
    o.cval = est;
    if (op == (uint32_t)kOpPeek || est + (int64_t)permits > L.max_permits) {  // :104
        const int64_t r = L.max_permits - est;
        o.remaining = r > 0 ? r : 0;
        return o;
    }
    // incrementAndExpire(currentKey, w) (:114-116, RedisRateLimitStorage.java:38-49)
    uint32_t new_count;
    if (s.b1_start == curr_start) {
        const bool alive = s.b1_cnt != 0 && !(now > s.b1_start + s.b1_off + w);
        s.b1_cnt = alive ? s.b1_cnt + 1 : 1;
        s.b1_off = (int32_t)(now - curr_start);
        new_count = s.b1_cnt;
    } else if (curr_start > s.b1_start || (s.b1_cnt == 0 && s.b0_cnt == 0)) {   // a newer window
        if (s.b1_start == curr_start - w) { s.b0_cnt = s.b1_cnt; s.b0_off = s.b1_off; }
        else { s.b0_cnt = 0; s.b0_off = 0; }
        s.b1_start = curr_start;
        s.b1_cnt = 1;
        s.b1_off = (int32_t)(now - curr_start);
        new_count = 1;
    } else if (curr_start == s.b1_start - w) {
        // time regression into the previous window (e.g. front-ends with skewed clocks):
        // Redis keeps every window's key, so the INCR lands on bucket b0 and the newer bucket
        // is untouched. PEXPIRE sets its deadline from this request's now.
        const int64_t b0_start = s.b1_start - w;
        const bool alive = s.b0_cnt != 0 && !(now > b0_start + s.b0_off + w);
        s.b0_cnt = alive ? s.b0_cnt + 1 : 1;
        s.b0_off = (int32_t)(now - b0_start);
        new_count = s.b0_cnt;
    } else {
        // regression past both tracked buckets: the bucket it increments (and the one before
        // it) are older than the key's newest two and are not kept; they read as absent, so
        // the INCR yields 1 (documented divergence). The newer buckets are
        // never rolled back.
        o.mutate = false;
        o.allowed = 1 <= L.max_permits;
        o.cval = 1;
        const int64_t r = L.max_permits - 1;              // estimate after: 0 * pw + 1
        o.remaining = r > 0 ? r : 0;
        return o;
    }
    o.mutate = true;
    o.cval = new_count;
    o.allowed = (int64_t)new_count <= L.max_permits;  // :123
    const int64_t est2 = sw_estimate(s, geo, now, w);  // remaining after the request (A4)
    const int64_t r = L.max_permits - est2;
    o.remaining = r > 0 ? r : 0;
    o.a = (uint64_t)s.b1_start;
    o.b = (uint64_t)s.b1_cnt | ((uint64_t)s.b0_cnt << 32);
    o.c = (uint64_t)(uint32_t)s.b1_off | ((uint64_t)(uint32_t)s.b0_off << 32);
    return o;
}

// tryAcquire / reset with the Caffeine local cache on (SlidingWindowRateLimiter.java:93-121,
// :148-150). The cache entry (value, write time) matters only through x = write time + ttl
// when value >= maxPermits (0 otherwise): getIfPresent returns it iff now - write < ttl
// (expireAfterWrite, :57-64) and only a value >= maxPermits short-circuits (:95); every put
// overwrites. `hit` = rejected from the cache without touching the Redis state.
__device__ inline Outcome sw_step_cache(const DevLimiter& L, uint32_t op, int32_t permits,
                                        int64_t now, const SWGeo& geo, uint64_t a, uint64_t b,
                                        uint64_t c, uint64_t x, bool& hit) {
    hit = false;
    if (op == (uint32_t)kOpAcquire && x != 0 && now < (int64_t)x) {           // :93-100
        Outcome o = sw_step_g(L, kOpPeek, permits, now, geo, a, b, c);     // remaining only
        hit = true;
        o.x = x;
        return o;
    }
    Outcome o = sw_step_g(L, op, permits, now, geo, a, b, c);
    o.x = x;
    if (op == (uint32_t)kOpReset) {                                            // :148-150
        o.x = 0;
    } else if (op == (uint32_t)kOpAcquire) {                                   // :106-108, :119-121
        o.x = o.cval >= L.max_permits ? (uint64_t)(now + L.cache_ttl_ms) : 0;
        o.mutate |= o.x != x;
    }
    return o;
}

__device__ inline Outcome sw_step(const DevLimiter& L, uint32_t op, int32_t permits,
                                  int64_t now, uint64_t a, uint64_t b, uint64_t c) {
    return sw_step_g(L, op, permits, now, sw_geo(now, L), a, b, c);
}

// Sliding-window acquire at `now` assuming that k earlier requests of the same key, all
// in now's window and all after the state's newest bucket, were ALLOWED (each INCRs the
// current bucket by 1, :114-116). Exactly what sw_step returns after those k steps:
// the current bucket is then curr0 + k (alive: its last INCR is in this window) and the
// previous bucket is untouched (a roll into this window moves b1 to b0 with its offset).
struct SWAllow { bool allowed; int64_t remaining; };
__device__ inline SWAllow sw_try_after_allows(const DevLimiter& L, int32_t permits, int64_t now,
                                              const SWGeo& g, uint64_t a, uint64_t b, uint64_t c,
                                              uint32_t k) {
    const int64_t w = L.window_ms;
    const SW2 s = sw_unpack(a, b, c);
    const int64_t curr0 = (s.b1_start == g.curr_start) ? (int64_t)s.b1_cnt : 0;
    const int64_t prev = sw_get(s, g.prev_start, now, w);
    const double t = (double)prev * g.prev_weight;            // :174, as sw_estimate
    const int64_t est = d2l(t + (double)(curr0 + (int64_t)k));
    SWAllow r;
    r.allowed = !(est + (int64_t)permits > L.max_permits);
    const int64_t e2 = r.allowed ? d2l(t + (double)(curr0 + (int64_t)k + 1)) : est;
    const int64_t rem = L.max_permits - e2;
    r.remaining = rem > 0 ? rem : 0;
    return r;
}

// The state after n such allows, the last at time t_last (the roll of sw_step included).
__device__ inline void sw_commit_allows(const DevLimiter& L, const SWGeo& g, uint64_t& a,
                                        uint64_t& b, uint64_t& c, uint32_t n, int64_t t_last) {
    SW2 s = sw_unpack(a, b, c);
    if (s.b1_start == g.curr_start) {
        s.b1_cnt += n;
    } else {
        if (s.b1_start == g.curr_start - L.window_ms) { s.b0_cnt = s.b1_cnt; s.b0_off = s.b1_off; }
        else { s.b0_cnt = 0; s.b0_off = 0; }
        s.b1_start = g.curr_start;
        s.b1_cnt = n;
    }
    s.b1_off = (int32_t)(t_last - g.curr_start);
    a = (uint64_t)s.b1_start;
    b = (uint64_t)s.b1_cnt | ((uint64_t)s.b0_cnt << 32);
    c = (uint64_t)(uint32_t)s.b1_off | ((uint64_t)(uint32_t)s.b0_off << 32);
}

// A slot is kept when the region is loaded iff some request at now >= batch_min could
// still read it (x: its local-cache block-until, SW with the cache on); everything else is
// dropped (the region is rebuilt in LDS).
__device__ inline bool slot_live(const DevLimiter& L, const Slot& s, int64_t batch_min,
                                 uint64_t x = 0) {
    if (x != 0 && (int64_t)x > batch_min) return true;
    if (L.algo == kAlgoTB) {
        return (s.c & 1u) && !(batch_min > (int64_t)s.b + L.ttl_ms);
    }
    SW2 q = sw_unpack(s.a, s.b, s.c);
    const int64_t w = L.window_ms;
    const bool l1 = q.b1_cnt != 0 && !(batch_min > q.b1_start + q.b1_off + w);
    const bool l0 = q.b0_cnt != 0 && !(batch_min > q.b1_start - w + q.b0_off + w);
    return l1 || l0;
}

__device__ inline bool state_present(int algo, uint64_t b, uint64_t c) {
    return algo == kAlgoTB ? (c & 1u) != 0 : b != 0;
}

}  // namespace rl
