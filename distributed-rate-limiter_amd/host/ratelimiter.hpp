// ratelimiter.hpp — C++ mirror of the reference's Java API over the C-ABI engine.
//
// The reference (Java 17) API this mirrors, name for name:
//   com.ratelimiter.core.RateLimiter            core/RateLimiter.java:7-44
//   com.ratelimiter.core.RateLimitConfig        core/RateLimitConfig.java:12-81
//   com.ratelimiter.storage.StorageException    storage/StorageException.java:6-14
//   SlidingWindowRateLimiter / TokenBucketRateLimiter constructors and argument checks
//                                               algorithms/SlidingWindowRateLimiter.java:46-131
//                                               algorithms/TokenBucketRateLimiter.java:70-116
// Java's toolchain is not available in this build, so the host side above the C-ABI is
// C++ (INTEGRATION.md shows the JNI binding a Java maintainer adds instead). Every
// decision is made on the GPU through include/rl_engine.h; nothing here computes one.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rl_engine.h"

namespace ratelimiter {

// java.lang.IllegalArgumentException
struct IllegalArgumentException : std::invalid_argument {
    using std::invalid_argument::invalid_argument;
};

// com.ratelimiter.storage.StorageException (unchecked; thrown on backend failure,
// RedisRateLimitStorage.java:177) — here: a HIP/device error from the engine.
struct StorageException : std::runtime_error {
    int status;
    StorageException(const std::string& m, int st) : std::runtime_error(m), status(st) {}
};

// RateLimitConfig (RateLimitConfig.java:12-81). Immutable value; Duration fields are
// milliseconds here.
struct RateLimitConfig {
    int64_t maxPermits = 0;
    int64_t windowMs = 0;
    double refillRate = 0.0;          // permits per second (token bucket only)
    bool enableLocalCache = true;     // @Builder.Default true (RateLimitConfig.java:37-38)
    int64_t localCacheTtlMs = 100;    // @Builder.Default 100 ms (:43-44)
    uint64_t expectedKeys = 0;        // engine table sizing (not in the reference)

    // validate() (RateLimitConfig.java:46-56)
    void validate() const {
        if (maxPermits <= 0) throw IllegalArgumentException("maxPermits must be positive");
        if (windowMs <= 0) throw IllegalArgumentException("window must be a positive duration");
        if (refillRate < 0) throw IllegalArgumentException("refillRate cannot be negative");
    }
    // factories (RateLimitConfig.java:61-80)
    static RateLimitConfig perSecond(int64_t maxPermits) { return make(maxPermits, 1000); }
    static RateLimitConfig perMinute(int64_t maxPermits) { return make(maxPermits, 60000); }
    static RateLimitConfig perHour(int64_t maxPermits) { return make(maxPermits, 3600000); }

  private:
    static RateLimitConfig make(int64_t m, int64_t w) {
        RateLimitConfig c;
        c.maxPermits = m;
        c.windowMs = w;
        return c;
    }
};

// RateLimiter (RateLimiter.java:7-44).
class RateLimiter {
  public:
    virtual ~RateLimiter() = default;
    virtual bool tryAcquire(const std::string& key) = 0;               // :16
    virtual bool tryAcquire(const std::string& key, int permits) = 0;  // :26
    virtual int64_t getAvailablePermits(const std::string& key) = 0;   // :35 (-1 if unknown)
    virtual void reset(const std::string& key) = 0;                    // :43
};

// Micrometer counter stand-ins with the reference's meter names
// (SlidingWindowRateLimiter.java:67-77, TokenBucketRateLimiter.java:87-93).
struct Counter {
    std::string name;
    std::atomic<uint64_t> value{0};
    explicit Counter(std::string n) : name(std::move(n)) {}
    void increment(uint64_t d = 1) { value.fetch_add(d, std::memory_order_relaxed); }
    uint64_t count() const { return value.load(std::memory_order_relaxed); }
};

// String -> 64-bit key hash (build-defined): FNV-1a over the UTF-8
// bytes followed by the splitmix64 finaliser. Collisions between distinct strings make
// them share state (probability ~ n^2 / 2^65).
uint64_t keyHash(const std::string& key);

// One GPU engine (rl_create). Thread-safe: the engine serialises batches.
class GpuEngine {
  public:
    struct Options {
        int device = 0;
        uint64_t maxBatch = 1u << 20;
        uint64_t defaultCapacity = 1u << 20;
        int64_t maxSkewMs = 0;          // rl_opts.max_skew_ms
    };
    explicit GpuEngine(const Options& o);
    GpuEngine() : GpuEngine(Options{}) {}
    ~GpuEngine();
    GpuEngine(const GpuEngine&) = delete;
    GpuEngine& operator=(const GpuEngine&) = delete;
    rl_engine* handle() const { return e_; }
    // Page-lock a reused host buffer for the engine's DMA (rl_pin_host); best effort:
    // an unpinned buffer still works through pageable staging.
    void pin(void* p, size_t bytes) { if (p && bytes) (void)rl_pin_host(e_, p, bytes); }
    void unpin(void* p) { if (p) (void)rl_unpin_host(e_, p); }
    uint16_t addLimiter(int algo, const RateLimitConfig& c);
    // Runs one host batch and returns its status and cache-hit count atomically with
    // respect to the other limiters sharing this engine.
    int executeBatch(size_t n, const uint64_t* key, const int32_t* permits, const int64_t* now,
                     const uint16_t* limiter, const uint8_t* op, uint8_t* allowed,
                     int64_t* remaining, uint64_t* cacheHits);

  private:
    rl_engine* e_ = nullptr;
    std::mutex mu_;
};

// Clock in nanoseconds (the reference reads System.currentTimeMillis(); injectable so a
// trace can be replayed with a pinned clock).
using Clock = std::function<int64_t()>;
int64_t systemNanos();

// Drop-in GPU implementation of RateLimiter for one limiter configuration. The
// constructor performs the reference constructors' checks; single calls are batched by
// a micro-batcher (concurrent callers share one engine batch, arrival order = the order
// in which callers enter the queue).
class GpuRateLimiter : public RateLimiter {
  public:
    enum class Algorithm { SlidingWindow = RL_ALGO_SLIDING_WINDOW, TokenBucket = RL_ALGO_TOKEN_BUCKET };

    GpuRateLimiter(std::shared_ptr<GpuEngine> engine, Algorithm algo, const RateLimitConfig& cfg,
                   Clock clock = systemNanos, int batchWindowMicros = 0);
    ~GpuRateLimiter() override;

    bool tryAcquire(const std::string& key) override { return tryAcquire(key, 1); }
    bool tryAcquire(const std::string& key, int permits) override;
    int64_t getAvailablePermits(const std::string& key) override;
    void reset(const std::string& key) override;

    // tryAcquireBatch(keys[], permits[], nowNanos[]); remaining may be null.
    void tryAcquireBatch(size_t n, const uint64_t* keyHash, const int32_t* permits,
                         const int64_t* nowNanos, bool* allowed, int64_t* remaining);

    uint16_t limiterId() const { return id_; }
    const RateLimitConfig& config() const { return cfg_; }
    Counter allowedRequests;
    Counter rejectedRequests;
    Counter cacheHits{"ratelimiter.cache.hits"};     // SlidingWindowRateLimiter.java:75-77

  private:
    struct Pending {
        uint64_t key;
        int32_t permits;
        int64_t now;
        uint8_t op;
        bool done = false;
        uint8_t allowed = 0;
        int64_t remaining = 0;
        int status = RL_OK;
    };
    void submit(Pending& p);
    void flushLocked(std::unique_lock<std::mutex>& lk);
    void checkStatus(int st, const char* where);

    std::shared_ptr<GpuEngine> engine_;
    Algorithm algo_;
    RateLimitConfig cfg_;
    Clock clock_;
    uint16_t id_ = 0;
    int windowMicros_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<Pending*> queue_;
    bool flushing_ = false;
    // flush buffers, reused across flushes and page-locked (owned by the flush slot)
    struct FlushBufs {
        size_t cap = 0;
        std::vector<uint64_t> key;
        std::vector<int32_t> permits;
        std::vector<int64_t> now, remaining;
        std::vector<uint16_t> lim;
        std::vector<uint8_t> op, allowed;
    } fb_;
    void reserveFlush(size_t n);
    void unpinFlush();
};

}  // namespace ratelimiter
