// ratelimiter.cpp — see ratelimiter.hpp.
#include "ratelimiter.hpp"

#include <cstring>

namespace ratelimiter {

uint64_t keyHash(const std::string& key) {
    uint64_t h = 0xcbf29ce484222325ULL;                 // FNV-1a 64
    for (unsigned char c : key) {
        h ^= c;
        h *= 0x100000001b3ULL;
    }
    h ^= h >> 30; h *= 0xbf58476d1ce4e5b9ULL;           // splitmix64 finaliser
    h ^= h >> 27; h *= 0x94d049bb133111ebULL;
    h ^= h >> 31;
    return h;
}

int64_t systemNanos() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}

GpuEngine::GpuEngine(const Options& o) {
    rl_opts opts{};
    opts.device = o.device;
    opts.max_batch = o.maxBatch;
    opts.default_capacity = o.defaultCapacity;
    opts.shard_count = 1;
    opts.max_skew_ms = o.maxSkewMs;
    int st = rl_create(&opts, &e_);
    if (st != RL_OK) throw StorageException(std::string("rl_create: ") + rl_strerror(st), st);
}

GpuEngine::~GpuEngine() { rl_destroy(e_); }

uint16_t GpuEngine::addLimiter(int algo, const RateLimitConfig& c) {
    rl_limiter_config lc{};
    lc.algo = algo;
    lc.max_permits = c.maxPermits;
    lc.window_ms = c.windowMs;
    lc.refill_per_s = c.refillRate;
    lc.capacity = c.expectedKeys;
    if (algo == RL_ALGO_SLIDING_WINDOW && c.enableLocalCache && c.localCacheTtlMs > 0) {
        lc.flags = RL_LIM_LOCAL_CACHE;               // SlidingWindowRateLimiter.java:57-64
        lc.local_cache_ttl_ms = c.localCacheTtlMs;
    }
    uint16_t id = 0;
    int st = rl_add_limiter_ex(e_, &lc, &id);
    if (st == RL_E_INVALID_ARG)
        throw IllegalArgumentException(std::string("limiter configuration rejected: ") + rl_strerror(st));
    if (st != RL_OK) throw StorageException(std::string("rl_add_limiter: ") + rl_strerror(st), st);
    return id;
}

int GpuEngine::executeBatch(size_t n, const uint64_t* key, const int32_t* permits,
                            const int64_t* now, const uint16_t* limiter, const uint8_t* op,
                            uint8_t* allowed, int64_t* remaining, uint64_t* cacheHits) {
    std::lock_guard<std::mutex> lk(mu_);
    const int st = rl_execute_batch(e_, n, key, permits, now, limiter, op, allowed, remaining, nullptr);
    rl_batch_stats bs{};
    if (cacheHits) *cacheHits = rl_batch_stats_get(e_, &bs) == RL_OK ? bs.cache_hits : 0;
    return st;
}

GpuRateLimiter::GpuRateLimiter(std::shared_ptr<GpuEngine> engine, Algorithm algo,
                               const RateLimitConfig& cfg, Clock clock, int batchWindowMicros)
    : allowedRequests(algo == Algorithm::TokenBucket ? "ratelimiter.tokenbucket.allowed"
                                                      : "ratelimiter.requests.allowed"),
      rejectedRequests(algo == Algorithm::TokenBucket ? "ratelimiter.tokenbucket.rejected"
                                                       : "ratelimiter.requests.rejected"),
      engine_(std::move(engine)), algo_(algo), cfg_(cfg), clock_(std::move(clock)),
      windowMicros_(batchWindowMicros) {
    cfg_.validate();                                    // SlidingWindowRateLimiter.java:51
    if (algo == Algorithm::TokenBucket && !(cfg_.refillRate > 0))
        throw IllegalArgumentException(                // TokenBucketRateLimiter.java:77-79
            "Token bucket requires positive refillRate. Use RateLimitConfig.builder().refillRate(...)");
    id_ = engine_->addLimiter((int)algo, cfg_);
}

GpuRateLimiter::~GpuRateLimiter() { unpinFlush(); }

void GpuRateLimiter::unpinFlush() {
    if (fb_.cap == 0) return;
    engine_->unpin(fb_.key.data()); engine_->unpin(fb_.permits.data());
    engine_->unpin(fb_.now.data()); engine_->unpin(fb_.remaining.data());
    engine_->unpin(fb_.lim.data()); engine_->unpin(fb_.op.data()); engine_->unpin(fb_.allowed.data());
}

// Grow the flush buffers (doubling) and page-lock them once, so every later flush DMAs
// them directly (no pageable staging).
void GpuRateLimiter::reserveFlush(size_t n) {
    if (n <= fb_.cap) return;
    unpinFlush();
    size_t c = fb_.cap ? fb_.cap : 256;
    while (c < n) c *= 2;
    fb_.key.assign(c, 0); fb_.permits.assign(c, 0); fb_.now.assign(c, 0);
    fb_.remaining.assign(c, 0); fb_.lim.assign(c, id_); fb_.op.assign(c, 0); fb_.allowed.assign(c, 0);
    fb_.cap = c;
    engine_->pin(fb_.key.data(), c * 8); engine_->pin(fb_.permits.data(), c * 4);
    engine_->pin(fb_.now.data(), c * 8); engine_->pin(fb_.remaining.data(), c * 8);
    engine_->pin(fb_.lim.data(), c * 2); engine_->pin(fb_.op.data(), c);
    engine_->pin(fb_.allowed.data(), c);
}

void GpuRateLimiter::checkStatus(int st, const char* where) {
    if (st == RL_OK || st == RL_E_INVALID_REQUEST) return;
    if (st == RL_E_INVALID_ARG) throw IllegalArgumentException(std::string(where) + ": " + rl_strerror(st));
    throw StorageException(std::string(where) + ": " + rl_strerror(st), st);
}

// Leader-based micro-batcher: the first caller that finds no flush in progress waits
// `windowMicros_` for company, then runs every queued request as ONE engine batch in
// queue (arrival) order; the others sleep until their result is filled in.
// The request's clock is read here, under mu_, so queue order is clock order: two threads
// on one key can never enqueue their `now` values out of order (the engine's sliding
// window keeps a key's two newest buckets and assumes a key's time does not run
// backwards by more than a window).
void GpuRateLimiter::submit(Pending& p) {
    std::unique_lock<std::mutex> lk(mu_);
    p.now = clock_();
    queue_.push_back(&p);
    while (!p.done) {
        if (!flushing_) {
            flushing_ = true;
            if (windowMicros_ > 0) {
                lk.unlock();
                std::this_thread::sleep_for(std::chrono::microseconds(windowMicros_));
                lk.lock();
            }
            flushLocked(lk);
            flushing_ = false;
            cv_.notify_all();
        } else {
            cv_.wait(lk);
        }
    }
    if (p.status != RL_OK && p.status != RL_E_INVALID_REQUEST) checkStatus(p.status, "tryAcquire");
}

void GpuRateLimiter::flushLocked(std::unique_lock<std::mutex>& lk) {
    std::vector<Pending*> batch;
    batch.swap(queue_);
    lk.unlock();
    const size_t n = batch.size();
    reserveFlush(n);                    // the flush slot (flushing_) owns fb_
    uint64_t* k = fb_.key.data();
    int32_t* pm = fb_.permits.data();
    int64_t* t = fb_.now.data();
    uint8_t* op = fb_.op.data();
    for (size_t i = 0; i < n; ++i) {
        k[i] = batch[i]->key; pm[i] = batch[i]->permits; t[i] = batch[i]->now; op[i] = batch[i]->op;
    }
    uint64_t hits = 0;
    int st = engine_->executeBatch(n, k, pm, t, fb_.lim.data(), op, fb_.allowed.data(),
                                   fb_.remaining.data(), &hits);
    const uint8_t* al = fb_.allowed.data();
    const int64_t* rem = fb_.remaining.data();
    cacheHits.increment(hits);
    lk.lock();
    for (size_t i = 0; i < n; ++i) {
        batch[i]->allowed = al[i];
        batch[i]->remaining = rem[i];
        batch[i]->status = st;
        batch[i]->done = true;
    }
}

bool GpuRateLimiter::tryAcquire(const std::string& key, int permits) {
    if (permits <= 0) throw IllegalArgumentException("permits must be positive");  // :87-89 / :106-108
    Pending p{keyHash(key), permits, 0, RL_OP_ACQUIRE};
    submit(p);
    if (p.allowed) allowedRequests.increment();
    else rejectedRequests.increment();
    return p.allowed != 0;
}

int64_t GpuRateLimiter::getAvailablePermits(const std::string& key) {
    Pending p{keyHash(key), 1, 0, RL_OP_PEEK};
    submit(p);
    return p.remaining;
}

void GpuRateLimiter::reset(const std::string& key) {
    Pending p{keyHash(key), 1, 0, RL_OP_RESET};
    submit(p);
}

void GpuRateLimiter::tryAcquireBatch(size_t n, const uint64_t* keyHash, const int32_t* permits,
                                     const int64_t* nowNanos, bool* allowed, int64_t* remaining) {
    if (n == 0) return;
    std::vector<uint16_t> lim(n, id_);
    std::vector<uint8_t> al(n);
    std::vector<int64_t> rem(n);
    int st;
    {
        // keep arrival order with single calls: wait out a flush in progress (it runs with
        // mu_ released) and hold the flush slot while this batch runs
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !flushing_; });
        flushing_ = true;
        lk.unlock();
        uint64_t hits = 0;
        st = engine_->executeBatch(n, keyHash, permits, nowNanos, lim.data(), nullptr, al.data(),
                                   rem.data(), &hits);
        cacheHits.increment(hits);
        lk.lock();
        flushing_ = false;
        cv_.notify_all();
    }
    checkStatus(st, "tryAcquireBatch");
    uint64_t ok = 0;
    for (size_t i = 0; i < n; ++i) {
        allowed[i] = al[i] != 0;
        ok += al[i];
        if (remaining) remaining[i] = rem[i];
    }
    allowedRequests.increment(ok);
    rejectedRequests.increment(n - ok);
}

}  // namespace ratelimiter
