// The multi-GPU router through the C-ABI (include/rl_engine.h rl_router_*), checked
// bit-exactly against the CPU oracle (oracle/rl_oracle.c, test infrastructure) on the
// global arrival stream.
//   test_router loop : G = 2 and 4 routers (threads), each with its own engine shard, on the
//                      box's one GPU, over an in-process loopback transport; compact and wide
//                      layouts, token-bucket time regression (exception blocks), the hot-key
//                      directory, a collective error (a shard's region overflows), an
//                      engine failure on one rank, steps split into rounds (an owner receives
//                      more than its receive capacity), and what a router reserves
//   test_router rccl : one rank over the RCCL transport (librl_rccl.so), world 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rl_engine.h"
#include "../../include/rl_rccl.h"

extern "C" {   // oracle/rl_oracle.c (test infrastructure)
struct orc_state;
orc_state* orc_create(void);
void orc_destroy(orc_state*);
int orc_add_limiter(orc_state*, int algo, int64_t max, int64_t w, double refill);
size_t orc_run(orc_state*, size_t n, const uint64_t* key, const int32_t* permits,
               const int64_t* now_ns, const uint16_t* limiter, const uint8_t* op,
               uint8_t* allowed, int64_t* remaining, double* tokens_after);
}

static int failures = 0;
#define CHECK(c)                                                                      \
    do {                                                                              \
        if (!(c)) {                                                                   \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                               \
        }                                                                             \
    } while (0)
#define HIPC(x) CHECK((x) == hipSuccess)

static uint64_t mix(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

struct Trace {
    std::vector<uint64_t> key;
    std::vector<int32_t> permits;
    std::vector<int64_t> now;
    std::vector<uint16_t> lim;
};

// skewed keys (a few very hot), two limiters by key, arrival times over span_ms
static Trace make_trace(size_t total, uint64_t seed, int64_t span_ms, bool regress) {
    Trace t;
    const int64_t NS = 1000000, T0 = 1700000000000LL;
    for (size_t i = 0; i < total; ++i) {
        const double u = (double)(mix(seed ^ (i * 0x9E3779B97F4A7C15ULL)) >> 11) * 0x1.0p-53;
        const uint64_t rank = (uint64_t)(20000.0 * u * u * u * u);
        t.key.push_back(mix(rank + (seed << 32)));
        t.permits.push_back(1 + (int32_t)(mix(seed + 7 * i) % 4));
        int64_t ms = T0 + (int64_t)((double)i * (double)span_ms / (double)total);
        if (regress && (rank % 2) == 0 && mix(seed + 13 * i) % 200 == 0)
            ms -= (int64_t)(mix(seed + 17 * i) % 5000);          // TB keys: late arrivals
        t.now.push_back(ms * NS + (int64_t)(mix(i) % NS));
        t.lim.push_back((uint16_t)(rank % 2));
    }
    return t;
}

// ---- in-process loopback transport: G ranks in threads on one device ---------------
struct Loop {
    int G;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0, gen = 0;
    struct Post { const void* send; const uint64_t* so; const uint64_t* sb; } post[64];
    explicit Loop(int g) : G(g) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const int g = gen;
        if (++arrived == G) { arrived = 0; ++gen; cv.notify_all(); }
        else cv.wait(lk, [&] { return gen != g; });
    }
};
struct LoopRank { Loop* loop; int rank; };

static int loop_a2av(void* ctx, const void* send, const uint64_t* so, const uint64_t* sb, void* recv,
                     const uint64_t* ro, const uint64_t* rb, void* stream) {
    LoopRank* lr = (LoopRank*)ctx;
    Loop* L = lr->loop;
    hipStream_t s = (hipStream_t)stream;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;      // my send bytes are ready
    L->post[lr->rank] = {send, so, sb};
    L->barrier();
    int rc = 0;
    for (int p = 0; p < L->G; ++p) {
        const Loop::Post& q = L->post[p];
        if (q.sb[lr->rank] != rb[p]) rc = -1;                   // protocol mismatch
        if (rb[p] && hipMemcpyAsync((char*)recv + ro[p], (const char*)q.send + q.so[lr->rank], rb[p],
                                    hipMemcpyDeviceToDevice, s) != hipSuccess)
            rc = -1;
    }
    if (hipStreamSynchronize(s) != hipSuccess) rc = -1;
    L->barrier();                                               // peers may reuse their buffers
    return rc;
}

struct Result {
    std::vector<uint8_t> a; std::vector<int64_t> r; int finish = 0; uint32_t placed = 0; int step_rc = 0;
    int fail_step = -1;               // first step whose rl_router_step returned an error
    std::vector<int> rcs;             // every step's status
    rl_router_stats st{};
};

static const int64_t kLims[2][3] = {{1, 50, 60000}, {0, 30, 5000}};   // TB 50 @ 10/s, SW 30 / 5 s
static const double kRefill[2] = {10.0, 0.0};

static void run_rank(int G, int rank, Loop* loop, const Trace* tr, size_t n, int steps, bool dir,
                     uint64_t capacity, Result* out, rl_transport* ext_t = nullptr,
                     bool nosync_finish = false, size_t recv_cap = 0, int fail_at = -1) {
    HIPC(hipSetDevice(0));
    rl_opts o{};
    o.device = 0; o.max_batch = (uint64_t)G * n; o.default_capacity = capacity;
    o.shard_index = (uint32_t)rank; o.shard_count = (uint32_t)G;
    rl_engine* e = nullptr;
    CHECK(rl_create(&o, &e) == RL_OK);
    for (int l = 0; l < 2; ++l) {
        rl_limiter_config c{};
        c.algo = (int)kLims[l][0]; c.max_permits = kLims[l][1]; c.window_ms = kLims[l][2];
        c.refill_per_s = kRefill[l]; c.capacity = capacity;
        uint16_t id;
        CHECK(rl_add_limiter_ex(e, &c, &id) == RL_OK && id == l);
    }
    LoopRank lr{loop, rank};
    rl_transport t{&lr, loop_a2av};
    if (ext_t) t = *ext_t;
    rl_router* r = nullptr;
    rl_router_opts ro{};
    ro.max_batch = n; ro.recv_cap = recv_cap;
    CHECK(rl_router_create_ex(e, (uint32_t)G, (uint32_t)rank, &t, &ro, &r) == RL_OK);
    hipStream_t s;
    HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint64_t* dk; int32_t* dp; int64_t* dt; uint16_t* dl; uint8_t* da; int64_t* dr;
    HIPC(hipMalloc((void**)&dk, n * 8)); HIPC(hipMalloc((void**)&dp, n * 4)); HIPC(hipMalloc((void**)&dt, n * 8));
    HIPC(hipMalloc((void**)&dl, n * 2)); HIPC(hipMalloc((void**)&da, n)); HIPC(hipMalloc((void**)&dr, n * 8));
    if (dir) {                       // the hottest keys of this rank's whole slice as candidates
        std::map<uint64_t, uint64_t> cnt;
        for (int st = 0; st < steps; ++st)
            for (size_t i = 0; i < n; ++i) cnt[tr->key[((size_t)st * G + rank) * n + i]]++;
        std::vector<std::pair<uint64_t, uint64_t>> v(cnt.begin(), cnt.end());
        std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.second > b.second || (a.second == b.second && a.first < b.first); });
        v.resize(std::min<size_t>(v.size(), 64));
        std::vector<uint64_t> k, c;
        for (auto& x : v) { k.push_back(x.first); c.push_back(x.second); }
        CHECK(rl_router_plan_directory(r, k.size(), k.data(), c.data(), (uint64_t)steps * n, 16,
                                       &out->placed, s) == RL_OK);
    }
    out->a.resize((size_t)steps * n);
    out->r.resize((size_t)steps * n);
    for (int st = 0; st < steps; ++st) {
        const size_t b = ((size_t)st * G + rank) * n;
        HIPC(hipMemcpyAsync(dk, &tr->key[b], n * 8, hipMemcpyHostToDevice, s));
        HIPC(hipMemcpyAsync(dp, &tr->permits[b], n * 4, hipMemcpyHostToDevice, s));
        HIPC(hipMemcpyAsync(dt, &tr->now[b], n * 8, hipMemcpyHostToDevice, s));
        HIPC(hipMemcpyAsync(dl, &tr->lim[b], n * 2, hipMemcpyHostToDevice, s));
        if (st == fail_at) CHECK(rl_tune(e, "fail_batches", 1) == RL_OK);   // this rank's engine only
        const int rc = rl_router_step(r, n, dk, dp, dt, dl, da, dr, s);
        out->rcs.push_back(rc);
        if (rc != RL_OK && out->step_rc == RL_OK) { out->step_rc = rc; out->fail_step = st; }
        // nosync_finish: the last step's work is still queued on s when finish is called
        // (finish must wait for it itself)
        if (nosync_finish && st == steps - 1) out->finish = rl_router_finish(r);
        HIPC(hipMemcpyAsync(&out->a[(size_t)st * n], da, n, hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(&out->r[(size_t)st * n], dr, n * 8, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
    }
    if (!nosync_finish) out->finish = rl_router_finish(r);
    CHECK(rl_router_stats_get(r, &out->st) == RL_OK);
    rl_router_destroy(r);
    HIPC(hipFree(dk)); HIPC(hipFree(dp)); HIPC(hipFree(dt)); HIPC(hipFree(dl)); HIPC(hipFree(da)); HIPC(hipFree(dr));
    HIPC(hipStreamDestroy(s));
    rl_destroy(e);
}

static void compare(const Trace& tr, int G, size_t n, int steps, const std::vector<Result>& res,
                    const char* what) {
    const size_t N = tr.key.size();
    orc_state* o = orc_create();
    for (int l = 0; l < 2; ++l) orc_add_limiter(o, (int)kLims[l][0], kLims[l][1], kLims[l][2], kRefill[l]);
    std::vector<uint8_t> wa(N);
    std::vector<int64_t> wr(N);
    orc_run(o, N, tr.key.data(), tr.permits.data(), tr.now.data(), tr.lim.data(), nullptr, wa.data(),
            wr.data(), nullptr);
    orc_destroy(o);
    size_t bad = 0, neg = 0;
    for (int rank = 0; rank < G; ++rank)
        for (int st = 0; st < steps; ++st)
            for (size_t i = 0; i < n; ++i) {
                const size_t g = ((size_t)st * G + rank) * n + i, l = (size_t)st * n + i;
                if (res[rank].a[l] != wa[g] || res[rank].r[l] != wr[g]) {
                    if (bad < 3)
                        std::fprintf(stderr, "%s: rank %d step %d i %zu: got (%d,%lld) want (%d,%lld)\n", what,
                                     rank, st, i, res[rank].a[l], (long long)res[rank].r[l], wa[g], (long long)wr[g]);
                    ++bad;
                }
                neg += wr[g] < -3;
            }
    CHECK(bad == 0);
    std::printf("%s: %zu requests, %zu mismatches, %zu out-of-range remainders\n", what, N, bad, neg);
}

static void loop_case(int G, size_t n, int steps, int64_t span_ms, bool regress, bool dir,
                      const char* what, size_t recv_cap = 0) {
    Trace tr = make_trace((size_t)G * n * steps, 0xC0FFEE + G + (regress ? 7 : 0), span_ms, regress);
    Loop loop(G);
    std::vector<Result> res(G);
    std::vector<std::thread> th;
    for (int rank = 0; rank < G; ++rank)
        th.emplace_back(run_rank, G, rank, &loop, &tr, n, steps, dir, (uint64_t)1 << 16, &res[rank], nullptr,
                        false, recv_cap, -1);
    for (auto& x : th) x.join();
    for (int rank = 0; rank < G; ++rank) {
        CHECK(res[rank].step_rc == RL_OK);
        CHECK(res[rank].finish == RL_OK);
        CHECK(res[rank].st.steps == (uint64_t)steps);
        if (dir) CHECK(res[rank].placed == 16 && res[rank].placed == res[0].placed);
        if (recv_cap) {                          // every step split into the same rounds everywhere
            CHECK(res[rank].st.split_steps == (uint64_t)steps);
            CHECK(res[rank].st.rounds == res[0].st.rounds && res[rank].st.rounds > (uint64_t)steps);
            CHECK(res[rank].st.recv_cap == recv_cap);
        } else {
            CHECK(res[rank].st.split_steps == 0 && res[rank].st.rounds == (uint64_t)steps);
        }
    }
    compare(tr, G, n, steps, res, what);
    std::printf("  rounds %llu over %d steps, max received %llu, header sync %.3f ms/step\n",
                (unsigned long long)res[0].st.rounds, steps, (unsigned long long)res[0].st.max_recv,
                res[0].st.header_sync_ns * 1e-6 / steps);
}

// One rank's engine fails a batch (fail_batches, before anything is enqueued): that rank's
// step leaves its requests undecided and publishes the error; EVERY rank's next step returns
// it (the same status at the same step), and no rank hangs in a collective.
static void loop_engine_fail_case() {
    const int G = 4;
    const size_t n = 30000;
    const int steps = 4, fail_rank = 2, fail_at = 1;
    Trace tr = make_trace((size_t)G * n * steps, 0xFA11, 30000, false);
    Loop loop(G);
    std::vector<Result> res(G);
    std::vector<std::thread> th;
    for (int rank = 0; rank < G; ++rank)
        th.emplace_back(run_rank, G, rank, &loop, &tr, n, steps, false, (uint64_t)1 << 16, &res[rank],
                        nullptr, false, (size_t)0, rank == fail_rank ? fail_at : -1);
    for (auto& x : th) x.join();
    for (int rank = 0; rank < G; ++rank) {
        CHECK(res[rank].step_rc == RL_E_DEVICE);
        CHECK(res[rank].fail_step == fail_at + 1);
        CHECK(res[rank].finish == RL_OK);            // reported once, at the step
        // the step that returns the error did not decide its own batch: all of its outputs
        // say so (not the previous step's decisions, still in the caller's buffers)
        for (size_t i = 0; i < n; ++i) {
            const size_t l = (size_t)(fail_at + 1) * n + i;
            CHECK(res[rank].a[l] == 0 && res[rank].r[l] == RL_REMAINING_ERROR);
        }
    }
    std::printf("engine failure on rank %d at step %d: every rank's step %d returned %d %d %d %d\n",
                fail_rank, fail_at, res[0].fail_step, res[0].step_rc, res[1].step_rc, res[2].step_rc,
                res[3].step_rc);
}

// What a router reserves at creation: nothing proportional to world x max_batch (the receive
// side is recv_cap, default min(world, 2) x max_batch; the return trip is sized for the
// requests really exchanged, not world x max_batch per segment).
static void reserve_case() {
    const uint32_t G = 8;
    const size_t n = (size_t)1 << 20;
    rl_opts o{};
    o.device = 0; o.max_batch = 2 * n; o.default_capacity = 1 << 16; o.shard_index = 0; o.shard_count = G;
    rl_engine* e = nullptr;
    CHECK(rl_create(&o, &e) == RL_OK);
    rl_transport t{nullptr, [](void*, const void*, const uint64_t*, const uint64_t*, void*, const uint64_t*,
                               const uint64_t*, void*) { return -1; }};
    rl_router* r = nullptr;
    CHECK(rl_router_create(e, G, 0, &t, n, &r) == RL_OK);
    rl_router_stats st{};
    CHECK(rl_router_stats_get(r, &st) == RL_OK);
    CHECK(st.recv_cap == 2 * n);
    const uint64_t fixed = 4u << 20;                       // headers, directory, exception blocks
    CHECK(st.reserved_bytes <= 58 * (uint64_t)n + 65 * st.recv_cap + fixed);
    CHECK(st.reserved_bytes < (uint64_t)G * n * 47);      // round 3 reserved ~(47 G + 8 G^2) x n
    std::printf("router reserve: world %u, max_batch %zu -> recv_cap %llu, %.1f MB (%.1f B per request)\n",
                G, n, (unsigned long long)st.recv_cap, st.reserved_bytes / 1e6, (double)st.reserved_bytes / n);
    rl_router_destroy(r);
    // an explicit receive capacity is clamped to what the engine accepts
    rl_router_opts ro{};
    ro.max_batch = n; ro.recv_cap = 16 * n;
    CHECK(rl_router_create_ex(e, G, 0, &t, &ro, &r) == RL_OK);
    CHECK(rl_router_stats_get(r, &st) == RL_OK && st.recv_cap == 2 * n);
    rl_router_destroy(r);
    rl_destroy(e);
}

// finish called right after the last step, with that step still queued on the caller's
// stream (finish must order itself after it)
static void loop_nosync_finish_case() {
    const int G = 2;
    const size_t n = 60000;
    const int steps = 2;
    Trace tr = make_trace((size_t)G * n * steps, 0xF1515, 30000, true);
    Loop loop(G);
    std::vector<Result> res(G);
    std::vector<std::thread> th;
    for (int rank = 0; rank < G; ++rank)
        th.emplace_back(run_rank, G, rank, &loop, &tr, n, steps, false, (uint64_t)1 << 16, &res[rank],
                        nullptr, true, (size_t)0, -1);
    for (auto& x : th) x.join();
    for (int rank = 0; rank < G; ++rank) CHECK(res[rank].step_rc == RL_OK && res[rank].finish == RL_OK);
    compare(tr, G, n, steps, res, "G=2 finish without a caller sync");
}

// Sources whose first requests lie within 2^30 ms of each other, one of them spanning far
// past the other's compact window: the merged batch must run in full width (the router
// decides from the sources' real now ranges), not be rejected as a span overflow.
static void loop_span_case() {
    const int G = 2;
    const size_t n = 4000;
    Trace tr;
    const int64_t NS = 1000000, T0 = 1700000000000LL;
    for (size_t i = 0; i < (size_t)G * n; ++i) {
        const size_t rank = i / n, j = i % n;
        int64_t ms;
        if (rank == 0) ms = T0 + (int64_t)j;
        else ms = T0 + ((int64_t)1 << 30) - 1000 + (int64_t)j * (((int64_t)1 << 31) / (int64_t)n);
        tr.key.push_back(mix(i * 7919 + 3));                   // distinct keys
        tr.permits.push_back(1 + (int32_t)(mix(i) % 3));
        tr.now.push_back(ms * NS);
        tr.lim.push_back((uint16_t)(i % 2));
    }
    Loop loop(G);
    std::vector<Result> res(G);
    std::vector<std::thread> th;
    for (int rank = 0; rank < G; ++rank)
        th.emplace_back(run_rank, G, rank, &loop, &tr, n, 1, false, (uint64_t)1 << 14, &res[rank],
                        nullptr, false, (size_t)0, -1);
    for (auto& x : th) x.join();
    for (int rank = 0; rank < G; ++rank) CHECK(res[rank].step_rc == RL_OK && res[rank].finish == RL_OK);
    compare(tr, G, n, 1, res, "G=2 merged span > 2^31 ms (bases within 2^30)");
}

static void loop_error_case() {
    // a shard's table is far too small: its engine reports RL_E_CAPACITY, and every rank's
    // router reports it (two steps later or at finish), never just the one rank
    const int G = 2;
    const size_t n = 20000;
    const int steps = 4;
    Trace tr = make_trace((size_t)G * n * steps, 0xBAD, 60000, false);
    for (size_t i = 0; i < tr.key.size(); ++i) tr.key[i] = mix(i + 12345);   // all distinct keys
    Loop loop(G);
    std::vector<Result> res(G);
    std::vector<std::thread> th;
    for (int rank = 0; rank < G; ++rank)
        th.emplace_back(run_rank, G, rank, &loop, &tr, n, steps, false, (uint64_t)1, &res[rank], nullptr, false,
                        (size_t)0, -1);
    for (auto& x : th) x.join();
    for (int rank = 0; rank < G; ++rank) {
        const bool failed = res[rank].step_rc == RL_E_CAPACITY || res[rank].finish == RL_E_CAPACITY;
        CHECK(failed);
        CHECK(res[rank].step_rc == res[0].step_rc);
    }
    std::printf("collective error: step rc %d / %d, finish %d / %d\n", res[0].step_rc, res[1].step_rc,
                res[0].finish, res[1].finish);
}

// a rank that receives nothing in every round of a split step must not
// fold the previous batch's status again. Step 0 sends every request to owner 1 (distinct
// keys: its one-key table overflows, RL_E_CAPACITY) in split rounds, owner 0 receiving
// nothing; steps 1-3 send every request to owner 0 (64 keys), owner 1 receiving nothing in
// any round. The capacity error is reported exactly once by every rank, and owner 1's table
// grows once for it (not again for each empty step).
static void loop_empty_rounds_case() {
    const int G = 2;
    const size_t n = 20000;
    const int steps = 4;
    const int64_t NS = 1000000, T0 = 1700000000000LL;
    Trace tr;
    std::vector<uint64_t> own0, own1;
    for (uint64_t x = 1; own0.size() < 64 || own1.size() < (size_t)G * n; ++x) {
        const uint64_t k = mix(x * 0x9E3779B97F4A7C15ULL + 11);
        (rl_owner_of(k, 0, G) == 0 ? own0 : own1).push_back(k);
    }
    for (int st = 0; st < steps; ++st)
        for (size_t i = 0; i < (size_t)G * n; ++i) {
            tr.key.push_back(st == 0 ? own1[i] : own0[i % 64]);
            tr.permits.push_back(1);
            tr.now.push_back((T0 + st * 1000 + (int64_t)(i / 64)) * NS);
            tr.lim.push_back(0);
        }
    Loop loop(G);
    std::vector<Result> res(G);
    std::vector<std::thread> th;
    for (int rank = 0; rank < G; ++rank)
        th.emplace_back(run_rank, G, rank, &loop, &tr, n, steps, false, (uint64_t)1, &res[rank], nullptr,
                        false, (size_t)12000, -1);
    for (auto& x : th) x.join();
    for (int rank = 0; rank < G; ++rank) {
        int cap = res[rank].finish == RL_E_CAPACITY ? 1 : 0, other = 0;
        for (int rc : res[rank].rcs) {
            cap += rc == RL_E_CAPACITY;
            other += rc != RL_OK && rc != RL_E_CAPACITY;
        }
        CHECK(cap == 1 && other == 0);
        // every step splits, but the one returning the fatal status did not exchange its batch
        CHECK(res[rank].st.split_steps == (uint64_t)steps - 1);
        std::printf("empty split rounds: rank %d step statuses %d %d %d %d, finish %d\n", rank,
                    res[rank].rcs[0], res[rank].rcs[1], res[rank].rcs[2], res[rank].rcs[3], res[rank].finish);
    }
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "loop";
    if (mode == "loop") {
        loop_case(2, 100000, 3, 30000, false, false, "G=2 compact");
        loop_case(4, 50000, 3, 30000, false, false, "G=4 compact");
        loop_case(2, 50000, 2, (int64_t)1 << 36, false, false, "G=2 wide (span > 2^32 ms)");
        loop_case(4, 50000, 3, 30000, true, false, "G=4 TB regression (exception blocks)");
        loop_case(4, 50000, 3, 30000, false, true, "G=4 hot-key directory");
        loop_case(4, 50000, 3, 30000, false, false, "G=4 split rounds (recv_cap 20000)", 20000);
        loop_case(2, 50000, 2, (int64_t)1 << 36, false, false, "G=2 wide + split rounds", 30001);
        loop_case(4, 50000, 3, 30000, true, true, "G=4 directory + TB regression + split", 17777);
        loop_engine_fail_case();
        reserve_case();
        loop_nosync_finish_case();
        loop_span_case();
        loop_error_case();
        loop_empty_rounds_case();
    } else if (mode == "rccl") {
        char id[RL_RCCL_ID_BYTES];
        CHECK(rl_rccl_unique_id(id) == RL_OK);
        rl_transport t{};
        CHECK(rl_transport_rccl_create(id, 1, 0, 0, &t) == RL_OK);
        const size_t n = 200000;
        const int steps = 3;
        Trace tr = make_trace(n * steps, 0x5CC1, 30000, true);
        std::vector<Result> res(1);
        Loop loop(1);
        run_rank(1, 0, &loop, &tr, n, steps, false, (uint64_t)1 << 16, &res[0], &t);
        CHECK(res[0].step_rc == RL_OK && res[0].finish == RL_OK);
        compare(tr, 1, n, steps, res, "RCCL world 1");
        rl_transport_rccl_destroy(&t);
    }
    std::printf("%s: %s (%d failures)\n", mode.c_str(), failures ? "FAIL" : "ok", failures);
    return failures ? 1 : 0;
}
