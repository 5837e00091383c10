// C ABI of libtadpole_hip.so (include/tadpole_hip.h): device contexts, stage
// orchestration, and the host-side tail of find_params (R/TADpole.R:125-135:
// NA-padded score matrix, rowMeans(na.rm=TRUE) in long double as R does, first
// which.max) plus the hclust merge encoding of the chosen tree.
#include <atomic>
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tadpole_hip.h"
#include "tp_internal.h"

namespace tp {

static thread_local std::string g_err;
// status of the last fail() on this thread (-1: none since the last reset):
// lets a sharded call's scope guard tell data errors from device failures
static thread_local int t_fail_status = -1;

void fail(int status, const std::string &msg) {
    t_fail_status = status;
    throw Error{status, msg};
}

// TP_TRACE_SYNC=1 (debugging hangs): synchronise and report at stage marks
void trace_mark(hipStream_t s, const char *what) {
    static const bool on = getenv("TP_TRACE_SYNC") && getenv("TP_TRACE_SYNC")[0] == '1';
    if (!on) return;
    fprintf(stderr, "[tp] %s ...", what);
    fflush(stderr);
    const hipError_t e = hipStreamSynchronize(s);
    fprintf(stderr, " %s\n", e == hipSuccess ? "done" : hipGetErrorString(e));
    fflush(stderr);
}

void hip_check(hipError_t e, const char *what, const char *file, int line) {
    if (e != hipSuccess) {
        char b[512];
        snprintf(b, sizeof b, "HIP error %d (%s) at %s:%d: %s", (int)e, hipGetErrorString(e), file, line, what);
        fail(TP_ERR_HIP, b);
    }
}

std::atomic<int> g_devbuf_grows{0};   // knob 41 (read / reset): scratch regrowths so far
// knob 42: scratch grows in stream order (hipFreeAsync / hipMallocAsync on the
// context's stream, the device pool keeping what is freed) instead of a
// device-wide sync + hipFree + hipMalloc, which stalled every stream of a
// genome run (C4: ~35 regrowths a run while contexts meet larger chromosomes)

// The library's own stream-ordered pool per device (hipMemPoolCreate): scratch
// regrowth frees into it and takes from it without a device sync, and it keeps
// what is freed for reuse (release threshold: unlimited) -- but only this
// library's blocks: the device's default pool, which torch and other
// hipMallocAsync users share, is left as it was.  Retiring a context trims the
// pool (hipMemPoolTrimTo), so freed scratch goes back to the device.
static hipMemPool_t g_pool[64];
static std::mutex g_pool_mu;
static hipMemPool_t lib_pool(int device) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (device < 0 || device >= 64) return nullptr;
    if (!g_pool[device]) {
        hipMemPoolProps pp;
        memset(&pp, 0, sizeof pp);
        pp.allocType = hipMemAllocationTypePinned;
        pp.handleTypes = hipMemHandleTypeNone;
        pp.location.type = hipMemLocationTypeDevice;
        pp.location.id = device;
        hipMemPool_t pool = nullptr;
        if (hipMemPoolCreate(&pool, &pp) != hipSuccess) return nullptr;
        uint64_t keep = UINT64_MAX;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        g_pool[device] = pool;
    }
    return g_pool[device];
}
// give the pool's unused blocks back to the device (after a context's scratch went)
static void lib_pool_trim(int device) {
    hipMemPool_t pool = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (device >= 0 && device < 64) pool = g_pool[device];
    }
    if (pool) (void)hipMemPoolTrimTo(pool, 0);
}

// knob 51 (test hook): the next N scratch allocations fail as out-of-memory
// (after the old block is gone, where a real hipMalloc failure would strike)
std::atomic<int> g_devbuf_fail_inject{0};   // hook 51: the next N allocations fail
static void devbuf_inject_failure() {
    int inj = g_devbuf_fail_inject.load();
    while (inj > 0 && !g_devbuf_fail_inject.compare_exchange_weak(inj, inj - 1)) {
    }
    if (inj > 0) {
        fail(TP_ERR_HIP, "scratch allocation failed (injected out-of-memory, knob 51)");
    }
}

void *DevBuf::get(size_t b, bool exact) {
    if (b == 0) b = 8;
    if (b > bytes) {
        if (p) g_devbuf_grows.fetch_add(1, std::memory_order_relaxed);
        const size_t nb = exact ? b : std::max(b, bytes + bytes / 4);
        hipMemPool_t pool = (cfg_devbuf_async && owner && owner->cur) ? lib_pool(owner->device) : nullptr;
        // the old block goes first; bytes / pooled describe what p holds at every
        // point, so a failed allocation below leaves an empty buffer (p null,
        // bytes 0) that the next get() allocates again -- never a null block that
        // claims a size
        if (pool) {
            hipStream_t s = owner->cur;
            if (p) {
                // the old block's readers: this context's stream and its side
                // stream (joined into it first); no other stream uses it
                if (owner->side) {
                    TP_HIP(hipEventRecord(owner->join_ev, owner->side));
                    TP_HIP(hipStreamWaitEvent(s, owner->join_ev, 0));
                }
                void *old = p;
                const bool was_pooled = pooled;
                p = nullptr;
                bytes = 0;
                pooled = false;
                if (was_pooled) {
                    TP_HIP(hipFreeAsync(old, s));
                } else {
                    TP_HIP(hipDeviceSynchronize());
                    TP_HIP(hipFree(old));
                }
            }
            void *np = nullptr;
            devbuf_inject_failure();
            TP_HIP(hipMallocFromPoolAsync(&np, nb, pool, s));
            p = np;
            pooled = true;
        } else {
            // work queued on any stream may still read the old block
            if (p) {
                TP_HIP(hipDeviceSynchronize());
                void *old = p;
                const bool was_pooled = pooled;
                p = nullptr;
                bytes = 0;
                pooled = false;
                if (was_pooled) {
                    TP_HIP(hipFreeAsync(old, nullptr));
                    TP_HIP(hipDeviceSynchronize());
                } else {
                    TP_HIP(hipFree(old));
                }
            }
            void *np = nullptr;
            devbuf_inject_failure();
            TP_HIP(hipMalloc(&np, nb));
            p = np;
            pooled = false;
        }
        bytes = nb;
    }
    return p;
}
void DevBuf::release() {
    if (p) {
        if (pooled) {   // every call that queued work on the context synchronised before returning
            (void)hipDeviceSynchronize();
            (void)hipFreeAsync(p, nullptr);
            (void)hipDeviceSynchronize();
        } else {
            (void)hipFree(p);
        }
    }
    p = nullptr;
    bytes = 0;
    pooled = false;
}

void *Ctx::pinned(size_t b) {
    if (b > host_pinned_bytes) {
        if (host_pinned) TP_HIP(hipHostFree(host_pinned));
        host_pinned = nullptr;
        TP_HIP(hipHostMalloc(&host_pinned, b, hipHostMallocDefault));
        host_pinned_bytes = b;
    }
    return host_pinned;
}

hipStream_t side_fork(Ctx &c) {
    if (!c.side) {
        TP_HIP(hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking));
        TP_HIP(hipEventCreateWithFlags(&c.fork_ev, hipEventDisableTiming));
        TP_HIP(hipEventCreateWithFlags(&c.join_ev, hipEventDisableTiming));
    }
    TP_HIP(hipEventRecord(c.fork_ev, c.cur));
    TP_HIP(hipStreamWaitEvent(c.side, c.fork_ev, 0));
    return c.side;
}
void side_join(Ctx &c) {
    TP_HIP(hipEventRecord(c.join_ev, c.side));
    TP_HIP(hipStreamWaitEvent(c.cur, c.join_ev, 0));
}

static hipEvent_t next_event(Ctx &c) {
    if (c.evnext == c.evpool.size()) {
        hipEvent_t e;
        TP_HIP(hipEventCreate(&e));
        c.evpool.push_back(e);
    }
    return c.evpool[c.evnext++];
}
std::atomic<int> g_kprof_fine{1};
void kprof_begin(Ctx &c, int cls) {
    if (!c.prof || (cls == K_GQ_GEMM && !g_kprof_fine)) return;
    c.open_cls = cls;
    c.open_ev = next_event(c);
    TP_HIP(hipEventRecord(c.open_ev, c.cur));
}
void kprof_end(Ctx &c, int cls) {
    if (!c.prof || c.open_cls != cls) return;
    hipEvent_t e = next_event(c);
    TP_HIP(hipEventRecord(e, c.cur));
    c.recs.push_back({cls, c.open_ev, e});
    c.open_cls = -1;
}
void kprof_collect(Ctx &c, double *ms, int *cnt) {
    for (int q = 0; q < K_NCLASS; ++q) { ms[q] = 0; cnt[q] = 0; }
    for (auto &r : c.recs) {
        TP_HIP(hipEventSynchronize(r.b));
        float t = 0;
        TP_HIP(hipEventElapsedTime(&t, r.a, r.b));
        ms[r.cls] += t;
        cnt[r.cls] += 1;
    }
    c.recs.clear();
    c.evnext = 0;
}

// The registry lives on the heap and is never destroyed: contexts are freed by
// tp_shutdown / tp_release_stream / LRU retirement, never by static
// destructors at process exit (after the HIP runtime may be gone).
static std::mutex &g_mu = *new std::mutex;
static std::shared_ptr<Ctx> *const g_ctx = new std::shared_ptr<Ctx>[64];
// contexts of caller-supplied streams: one set of scratch buffers per stream,
// so pipelines on different streams of one device can run concurrently
static std::vector<std::pair<hipStream_t, std::shared_ptr<Ctx>>> *const g_sctx =
    new std::vector<std::pair<hipStream_t, std::shared_ptr<Ctx>>>[64];
// one sharded call at a time per device: an RCCL communicator is not for
// concurrent use from several streams, and an abort must not free it under
// another call
static std::mutex *const g_comm_mu = new std::mutex[64];
// the contexts this thread's current C-ABI call holds (locked)
static thread_local std::vector<std::shared_ptr<Ctx>> t_held;
static unsigned long long g_tick = 0;

// at most this many caller-stream contexts per device (env TP_MAX_STREAM_CONTEXTS,
// default 8): a new one retires the least recently used idle one
static size_t max_stream_ctx() {
    static const size_t v = [] {
        const char *e = getenv("TP_MAX_STREAM_CONTEXTS");
        const long x = e ? atol(e) : 8;
        return (size_t)(x < 1 ? 1 : x);
    }();
    return v;
}

static int g_created[64];   // contexts made per device (under g_mu)

static std::shared_ptr<Ctx> new_ctx(int device) {
    auto c = std::make_shared<Ctx>();
    c->device = device;
    for (auto &b : c->buf) b.owner = c.get();
    c->pinned_flag.owner = c.get();
    ++g_created[device];
    static bool pool_set[64];
    if (!pool_set[device]) {   // (under g_mu) the pool keeps what scratch regrowth frees, for reuse
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
            uint64_t keep = UINT64_MAX;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        }
        pool_set[device] = true;
    }
    return c;
}

static void ctx_stats(int device, int *live, int *created) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (device < 0 || device >= 64) fail(TP_ERR_ARG, "device index out of range");
    *live = (int)g_sctx[device].size();
    *created = g_created[device];
}

Ctx &ctx_for(int device, hipStream_t stream) {
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) fail(TP_ERR_HIP, "no HIP device available (libtadpole_hip has no CPU path)");
    if (device < 0 || device >= ndev || device >= 64) fail(TP_ERR_ARG, "device index out of range");
    std::shared_ptr<Ctx> c, retired;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        TP_HIP(hipSetDevice(device));
        if (!g_ctx[device]) {
            auto d = new_ctx(device);
            TP_HIP(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
            d->owns_stream = true;
            g_ctx[device] = d;
        }
        std::shared_ptr<Ctx> def = g_ctx[device];
        if (!stream || stream == def->stream) {
            c = def;
        } else {
            for (auto &pr : g_sctx[device])
                if (pr.first == stream) c = pr.second;
            if (!c) {
                auto &v = g_sctx[device];
                if (v.size() >= max_stream_ctx()) {
                    // retire the least recently used context no call is using
                    // (try_lock: not held; lookups need g_mu, which we hold)
                    size_t best = v.size();
                    for (size_t q = 0; q < v.size(); ++q)
                        if ((best == v.size() || v[q].second->last_use < v[best].second->last_use) &&
                            v[q].second->mu.try_lock()) {
                            v[q].second->mu.unlock();
                            best = q;
                        }
                    if (best < v.size()) {
                        retired = std::move(v[best].second);
                        v.erase(v.begin() + best);
                    }
                }
                c = new_ctx(device);
                c->stream = stream;
                c->owns_stream = false;
                v.push_back({stream, c});
            }
            // the communicator belongs to the device: every stream's context uses it
            c->shard.comm = def->shard.comm;
            c->shard.rank = def->shard.rank;
            c->shard.nranks = def->shard.nranks;
            c->shard.nvirt = def->shard.nvirt;
            c->shard.dead = def->shard.dead;
        }
        c->last_use = ++g_tick;
    }
    retired.reset();   // frees its device memory (outside the registry lock)
    // outside the registry lock: a long call on one stream does not block
    // lookups of the others
    c->mu.lock();
    t_held.push_back(c);
    TP_HIP(hipSetDevice(device));
    c->cur = c->stream;
    return *c;
}

void shard_lease_begin(Ctx &c) {
    g_comm_mu[c.device].lock();
    {
        std::lock_guard<std::mutex> lk(g_mu);
        const std::shared_ptr<Ctx> &def = g_ctx[c.device];
        if (def && def.get() != &c) {
            c.shard.comm = def->shard.comm;
            c.shard.rank = def->shard.rank;
            c.shard.nranks = def->shard.nranks;
            c.shard.nvirt = def->shard.nvirt;
            c.shard.dead = def->shard.dead;
        }
    }
    if (c.shard.dead && !c.shard.comm) {
        g_comm_mu[c.device].unlock();
        fail(TP_ERR_HIP, "sharded call: this device's RCCL communicator was aborted after an earlier failure; "
                         "make a new one (tp_comm_init / tadpole_amd.multi.init_comm) first");
    }
}

void shard_lease_end(Ctx &c) { g_comm_mu[c.device].unlock(); }

bool ctx_comm_retire(Ctx &c, void *comm) {
    std::lock_guard<std::mutex> lk(g_mu);
    const std::shared_ptr<Ctx> &def = g_ctx[c.device];
    if (!def || def->shard.comm != comm) return false;   // already retired (or replaced by tp_comm_init)
    def->shard.comm = nullptr;
    def->shard.rank = 0;
    def->shard.nranks = 1;
    def->shard.dead = true;
    // idle stream contexts keep a stale copy until their next lookup / lease,
    // both of which re-copy it from the device's context
    return true;
}

void ctx_unlock_held() {
    // unlock in reverse order; dropping the last reference frees a context
    // that tp_release_stream / tp_shutdown retired during the call
    while (!t_held.empty()) {
        std::shared_ptr<Ctx> c = std::move(t_held.back());
        t_held.pop_back();
        c->mu.unlock();
    }
}

Ctx::~Ctx() {
    (void)hipSetDevice(device);
    // a caller's stream may already be destroyed: every C-ABI call that queued
    // work on it synchronised before returning, and hipFree waits for the device
    if (stream && owns_stream) (void)hipStreamSynchronize(stream);
    for (auto &b : buf) b.release();
    pinned_flag.release();
    if (host_pinned) (void)hipHostFree(host_pinned);
    if (side) {
        (void)hipStreamSynchronize(side);
        (void)hipStreamDestroy(side);
        (void)hipEventDestroy(fork_ev);
        (void)hipEventDestroy(join_ev);
    }
    for (auto e : evpool) (void)hipEventDestroy(e);
    if (sync_ev) (void)hipEventDestroy(sync_ev);
    for (auto e : ring_ev)
        if (e) (void)hipEventDestroy(e);
    if (owns_stream) (void)hipStreamDestroy(stream);
    lib_pool_trim(device);   // the freed scratch goes back to the device
}

void ctx_shutdown_all() {
    std::vector<std::shared_ptr<Ctx>> dead;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (int d = 0; d < 64; ++d) {
            for (auto &pr : g_sctx[d]) dead.push_back(std::move(pr.second));
            g_sctx[d].clear();
            if (g_ctx[d]) dead.push_back(std::move(g_ctx[d]));
        }
    }
    // contexts in use by another thread are freed when that call ends
}

bool ctx_release_stream(int device, hipStream_t stream) {
    std::shared_ptr<Ctx> dead;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (device < 0 || device >= 64) return false;
        auto &v = g_sctx[device];
        for (size_t q = 0; q < v.size(); ++q)
            if (v[q].first == stream) {
                dead = std::move(v[q].second);
                v.erase(v.begin() + q);
                break;
            }
    }
    return dead != nullptr;   // freed here, or by the call that still holds it
}

// ---------------------------------------------------------- host helpers
// R/TADpole.R:134-135: which.max(rowMeans(scores, na.rm = TRUE)) and
// which.max(scores[n_PCs, ]); rowMeans sums in LDOUBLE (R array.c).
static void select_params(const double *scores, int k, int w, int *n_pcs, int *n_clusters) {
    int best = -1;
    double bestv = 0.0;
    // row sums in R's rowMeans order (j ascending per row, long double),
    // four rows at a time: four independent x87 chains held in registers (one
    // chain per row, or sums kept in memory, cost ~0.1 ms at k = 200, w = 210)
    std::vector<long double> s(k, 0.0L);
    std::vector<int> cnt(k, 0);
    int i0 = 0;
    for (; i0 + 4 <= k; i0 += 4) {
        long double a0 = 0.0L, a1 = 0.0L, a2 = 0.0L, a3 = 0.0L;
        int n0 = 0, n1 = 0, n2 = 0, n3 = 0;
        for (int j = 0; j < w; ++j) {
            const double *col = scores + (size_t)j * k + i0;
            const double v0 = col[0], v1 = col[1], v2 = col[2], v3 = col[3];
            if (!std::isnan(v0)) { a0 += v0; ++n0; }
            if (!std::isnan(v1)) { a1 += v1; ++n1; }
            if (!std::isnan(v2)) { a2 += v2; ++n2; }
            if (!std::isnan(v3)) { a3 += v3; ++n3; }
        }
        s[i0] = a0; s[i0 + 1] = a1; s[i0 + 2] = a2; s[i0 + 3] = a3;
        cnt[i0] = n0; cnt[i0 + 1] = n1; cnt[i0 + 2] = n2; cnt[i0 + 3] = n3;
    }
    for (; i0 < k; ++i0) {
        long double a = 0.0L;
        int c = 0;
        for (int j = 0; j < w; ++j) {
            const double v = scores[(size_t)j * k + i0];
            if (!std::isnan(v)) { a += v; ++c; }
        }
        s[i0] = a;
        cnt[i0] = c;
    }
    for (int i = 0; i < k; ++i) {
        if (cnt[i] == 0) continue;                 // NaN row mean: skipped by which.max
        double mean = (double)(s[i] / cnt[i]);
        if (std::isnan(mean)) continue;
        if (best < 0 || mean > bestv) { best = i; bestv = mean; }
    }
    if (best < 0) fail(TP_ERR_NUMERIC, "no finite Calinski-Harabasz row mean (which.max is empty)");
    int bj = -1;
    double bv = 0.0;
    for (int j = 0; j < w; ++j) {
        double v = scores[(size_t)best + (size_t)j * k];
        if (std::isnan(v)) continue;
        if (bj < 0 || v > bv) { bj = j; bv = v; }
    }
    *n_pcs = best + 1;
    *n_clusters = bj + 1;
}

// rioja chclust `merge` (R/TADpole.R:465, consumed by cutree / ggdendro at
// :231-232) in stats::hclust encoding: row s joins the clusters starting at
// mrg_a[s] (left) and mrg_b[s] (right); an observation is -(bin + 1), a cluster
// the 1-based step that made it (a merged cluster keeps its left part's id, as
// hclust keeps the smaller index).  hcass2's row order: a singleton before a
// cluster, the earlier step first of two clusters, two singletons left to right.
static void encode_merge(const int *mrg_a, const int *mrg_b, int n, int *merge) {
    std::vector<int> id(n);
    for (int p = 0; p < n; ++p) id[p] = -(p + 1);
    for (int s = 0; s < n - 1; ++s) {
        const int a = mrg_a[s], b = mrg_b[s];
        int x = id[a], y = id[b];
        if ((x > 0 && y < 0) || (x > 0 && y > 0 && x > y)) std::swap(x, y);
        merge[s] = x;
        merge[s + (n - 1)] = y;
        id[a] = s + 1;
    }
}

struct Timer {
    hipEvent_t ev[8];
    int n = 0;
    bool on;
    hipStream_t s;
    Timer(bool enable, hipStream_t st) : on(enable), s(st) {
        if (on) for (auto &e : ev) TP_HIP(hipEventCreate(&e));
    }
    void mark() {
        if (on && n < 8) TP_HIP(hipEventRecord(ev[n++], s));
    }
    void read(double *out) {
        if (!on || !out) return;
        TP_HIP(hipEventSynchronize(ev[n - 1]));
        for (int t = 1; t < n; ++t) {
            float ms = 0;
            TP_HIP(hipEventElapsedTime(&ms, ev[t - 1], ev[t]));
            out[t - 1] = ms;
        }
        float tot = 0;
        TP_HIP(hipEventElapsedTime(&tot, ev[0], ev[n - 1]));
        out[4] = tot;
    }
    ~Timer() {
        if (on) for (auto &e : ev) (void)hipEventDestroy(e);
    }
};

// ------------------------------------------------------------- sweep host
struct SweepOut {
    int w = 0, n_pcs = 0, n_clusters = 0;
};

// Runs the sweep for trees 1..k on device scores Pt (n x k row-major), copies
// n_cluster and the NA-padded scores to the host, selects (n_pcs, n_clusters)
// and fetches the merge record / heights of tree n_pcs.
static SweepOut run_sweep(Ctx &c, const double *d_Pt, int n, int k, int min_clusters, int w_cap_host,
                          int *n_cluster, double *scores, int *merge, double *height, int *boundary,
                          std::vector<int> *all_a = nullptr, std::vector<int> *all_b = nullptr,
                          std::vector<double> *all_cost = nullptr, std::vector<double> *all_h = nullptr) {
    hipStream_t s = c.cur;
    // trees 1..k, split in contiguous ranges over the shards (one range when
    // not sharded); per-shard outputs are packed blocks: n_cluster[t0..t1),
    // scores (t1 - t0) x w_cap column-major at offset t0 * w_cap
    const int R = shard_count(c);
    std::vector<int> tb(R + 1);
    shard_plan(k, R, 2, tb.data());
    SweepDev sd{};
    sd.Pt = d_Pt;
    sd.n = n;
    sd.ldp = k;
    sd.k = k;
    sd.min_clusters = min_clusters;
    // lean: asked for, or another pipeline is in flight on this device now
    // (concurrent streams: a tree of each fits on one CU; the same bits)
    sd.lds_lean = c.lds_lean || (cfg_lean_auto && pipelines_in_flight(c.device) > 1);
    double *sums = c.buf[S_SWEEP].as<double>(sweep_sums_doubles(n, 0, k));
    const size_t rec = (size_t)k * (n - 1);
    char *recbuf = c.buf[S_SWEEP2].as<char>(rec * (4 + 4 + 8 + 8) + 256);
    int *mrg_a = (int *)recbuf;
    int *mrg_b = mrg_a + rec;
    double *cost = (double *)(((uintptr_t)(mrg_b + rec) + 15) & ~(uintptr_t)15);
    double *hgt = cost + rec;
    sd.w_cap = std::max(1, n - 1);
    sd.seg_cap = std::min(sd.w_cap, 1024);
    char *sc = c.buf[S_SCORES].as<char>((size_t)k * sd.w_cap * 8 + (size_t)k * 4 + (size_t)R * 4 + 64);
    double *sc_all = (double *)sc;
    int *nc_all = (int *)(sc_all + (size_t)k * sd.w_cap);
    int *err_all = nc_all + k;   // one flag per shard
    sd.seg = c.buf[S_PARTIAL].as<double>((size_t)k * sd.seg_cap * (k + 1));
    sd.iseg = c.buf[S_MISC].as<int>((size_t)k * (2 * sd.seg_cap + 2) + 64) + 64;
    sd.trS = (double *)(c.buf[S_NGOOD].as<char>(64)) + 2;
    sd.cost0 = c.buf[S_SMALL].as<double>(sweep_cost0_doubles(n, k, k));
    if (cfg_ch_dedup) {   // CH segment statistics shared across trees
        int hcap = 0, ucap = 0;
        const size_t bytes = sweep_dedup_bytes(n, k, k, sd.seg_cap, &hcap, &ucap);
        sweep_dedup_bind(sd, c.buf[S_DEDUP].as<char>(bytes), hcap, ucap);
    }
    TP_HIP(hipMemsetAsync(err_all, 0, (size_t)R * sizeof(int), s));
    std::vector<SweepDev> mine;   // this rank's launched shards
    for (int r = 0; r < R; ++r) {
        const int t0 = tb[r], nt = tb[r + 1] - tb[r];
        if (!shard_mine(c, r) || nt == 0) continue;
        SweepDev d = sd;
        d.tree0 = t0;
        d.ntrees = nt;
        d.sums = sums + sweep_sums_doubles(n, 0, t0);   // offset of tree t0 + 1
        d.mrg_a = mrg_a + (size_t)t0 * (n - 1);
        d.mrg_b = mrg_b + (size_t)t0 * (n - 1);
        d.cost = cost + (size_t)t0 * (n - 1);
        d.height = hgt + (size_t)t0 * (n - 1);
        d.n_cluster = nc_all + t0;
        d.scores = sc_all + (size_t)t0 * sd.w_cap;   // ld = nt
        d.err = err_all + r;
        launch_sweep(d, s, &c);
        mine.push_back(d);
    }
    {
        std::vector<size_t> off(R + 1);
        for (int r = 0; r <= R; ++r) off[r] = (size_t)tb[r] * 4;
        shard_gather_bytes(c, nc_all, off);
        std::vector<size_t> off2(R + 1, 0);
        for (int r = 0; r < R; ++r) off2[r + 1] = (size_t)(r + 1) * 4;
        shard_gather_bytes(c, err_all, off2);
    }
    // host read-backs go through the context's pinned staging (one sync per
    // phase; pageable copies each stage and synchronise on their own)
    std::vector<int> h_nc(k), h_err(R);
    {
        int *pi = (int *)c.pinned((size_t)(k + R) * sizeof(int));   // nc_all and err_all are contiguous
        TP_HIP(hipMemcpyAsync(pi, nc_all, (size_t)(k + R) * sizeof(int), hipMemcpyDeviceToHost, s));
        stream_sync(c, s);
        memcpy(h_nc.data(), pi, k * sizeof(int));
        memcpy(h_err.data(), pi + k, R * sizeof(int));
    }
    for (int i = 0; i < k; ++i)
        if (h_nc[i] < 1)
            fail(TP_ERR_NO_BSTICK, "no broken-stick level is significant for PC prefix " + std::to_string(i + 1) +
                                       " (R: invalid 'times' argument at R/TADpole.R:115)");
    // trees whose finest cut exceeds k_ch's 1024 LDS segments (R's loop at
    // R/TADpole.R:117-120 has no limit): the global-memory CH kernel scores
    // them (on the rank that owns them, before the scores are gathered)
    for (const SweepDev &d : mine) {
        std::vector<int> slot(d.ntrees, -1);
        int nbig = 0, ncmax = 0;
        for (int ti = 0; ti < d.ntrees; ++ti) {
            const int nc = h_nc[d.tree0 + ti];
            if (nc > d.seg_cap) {
                slot[ti] = nbig++;
                ncmax = std::max(ncmax, nc);
            }
        }
        if (!nbig) continue;
        const size_t sd_d = ch_glb_slot_doubles(ncmax, d.k);
        char *big = c.buf[S_CHBIG].as<char>((size_t)nbig * sd_d * 8 + (size_t)d.ntrees * 4 + 256);
        int *d_slot = (int *)big;
        double *scr = (double *)(big + (((size_t)d.ntrees * 4 + 255) & ~(size_t)255));
        TP_HIP(hipMemcpyAsync(d_slot, slot.data(), (size_t)d.ntrees * 4, hipMemcpyHostToDevice, s));
        launch_ch_glb(d, d_slot, scr, sd_d, s);
        stream_sync(c, s);   // the host slot list lives on this stack frame
    }
    SweepOut o;
    o.w = *std::max_element(h_nc.begin(), h_nc.end());
    if (o.w > w_cap_host) fail(TP_ERR_CAPACITY, "scores capacity (w_cap) too small: need " + std::to_string(o.w));
    if (n_cluster) memcpy(n_cluster, h_nc.data(), k * sizeof(int));
    {
        std::vector<size_t> off(R + 1);
        for (int r = 0; r <= R; ++r) off[r] = (size_t)tb[r] * sd.w_cap;
        shard_gather(c, sc_all, off);   // whole blocks (each rank's w may differ)
    }
    // scores and the chosen tree's records are read straight out of the
    // context's pinned staging (no fresh host vectors: a k x w vector is a
    // new mmap per call, ~0.1 ms of page faults)
    const size_t sc_bytes = (size_t)k * o.w * sizeof(double);
    const size_t mrec_off = (sc_bytes * (R > 1 ? 2 : 1) + 255) & ~(size_t)255;
    char *pin = (char *)c.pinned(mrec_off + (size_t)(n - 1) * 16);
    double *ps = (double *)pin;
    const double *h_sc = ps;
    for (int r = 0; r < R; ++r) {
        const int t0 = tb[r], nt = tb[r + 1] - tb[r];
        if (nt == 0) continue;
        TP_HIP(hipMemcpyAsync(ps + (size_t)t0 * o.w, sc_all + (size_t)t0 * sd.w_cap,
                              (size_t)nt * o.w * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    stream_sync(c, s);
    if (R > 1) {
        // every shard's block (nt x w at offset t0 * w, ld nt) reordered to k x w
        double *sc = ps + (size_t)k * o.w;
        for (int r = 0; r < R; ++r) {
            const int t0 = tb[r], nt = tb[r + 1] - tb[r];
            const double *blk = ps + (size_t)t0 * o.w;
            for (int j = 0; j < o.w; ++j)
                for (int ti = 0; ti < nt; ++ti) sc[(size_t)(t0 + ti) + (size_t)j * k] = blk[(size_t)ti + (size_t)j * nt];
        }
        h_sc = sc;
    }
    select_params(h_sc, k, o.w, &o.n_pcs, &o.n_clusters);
    const int t = o.n_pcs - 1;
    {
        int owner = 0;
        while (owner + 1 < R && t >= tb[owner + 1]) ++owner;
        shard_bcast_bytes(c, mrg_a + (size_t)t * (n - 1), (size_t)(n - 1) * 4, owner);
        shard_bcast_bytes(c, mrg_b + (size_t)t * (n - 1), (size_t)(n - 1) * 4, owner);
        shard_bcast_bytes(c, hgt + (size_t)t * (n - 1), (size_t)(n - 1) * 8, owner);
    }
    char *pm = pin + mrec_off;   // a, b (ints), then heights (8-byte aligned)
    int *pa = (int *)pm, *pb = pa + (n - 1);
    double *ph = (double *)(pm + (size_t)(n - 1) * 8);
    TP_HIP(hipMemcpyAsync(pa, mrg_a + (size_t)t * (n - 1), (n - 1) * sizeof(int), hipMemcpyDeviceToHost, s));
    TP_HIP(hipMemcpyAsync(pb, mrg_b + (size_t)t * (n - 1), (n - 1) * sizeof(int), hipMemcpyDeviceToHost, s));
    TP_HIP(hipMemcpyAsync(ph, hgt + (size_t)t * (n - 1), (n - 1) * sizeof(double), hipMemcpyDeviceToHost, s));
    if (all_a) {
        if (R > 1 && c.shard.comm) fail(TP_ERR_ARG, "all-tree records are not gathered across ranks");
        all_a->resize(rec); all_b->resize(rec); all_cost->resize(rec); all_h->resize(rec);
        TP_HIP(hipMemcpyAsync(all_a->data(), mrg_a, rec * 4, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(all_b->data(), mrg_b, rec * 4, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(all_cost->data(), cost, rec * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(all_h->data(), hgt, rec * 8, hipMemcpyDeviceToHost, s));
    }
    // the caller's score matrix is filled while the chosen tree's records are
    // in flight (different parts of the pinned staging)
    if (scores) memcpy(scores, h_sc, sc_bytes);
    stream_sync(c, s);
    if (merge) encode_merge(pa, pb, n, merge);
    if (height) memcpy(height, ph, (n - 1) * sizeof(double));
    if (boundary)
        for (int q = 0; q < n - 1; ++q) boundary[q] = pb[q] + 1;
    return o;
}

// ------------------------------------------------------------ pipeline
static std::atomic<int> g_in_flight[64];
int pipelines_in_flight(int device) { return g_in_flight[device & 63].load(); }

struct PipeOut {
    int n_good = 0, k = 0;
    SweepOut sw;
};

static PipeOut pipeline_dev(Ctx &c, double *d_M, int n0, int max_pcs, int min_clusters, double bad_frac, int flags,
                            int k_cap, int w_cap, int *bad, int *good_idx, int *n_cluster, double *scores,
                            int *merge, double *height, int *boundary, double *timings, int n_sub = 0) {
    hipStream_t s = c.cur;
    if (n0 < 1) fail(TP_ERR_ARG, "empty matrix");
    if (max_pcs < 1) fail(TP_ERR_ARG, "max_pcs must be >= 1");
    if (!(bad_frac >= 0.0 && bad_frac <= 1.0)) fail(TP_ERR_ARG, "bad_frac must be in [0, 1]");
    Timer tm(timings != nullptr, s);
    // TP_FLAG_SHARDED: this call splits its products over the ranks of the
    // device's communicator (or its virtual shards), holding the device's
    // communicator lease for the whole call; reset on every exit.  A sharded
    // call that fails on a device / RCCL error (or anything that is not one of
    // the data errors below) aborts the communicator: its peers then leave
    // their collectives through their deadline (see stream_sync).  Data errors
    // (bad arguments, no broken-stick level, capacity, no convergence) come
    // from the replicated inputs and hit every rank at the same point, so the
    // communicator stays usable.  Checks of rank-local state (a shard's rows
    // against its slab or digit image) fail with TP_ERR_INTERNAL, which
    // aborts: its peers would otherwise wait in their collectives until the
    // deadline.
    struct ShardScope {
        Ctx &c;
        int pending;
        bool on;
        ShardScope(Ctx &cc, bool sharded) : c(cc), pending(std::uncaught_exceptions()), on(sharded) {
            if (on) shard_lease_begin(c);
            t_fail_status = -1;
            c.shard.active = on;
        }
        ~ShardScope() {
            const bool data_error = t_fail_status == TP_ERR_ARG || t_fail_status == TP_ERR_NO_BSTICK ||
                                    t_fail_status == TP_ERR_CAPACITY || t_fail_status == TP_ERR_NUMERIC ||
                                    t_fail_status == TP_ERR_UNSUPPORTED;
            if (c.shard.active && c.shard.comm && std::uncaught_exceptions() > pending && !data_error) comm_abort(c);
            c.shard.active = false;
            if (on) shard_lease_end(c);
        }
    } shard_scope(c, (flags & TP_FLAG_SHARDED) != 0);
    c.prof = timings != nullptr;
    c.lds_lean = (flags & TP_FLAG_LDS_LEAN) != 0;
    struct InFlight {   // this device's pipelines in flight (the sweep's lean choice)
        int d;
        explicit InFlight(int dev) : d(dev & 63) { g_in_flight[d].fetch_add(1); }
        ~InFlight() { g_in_flight[d].fetch_sub(1); }
    } in_flight(c.device);
    c.recs.clear();
    c.evnext = 0;
    // the caller's progress word (tp_progress_attach): 0 started, 1 mask read
    // back, 2 correlation queued, 3 PCA done (its last read-back) and the sweep
    // about to be queued, 4 done -- set on every exit too (a failure reads 4)
    struct Progress {
        int *p;
        void set(int v) {
            if (p) __atomic_store_n(p, v, __ATOMIC_RELEASE);
        }
        ~Progress() { set(4); }
    } progress{c.progress};
    progress.set(0);
    tm.mark();
    // ---- load_mat cleaning + mask + subset (R/TADpole.R:19-20,35-37,88-89)
    if (!(flags & TP_FLAG_CLEAN)) launch_clean_symmetrize(d_M, n0, !(flags & TP_FLAG_ROW_MAJOR), s);
    double *rm = c.buf[S_ROWMEAN].as<double>(n0);
    double *dg = c.buf[S_DIAG].as<double>(n0);
    int *d_bad = c.buf[S_BAD].as<int>(n0);
    int *d_good = c.buf[S_GOOD].as<int>(n0);
    int *d_ng = (int *)c.buf[S_NGOOD].as<char>(64);
    int n = 0;
    if (flags & TP_FLAG_SUBSET) {
        // the principal submatrix the caller names (a centromere arm's kept
        // bins, R/TADpole.R:362): the gather below reads only its rows and
        // columns, so the submatrix is never formed
        if (!good_idx || n_sub < 1 || n_sub > n0) fail(TP_ERR_ARG, "TP_FLAG_SUBSET: *n_good must be in 1..n0");
        std::vector<int> g(n_sub);
        for (int q = 0; q < n_sub; ++q) {
            g[q] = good_idx[q] - 1;
            if (g[q] < 0 || g[q] >= n0 || (q > 0 && g[q] <= g[q - 1]))
                fail(TP_ERR_ARG, "TP_FLAG_SUBSET: good_idx must hold strictly ascending 1-based indices into the matrix");
        }
        TP_HIP(hipMemcpyAsync(d_good, g.data(), n_sub * sizeof(int), hipMemcpyHostToDevice, s));
        TP_HIP(hipMemsetAsync(d_bad, 0, n0 * sizeof(int), s));
        stream_sync(c, s);
        n = n_sub;
    } else if (flags & TP_FLAG_NO_MASK) {
        std::vector<int> iota(n0);
        for (int q = 0; q < n0; ++q) iota[q] = q;
        TP_HIP(hipMemcpyAsync(d_good, iota.data(), n0 * sizeof(int), hipMemcpyHostToDevice, s));
        TP_HIP(hipMemsetAsync(d_bad, 0, n0 * sizeof(int), s));
        stream_sync(c, s);
        n = n0;
    } else {
        launch_rowmean_diag(d_M, n0, rm, dg, s);
        const double qindex = 1.0 + (double)(n0 - 1) * bad_frac;
        launch_mask_select(rm, dg, n0, bad_frac, qindex, d_bad, d_good, d_ng, s);
    }
    {
        // n_good, the mask and the good indices through the pinned staging:
        // one sync, then the gather is launched at once
        int *pi = (int *)c.pinned((size_t)(2 * n0 + 1) * sizeof(int));
        TP_HIP(hipMemcpyAsync(pi + 2 * n0, d_ng, sizeof(int), hipMemcpyDeviceToHost, s));
        if (bad) TP_HIP(hipMemcpyAsync(pi, d_bad, n0 * sizeof(int), hipMemcpyDeviceToHost, s));
        if (good_idx) TP_HIP(hipMemcpyAsync(pi + n0, d_good, n0 * sizeof(int), hipMemcpyDeviceToHost, s));
        stream_sync(c, s);
        if (!(flags & (TP_FLAG_NO_MASK | TP_FLAG_SUBSET))) n = pi[2 * n0];
        if (bad && !(flags & TP_FLAG_SUBSET)) memcpy(bad, pi, n0 * sizeof(int));
        if (good_idx) memcpy(good_idx, pi + n0, (size_t)n * sizeof(int));
    }
    PipeOut o;
    o.n_good = n;
    progress.set(1);
    if (n < 3) fail(TP_ERR_NO_BSTICK, "fewer than 3 good bins after masking");
    double *m = c.buf[S_COLMEAN].as<double>(n);
    // the gather also scans X for the exact int8 X'X (integrality, maximum,
    // S_jj) and builds its 2-slice image: no separate passes over X for them,
    // and X itself is written only if the fp64 product turns out to be needed
    // (non-integer counts: cor_product gathers it then)
    const bool prep = t_knob.xtx_fused && t_knob.xtx_int8 && n >= 1024 && n <= 130000;
    GatherStats gs{};
    double *X = nullptr;
    if (prep) {
        const int Kp = xtx_kp(n), Np = (n + 127) / 128 * 128;
        char *gb = c.buf[S_GSTAT].as<char>((size_t)n * 24 + 256);
        double *cmax = (double *)gb;
        long long *css = (long long *)(cmax + n);
        int *cbad = (int *)(css + n);
        int8_t *sl = xtx_slice_buf(c, n, 2);
        launch_gather_prep(d_M, n0, d_good, n, nullptr, m, cmax, cbad, css, sl, Kp, Np, s);
        gs = GatherStats{cmax, cbad, css, true, d_M, n0, d_good};
    } else {
        X = c.buf[S_X].as<double>((size_t)n * n);
        launch_gather_colmean(d_M, n0, d_good, n, X, m, s);
    }
    trace_mark(s, "mask");
    tm.mark();
    // ---- sparse_cor (R/TADpole.R:94-100,448-449)
    const int k = std::min(max_pcs, n);
    // C5 (one matrix over R > 1 shards, Krylov PCA, int8-exact X'X): C stays
    // row-sharded -- shard r computes and keeps only the columns (= rows, C is
    // symmetric) its Krylov products read, so C is never gathered; with real
    // ranks a rank allocates only its slab
    CorSlab slab;
    bool use_slab = false;
    {
        const int R = shard_count(c);
        const int b_est = std::min(n, ((k + std::max(32, k / 4) + 31) / 32) * 32);
        if (t_knob.shard_slab && c.shard.active && R > 1 && prep && n >= t_knob.pca_krylov_min && b_est < n) {
            const int ns = xtx_int_slices_cols(c, gs.cmax, gs.cbad, n);
            if (ns == 1 || ns == 2) {
                use_slab = true;
                slab.ns = ns;
                slab.rb.resize(R + 1);
                shard_plan(n + 2, R, 1, slab.rb.data());   // rows_gemm_sharded's row plan over [C | m | 1]
                slab.narrow = c.shard.comm != nullptr;
            }
        }
    }
    const int sc0 = use_slab && slab.narrow ? slab.rb[c.shard.rank] : 0;
    const int sc1 = use_slab && slab.narrow ? slab.rb[c.shard.rank + 1] : -1;
    double *C = use_slab && slab.narrow ? c.buf[S_C].as<double>((size_t)n * (sc1 - sc0) + 64)
                                        : c.buf[S_C].as<double>(pca_c_doubles(n));
    // C's column means, for prcomp (C's tail, or the [m | 1] buffer of a slab)
    double *cmean = use_slab ? c.buf[S_MEXT].as<double>(2 * (size_t)n) : (cfg_cor_fused ? C + (size_t)n * n : nullptr);
    trace_mark(s, "cor: start");
    bool cm_defer = !use_slab;   // C's means in the PCA's digit pass when C comes from the int8 X'X
    cor_product(c, X, n, m, prep ? &gs : nullptr, nullptr, C, c.buf[S_DIAG].as<double>(n), cmean,
                use_slab ? &slab : nullptr, &cm_defer);
    trace_mark(s, "cor");
    tm.mark();
    progress.set(2);
    // ---- prcomp (R/TADpole.R:452-453)
    o.k = k;
    if (k > k_cap) fail(TP_ERR_CAPACITY, "k_cap smaller than min(max_pcs, n_good)");
    double *P = c.buf[S_P].as<double>((size_t)n * k);
    double *Pt = c.buf[S_PT].as<double>(pt_doubles(n, k));
    PcaStats ps = pca_dev(c, C, n, k, P, Pt, nullptr, cmean, sc0, sc1, cm_defer);
    trace_mark(s, "pca");
    tm.mark();
    // ---- find_params + final tree (R/TADpole.R:456-460)
    progress.set(3);
    o.sw = run_sweep(c, Pt, n, k, min_clusters, w_cap, n_cluster, scores, merge, height, boundary);
    tm.mark();
    if (good_idx)
        for (int q = 0; q < n; ++q) good_idx[q] += 1;
    if (timings) {
        double t[8] = {0};
        tm.read(t);
        for (int q = 0; q < 5; ++q) timings[q] = t[q];
        double kms[K_NCLASS];
        int kcnt[K_NCLASS];
        kprof_collect(c, kms, kcnt);
        timings[5] = kms[K_COR_GEMM];
        timings[6] = kms[K_G_GEMM];
        timings[7] = kms[K_GQ_GEMM];
        timings[8] = kcnt[K_GQ_GEMM];
        timings[9] = kms[K_CONISS];
        timings[10] = kms[K_CH];
        timings[11] = ps.iters;
        timings[12] = ps.block;
        timings[13] = ps.resid;
        timings[14] = n;
        timings[15] = k;
        timings[16] = ps.krylov_steps;
        timings[17] = ps.krylov_dim;
        timings[18] = c.last_xtx_ns;
        timings[19] = ps.prod_pairs;
        for (int q = 20; q < 32; ++q) timings[q] = 0.0;
    }
    c.prof = false;
    return o;
}

thread_local Knobs t_knob;
static std::mutex &knob_mu() {
    static std::mutex m;
    return m;
}
static Knobs &knob_set() {   // the process-wide values tp_debug_knob sets
    static Knobs k;
    return k;
}

template <class F> static void guarded(int *status, F &&f) {
    struct Unlock {
        ~Unlock() { ctx_unlock_held(); }
    } unlock;
    {
        std::lock_guard<std::mutex> lk(knob_mu());
        t_knob = knob_set();   // this call's switches
    }
    try {
        f();
        if (status) *status = TP_OK;
    } catch (const Error &e) {
        g_err = e.msg;
        if (status) *status = e.status;
    } catch (const std::exception &e) {
        g_err = e.what();
        if (status) *status = TP_ERR_HIP;
    } catch (...) {
        g_err = "unknown error";
        if (status) *status = TP_ERR_HIP;
    }
}

static int dev_of(const int *device) { return device ? *device : 0; }

}  // namespace tp

using namespace tp;

extern "C" {

int tp_version(void) { return 2; }

int tp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void tp_shutdown(void) { ctx_shutdown_all(); }

void tp_release_stream(const int *device, void *stream, int *status) {
    guarded(status, [&] {
        if (!stream) fail(TP_ERR_ARG, "tp_release_stream: NULL stream (the library stream is freed by tp_shutdown)");
        (void)ctx_release_stream(dev_of(device), (hipStream_t)stream);
    });
}

/* Size the scratch of the contexts of `nstreams` caller streams alike: every
 * scratch buffer of each becomes at least as large as the largest of that
 * buffer over the set (stream-ordered allocation on each stream, no data
 * kept).  A pool of streams that any matrix of a workload may land on (genome
 * runs) then regrows no scratch once each matrix has run on one of them. */
void tp_reserve_streams(const int *device, void *const *streams, const int *nstreams, int *status) {
    guarded(status, [&] {
        const int ns = *nstreams;
        if (ns < 1 || !streams) fail(TP_ERR_ARG, "tp_reserve_streams: no streams");
        std::vector<Ctx *> cs;
        for (int q = 0; q < ns; ++q) {
            if (!streams[q]) fail(TP_ERR_ARG, "tp_reserve_streams: NULL stream");
            cs.push_back(&ctx_for(dev_of(device), (hipStream_t)streams[q]));   // locked until the call ends
        }
        for (int b = 0; b < S_NSLOT; ++b) {
            size_t mx = 0;
            for (Ctx *c : cs) mx = std::max(mx, c->buf[b].bytes);
            if (!mx) continue;
            for (Ctx *c : cs) {
                if (c->buf[b].bytes >= mx) continue;
                c->cur = c->stream;
                (void)c->buf[b].get(mx, true);   // exactly the largest: no headroom to leapfrog it
            }
        }
        for (Ctx *c : cs) TP_HIP(hipStreamSynchronize(c->stream));
    });
}

void tp_progress_attach(const int *device, void *stream, int *progress, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(dev_of(device), (hipStream_t)stream);
        c.progress = progress;
    });
}

void tp_context_stats(const int *device, int *live, int *created, int *status) {
    guarded(status, [&] {
        if (!live || !created) fail(TP_ERR_ARG, "tp_context_stats: NULL argument");
        ctx_stats(dev_of(device), live, created);
    });
}

/* ------------------------------------------------------------ multi-GPU */
void tp_comm_unique_id(char *id, int *status) {
    guarded(status, [&] { comm_unique_id(id); });
}

void tp_comm_init(const char *id, const int *nranks, const int *rank, const int *device, int *status) {
    guarded(status, [&] {
        if (!id || !nranks || !rank) fail(TP_ERR_ARG, "tp_comm_init: NULL argument");
        Ctx &c = ctx_for(dev_of(device));
        std::lock_guard<std::mutex> lease(g_comm_mu[c.device]);   // no sharded call is using the old one
        comm_init(c, id, *nranks, *rank);
    });
}

void tp_comm_destroy(const int *device) {
    int st = 0;
    guarded(&st, [&] {
        Ctx &c = ctx_for(dev_of(device));
        std::lock_guard<std::mutex> lease(g_comm_mu[c.device]);
        comm_destroy(c);
        c.shard.dead = false;   // destroyed on purpose: the next sharded call runs on virtual shards / one rank
    });
}

void tp_set_virtual_shards(const int *device, const int *nvirt, int *status) {
    guarded(status, [&] {
        if (!nvirt || *nvirt < 1 || *nvirt > 64) fail(TP_ERR_ARG, "virtual shards must be in 1..64");
        Ctx &c = ctx_for(dev_of(device));
        if (c.shard.comm) fail(TP_ERR_ARG, "device has a communicator: virtual shards are a single-device hook");
        c.shard.nvirt = *nvirt;
    });
}

void tp_shard_plan(const int *n, const int *nranks, const int *kind, int *bounds, int *status) {
    guarded(status, [&] {
        if (!n || !nranks || !kind || !bounds || *n < 0 || *kind < 0 || *kind > 2) fail(TP_ERR_ARG, "tp_shard_plan");
        shard_plan(*n, *nranks, *kind, bounds);
    });
}

int tp_last_error(char *buf, int len) {
    if (!buf || len <= 0) return (int)g_err.size();
    snprintf(buf, (size_t)len, "%s", g_err.c_str());
    return (int)g_err.size();
}

void tp_last_error_r(char **buf, int *len) {
    if (buf && buf[0] && len && *len > 0) snprintf(buf[0], (size_t)*len, "%s", g_err.c_str());
}

static void mask_core(Ctx &c, double *dM, int N0, double bf, int fl, int *bad, double *rowmean, int *n_good,
                      int *good_idx) {
    hipStream_t s = c.cur;
    if (!(fl & TP_FLAG_CLEAN)) launch_clean_symmetrize(dM, N0, !(fl & TP_FLAG_ROW_MAJOR), s);
    double *rm = c.buf[S_ROWMEAN].as<double>(N0);
    double *dg = c.buf[S_DIAG].as<double>(N0);
    int *d_bad = c.buf[S_BAD].as<int>(N0);
    int *d_good = c.buf[S_GOOD].as<int>(N0);
    int *d_ng = (int *)c.buf[S_NGOOD].as<char>(64);
    launch_rowmean_diag(dM, N0, rm, dg, s);
    launch_mask_select(rm, dg, N0, bf, 1.0 + (double)(N0 - 1) * bf, d_bad, d_good, d_ng, s);
    int ng = 0;
    TP_HIP(hipMemcpyAsync(&ng, d_ng, 4, hipMemcpyDeviceToHost, s));
    if (bad) TP_HIP(hipMemcpyAsync(bad, d_bad, N0 * 4, hipMemcpyDeviceToHost, s));
    if (rowmean) TP_HIP(hipMemcpyAsync(rowmean, rm, N0 * 8, hipMemcpyDeviceToHost, s));
    if (good_idx) TP_HIP(hipMemcpyAsync(good_idx, d_good, N0 * 4, hipMemcpyDeviceToHost, s));
    TP_HIP(hipStreamSynchronize(s));
    if (n_good) *n_good = ng;
    if (good_idx)
        for (int q = 0; q < ng; ++q) good_idx[q] += 1;
}

void tp_mask(const double *M, const int *n0, const double *bad_frac, const int *flags, const int *device, int *bad,
             double *rowmean, int *n_good, int *good_idx, int *status) {
    guarded(status, [&] {
        if (!M || !n0 || *n0 < 1) fail(TP_ERR_ARG, "bad matrix");
        Ctx &c = ctx_for(dev_of(device));
        const int N0 = *n0;
        double *dM = c.buf[S_M].as<double>((size_t)N0 * N0);
        TP_HIP(hipMemcpyAsync(dM, M, (size_t)N0 * N0 * 8, hipMemcpyHostToDevice, c.cur));
        mask_core(c, dM, N0, bad_frac ? *bad_frac : 0.01, flags ? *flags : 0, bad, rowmean, n_good, good_idx);
    });
}

void tp_mask_dev(double *d_M, const int *n0, const double *bad_frac, const int *flags, const int *device,
                 void *stream, int *bad, double *rowmean, int *n_good, int *good_idx, int *status) {
    guarded(status, [&] {
        if (!d_M || !n0 || *n0 < 1) fail(TP_ERR_ARG, "bad matrix");
        Ctx &c = ctx_for(dev_of(device), (hipStream_t)stream);
        mask_core(c, d_M, *n0, bad_frac ? *bad_frac : 0.01, flags ? *flags : 0, bad, rowmean, n_good, good_idx);
    });
}

void tp_cor(const double *X, const int *n, const int *device, double *cor, int *status) {
    guarded(status, [&] {
        if (!X || !n || *n < 2 || !cor) fail(TP_ERR_ARG, "bad arguments");
        Ctx &c = ctx_for(dev_of(device));
        hipStream_t s = c.cur;
        const int N = *n;
        double *dX = c.buf[S_X].as<double>((size_t)N * N);
        TP_HIP(hipMemcpyAsync(dX, X, (size_t)N * N * 8, hipMemcpyHostToDevice, s));
        double *m = c.buf[S_COLMEAN].as<double>(N);
        launch_colmean(dX, N, N, m, s);
        double *S = c.buf[S_S].as<double>((size_t)N * N);
        double *C = c.buf[S_C].as<double>((size_t)N * N);
        xtx_product(c, dX, N, S);
        launch_cor_epilogue(S, m, N, C, c.buf[S_DIAG].as<double>(N), s);
        TP_HIP(hipMemcpyAsync(cor, C, (size_t)N * N * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
    });
}

void tp_pca(const double *C, const int *n, const int *k, const int *device, double *P, double *sdev, int *status) {
    guarded(status, [&] {
        if (!C || !n || !k || *n < 2 || *k < 1 || *k > *n || !P) fail(TP_ERR_ARG, "bad arguments");
        Ctx &c = ctx_for(dev_of(device));
        hipStream_t s = c.cur;
        const int N = *n, K = *k;
        double *dC = c.buf[S_C].as<double>(pca_c_doubles(N));
        TP_HIP(hipMemcpyAsync(dC, C, (size_t)N * N * 8, hipMemcpyHostToDevice, s));
        double *dP = c.buf[S_P].as<double>((size_t)N * K);
        pca_dev(c, dC, N, K, dP, nullptr, sdev);
        TP_HIP(hipMemcpyAsync(P, dP, (size_t)N * K * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
    });
}

void tp_sweep(const double *P, const int *n, const int *k, const int *min_clusters, const int *device,
              const int *w_cap, int *n_cluster, double *scores, int *w, int *n_pcs, int *n_clusters, int *merge,
              double *height, int *status) {
    guarded(status, [&] {
        if (!P || !n || !k || *n < 3 || *k < 1 || !w_cap) fail(TP_ERR_ARG, "bad arguments");
        Ctx &c = ctx_for(dev_of(device));
        hipStream_t s = c.cur;
        const int N = *n, K = *k;
        double *dP = c.buf[S_P].as<double>((size_t)N * K);
        double *dPt = c.buf[S_PT].as<double>(pt_doubles(N, K));
        TP_HIP(hipMemcpyAsync(dP, P, (size_t)N * K * 8, hipMemcpyHostToDevice, s));
        launch_transpose(dP, N, K, N, dPt, K, s);
        SweepOut o = run_sweep(c, dPt, N, K, min_clusters ? *min_clusters : 2, *w_cap, n_cluster, scores, merge,
                               height, nullptr);
        if (w) *w = o.w;
        if (n_pcs) *n_pcs = o.n_pcs;
        if (n_clusters) *n_clusters = o.n_clusters;
    });
}

void tp_sweep_dev(const double *d_P, const int *n, const int *k, const int *min_clusters, const int *device,
                  void *stream, const int *w_cap, int *n_cluster, double *scores, int *w, int *mrg_a_all,
                  int *mrg_b_all, double *cost_all, double *height_all, int *status) {
    guarded(status, [&] {
        if (!d_P || !n || !k || *n < 3 || *k < 1 || !w_cap) fail(TP_ERR_ARG, "bad arguments");
        Ctx &c = ctx_for(dev_of(device), (hipStream_t)stream);
        hipStream_t s = c.cur;
        const int N = *n, K = *k;
        double *dPt = c.buf[S_PT].as<double>(pt_doubles(N, K));
        launch_transpose(d_P, N, K, N, dPt, K, s);
        std::vector<int> A, B;
        std::vector<double> Co, H;
        bool want = mrg_a_all || mrg_b_all || cost_all || height_all;
        SweepOut o = run_sweep(c, dPt, N, K, min_clusters ? *min_clusters : 2, *w_cap, n_cluster, scores, nullptr,
                               nullptr, nullptr, want ? &A : nullptr, want ? &B : nullptr, want ? &Co : nullptr,
                               want ? &H : nullptr);
        if (w) *w = o.w;
        if (want) {
            if (mrg_a_all) memcpy(mrg_a_all, A.data(), A.size() * 4);
            if (mrg_b_all) memcpy(mrg_b_all, B.data(), B.size() * 4);
            if (cost_all) memcpy(cost_all, Co.data(), Co.size() * 8);
            if (height_all) memcpy(height_all, H.data(), H.size() * 8);
        }
    });
}

void tp_coniss(const double *P, const int *n, const int *ncols, const int *device, int *merge, double *height,
               int *boundary, int *status) {
    guarded(status, [&] {
        if (!P || !n || !ncols || *n < 2 || *ncols < 1 || *ncols > 1024) fail(TP_ERR_ARG, "bad arguments");
        Ctx &c = ctx_for(dev_of(device));
        hipStream_t s = c.cur;
        const int N = *n, K = *ncols;
        double *dP = c.buf[S_P].as<double>((size_t)N * K);
        double *dPt = c.buf[S_PT].as<double>(pt_doubles(N, K));
        TP_HIP(hipMemcpyAsync(dP, P, (size_t)N * K * 8, hipMemcpyHostToDevice, s));
        launch_transpose(dP, N, K, N, dPt, K, s);
        SweepDev sd{};
        sd.Pt = dPt;
        sd.n = N;
        sd.ldp = K;
        sd.k = K;
        sd.tree0 = K - 1;
        sd.ntrees = 1;
        sd.min_clusters = 2;
        sd.sums = c.buf[S_SWEEP].as<double>(sweep_sums_doubles(N, K - 1, 1));
        char *recbuf = c.buf[S_SWEEP2].as<char>((size_t)(N - 1) * 24 + 256);
        sd.mrg_a = (int *)recbuf;
        sd.mrg_b = sd.mrg_a + (N - 1);
        sd.cost = (double *)(((uintptr_t)(sd.mrg_b + (N - 1)) + 15) & ~(uintptr_t)15);
        sd.height = sd.cost + (N - 1);
        sd.n_cluster = c.buf[S_MISC].as<int>(64);
        sd.cost0 = c.buf[S_SMALL].as<double>(sweep_cost0_doubles(N, 1, K));
        sd.w_cap = std::max(1, N - 1);
        // CONISS only (the CH half needs a broken-stick cut; not wanted here)
        launch_coniss_only(sd, s);
        std::vector<int> ma(N - 1), mb(N - 1);
        std::vector<double> he(N - 1);
        TP_HIP(hipMemcpyAsync(ma.data(), sd.mrg_a, (N - 1) * 4, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(mb.data(), sd.mrg_b, (N - 1) * 4, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(he.data(), sd.height, (N - 1) * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
        if (merge) encode_merge(ma.data(), mb.data(), N, merge);
        if (height) memcpy(height, he.data(), (N - 1) * 8);
        if (boundary)
            for (int q = 0; q < N - 1; ++q) boundary[q] = mb[q] + 1;
    });
}

void tp_dist(const double *P, const int *n, const int *ncols, const int *device, double *d, int *status) {
    guarded(status, [&] {
        if (!P || !n || !ncols || *n < 2 || *ncols < 1 || !d) fail(TP_ERR_ARG, "bad arguments");
        Ctx &c = ctx_for(dev_of(device));
        hipStream_t s = c.cur;
        const int N = *n, K = *ncols;
        double *dP = c.buf[S_P].as<double>((size_t)N * K);
        size_t nd = (size_t)N * (N - 1) / 2;
        double *dd = c.buf[S_S].as<double>(nd);
        TP_HIP(hipMemcpyAsync(dP, P, (size_t)N * K * 8, hipMemcpyHostToDevice, s));
        launch_dist(dP, N, N, K, dd, s);
        TP_HIP(hipMemcpyAsync(d, dd, nd * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
    });
}

void tp_ch(const double *P, const int *n, const int *k, const int *labels, const int *cn, const int *device,
           double *ch, int *status) {
    guarded(status, [&] {
        if (!P || !n || !k || !labels || !cn || *n < 2 || *k < 1 || *k > 1024 || *cn < 1 || !ch)
            fail(TP_ERR_ARG, "bad arguments");
        const int N = *n, K = *k, CN = *cn;
        std::vector<int> bnd(CN + 1);
        bnd[0] = 0;
        int g = 0;
        if (labels[0] != 1) fail(TP_ERR_ARG, "labels must be contiguous 1..cn in order");
        for (int a = 1; a < N; ++a) {
            if (labels[a] == labels[a - 1]) continue;
            if (labels[a] != labels[a - 1] + 1) fail(TP_ERR_ARG, "labels must be contiguous 1..cn in order");
            bnd[++g] = a;
        }
        if (g + 1 != CN) fail(TP_ERR_ARG, "cn does not match the number of label runs");
        bnd[CN] = N;
        Ctx &c = ctx_for(dev_of(device));
        hipStream_t s = c.cur;
        double *dP = c.buf[S_P].as<double>((size_t)N * K);
        double *dPt = c.buf[S_PT].as<double>(pt_doubles(N, K));
        int *dB = c.buf[S_GOOD].as<int>(CN + 1);
        double *seg = c.buf[S_PARTIAL].as<double>(CN + 8);
        double *out = c.buf[S_SMALL].as<double>(8);
        TP_HIP(hipMemcpyAsync(dP, P, (size_t)N * K * 8, hipMemcpyHostToDevice, s));
        TP_HIP(hipMemcpyAsync(dB, bnd.data(), (CN + 1) * 4, hipMemcpyHostToDevice, s));
        launch_transpose(dP, N, K, N, dPt, K, s);
        launch_ch_only(dPt, N, K, K, dB, CN, seg, out, s);
        TP_HIP(hipMemcpyAsync(ch, out, 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
    });
}

static void pipeline_common(double *dM, const int *n0, const int *max_pcs, const int *min_clusters,
                            const double *bad_frac, const int *flags, Ctx &c, const int *k_cap, const int *w_cap,
                            int *bad, int *n_good, int *good_idx, int *k, int *n_cluster, double *scores, int *w,
                            int *n_pcs, int *n_clusters, int *merge, double *height, int *boundary,
                            double *timings_ms) {
    PipeOut o = pipeline_dev(c, dM, *n0, max_pcs ? *max_pcs : 200, min_clusters ? *min_clusters : 2,
                             bad_frac ? *bad_frac : 0.01, flags ? *flags : 0, k_cap ? *k_cap : 0,
                             w_cap ? *w_cap : 0, bad, good_idx, n_cluster, scores, merge, height, boundary,
                             timings_ms, flags && (*flags & TP_FLAG_SUBSET) && n_good ? *n_good : 0);
    if (n_good) *n_good = o.n_good;
    if (k) *k = o.k;
    if (w) *w = o.sw.w;
    if (n_pcs) *n_pcs = o.sw.n_pcs;
    if (n_clusters) *n_clusters = o.sw.n_clusters;
}

void tp_pipeline(const double *M, const int *n0, const int *max_pcs, const int *min_clusters,
                 const double *bad_frac, const int *flags, const int *device, const int *k_cap, const int *w_cap,
                 int *bad, int *n_good, int *good_idx, int *k, int *n_cluster, double *scores, int *w, int *n_pcs,
                 int *n_clusters, int *merge, double *height, int *boundary, double *timings_ms, int *status) {
    guarded(status, [&] {
        if (!M || !n0 || *n0 < 1) fail(TP_ERR_ARG, "bad matrix");
        Ctx &c = ctx_for(dev_of(device));
        const size_t bytes = (size_t)(*n0) * (*n0) * 8;
        double *dM = c.buf[S_M].as<double>((size_t)(*n0) * (*n0));
        // through the context's pinned ring, count blocks packed to 16 bits
        upload_host(c, M, bytes, dM, bytes >= ((size_t)256 << 20) ? 8 : (bytes >= ((size_t)64 << 20) ? 4 : 1), true);
        pipeline_common(dM, n0, max_pcs, min_clusters, bad_frac, flags, c, k_cap, w_cap, bad, n_good, good_idx, k,
                        n_cluster, scores, w, n_pcs, n_clusters, merge, height, boundary, timings_ms);
    });
}

void tp_pipeline_dev(const double *d_M, const int *n0, const int *max_pcs, const int *min_clusters,
                     const double *bad_frac, const int *flags, const int *device, void *stream, const int *k_cap,
                     const int *w_cap, int *bad, int *n_good, int *good_idx, int *k, int *n_cluster, double *scores,
                     int *w, int *n_pcs, int *n_clusters, int *merge, double *height, int *boundary,
                     double *timings_ms, int *status) {
    guarded(status, [&] {
        if (!d_M || !n0 || *n0 < 1) fail(TP_ERR_ARG, "bad matrix");
        Ctx &c = ctx_for(dev_of(device), (hipStream_t)stream);
        pipeline_common(const_cast<double *>(d_M), n0, max_pcs, min_clusters, bad_frac, flags, c, k_cap, w_cap,
                        bad, n_good, good_idx, k, n_cluster, scores, w, n_pcs, n_clusters, merge, height, boundary,
                        timings_ms);
    });
}

/* R/TADpole.R:470-488 for every level at once: the cuts of the constrained
 * tree are nested (the cut into kk clusters is the cut into kk - 1 plus
 * boundary[n - kk]), so one stable sort of the deepest level's boundaries
 * gives every level's boundaries in order.  Host-only (no device). */
void tp_level_coords(const int *boundary, const int *n, const int *levels, const int *nlev, const int *pos, int *out,
                     int *status) {
    guarded(status, [&] {
        if (!n || *n < 1 || !nlev || *nlev < 0 || (*nlev && (!levels || !pos || !out)) || (*n > 1 && !boundary))
            fail(TP_ERR_ARG, "tp_level_coords: bad arguments");
        const int N = *n, NL = *nlev;
        int L = 1;
        for (int l = 0; l < NL; ++l) {
            if (levels[l] < 1 || levels[l] > N) fail(TP_ERR_ARG, "tp_level_coords: level outside 1..n");
            L = std::max(L, levels[l]);
        }
        // B[j] = boundary[n - L + j] (j < L - 1) joins the cut at level L - j
        std::vector<std::pair<int, int>> vb;   // (boundary, join level), stable by boundary
        vb.reserve(L - 1);
        for (int j = 0; j < L - 1; ++j) {
            const int v = boundary[N - L + j];
            if (v < 2 || v > N) fail(TP_ERR_ARG, "tp_level_coords: boundary outside 2..n");
            vb.push_back({v, L - j});
        }
        std::stable_sort(vb.begin(), vb.end(),
                         [](const std::pair<int, int> &a, const std::pair<int, int> &b) { return a.first < b.first; });
        int *o = out;
        for (int l = 0; l < NL; ++l) {
            const int kk = levels[l];
            o[0] = pos[0];
            for (const auto &e : vb) {
                if (e.second > kk) continue;
                o[1] = pos[e.first - 2];   // the run before the boundary ends at bin v - 1
                o += 2;
                o[0] = pos[e.first - 1];   // the next starts at bin v
            }
            o[1] = pos[N - 1];
            o += 2;
        }
    });
}


/* ---- diagnostics (not part of include/tadpole_hip.h) -------------------- */

/* k_chol + k_trsm_ru on a b x b SPD matrix W: U (upper) and Q = Z U^{-1}
 * for Z = identity (so Q = U^{-1}); mean ms of `reps` (chol, trsm). */
void tp_debug_chol(const double *W, const int *b, const double *rel, const int *reps, double *U, double *Xinv,
                   double *ms, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int B = *b;
        double *dW = c.buf[S_SMALL].as<double>((size_t)3 * B * B + B);
        double *dI = dW + (size_t)B * B;
        double *dX = dI + (size_t)B * B;
        double *rd = dX + (size_t)B * B;
        int *info = c.buf[S_MISC].as<int>(64);
        std::vector<double> eye((size_t)B * B, 0.0);
        for (int q = 0; q < B; ++q) eye[(size_t)q * B + q] = 1.0;
        TP_HIP(hipMemcpyAsync(dI, eye.data(), (size_t)B * B * 8, hipMemcpyHostToDevice, s));
        hipEvent_t e0, e1, e2;
        TP_HIP(hipEventCreate(&e0));
        TP_HIP(hipEventCreate(&e1));
        TP_HIP(hipEventCreate(&e2));
        float t1 = 0, t2 = 0;
        for (int r = 0; r < *reps; ++r) {
            TP_HIP(hipMemcpyAsync(dW, W, (size_t)B * B * 8, hipMemcpyHostToDevice, s));
            TP_HIP(hipEventRecord(e0, s));
            launch_chol(dW, rd, B, *rel, info, s);
            TP_HIP(hipEventRecord(e1, s));
            launch_trsm_ru(dI, B, B, dW, rd, dX, s);
            TP_HIP(hipEventRecord(e2, s));
            TP_HIP(hipEventSynchronize(e2));
            float a = 0, bb = 0;
            TP_HIP(hipEventElapsedTime(&a, e0, e1));
            TP_HIP(hipEventElapsedTime(&bb, e1, e2));
            t1 += a;
            t2 += bb;
        }
        // one stamped run: cycles of (a) diag factor, (b) panel solve, (c) trailing, prologue
        long long *dst = (long long *)c.buf[S_MISC].as<char>(1024) + 32;
        TP_HIP(hipMemcpyAsync(dW, W, (size_t)B * B * 8, hipMemcpyHostToDevice, s));
        launch_chol_stamped(dW, rd, B, *rel, info, dst, s);
        long long hst[4];
        TP_HIP(hipMemcpyAsync(hst, dst, 32, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
        for (int q = 0; q < 4; ++q) ms[2 + q] = (double)hst[q];
        TP_HIP(hipMemcpyAsync(U, dW, (size_t)B * B * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(Xinv, dX, (size_t)B * B * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipEventDestroy(e2);
        ms[0] = t1 / *reps;
        ms[1] = t2 / *reps;
    });
}

/* Out = A'B (A: K x M col-major, B: K x N, N = 64, K >= 64) by the
 * int8-digit product (rows_gemm_sharded's path, rank-1 epilogue against row
 * vrow = M - 1) into O8 and by the fp64 k_gemm_ts path into O64 (M - 1 rows
 * each, ld M - 1); ms[0..1] the two products' device time. */
void tp_debug_prod_i8(const double *A, const int *K, const int *M, const double *B, const int *N, double *O8,
                      double *O64, double *ms, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int k = *K, m = *M, nn = *N;
        if (!prod_i8_ok(k, nn) || m < 2) fail(TP_ERR_ARG, "prod_i8: N must be 32 or 64 and K >= 64");
        double *dA = c.buf[S_C].as<double>((size_t)k * m);
        double *dB = c.buf[S_Q].as<double>((size_t)k * nn);
        double *dO = c.buf[S_Z].as<double>(2 * (size_t)(m - 1) * nn);
        TP_HIP(hipMemcpyAsync(dA, A, (size_t)k * m * 8, hipMemcpyHostToDevice, s));
        TP_HIP(hipMemcpyAsync(dB, B, (size_t)k * nn * 8, hipMemcpyHostToDevice, s));
        ProdDigits pd;
        prod_digits_build(c, dA, k, k, m, 0, pd);
        const R1 r1{m - 1, nullptr, m - 1};
        hipEvent_t e0, e1, e2;
        TP_HIP(hipEventCreate(&e0));
        TP_HIP(hipEventCreate(&e1));
        TP_HIP(hipEventCreate(&e2));
        float t8 = 0, t64 = 0;
        for (int r = 0; r < 4; ++r) {
            TP_HIP(hipEventRecord(e0, s));
            rows_gemm_sharded(c, dA, k, m, dB, k, nn, k, dO, 0, 1, &r1, 0, &pd);
            TP_HIP(hipEventRecord(e1, s));
            rows_gemm_sharded(c, dA, k, m, dB, k, nn, k, dO + (size_t)(m - 1) * nn, 0, 1, &r1, 0, nullptr);
            TP_HIP(hipEventRecord(e2, s));
            TP_HIP(hipEventSynchronize(e2));
            float a = 0, b = 0;
            TP_HIP(hipEventElapsedTime(&a, e0, e1));
            TP_HIP(hipEventElapsedTime(&b, e1, e2));
            if (r) {   // the first round loads the code objects
                t8 += a;
                t64 += b;
            }
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipEventDestroy(e2);
        ms[0] = t8 / 3;
        ms[1] = t64 / 3;
        TP_HIP(hipMemcpyAsync(O8, dO, (size_t)(m - 1) * nn * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(O64, dO + (size_t)(m - 1) * nn, (size_t)(m - 1) * nn * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
    });
}

/* int8-digit product rows (test hook): the digit image of columns [col0, M)
 * of A (K x M, the column slab a rank keeps), then rows [r0, r0 + rows) of
 * A'B, no rank-1 epilogue, into O (rows x N, column-major): a shard's rows
 * must carry the whole product's bits.  *which: the product kernel (knob 36). */
void tp_debug_prod_i8_rows(const double *A, const int *K, const int *M, const double *B, const int *N,
                           const int *col0, const int *r0, const int *rows, double *O, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int k = *K, m = *M, nn = *N, c0 = *col0, q0 = *r0, nr = *rows;
        if (!prod_i8_ok(k, nn) || c0 < 0 || c0 % 64 || c0 >= m || q0 < c0 || nr < 1 || q0 + nr > m)
            fail(TP_ERR_ARG, "prod_i8_rows: N must be 64, col0 a multiple of 64, rows inside [col0, M)");
        double *dA = c.buf[S_C].as<double>((size_t)k * (m - c0));
        double *dB = c.buf[S_Q].as<double>((size_t)k * nn);
        double *dO = c.buf[S_Z].as<double>((size_t)nr * nn);
        TP_HIP(hipMemcpyAsync(dA, A + (size_t)c0 * k, (size_t)k * (m - c0) * 8, hipMemcpyHostToDevice, s));
        TP_HIP(hipMemcpyAsync(dB, B, (size_t)k * nn * 8, hipMemcpyHostToDevice, s));
        ProdDigits pd;
        prod_digits_build(c, dA, k, k, m - c0, c0, pd);
        double *part = nullptr;
        const int S = prod_i8_partials(c, pd, q0, nr, dB, k, nn, k, c.buf[S_PARTIAL], &part);
        launch_splitk_reduce(part, (size_t)nr * nn, S, nr, nn, dO, nr, 0, s);
        TP_HIP(hipMemcpyAsync(O, dO, (size_t)nr * nn * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
    });
}

/* A's int8 digit image (test hook): columns of A (K x M) digitised as the
 * PCA does -- fused = 1: the first M - 2 columns with their means in one pass
 * (k_pd_digits_cm), then the last two; 0: k_pd_digits_reg / k_pd_digits.
 * img: ND x ceil(M / 64) 64 x Kp bytes in the pd_off layout (ND = *nd on
 * return), scale[ceil(M/64) 64], cm[M - 2] (fused only) and cm_ref[M - 2]
 * (k_colmean on the same columns). */
void tp_debug_pd_image(const double *A, const int *K, const int *M, const int *fused, int8_t *img, double *scale,
                       double *cm, double *cm_ref, int *nd, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int k = *K, m = *M;
        if (k < 64 || m < 3) fail(TP_ERR_ARG, "pd_image: K >= 64, M >= 3");
        double *dA = c.buf[S_C].as<double>((size_t)k * m);
        double *dm = c.buf[S_Q].as<double>(2 * (size_t)m);
        TP_HIP(hipMemcpyAsync(dA, A, (size_t)k * m * 8, hipMemcpyHostToDevice, s));
        ProdDigits pd;
        if (*fused) {
            prod_digits_build(c, dA, k, k, m, 0, pd, dm, m - 2);
            prod_digits_finish(c, dA, k, k, pd);
        } else {
            prod_digits_build(c, dA, k, k, m, 0, pd);
        }
        launch_colmean_cols(dA, k, m - 2, k, dm + m, s);
        const int cp = (m + 63) / 64 * 64;
        *nd = prod_i8_adig();
        TP_HIP(hipMemcpyAsync(img, pd.d, (size_t)prod_i8_adig() * pd.slice, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(scale, pd.rs, (size_t)cp * 8, hipMemcpyDeviceToHost, s));
        if (*fused) TP_HIP(hipMemcpyAsync(cm, dm, (size_t)(m - 2) * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(cm_ref, dm + m, (size_t)(m - 2) * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
    });
}

/* CholQR kernels for b <= 256 on Z = I: k_chol_inv + k_trsm_frag give
 * Y = U^{-1} (W = U'U, S-scaled, + rel on the scaled diagonal); diag[b] =
 * diag(U).  ms[0] chol kernel (the product's choice of waves), ms[1] info,
 * ms[2] chol kernel (16 waves), ms[3..4] stamps (prologue, factor cycles), ms[5] diag-factor cycles,
 * ms[6] trsm kernel (n = b). */
void tp_debug_chol_inv(const double *W, const int *b, const double *rel, const int *reps, double *diag, double *Y,
                       double *ms, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int B = *b;
        double *dW = c.buf[S_SMALL].as<double>((size_t)4 * B * B + 2 * B);
        double *dF = dW + (size_t)B * B;
        double *dI = dF + (size_t)B * B;
        double *dY = dI + (size_t)B * B;
        double *rd = dY + (size_t)B * B;
        double *sc = rd + B;
        int *info = c.buf[S_MISC].as<int>(64);
        std::vector<double> eye((size_t)B * B, 0.0);
        for (int q = 0; q < B; ++q) eye[(size_t)q * B + q] = 1.0;
        TP_HIP(hipMemcpyAsync(dI, eye.data(), (size_t)B * B * 8, hipMemcpyHostToDevice, s));
        hipEvent_t e0, e1, e2;
        TP_HIP(hipEventCreate(&e0));
        TP_HIP(hipEventCreate(&e1));
        TP_HIP(hipEventCreate(&e2));
        const int R = std::max(1, *reps);
        const int keep = g_chol_inv_waves;
        for (int pass = 0; pass < 2; ++pass) {
            g_chol_inv_waves = pass == 0 ? 0 : 16;
            float tc = 0, tt = 0;
            for (int r = 0; r < R; ++r) {
                TP_HIP(hipMemcpyAsync(dW, W, (size_t)B * B * 8, hipMemcpyHostToDevice, s));
                TP_HIP(hipEventRecord(e0, s));
                launch_chol_inv(dW, dF, sc, rd, B, *rel, info, s);
                TP_HIP(hipEventRecord(e1, s));
                launch_trsm_frag(dI, B, B, dF, sc, dY, s);
                TP_HIP(hipEventRecord(e2, s));
                TP_HIP(hipEventSynchronize(e2));
                float a = 0, bb = 0;
                TP_HIP(hipEventElapsedTime(&a, e0, e1));
                TP_HIP(hipEventElapsedTime(&bb, e1, e2));
                tc += a;
                tt += bb;
            }
            ms[pass == 0 ? 0 : 2] = tc / R;
            if (pass == 0) ms[6] = tt / R;
        }
        g_chol_inv_waves = keep;
        TP_HIP(hipMemcpyAsync(dW, W, (size_t)B * B * 8, hipMemcpyHostToDevice, s));
        long long *dst = (long long *)c.buf[S_MISC].as<char>(1024) + 32;
        launch_chol_inv(dW, dF, sc, rd, B, *rel, info, s, dst);
        launch_trsm_frag(dI, B, B, dF, sc, dY, s);
        long long hst[5];
        TP_HIP(hipMemcpyAsync(hst, dst, sizeof(hst), hipMemcpyDeviceToHost, s));
        int hinfo = 0;
        std::vector<double> hw((size_t)B * B);
        TP_HIP(hipMemcpyAsync(hw.data(), dW, (size_t)B * B * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(Y, dY, (size_t)B * B * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
        for (int q = 0; q < B; ++q) diag[q] = hw[(size_t)q * B + q];
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipEventDestroy(e2);
        ms[1] = hinfo;
        ms[3] = (double)hst[0];
        ms[4] = (double)hst[1];
        ms[5] = (double)hst[4];
    });
}

/* stamped CONISS for trees 1..k on P (n x k col-major): stamps[k * 16]
 * (cycles per phase, wave A 0..7 and wave B 8..15, tp_sweep.hip), kernel ms. */
void tp_debug_coniss_stamps(const double *P, const int *n, const int *k, long long *stamps, double *ms,
                            int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int N = *n, K = *k;
        double *dP = c.buf[S_P].as<double>((size_t)N * K);
        double *dPt = c.buf[S_PT].as<double>(pt_doubles(N, K));
        TP_HIP(hipMemcpyAsync(dP, P, (size_t)N * K * 8, hipMemcpyHostToDevice, s));
        launch_transpose(dP, N, K, N, dPt, K, s);
        SweepDev sd{};
        sd.Pt = dPt;
        sd.n = N;
        sd.ldp = K;
        sd.k = K;
        sd.tree0 = 0;
        sd.ntrees = K;
        sd.sums = c.buf[S_SWEEP].as<double>(sweep_sums_doubles(N, 0, K));
        const size_t rec = (size_t)K * (N - 1);
        char *recbuf = c.buf[S_SWEEP2].as<char>(rec * 24 + 256);
        sd.mrg_a = (int *)recbuf;
        sd.mrg_b = sd.mrg_a + rec;
        sd.cost = (double *)(((uintptr_t)(sd.mrg_b + rec) + 15) & ~(uintptr_t)15);
        sd.height = sd.cost + rec;
        sd.n_cluster = c.buf[S_MISC].as<int>(K + 64);
        long long *dst = (long long *)c.buf[S_SCORES].as<char>((size_t)K * 16 * 8);
        sd.stamps = dst;
        sd.cost0 = c.buf[S_SMALL].as<double>(sweep_cost0_doubles(N, K, K));
        hipEvent_t e0, e1;
        TP_HIP(hipEventCreate(&e0));
        TP_HIP(hipEventCreate(&e1));
        TP_HIP(hipEventRecord(e0, s));
        launch_coniss_stamped(sd, s);
        TP_HIP(hipEventRecord(e1, s));
        TP_HIP(hipEventSynchronize(e1));
        float t = 0;
        TP_HIP(hipEventElapsedTime(&t, e0, e1));
        *ms = t;
        TP_HIP(hipMemcpy(stamps, dst, (size_t)K * 16 * 8, hipMemcpyDeviceToHost));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    });
}


}  // extern "C"

extern "C" {
// Test hook for the PCA's Rayleigh-Ritz eigensolver (tp_eig.hip, not part of the
// reference-facing ABI): H (b x b, column-major, symmetric, b <= 1280) -> theta
// ascending, V eigenvectors (columns): tridiagonalisation + bisection + inverse
// iteration (the product path; *method is ignored -- the rocSOLVER dstedc
// variant of earlier builds is gone).
void tp_debug_eigsym(const double *H, const int *b, const int *method, double *theta, double *V, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int B = *b;
        (void)method;
        if (!tp::eig_sym_supported(B)) fail(TP_ERR_UNSUPPORTED, "b > 1280 (EIG_BMAX)");
        double *dA = c.buf[S_SMALL].as<double>((size_t)B * B + B + 64);
        double *dW = dA + (size_t)B * B;
        double *dWork = c.buf[S_PARTIAL].as<double>((size_t)B * B + 4 * B + 64);
        TP_HIP(hipMemcpyAsync(dA, H, (size_t)B * B * 8, hipMemcpyHostToDevice, s));
        tp::eig_sym(dA, B, dW, dWork, s);
        TP_HIP(hipMemcpyAsync(theta, dW, (size_t)B * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipMemcpyAsync(V, dA, (size_t)B * B * 8, hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
    });
}
}  // extern "C"

extern "C" {
// ------------------------------------------------------------------ load_mat
// bigmemory::read.big.matrix(mat_file, type = 'double', sep = '\t')
// (R/TADpole.R:17,160) natively: path is a char** (R .C passes strings so).
void tp_tsv_dims(const char **path, int *nrow, int *ncol, int *status) {
    guarded(status, [&] {
        if (!path || !*path) fail(TP_ERR_ARG, "null path");
        tp::tsv_dims(*path, nrow, ncol);
    });
}

void tp_read_tsv(const char **path, const int *nrow, const int *ncol, const int *nthreads, const int *flags,
                 double *out, int *status) {
    guarded(status, [&] {
        if (!path || !*path || !nrow || !ncol || !out) fail(TP_ERR_ARG, "null argument");
        const int th = (nthreads && *nthreads > 0) ? *nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
        tp::tsv_read(*path, *nrow, *ncol, th, flags && (*flags & TP_FLAG_ROW_MAJOR), out);
    });
}

// host -> device copy of a pageable buffer through this stream's context's
// pinned staging (tp_upload.hip): a pageable hipMemcpy goes through the
// runtime's one staging path, which the 8 streams of a genome run shared
void tp_upload_dev(const void *host, const long long *bytes, void *d_dst, const int *nthreads, const int *device,
                   void *stream, int *status) {
    guarded(status, [&] {
        if (!host || !bytes || !d_dst || *bytes < 0) fail(TP_ERR_ARG, "null argument");
        Ctx &c = ctx_for(dev_of(device), (hipStream_t)stream);
        upload_host(c, host, (size_t)*bytes, d_dst, nthreads && *nthreads > 0 ? *nthreads : 1, false);
    });
}

// the same for a float64 matrix of counts: blocks whose values are all exact
// integers in [0, 65535] travel as 16-bit integers (widened on the device to
// the same doubles), any other block as float64; *packed = bytes of float64
// that travelled packed (may be NULL)
void tp_upload_counts_dev(const double *host, const long long *count, double *d_dst, const int *nthreads,
                          const int *device, void *stream, long long *packed, int *status) {
    guarded(status, [&] {
        if (!host || !count || !d_dst || *count < 0) fail(TP_ERR_ARG, "null argument");
        Ctx &c = ctx_for(dev_of(device), (hipStream_t)stream);
        const size_t pk = upload_host(c, host, (size_t)*count * sizeof(double), d_dst,
                                      nthreads && *nthreads > 0 ? *nthreads : 1, true);
        if (packed) *packed = (long long)pk;
    });
}

void tp_read_tsv_dev(const char **path, const int *nrow, const int *ncol, const int *nthreads, const int *device,
                     void *stream, double *d_out, int *status) {
    guarded(status, [&] {
        if (!path || !*path || !nrow || !ncol || !d_out || *nrow < 0 || *ncol < 0) fail(TP_ERR_ARG, "null argument");
        const int th = (nthreads && *nthreads > 0) ? *nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
        Ctx &c = ctx_for(dev_of(device), (hipStream_t)stream);
        const size_t ld = (size_t)*ncol;
        // a ring of 3 pinned row-block slots (~16 MB each, the context's pinned
        // staging, kept across calls): each parsed block is copied to the device
        // while the next ones are parsed, and a slot is refilled once its copy
        // is done -- the staging is 3 blocks, not the matrix
        constexpr int kSlots = 3;
        static_assert(kSlots <= (int)(sizeof(c.ring_ev) / sizeof(c.ring_ev[0])), "Ctx::ring_ev too small");
        for (int q = 0; q < kSlots; ++q)
            if (!c.ring_ev[q]) TP_HIP(hipEventCreateWithFlags(&c.ring_ev[q], hipEventDisableTiming));
        hipEvent_t *ev = c.ring_ev;
        tp::tsv_read_rows(
            *path, *nrow, *ncol, th, (size_t)16 << 20, kSlots,
            [&](size_t slot_rows) { return (double *)c.pinned(kSlots * slot_rows * ld * sizeof(double)); },
            [&](size_t r0, size_t r1, const double *rows, int slot) {
                if (r1 > r0)
                    TP_HIP(hipMemcpyAsync(d_out + r0 * ld, rows, (r1 - r0) * ld * sizeof(double),
                                          hipMemcpyHostToDevice, c.cur));
                TP_HIP(hipEventRecord(ev[slot], c.cur));
            },
            [&](int slot) {   // a ~16 MB copy (< 1 ms): poll with short sleeps, no spinning
                hipError_t q;
                while ((q = hipEventQuery(ev[slot])) == hipErrorNotReady)
                    std::this_thread::sleep_for(std::chrono::microseconds(20));
                TP_HIP(q);
            });
        stream_sync(c, c.cur);   // the staging is reused by the next call on this context
    });
}
}  // extern "C"

extern "C" {
// diagnostic: k_sytrd_l time and per-phase cycles for H (b x b)
void tp_debug_sytrd(const double *H, const int *b, double *ms, long long *stamps, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int B = *b;
        double *dA = c.buf[S_SMALL].as<double>((size_t)B * B + 64);
        double *dWork = c.buf[S_PARTIAL].as<double>((size_t)4 * B + 64);
        long long *dst = (long long *)c.buf[S_MISC].as<int>(64);
        hipEvent_t e0, e1;
        TP_HIP(hipEventCreate(&e0));
        TP_HIP(hipEventCreate(&e1));
        TP_HIP(hipMemcpyAsync(dA, H, (size_t)B * B * 8, hipMemcpyHostToDevice, s));
        TP_HIP(hipEventRecord(e0, s));
        tp::sytrd_stamped(dA, B, dWork, dst, s);
        TP_HIP(hipEventRecord(e1, s));
        TP_HIP(hipEventSynchronize(e1));
        float t = 0;
        TP_HIP(hipEventElapsedTime(&t, e0, e1));
        *ms = t;
        TP_HIP(hipMemcpy(stamps, dst, 4 * sizeof(long long), hipMemcpyDeviceToHost));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    });
}
/* one tridiagonalisation of H (b x b, lower triangle used) by k_sytrd_l
 * (which 0) or k_sytrd32 (which 2): d[b], e[b-1], tau[b-1], Aout = A with
 * the reflectors below the subdiagonal; ms[0] = kernel time (mean of 3). */
void tp_debug_sytrd2(const double *H, const int *b, const int *which, double *ms, double *d, double *e, double *tau,
                     double *Aout, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int B = *b;
        double *dA = c.buf[S_SMALL].as<double>((size_t)B * B + 64);
        double *dWork = c.buf[S_PARTIAL].as<double>((size_t)4 * B + 64);
        hipEvent_t e0, e1;
        TP_HIP(hipEventCreate(&e0));
        TP_HIP(hipEventCreate(&e1));
        float tot = 0;
        for (int r = 0; r < 3; ++r) {
            TP_HIP(hipMemcpyAsync(dA, H, (size_t)B * B * 8, hipMemcpyHostToDevice, s));
            TP_HIP(hipEventRecord(e0, s));
            sytrd_which(dA, B, dWork, *which, s);
            TP_HIP(hipEventRecord(e1, s));
            TP_HIP(hipEventSynchronize(e1));
            float t = 0;
            TP_HIP(hipEventElapsedTime(&t, e0, e1));
            tot += t;
        }
        ms[0] = tot / 3;
        TP_HIP(hipMemcpy(Aout, dA, (size_t)B * B * 8, hipMemcpyDeviceToHost));
        TP_HIP(hipMemcpy(e, dWork, (size_t)(B > 1 ? B - 1 : 1) * 8, hipMemcpyDeviceToHost));
        TP_HIP(hipMemcpy(tau, dWork + B, (size_t)(B > 1 ? B - 1 : 1) * 8, hipMemcpyDeviceToHost));
        TP_HIP(hipMemcpy(d, dWork + 2 * B, (size_t)B * 8, hipMemcpyDeviceToHost));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    });
}
}  // extern "C"

extern "C" {
/* S = X'X (n x n, column-major in and out) by mode 0 = fp64 MFMA GEMM, 1 = the
 * int8-exact path with 64-column tiles, 2 = the 128-column tile kernels of the
 * pipeline (k_xtx_i8_w, or with knob 44 = 0 the 128-tile LDS-DMA kernel;
 * counts below 16384) (fails with TP_ERR_ARG when X is not non-negative integer
 * counts below 2^21); *slices = slices used (0 for fp64); ms = mean of 3. */
void tp_debug_xtx(const double *X, const int *n, const int *mode, double *S, int *slices, double *ms,
                  int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int N = *n;
        double *dX = c.buf[S_X].as<double>((size_t)N * N);
        double *dS = c.buf[S_S].as<double>((size_t)N * N);
        TP_HIP(hipMemcpyAsync(dX, X, (size_t)N * N * 8, hipMemcpyHostToDevice, s));
        int ns = 0;
        if (*mode >= 1) {
            ns = xtx_int_slices(c, dX, N);
            if (ns == 0) fail(TP_ERR_ARG, "X is not non-negative integer counts < 2^21");
            if (*mode == 2 && ns > 2) fail(TP_ERR_ARG, "128-tile kernels: counts < 16384");
        }
        hipEvent_t e0, e1;
        TP_HIP(hipEventCreate(&e0));
        TP_HIP(hipEventCreate(&e1));
        float tot = 0;
        for (int r = 0; r < 3; ++r) {
            TP_HIP(hipEventRecord(e0, s));
            if (ns) {
                const int8_t *sl = xtx_slices(c, dX, N, ns);
                if (*mode == 2) xtx_int8_tiles128(c, sl, N, ns, dS, 0, -1, nullptr, nullptr);
                else xtx_int8_tiles(c, sl, N, ns, dS, 0, -1);
            } else {
                GemmArgs g{N, N, N, dX, N, true, dX, N, dS, N};
                g.sym_upper = true;
                gemm_f64(g, c.buf[S_PARTIAL], s);
            }
            TP_HIP(hipEventRecord(e1, s));
            TP_HIP(hipEventSynchronize(e1));
            float t = 0;
            TP_HIP(hipEventElapsedTime(&t, e0, e1));
            tot += t;
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        *ms = tot / 3;
        *slices = ns;
        TP_HIP(hipMemcpy(S, dS, (size_t)N * N * 8, hipMemcpyDeviceToHost));
    });
}
}  // extern "C"

extern "C" {
/* Test hook: set a run-time switch, *old = its previous value.  Switches (the
 * process-wide values each C-ABI entry copies into its calling thread's set
 * when it starts, so a call in flight keeps the set it started with):
 *   1 cap on the shared CH segment store (0 = automatic; > 0 tests its
 *     overflow path),
 *   5 exact int8 X'X for integer counts (0: the fp64 MFMA product),
 *   8 bins from which the block Krylov PCA replaces forming G,
 *  18 the correlation epilogue in the int8 X'X store (0: X'X into S, then the
 *     separate epilogue -- the path of counts past two slices and real data),
 *  20 the PCA's Krylov space: 1 of C, 0 of G, -1 (default) of C from 10 000 bins,
 *  24 C5 shards keep C row-sharded (0: C gathered whole),
 *  36 the G-space Krylov products on int8 digit images (0: the fp64
 *     k_gemm_ts; 1: k_pd_prod's 64-row tiles; 5, default: k_pd_prodA),
 *  43 host uploads (bit 1: exact 16-bit count blocks travel packed, bit 0:
 *     one block at a time),
 *  44 the whole-triangle int8 X'X by k_xtx_i8_w's 256 x 128 tiles (0: 128-tiles),
 *  45 the C-space Krylov products on int8 digit images (0: fp64),
 *  48 the bins from which a lean sweep of a matrix that fits LDS takes the
 *     global link-only CONISS (0: never),
 *  49 the LDS CONISS with one 16-bit link array (3, default: where the 16-byte
 *     variant does not fit; 1: lean sweeps; 2: every sweep; 0: never),
 *  52 the batched CONISS (3, default: every sweep, lean ones in storage mode 1
 *     where it fits; 2: every sweep; 1: not lean ones; 0: never).
 * Process-wide hooks (not path choices):
 *  25 events around every Krylov product when timings are requested,
 *  30 the next N sharded waits with a live communicator fail as device errors,
 *  41 scratch regrowths so far (a counter: returned, then set to *value),
 *  51 the next N scratch allocations fail as out-of-memory.
 * Every other switch of earlier rounds is a compile-time constant now
 * (tp_internal.h, cfg_*). */
void tp_debug_knob(const int *which, const int *value, int *old, int *status) {
    guarded(status, [&] {
        std::atomic<int> *h = nullptr;
        switch (*which) {
        case 25: h = &g_kprof_fine; break;
        case 30: h = &g_shard_inject; break;
        case 41: h = &g_devbuf_grows; break;
        case 51: h = &g_devbuf_fail_inject; break;
        default: break;
        }
        if (h) {
            *old = h->exchange(*value);
            return;
        }
        std::lock_guard<std::mutex> lk(knob_mu());
        Knobs &k = knob_set();
        int *p = nullptr;
        switch (*which) {
        case 1: p = &k.ch_dedup_ucap; break;
        case 5: p = &k.xtx_int8; break;
        case 8: p = &k.pca_krylov_min; break;
        case 18: p = &k.xtx_fused; break;
        case 20: p = &k.pca_ckrylov; break;
        case 24: p = &k.shard_slab; break;
        case 36: p = &k.prod_i8; break;
        case 43: p = &k.upload_mode; break;
        case 44: p = &k.xtx_w; break;
        case 45: p = &k.pd_cspace; break;
        case 48: p = &k.coniss_lean_min; break;
        case 49: p = &k.coniss_lds2; break;
        case 52: p = &k.coniss_batch; break;
        default: fail(TP_ERR_ARG, "unknown knob");
        }
        if (*which == 36 && *value != 0 && *value != 1 && *value != 5) fail(TP_ERR_ARG, "knob 36 takes 0, 1 or 5");
        *old = *p;
        *p = *value;
    });
}

/* The int8 MACs the last whole-triangle X'X (k_xtx_i8_w) of this stream's
 * context executed (out[0]), its slice-0 MACs (out[1]), high-slice k-blocks
 * over all tiles (out[2]), tiles (out[3]), k-blocks a tile (out[4]); out[0] = -1
 * when the context ran none.  Reads the high slice's block map back (a sync):
 * call it outside timed regions. */
void tp_debug_xtx_exec(const int *device, void *stream, double *out, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(dev_of(device), (hipStream_t)stream);
        for (int q = 0; q < 5; ++q) out[q] = 0.0;
        if (!xtx_w_exec(c, out)) out[0] = -1.0;
    });
}

/* The scores P (n x k, column-major) of the last pipeline on device 0's default
 * context (test hook: compares the PCA of two schedules). */
void tp_debug_last_scores(const int *n, const int *k, double *P, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        const size_t cnt = (size_t)(*n) * (*k);
        if (c.buf[S_P].bytes < cnt * 8) fail(TP_ERR_ARG, "no scores of that size");
        TP_HIP(hipStreamSynchronize(c.cur));
        TP_HIP(hipMemcpy(P, c.buf[S_P].p, cnt * 8, hipMemcpyDeviceToHost));
    });
}

/* C = A'B (trans_a) or AB, fp64 MFMA, kernel 0 = 64 x 64 tiles, 1 = 128 x 128
 * tiles (both without split-K); sym = upper tiles mirrored (M == N). */
void tp_debug_gemm(const double *A, const double *B, const int *M, const int *N, const int *K, const int *trans_a,
                   const int *sym, const int *kernel, double *C, double *ms, int *status) {
    guarded(status, [&] {
        Ctx &c = ctx_for(0);
        hipStream_t s = c.cur;
        const int m = *M, n = *N, k = *K;
        const bool ta = *trans_a != 0;
        const size_t na = (size_t)m * k, nb = (size_t)k * n, nc = (size_t)m * n;
        double *dA = c.buf[S_X].as<double>(na), *dB = c.buf[S_S].as<double>(nb), *dC = c.buf[S_C].as<double>(nc);
        TP_HIP(hipMemcpyAsync(dA, A, na * 8, hipMemcpyHostToDevice, s));
        TP_HIP(hipMemcpyAsync(dB, B, nb * 8, hipMemcpyHostToDevice, s));
        TP_HIP(hipMemsetAsync(dC, 0, nc * 8, s));
        GemmArgs g{m, n, k, dA, ta ? k : m, ta, dB, k, dC, m};
        g.sym_upper = *sym != 0;
        // kernel: 0 = 64 x 64 tiles, 1 = 128 x 128 (when the tile count allows),
        // 2 = the library's policy (panel kernel for tall-skinny products),
        // 3 = the split-K policy without the panel kernel, 4 = row-shardable
        // kernel 10..99: 64 x 64 tiles with split-K (kernel - 10); 110..199: the
        // same with 16-deep LDS stages
        const int kern = *kernel >= 110 ? *kernel - 100 : *kernel;
        g.splitk = kern >= 10 ? kern - 10 : (kern >= 2 ? 0 : 1);
        const int keep_kb = g_gemm_kb;
        if (*kernel >= 110) g_gemm_kb = 16;
        else if (*kernel >= 10) g_gemm_kb = 32;
        g.big_cols = *kernel == 1;
        g.rows = *kernel == 4 || *kernel == 5;   // 4: a row-shardable product (128 x 64 kernel, k chunks by K)
        if (*kernel == 5) {   // 5: the same, stored transposed (C row-major m x n, as a row shard writes it)
            g.store_t = true;
            g.ldc = n;
        }
        const int keep_panel = g_gemm_panel;
        g_gemm_panel = *kernel == 2 ? 1 : 0;
        hipEvent_t e0, e1;
        TP_HIP(hipEventCreate(&e0));
        TP_HIP(hipEventCreate(&e1));
        TP_HIP(hipEventRecord(e0, s));
        if (*kernel == 6) {   // 6: the row-sharded schedule (virtual shards of tp_set_virtual_shards), A'B
            c.shard.active = true;
            rows_gemm_sharded(c, dA, k, m, dB, k, n, k, dC, 0, 0);
            c.shard.active = false;
        } else
        gemm_f64(g, c.buf[S_PARTIAL], s);
        g_gemm_panel = keep_panel;
        g_gemm_kb = keep_kb;
        TP_HIP(hipEventRecord(e1, s));
        TP_HIP(hipEventSynchronize(e1));
        float t = 0;
        TP_HIP(hipEventElapsedTime(&t, e0, e1));
        *ms = t;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        TP_HIP(hipMemcpy(C, dC, nc * 8, hipMemcpyDeviceToHost));
    });
}
}  // extern "C"
