// One matrix sharded over several GPUs (C5, chr1 @5kb, an
// arm of ~24k bins).  One process (or host thread) per GPU; the ranks share an
// RCCL communicator (xGMI) created from a unique id the host distributes
// (tp_comm_unique_id / tp_comm_init).  Every rank holds the full matrix and
// runs the same pipeline; only the O(N^3) / O(N^2 b) products are split:
//
//   S = X'X, G = Xc'Xc   upper tiles of a contiguous range of 64-column tile
//                        columns per rank (balanced by tile count), gathered
//                        by one in-place ncclBroadcast per owner inside a
//                        group, then the lower triangle mirrored locally
//   Y = G Q, P = Xc V    rows split in 64-row blocks; each rank writes its rows
//                        transposed (b-contiguous), gathered the same way,
//                        transposed back
//   the sweep            PC prefixes (trees) split in contiguous ranges;
//                        n_cluster / CH rows gathered, the chosen tree's merge
//                        record broadcast by its owner
//
// Every output element is computed by the same tile code with the same K order
// whatever the rank count (split-K is off in the sharded products), and all
// replicated stages see identical inputs, so results are bit-identical for 1,
// 2, 4 or 8 ranks.  A test hook (tp_set_virtual_shards) runs the same sharded
// schedule as V shards on one device with the gathers as no-ops.
//
// RCCL is bound at tp_comm_init with dlopen("librccl.so.1"): in a torch
// process that is torch's own RCCL (same SONAME), so there is one RCCL and one
// HIP runtime per process; the library itself has no link-time dependency.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

// ------------------------------------------------------------------ RCCL
struct Rccl {
    void *h = nullptr;
    decltype(&ncclGetUniqueId) get_uid = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclBroadcast) bcast = nullptr;
    decltype(&ncclGroupStart) gstart = nullptr;
    decltype(&ncclGroupEnd) gend = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
    decltype(&ncclCommGetAsyncError) async_err = nullptr;
};
static Rccl g_rccl;

static Rccl &rccl() {
    if (g_rccl.h) return g_rccl;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) fail(TP_ERR_HIP, std::string("cannot load RCCL (librccl.so.1): ") + dlerror());
    Rccl r;
    r.h = h;
#define TP_SYM(f, name)                                                             \
    r.f = (decltype(r.f))dlsym(h, name);                                            \
    if (!r.f) fail(TP_ERR_HIP, std::string("RCCL symbol missing: ") + name);
    TP_SYM(get_uid, "ncclGetUniqueId")
    TP_SYM(init_rank, "ncclCommInitRank")
    TP_SYM(destroy, "ncclCommDestroy")
    TP_SYM(bcast, "ncclBroadcast")
    TP_SYM(gstart, "ncclGroupStart")
    TP_SYM(gend, "ncclGroupEnd")
    TP_SYM(errstr, "ncclGetErrorString")
    TP_SYM(abort, "ncclCommAbort")
    TP_SYM(async_err, "ncclCommGetAsyncError")
#undef TP_SYM
    g_rccl = r;
    return g_rccl;
}

static void nccl_ok(ncclResult_t r, const char *what) {
    if (r != ncclSuccess)
        fail(TP_ERR_HIP, std::string("RCCL failure in ") + what + ": " + (g_rccl.errstr ? g_rccl.errstr(r) : "?"));
}

void comm_unique_id(char *id128) {
    ncclUniqueId u;
    nccl_ok(rccl().get_uid(&u), "ncclGetUniqueId");
    static_assert(sizeof(u) == 128, "ncclUniqueId is 128 bytes");
    memcpy(id128, &u, 128);
}

void comm_init(Ctx &c, const char *id128, int nranks, int rank) {
    if (nranks < 1 || rank < 0 || rank >= nranks) fail(TP_ERR_ARG, "comm_init: bad rank / nranks");
    comm_destroy(c);
    ncclUniqueId u;
    memcpy(&u, id128, 128);
    ncclComm_t comm = nullptr;
    nccl_ok(rccl().init_rank(&comm, nranks, u, rank), "ncclCommInitRank");
    c.shard.comm = comm;
    c.shard.rank = rank;
    c.shard.nranks = nranks;
    c.shard.dead = false;
}

void comm_destroy(Ctx &c) {
    if (c.shard.comm) {
        (void)hipStreamSynchronize(c.stream);
        rccl().destroy((ncclComm_t)c.shard.comm);
    }
    c.shard.comm = nullptr;
    c.shard.rank = 0;
    c.shard.nranks = 1;
}

// ------------------------------------------------- failure containment
// A rank that fails inside a sharded call leaves its peers waiting in a
// collective.  Sharded calls therefore never block in hipStreamSynchronize:
// stream_sync polls the stream, the communicator's asynchronous error and a
// deadline (TP_SHARD_TIMEOUT_S, default 300 s), and on either aborts the
// communicator (ncclCommAbort) and fails the call; a rank whose own host code
// throws aborts it too (comm_abort from the pipeline's scope guard).  Peers
// then leave their collectives through their own deadline instead of hanging.
static double shard_timeout_s() {
    static const double v = [] {
        const char *e = getenv("TP_SHARD_TIMEOUT_S");
        const double x = e ? atof(e) : 300.0;
        return x > 0 ? x : 300.0;
    }();
    return v;
}

// The communicator belongs to the device (every stream's context copies it):
// the device's registry entry forgets it first, so no later call -- and no
// tp_comm_destroy -- touches the aborted communicator, and exactly one caller
// aborts it.
void comm_abort(Ctx &c) {
    void *comm = c.shard.comm;
    if (!comm) return;
    const bool owner = ctx_comm_retire(c, comm);
    c.shard.comm = nullptr;
    c.shard.rank = 0;
    c.shard.nranks = 1;
    c.shard.dead = true;
    if (owner) (void)rccl().abort((ncclComm_t)comm);
}

std::atomic<int> g_shard_inject{0};   // test hook (knob 30): the next N sharded waits fail as a device error

// Unsharded waits poll the stream (yielding the core) before blocking: the
// pipeline's read-backs are short waits, and hipStreamSynchronize's blocking
// wake-up put ~45 us between a copy and the next command (rocprof trace, four
// such host round trips after the sweep, two in the mask).  Waits longer than
// cfg_sync_spin_us block as before.
template <typename Query, typename Block>
static void poll_then_block(Query query, Block block) {
    if (cfg_sync_spin_us > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t e = query();
            if (e == hipSuccess) return;
            if (e != hipErrorNotReady) TP_HIP(e);
            if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() >
                cfg_sync_spin_us)
                break;
            std::this_thread::yield();
        }
    }
    TP_HIP(block());
}

void stream_sync(Ctx &c, hipStream_t s) {
    if (!(c.shard.active && c.shard.comm)) {
        poll_then_block([&] { return hipStreamQuery(s); }, [&] { return hipStreamSynchronize(s); });
        return;
    }
    int inj = g_shard_inject.load();
    while (inj > 0 && !g_shard_inject.compare_exchange_weak(inj, inj - 1)) {
    }
    if (inj > 0) {
        TP_HIP(hipStreamSynchronize(s));
        comm_abort(c);
        fail(TP_ERR_HIP, "injected device failure in a sharded call (knob 30); communicator aborted");
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) {
            comm_abort(c);
            TP_HIP(e);
        }
        ncclResult_t ae = ncclSuccess;
        if (rccl().async_err((ncclComm_t)c.shard.comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
            comm_abort(c);
            fail(TP_ERR_HIP, std::string("RCCL asynchronous error in a sharded call: ") + rccl().errstr(ae) +
                                 " (communicator aborted)");
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > shard_timeout_s()) {
            comm_abort(c);
            fail(TP_ERR_HIP, "sharded call timed out waiting for its peers (TP_SHARD_TIMEOUT_S); communicator aborted");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

void event_mark(Ctx &c, hipStream_t s) {
    if (!c.sync_ev) TP_HIP(hipEventCreateWithFlags(&c.sync_ev, hipEventDisableTiming));
    TP_HIP(hipEventRecord(c.sync_ev, s));
}

void event_sync(Ctx &c) {
    if (!(c.shard.active && c.shard.comm)) {
        poll_then_block([&] { return hipEventQuery(c.sync_ev); }, [&] { return hipEventSynchronize(c.sync_ev); });
        return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipEventQuery(c.sync_ev);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) {
            comm_abort(c);
            TP_HIP(e);
        }
        ncclResult_t ae = ncclSuccess;
        if (rccl().async_err((ncclComm_t)c.shard.comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
            comm_abort(c);
            fail(TP_ERR_HIP, std::string("RCCL asynchronous error in a sharded call: ") + rccl().errstr(ae) +
                                 " (communicator aborted)");
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > shard_timeout_s()) {
            comm_abort(c);
            fail(TP_ERR_HIP, "sharded call timed out waiting for its peers (TP_SHARD_TIMEOUT_S); communicator aborted");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// -------------------------------------------------------------- planning
int shard_count(const Ctx &c) {
    if (!c.shard.active) return 1;
    return c.shard.comm ? c.shard.nranks : std::max(1, c.shard.nvirt);
}
bool shard_mine(const Ctx &c, int r) { return !c.shard.comm || r == c.shard.rank; }

// kind 0: tile-column bounds (in 64-column tiles) of the symmetric products,
//   balanced by upper-tile count (tile column j holds j + 1 tiles);
// kind 1: row bounds of the row-split products, whole 64-row blocks;
// kind 2: tree (PC prefix) bounds of the sweep.
// bounds[0..R]: shard r covers [bounds[r], bounds[r+1]).
void shard_plan(int n, int R, int kind, int *bounds) {
    if (R < 1) fail(TP_ERR_ARG, "shard_plan: nranks < 1");
    bounds[0] = 0;
    if (kind == 0) {
        const int tn = (n + 63) / 64;
        const double tot = (double)tn * (tn + 1) / 2.0;
        int j = 0;
        double cum = 0.0;
        for (int r = 1; r < R; ++r) {
            const double target = tot * r / R;
            while (j < tn && cum + (j + 1) * 0.5 <= target) {   // take column j while its midpoint fits
                cum += j + 1;
                ++j;
            }
            bounds[r] = j;
        }
        bounds[R] = tn;
    } else if (kind == 1) {
        const int nb = (n + 63) / 64;
        for (int r = 1; r < R; ++r) bounds[r] = std::min(n, (int)(((long)nb * r / R) * 64));
        bounds[R] = n;
    } else {
        for (int r = 1; r < R; ++r) bounds[r] = (int)((long)n * r / R);
        bounds[R] = n;
    }
    for (int r = 1; r <= R; ++r) bounds[r] = std::max(bounds[r], bounds[r - 1]);
}

// ------------------------------------------------------------- gathers
// The owner of each contiguous chunk [off[r], off[r+1]) (doubles) of buf sends
// it to every rank, in place.  No-op for virtual shards / one rank.
void shard_gather(Ctx &c, double *buf, const std::vector<size_t> &off) {
    if (!c.shard.active || !c.shard.comm || c.shard.nranks == 1) return;
    Rccl &R = rccl();
    nccl_ok(R.gstart(), "ncclGroupStart");
    for (int r = 0; r + 1 < (int)off.size(); ++r) {
        const size_t cnt = off[r + 1] - off[r];
        if (cnt == 0) continue;
        nccl_ok(R.bcast(buf + off[r], buf + off[r], cnt, ncclFloat64, r, (ncclComm_t)c.shard.comm, c.cur),
                "ncclBroadcast");
    }
    nccl_ok(R.gend(), "ncclGroupEnd");
}
void shard_gather_bytes(Ctx &c, void *buf, const std::vector<size_t> &off) {
    if (!c.shard.active || !c.shard.comm || c.shard.nranks == 1) return;
    Rccl &R = rccl();
    char *b = (char *)buf;
    nccl_ok(R.gstart(), "ncclGroupStart");
    for (int r = 0; r + 1 < (int)off.size(); ++r) {
        const size_t cnt = off[r + 1] - off[r];
        if (cnt == 0) continue;
        nccl_ok(R.bcast(b + off[r], b + off[r], cnt, ncclUint8, r, (ncclComm_t)c.shard.comm, c.cur), "ncclBroadcast");
    }
    nccl_ok(R.gend(), "ncclGroupEnd");
}
void shard_bcast_bytes(Ctx &c, void *buf, size_t bytes, int root) {
    if (!c.shard.active || !c.shard.comm || c.shard.nranks == 1) return;
    nccl_ok(rccl().bcast(buf, buf, bytes, ncclUint8, root, (ncclComm_t)c.shard.comm, c.cur), "ncclBroadcast");
}

// ------------------------------------------------------ sharded products
// C = A'A-style symmetric product (g.sym_upper): each shard computes the upper
// tiles of its tile columns; columns gathered; lower triangle mirrored.
void sym_gemm_sharded(Ctx &c, GemmArgs g) {
    const int R = shard_count(c);
    // 128 x 128 tiles for n >= 8192 (measured: slower than 64 x 64 at 3000,
    // ~3 % faster at 10k-24k); both kernels give the same bits, so the choice
    // never changes results
    const bool big = g.sym_upper && g.splitk <= 1 && g.M >= 8192;
    g.big_cols = big;
    if (R == 1 && !c.shard.active) {
        gemm_f64(g, c.buf[S_PARTIAL], c.cur);
        return;
    }
    if (!g.sym_upper || g.M != g.N || g.ldc != g.M) fail(TP_ERR_ARG, "sym_gemm_sharded: square packed output only");
    const int n = g.M;
    const int tw = big ? 128 : 64;
    std::vector<int> tb(R + 1);
    shard_plan((n + tw / 64 - 1) / (tw / 64), R, 0, tb.data());   // kind 0 counts 64-wide tiles
    g.splitk = 1;   // the same K order for every rank count
    for (int r = 0; r < R; ++r) {
        if (!shard_mine(c, r) || tb[r + 1] <= tb[r]) continue;
        GemmArgs h = g;
        h.tcol0 = tb[r];
        h.tcol1 = tb[r + 1];
        gemm_f64(h, c.buf[S_PARTIAL], c.cur);
    }
    std::vector<size_t> off(R + 1);
    for (int r = 0; r <= R; ++r) off[r] = (size_t)std::min(n, tb[r] * tw) * n;
    shard_gather(c, g.C, off);
    launch_clean_symmetrize(g.C, n, true, c.cur);   // lower <- upper (finite: NaN->0 is a no-op)
}

// S = X'X: int8-exact for integer counts, else the fp64 MFMA product; split by
// tile columns over the shards exactly as sym_gemm_sharded.
void xtx_product(Ctx &c, const double *X, int n, double *S) {
    const int ns = xtx_int_slices(c, X, n);
    c.last_xtx_ns = ns;
    if (ns == 0) {
        GemmArgs g{n, n, n, X, n, true, X, n, S, n};
        g.sym_upper = true;
        sym_gemm_sharded(c, g);
        return;
    }
    const int8_t *sl = xtx_slices(c, X, n, ns);
    trace_mark(c.cur, "xtx: slices");
    // 128-column tiles (the LDS-staged kernel) for n >= 1024 and <= 2 slices,
    // else 64-column tiles; the products are exact, so any split gives the same bits
    const bool big = n >= 1024 && ns <= 2;
    const int tw = big ? 128 : 64;
    auto tiles = [&](int t0, int t1) {
        if (big) xtx_int8_tiles128(c, sl, n, ns, S, t0, t1);
        else xtx_int8_tiles(c, sl, n, ns, S, t0, t1);
    };
    if (!c.shard.active) {
        tiles(0, -1);
        trace_mark(c.cur, "xtx: tiles");
        return;
    }
    const int R = shard_count(c);
    std::vector<int> tb(R + 1);
    shard_plan((n + tw / 64 - 1) / (tw / 64), R, 0, tb.data());   // kind 0 counts 64-wide tiles
    for (int r = 0; r < R; ++r)
        if (shard_mine(c, r)) tiles(tb[r], tb[r + 1]);
    std::vector<size_t> off(R + 1);
    for (int r = 0; r <= R; ++r) off[r] = (size_t)std::min(n, tb[r] * tw) * n;
    shard_gather(c, S, off);
    launch_clean_symmetrize(S, n, true, c.cur);
}


void cor_product(Ctx &c, const double *X, int n, const double *m, const GatherStats *gs, double *S, double *C,
                 double *sd, double *cmean, const CorSlab *slab, bool *cm_defer) {
    hipStream_t s = c.cur;
    const bool defer = cm_defer && *cm_defer && cmean;
    if (cm_defer) *cm_defer = false;   // set again where the means are left out
    if (slab) {
        // C5 row-sharded C: each shard computes only its columns (the tiles of
        // xtx_int8_slab128: same tiles and arithmetic, so the same bits) and
        // their means; the n means are gathered, C itself never is
        if (!gs || !gs->slices2 || !cmean || !(slab->ns == 1 || slab->ns == 2))
            fail(TP_ERR_ARG, "cor_product: the column slab needs the gather's int8 image and the means buffer");
        c.last_xtx_ns = slab->ns;
        const int8_t *sl = xtx_slice_buf(c, n, 2);
        launch_cor_sd_ss(gs->css, m, n, sd, s);
        const int R = (int)slab->rb.size() - 1;
        kprof_begin(c, K_COR_GEMM);
        for (int r = 0; r < R; ++r) {
            if (!shard_mine(c, r)) continue;
            const int c0 = std::min(n, slab->rb[r]), c1 = std::min(n, slab->rb[r + 1]);
            double *dst = slab->narrow ? C : C + (size_t)c0 * n;
            xtx_int8_slab128(c, sl, n, slab->ns, dst, c0, c1, m, sd);
            launch_colmean_cols(dst, n, c1 - c0, n, cmean + c0, s);
        }
        kprof_end(c, K_COR_GEMM);
        std::vector<size_t> off(R + 1);
        for (int r = 0; r <= R; ++r) off[r] = (size_t)std::min(n, slab->rb[r]);
        shard_gather(c, cmean, off);
        return;
    }
    int ns = -1;
    if (gs && t_knob.xtx_fused && n >= 1024) ns = xtx_int_slices_cols(c, gs->cmax, gs->cbad, n);
    if (!(ns == 1 || ns == 2)) {
        if (!X) {   // the gather skipped X (int8 path expected): gather it now, same means
            if (!gs || !gs->M) fail(TP_ERR_ARG, "cor_product: no X and no gather source");
            double *Xg = c.buf[S_X].as<double>((size_t)n * n);
            launch_gather_colmean(gs->M, gs->n0, gs->good, n, Xg, const_cast<double *>(m), s);
            X = Xg;
        }
        if (!S) S = c.buf[S_S].as<double>((size_t)n * n);
        kprof_begin(c, K_COR_GEMM);
        xtx_product(c, X, n, S);
        kprof_end(c, K_COR_GEMM);
        launch_cor_epilogue(S, m, n, C, sd, s, cmean);
        return;
    }
    c.last_xtx_ns = ns;
    // the gather's 2-slice image serves ns = 1 too (its slice 1 is zero then)
    if (!gs->slices2 && !X) fail(TP_ERR_ARG, "cor_product: no X and no int8 image");
    const int8_t *sl = gs->slices2 ? xtx_slice_buf(c, n, 2) : xtx_slices(c, X, n, ns);
    launch_cor_sd_ss(gs->css, m, n, sd, s);
    kprof_begin(c, K_COR_GEMM);
    if (!c.shard.active) {
        xtx_int8_tiles128(c, sl, n, ns, C, 0, -1, m, sd);
    } else {
        // 128-column tiles split by tile columns exactly as xtx_product's big path
        const int R = shard_count(c);
        std::vector<int> tb(R + 1);
        shard_plan((n + 1) / 2, R, 0, tb.data());   // kind 0 counts 64-wide tiles: (n + 127) / 128 of 128
        for (int r = 0; r < R; ++r)
            if (shard_mine(c, r)) xtx_int8_tiles128(c, sl, n, ns, C, tb[r], tb[r + 1], m, sd);
        std::vector<size_t> off(R + 1);
        for (int r = 0; r <= R; ++r) off[r] = (size_t)std::min(n, tb[r] * 128) * n;
        shard_gather(c, C, off);
        launch_clean_symmetrize(C, n, true, s);   // lower <- upper (cor is finite: NaN -> 0 done)
    }
    kprof_end(c, K_COR_GEMM);
    if (defer) *cm_defer = true;                         // the PCA's digit pass forms them
    else if (cmean) launch_colmean(C, n, n, cmean, s);   // k_cor_epilogue_mean's bits
}

// Out (M x N col-major, ld M) = A' B with A stored K x M (col-major, lda) and
// B K x N: rows of Out split in 64-row blocks, each written transposed into
// the packed T (N x M col-major = Out row-major), gathered, transposed back.
void rows_gemm_sharded(Ctx &c, const double *A, int lda, int M, const double *B, int ldb, int N, int K,
                       double *Out, int splitk_plain, int tag, const R1 *r1, int a_col0, const ProdDigits *pd) {
    // int8 digits: row shards (the rows plan's 64-row blocks) start on the image's 64-column tiles
    const bool i8 = pd && pd->d && prod_i8_ok(K, N) && splitk_plain <= 1 && pd->col0 % 64 == 0;
    if (!c.shard.active) {
        if (a_col0 != 0) fail(TP_ERR_ARG, "rows_gemm_sharded: a column slab needs the sharded schedule");
        if (i8 && r1) {   // int8-digit partials, then the fp64 path's rank-1 reduction
            double *part = nullptr;
            const int S = prod_i8_partials(c, *pd, 0, M, B, ldb, N, K, c.buf[S_PARTIAL], &part);
            launch_splitk_reduce_r1(part, (size_t)M * N, S, M, N, r1->rows, r1->vrow, r1->u, Out, r1->rows, c.cur);
            return;
        }
        const bool fused = r1 && rows_ts(K, N) && splitk_plain <= 1;   // the epilogue rides in the reduction
        double *dst = (r1 && !fused) ? c.buf[S_SHARD].as<double>((size_t)M * N) : Out;
        GemmArgs g{M, N, K, A, lda, true, B, ldb, dst, fused ? r1->rows : M};
        g.splitk = splitk_plain;
        g.tag = tag;
        g.rows = true;
        if (fused) {
            g.r1_vrow = r1->vrow;
            g.r1_u = r1->u;
            g.r1_rows = r1->rows;
        }
        gemm_f64(g, c.buf[S_PARTIAL], c.cur);
        if (r1 && !fused) launch_r1_apply(dst, 1, (size_t)M, N, r1->rows, r1->vrow, r1->u, Out, c.cur);
        return;
    }
    const int R = shard_count(c);
    std::vector<int> rb(R + 1);
    shard_plan(M, R, 1, rb.data());
    double *T = c.buf[S_SHARD].as<double>((size_t)M * N);
    for (int r = 0; r < R; ++r) {
        if (!shard_mine(c, r) || rb[r + 1] <= rb[r]) continue;
        if (rb[r] < a_col0) fail(TP_ERR_INTERNAL, "rows_gemm_sharded: shard rows outside this rank's slab");
        if (i8) {   // the same k chunks as unsharded: the same element bits
            const int Mr = rb[r + 1] - rb[r];
            double *part = nullptr;
            const int S = prod_i8_partials(c, *pd, rb[r], Mr, B, ldb, N, K, c.buf[S_PARTIAL], &part);
            launch_splitk_reduce(part, (size_t)Mr * N, S, Mr, N, T + (size_t)rb[r] * N, N, 1, c.cur);
            continue;
        }
        GemmArgs g{rb[r + 1] - rb[r], N, K, A + (size_t)(rb[r] - a_col0) * lda, lda, true, B, ldb,
                   T + (size_t)rb[r] * N, N};
        g.store_t = true;
        // long-K products (128 x 64 kernel): k chunks fixed by K, the same bits
        // as unsharded; otherwise no split (chunks would follow the shard's tiles)
        g.splitk = rows_ts(K, N) ? splitk_plain : 1;
        g.tag = tag;
        g.rows = true;
        gemm_f64(g, c.buf[S_PARTIAL], c.cur);
    }
    std::vector<size_t> off(R + 1);
    for (int r = 0; r <= R; ++r) off[r] = (size_t)rb[r] * N;
    shard_gather(c, T, off);
    if (r1)   // same element values as unsharded, then the same rank-1 arithmetic
        launch_r1_apply(T, (size_t)N, 1, N, r1->rows, r1->vrow, r1->u, Out, c.cur);
    else
        launch_transpose(T, N, M, N, Out, M, c.cur);
}

}  // namespace tp
