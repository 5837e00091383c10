// Internal declarations shared by the HIP translation units of libtadpole_hip.
// Nothing here is part of the C ABI (include/tadpole_hip.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <atomic>
#include <mutex>
#include <string>
#include <functional>
#include <vector>

#include "../../include/tadpole_hip.h"

namespace tp {

// Run-time switches (tp_debug_knob, tp_api.hip).  tp_debug_knob sets the
// process-wide values; every C-ABI entry copies them into its calling
// thread's t_knob when it starts (guarded), so a call runs on the one set it
// started with whatever another thread sets meanwhile.
struct Knobs {
    int ch_dedup_ucap = 0;       // 1: cap on the shared CH segment store (> 0: tests of its overflow path)
    int xtx_int8 = 1;            // 5: exact int8 X'X for integer counts (0: the fp64 MFMA product)
    int pca_krylov_min = 4096;   // 8: bins from which the block Krylov PCA replaces forming G
    int xtx_fused = 1;           // 18: the correlation epilogue in the int8 X'X store
    int pca_ckrylov = -1;        // 20: Krylov space of C (1), of G (0), of C from cfg_ckry_min bins (-1)
    int shard_slab = 1;          // 24: C5 shards keep C row-sharded (0: C gathered whole)
    int prod_i8 = 5;             // 36: G-space Krylov products on int8 digits (0: fp64; 1: k_pd_prod; 5: k_pd_prodA)
    int upload_mode = 2;         // 43: bit 1: exact count blocks travel packed; bit 0: one block at a time
    int xtx_w = 1;               // 44: whole-triangle X'X by 256 x 128 tiles
    int pd_cspace = 1;           // 45: C-space Krylov products on int8 digits
    int coniss_lean_min = 0;     // 48: lean sweeps from this many bins take the global link-only CONISS
    int coniss_lds2 = 3;         // 49: LDS CONISS with one 16-bit link array (3: where 16 bytes a bin do not fit)
    int coniss_batch = 3;        // 52: batched CONISS (3: every sweep, lean ones in mode 1 where it fits;
                                 // 2: every sweep; 1: not lean ones; 0: never)
};
extern thread_local Knobs t_knob;

// Former A/B switches, now compile-time constants at their measured settings
// (the alternatives were measured slower or equal; git history has them).
constexpr int cfg_ch_dedup = 1;          // CH segment statistics shared across trees
constexpr int cfg_pca_margin = 0;        // extra Chebyshev degrees over the planned count
constexpr int cfg_gemm_xcd = 1;          // XCD-aware workgroup order of the 64 x 64 GEMM
constexpr int cfg_pca_krylov_block = 0;  // Krylov block p (0: 64 for k >= 128, else 32)
constexpr int cfg_pca_krylov_steps = 0;  // Krylov steps before the first check (0: ceil(5 k / p))
constexpr int cfg_gemm_splitk = 1;       // deep split-K for few-tile long-K products
constexpr int cfg_gemm_ts = 8;           // k_gemm_ts: most k chunks (64-column tile)
constexpr int cfg_gemm_ts32 = 8;         // the same for the 32-column tile
constexpr int cfg_xtx_supertile = 1;     // int8 X'X: XCD-contiguous supertile order
constexpr int cfg_pca_over = 0;          // subspace oversampling (0: max(32, k / 4), b rounded to 32)
constexpr int cfg_coniss_lu = 1;         // the global CONISS keeps its links as 16-bit indices in LDS
constexpr int cfg_cor_fused = 1;         // C's column means in the correlation epilogue
constexpr int cfg_pca_cheb_fused = 1;    // Chebyshev step in the T Y product's reduction
constexpr int cfg_ckry_chunk = 0;        // rows per Z partial of the PIP passes (0: from n and D)
constexpr int cfg_ckry_steps = 0;        // C-Krylov blocks before the first check (0: from k and n)
constexpr int cfg_pca_band = 1;          // products with the block-tridiagonal T skip its zero blocks
constexpr int cfg_krylov_local = 1;      // G-space CGS pass 0 against the last two blocks only
constexpr int cfg_ckry_min = 10000;      // bins from which pca_ckrylov = -1 takes the Krylov space of C
constexpr int cfg_ckry_local = 1;        // C-space first PIP pass against K_0 and the last two blocks
constexpr int cfg_xtx_nz = 1;            // int8 X'X skips the high slice's all-zero blocks
constexpr int cfg_pd_digits_blk = 1;     // the block's digits by (column, slice) workgroups
constexpr int cfg_pd_cm = 1;             // C's column means in A's digit pass
constexpr int cfg_sync_spin_us = 20000;  // sharded waits spin this long before blocking
constexpr int cfg_devbuf_async = 1;      // scratch from the library's stream-ordered pool
constexpr int cfg_pd_digits_big = 1;     // long columns' digit image in one read
constexpr int cfg_lean_auto = 1;         // sweeps lean while another pipeline is in flight on the device
constexpr int cfg_clean_tile = 0;        // NA -> 0 / symmetrise tile edge (0: 128 from 16 384 bins, else 64)

constexpr uint64_t kRNaBits = 0x7FF00000000007A2ULL;  // R NA_real_
constexpr uint64_t kRNanBits = 0x7FF8000000000000ULL; // R NaN

struct Error {
    int status;
    std::string msg;
};

[[noreturn]] void fail(int status, const std::string &msg);
void trace_mark(hipStream_t s, const char *what);   // TP_TRACE_SYNC=1: sync + stderr mark
void hip_check(hipError_t e, const char *what, const char *file, int line);
#define TP_HIP(x) ::tp::hip_check((x), #x, __FILE__, __LINE__)

// Growable device scratch buffer.
struct Ctx;
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    Ctx *owner = nullptr;   // the context whose streams use the block
    bool pooled = false;    // from the device's stream-ordered pool (hipMallocAsync)
    void *get(size_t b, bool exact = false);   // exact: grow to b, not b or 1.25x the old size
    template <class T> T *as(size_t count) { return static_cast<T *>(get(count * sizeof(T))); }
    void release();
};

// Kernel classes timed with HIP events when a caller asks for timings.
enum KClass { K_COR_GEMM = 0, K_G_GEMM, K_GQ_GEMM, K_CONISS, K_CH, K_NCLASS };

// Multi-GPU sharding of one matrix (tp_shard.hip).
struct Shard {
    void *comm = nullptr;   // ncclComm_t of this device's rank (tp_comm_init)
    int rank = 0, nranks = 1;
    int nvirt = 1;          // test hook: virtual shards on one device (no comm)
    bool active = false;    // this call runs sharded (TP_FLAG_SHARDED)
    bool dead = false;      // the device's communicator was aborted after a failure (until tp_comm_init)
};

// Per-stream state: one stream, named scratch buffers.  Every C-ABI entry
// holds the context's lock for the whole call (ctx_for takes it, the entry's
// guard releases it), so callers sharing a stream -- or the default context --
// serialise instead of racing on the scratch.  Contexts are reference counted:
// tp_release_stream / tp_shutdown drop the registry's reference and the last
// holder frees the device memory (~Ctx).
struct Ctx {
    ~Ctx();
    std::recursive_mutex mu;
    Shard shard;
    bool prof = false;                  // record per-kernel events this call
    bool lds_lean = false;              // TP_FLAG_LDS_LEAN this call (or another pipeline in flight on the device)
    std::vector<hipEvent_t> evpool;
    size_t evnext = 0;
    struct Rec { int cls; hipEvent_t a, b; };
    std::vector<Rec> recs;
    int open_cls = -1;
    hipEvent_t open_ev = nullptr;
    int device = 0;
    unsigned long long last_use = 0;   // registry tick of the last lookup (LRU retirement)
    int last_xtx_ns = 0;            // int8 slices of the last X'X product (0: fp64 MFMA product)
    // the last whole-triangle k_xtx_i8_w launch (tp_debug_xtx_exec: its executed
    // int8 MACs from the high slice's block map, still in S_XNZ)
    int xtx_w_n = 0, xtx_w_kp = 0, xtx_w_np = 0, xtx_w_ns = 0;
    bool xtx_w_map = false;
    hipStream_t stream = nullptr;   // library stream (or the caller's, owns_stream = false)
    bool owns_stream = false;
    hipStream_t cur = nullptr;      // stream used by the current call
    hipStream_t side = nullptr;     // fork-join helper stream (side_stream())
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    DevBuf buf[48];   // indexed by Slot (static_assert below)
    DevBuf pinned_flag;
    void *host_pinned = nullptr;    // small pinned staging area
    size_t host_pinned_bytes = 0;
    hipEvent_t ring_ev[4] = {};     // tp_read_tsv_dev: one event per staging-ring slot
    hipEvent_t sync_ev = nullptr;   // event_sync: a read-back point with more work queued behind it
    int *progress = nullptr;        // tp_progress_attach: host word, the pipeline's stage (1 mask .. 4 done)
    void *pinned(size_t b);
};

// device context; a non-null stream other than the library's selects that
// stream's own context (scratch buffers), so streams can run concurrently
Ctx &ctx_for(int device, hipStream_t stream = nullptr);
// a second stream of this context for work that overlaps the current stream's
// (fork: side waits for cur's work so far; join: cur waits for side's)
hipStream_t side_fork(Ctx &c);
void side_join(Ctx &c);
void kprof_begin(Ctx &c, int cls);
void kprof_end(Ctx &c, int cls);
void kprof_collect(Ctx &c, double *ms_per_class, int *count_per_class);
void ctx_shutdown_all();
bool ctx_release_stream(int device, hipStream_t stream);   // false: no context for that stream
void ctx_unlock_held();   // end of a C-ABI call: unlock (and maybe free) the contexts it used
// sharded calls: exclusive use of the device's communicator for the call, with
// the context's copy of it refreshed from the device's (shard_lease_begin
// fails when the communicator was aborted); shard_lease_end releases it
void shard_lease_begin(Ctx &c);
void shard_lease_end(Ctx &c);
// the device's communicator `comm` failed: the device forgets it (and
// remembers that it died); true for the one caller that must ncclCommAbort it
bool ctx_comm_retire(Ctx &c, void *comm);

// Scratch slots (indices into Ctx::buf) so stages can share one context.
enum Slot {
    S_M = 0, S_ROWMEAN, S_DIAG, S_BAD, S_GOOD, S_NGOOD, S_X, S_COLMEAN,
    S_S, S_C, S_XC, S_XCT, S_G, S_Q, S_Z, S_W, S_SMALL, S_P, S_PT,
    S_SWEEP, S_SWEEP2, S_SCORES, S_PARTIAL, S_MISC, S_SHARD, S_SHARD2, S_DEDUP,
    S_KRY, S_KRYG, S_KRYT, S_KRYV, S_KRYX, S_CMEAN, S_CHBIG, S_CHOLP, S_SMALL2, S_GSTAT, S_XTXT, S_MEXT, S_KRYA,
    S_KRYH, S_XNZ, S_PDIGA, S_PDIGB, S_UPLD,
    S_NSLOT
};
static_assert(S_NSLOT <= (int)(sizeof(Ctx::buf) / sizeof(Ctx::buf[0])), "Ctx::buf too small for the slots");

// ---------------------------------------------------------------- kernels
// mask / correlation / centering  (tp_prep.hip)
void launch_clean_symmetrize(double *d_M, int n0, bool src_upper, hipStream_t s);
void launch_rowmean_diag(const double *d_M, int n0, double *d_rowmean, double *d_diag,
                         hipStream_t s);
void launch_mask_select(const double *d_rowmean, const double *d_diag, int n0,
                        double bad_frac, double qindex, int *d_bad, int *d_good,
                        int *d_ngood, hipStream_t s);
void launch_gather_colmean(const double *d_M, int n0, const int *d_good, int n,
                           double *d_X, double *d_colmean, hipStream_t s);
void launch_colmean(const double *d_A, int n, int ld, double *d_mean, hipStream_t s);
void launch_colmean_cols(const double *d_A, int n, int ncols, int ld, double *d_mean, hipStream_t s);
// the gather with what the int8 X'X needs (per-column max / non-integer flag /
// exact sum of squares, speculative 2-slice int8 image), tp_prep.hip
void launch_gather_prep(const double *d_M, int n0, const int *d_good, int n, double *d_X, double *d_colmean,
                        double *d_cmax, int *d_cbad, long long *d_css, int8_t *d_sl, int Kp, int Np, hipStream_t s);
void launch_cor_sd_ss(const long long *d_css, const double *d_m, int n, double *d_sd, hipStream_t s);
// d_cmean != nullptr: the column means of C are formed in the same pass (k_colmean's order)
void launch_cor_epilogue(const double *d_S, const double *d_m, int n, double *d_C, double *d_sd,
                         hipStream_t s, double *d_cmean = nullptr);
void launch_center(const double *d_C, const double *d_mean, int n, double *d_Xc,
                   double *d_XcT, hipStream_t s);

// fp64 MFMA GEMM (tp_gemm.hip).  C[i,j] = sum_k A'(i,k) B(k,j); A' = A^T when
// trans_a (A stored K x M col-major), else A (M x K col-major).  B: K x N
// col-major.  C: M x N col-major (ldc) or, if store_t, C^T (C[j + i*ldc]).
// sym_upper: compute tiles with row-block <= col-block only and mirror them.
// splitk > 1: partial sums in workspace, reduced in a fixed order.
struct GemmArgs {
    int M, N, K;
    const double *A; int lda; bool trans_a;
    const double *B; int ldb;
    double *C; int ldc;
    bool store_t = false;
    bool sym_upper = false;
    int splitk = 1;     // 0 = choose from the tile count
    int tcol0 = 0, tcol1 = -1;   // sym_upper: only tile columns [tcol0, tcol1) (-1 = all)
    bool big_cols = false;       // use the 128 x 128 kernel; tcol0/tcol1 then count 128-column tiles
    int tag = 0;                 // 1: the PCA's G Y products (own kernel symbols for profiles)
    bool rows = false;           // row-shardable long-K product (rows_gemm_sharded): 128 x 64 kernel, k chunks by K
    const double *sub_from = nullptr;   // C = sub_from - A'B (plain column-major C; may alias C): same bits as
                                        // the product into a temporary and a separate subtraction
    // rank-1 epilogue of the row-shardable long-K product (rows_ts path): rows
    // [0, r1_rows) of C (ldc) = (A'B)[i, j] - u_i (A'B)[r1_vrow, j], u = r1_u or
    // all ones; the M - r1_rows extra rows are computed, not stored
    int r1_vrow = -1;
    const double *r1_u = nullptr;
    int r1_rows = 0;
    // affine epilogue (the Chebyshev three-term step): C = af_a (A'B) + af_b af_y
    // [+ af_c af_z], elementwise over C's column-major layout (ldc), in the
    // split-K reduction; plain (not sym/store_t/sub_from/rows) products only
    bool affine = false;
    double af_a = 1.0, af_b = 0.0, af_c = 0.0;
    const double *af_y = nullptr, *af_z = nullptr;
};
void gemm_f64(const GemmArgs &g, DevBuf &work, hipStream_t s);
void launch_r1_apply(const double *T, size_t rs, size_t cs, int N, int rows, int vrow, const double *u, double *Out,
                     hipStream_t s);
void launch_splitk_reduce_r1(const double *part, size_t stride, int S, int M, int N, int rows, int vrow,
                             const double *u, double *C, int ldc, hipStream_t s);
void launch_splitk_reduce(const double *part, size_t stride, int S, int M, int N, double *C, int ldc, int store_t,
                          hipStream_t s);
// set only by the tp_debug_gemm hook around its own call (this thread)
extern thread_local int g_gemm_panel;   // short-K tall-skinny 32 x 64 kernel enabled (default 1)
extern thread_local int g_gemm_kb;      // LDS stage depth of the 64 x 64 kernel (16 / 32)
// b <= 1280 (a multiple of 32); b > 480 needs chol_panel_doubles(b) of scratch
size_t chol_panel_doubles(int b);
void launch_chol(double *d_W, double *d_rdiag, int b, double rel, int *d_info, hipStream_t s,
                 double *d_panel = nullptr);
void launch_chol_stamped(double *d_W, double *d_rdiag, int b, double rel, int *d_info, long long *d_st,
                         hipStream_t s);
void launch_trsm_ru(const double *d_Z, int n, int b, const double *d_U, const double *d_rdiag, double *d_Q,
                    hipStream_t s);
// CholQR for b <= 256 (b % 16 == 0), tp_chol.hip: k_chol_inv factors
// S W S + rel I = U'^T U' (S = diag(W)^-1/2) in one register-resident
// workgroup and leaves U' tiles and E_p = U'_pp^-T as MFMA operand fragments
// in F (b x b doubles), S in sc (b), 1/diag(U) in rdiag (b), diag(U) on W's
// diagonal; k_trsm_frag then forms Q = Z U^-1 (U = U' S^-1), n/16 waves.
constexpr int kCholInvMax = 256;
extern thread_local int g_chol_inv_waves;   // set only by the CholQR debug hook (this thread)
// row-shardable products that take the 128 x 64 kernel with k chunks fixed by K
// (tp_gemm.hip); shards and the unsharded call must agree on it
inline bool rows_ts(int K, int N) { return cfg_gemm_ts > 0 && K >= 4096 && N <= 256; }
void launch_chol_inv(double *d_W, double *d_F, double *d_sc, double *d_rdiag, int b, double rel, int *d_info,
                     hipStream_t s, long long *d_stamps = nullptr);
void launch_trsm_frag(const double *d_Z, int n, int b, const double *d_F, const double *d_sc, double *d_Q,
                      hipStream_t s);

// sweep (tp_sweep.hip)
struct SweepDev {
    const double *Pt;   // n x ldp row-major PC scores
    int n, ldp, k;      // k = columns used by CH (all PCs)
    int tree0 = 0;      // trees tree0+1 .. tree0+ntrees (grid = ntrees)
    int ntrees = 0;
    int min_clusters;
    double *sums;       // per-tree cluster sums, see sweep_sums_doubles
    int *mrg_a, *mrg_b; // k x (n-1)
    double *cost, *height;
    int *n_cluster;     // ntrees
    double *scores;     // ntrees x w_cap, column-major (ld ntrees)
    int w_cap;
    double *seg;        // CH scratch: k trees x seg_cap x (k + 1) doubles
    int *iseg;          // CH scratch: k trees x (2 seg_cap + 2) ints
    int seg_cap;        // max cut size the CH kernel handles
    double *trS;        // 1
    int *err;           // device flag: 1 = a cut exceeded seg_cap / w_cap
    long long *stamps = nullptr;   // diagnostic builds only (k_coniss_t<true>)
    double *cost0 = nullptr;       // ntrees x roundup(n, 64) initial costs (scratch)
    const double *pt2 = nullptr;   // CONISS: the scores with slots 0 and 1 paired (set by the launcher, inside cost0)
    int pt2_ld = 256;              // its row stride: 64 x the widest tree's slots rounded to 4 or 8
    const double *pt4 = nullptr;   // CONISS, trees of exactly 4 slots: slots (0,1) and (2,3) paired, row stride 256
    // CH segment statistics shared across trees (null: every tree computes its
    // own): the finest cuts' segments [s, e) go into an open-addressing set
    // (hkeys, empty = ~0), each distinct one gets a slot of ustore (k column
    // sums + SS) computed once; see sweep_dedup_bytes
    unsigned long long *hkeys = nullptr;
    int *hidx = nullptr;                  // hcap: ustore index per set slot (-1: store full)
    int hcap = 0;                         // power of two >= 2 x the segments inserted
    unsigned long long *ukey = nullptr;   // ucap: key of each stored segment
    double *ustore = nullptr;             // ucap x (k + 1)
    int ucap = 0;
    int *ucount = nullptr;                // distinct segments inserted (may exceed ucap)
    bool lds_lean = false;                // CONISS: links in global memory (a few bytes of LDS a tree)
};
// scratch of the shared CH segment statistics for ntrees trees
int pipelines_in_flight(int device);
size_t sweep_dedup_bytes(int n, int k, int ntrees, int seg_cap, int *hcap, int *ucap);
void sweep_dedup_bind(SweepDev &sd, void *base, int hcap, int ucap);
// CONISS per-tree rows: roundup(n, 64) costs + 64 (a dummy slot, index
// roundup(n, 64), that takes the branch-free writes of absent positions); link
// and right-end arrays of n + 64 ints (dummy slot n)
__host__ __device__ inline size_t coniss_cost_stride(int n) { return (size_t)((n + 63) / 64) * 64 + 64; }
__host__ __device__ inline size_t coniss_link_stride(int n) { return (size_t)n + 64; }
// initial costs (ntrees x cost stride) + link scratch of the global-memory
// CONISS variant (ntrees x 2 link strides of ints)
// row-major scores Pt (n x k) + slack: CONISS reads whole 64-column slots of a
// row (up to 1024 columns) and masks the columns past its prefix
inline size_t pt_doubles(int n, int k) { return (size_t)n * k + 1024; }
// + the copy of the scores with column pairs (l, l + 64) adjacent that CONISS
// reads (n x 64 KS: 256, 512 for k > 256, 1024 for k > 512; see k_pt_pairs in
// tp_sweep.hip), + the fully paired copy the 4-slot trees read (n x 256, when k > 192)
inline size_t sweep_cost0_doubles(int n, int ntrees, int k = 256) {
    return (size_t)ntrees * (coniss_cost_stride(n) + coniss_link_stride(n)) + 2 +
           (size_t)n * (k > 512 ? 1024 : (k > 256 ? 512 : 256)) + (k > 192 ? (size_t)n * 256 : 0);
}
size_t sweep_sums_doubles(int n, int tree0, int ntrees);
void launch_sweep(const SweepDev &sd, hipStream_t s, Ctx *prof = nullptr);
void launch_coniss_only(const SweepDev &sd, hipStream_t s);
// CH of the trees whose finest cut has more than 1024 segments (k_ch's LDS
// capacity): d_slot_of[ntrees] = scratch slot or -1
size_t ch_glb_slot_doubles(int nc, int k);
void launch_ch_glb(const SweepDev &sd, const int *d_slot_of, double *scratch, size_t slot_doubles, hipStream_t s);
void launch_coniss_stamped(const SweepDev &sd, hipStream_t s);
void launch_ch_only(const double *d_Pt, int n, int ldp, int k, const int *d_bnd,
                    int cn, double *d_seg, double *d_out, hipStream_t s);
void launch_dist(const double *d_P, int n, int ldp, int ncols, double *d_d, hipStream_t s);
void launch_transpose(const double *d_A, int rows, int cols, int lda, double *d_T, int ldt,
                      hipStream_t s);

// PCA (tp_pca.hip): P (n x k col-major, ld n) and Pt (n x k row-major) from C.
// Symmetric eigendecomposition for b <= 1280 (tp_eig.hip): A (b x b, lower
// triangle) <- eigenvectors, theta <- ascending eigenvalues.  work >= b*b + 4b + 8.
bool eig_sym_supported(int b);
void sytrd_stamped(double *A, int b, double *work, long long *d_stamps, hipStream_t s);
void sytrd_which(double *A, int b, double *work, int which, hipStream_t s,
                 long long *d_stamps = nullptr);   // work: 3b (e, tau, d)
void eig_sym(double *A, int b, double *theta, double *work, hipStream_t s);

// tp_io.hip: native reader of read.big.matrix(sep = '\t') files (host code)
void tsv_dims(const char *path, int *nrow, int *ncol);
void tsv_read(const char *path, int nrow, int ncol, int nthreads, bool row_major, double *out);
// row-major, in row blocks of ~block_bytes of doubles through a ring of nslots
// staging slots (alloc(slot_rows) -> nslots x slot_rows x ncol doubles):
// on_block(r0, r1, rows, slot) as each block completes; slot_free(slot) must
// return only when the slot may be overwritten (see tp_io.hip)
void tsv_read_rows(const char *path, int nrow, int ncol, int nthreads, size_t block_bytes, int nslots,
                   const std::function<double *(size_t)> &alloc,
                   const std::function<void(size_t, size_t, const double *, int)> &on_block,
                   const std::function<void(int)> &slot_free);

// sharding (tp_shard.hip)
void comm_unique_id(char *id128);
void comm_init(Ctx &c, const char *id128, int nranks, int rank);
void comm_destroy(Ctx &c);
// host waits of a call that may be sharded: bounded and abort-on-failure with a
// live communicator (see tp_shard.hip), hipStreamSynchronize otherwise
void stream_sync(Ctx &c, hipStream_t s);
// Record the context's sync event on s (behind the work queued so far); then
// event_sync waits for that point only, so work queued after the record keeps
// the device busy while the host reads the results (sharded: same watchdog as
// stream_sync)
void event_mark(Ctx &c, hipStream_t s);
void event_sync(Ctx &c);
void comm_abort(Ctx &c);
extern std::atomic<int> g_shard_inject;   // test hook: the next N sharded waits fail as device errors
int shard_count(const Ctx &c);
bool shard_mine(const Ctx &c, int r);
void shard_plan(int n, int R, int kind, int *bounds);
void shard_gather(Ctx &c, double *buf, const std::vector<size_t> &off);
void shard_gather_bytes(Ctx &c, void *buf, const std::vector<size_t> &off);
void shard_bcast_bytes(Ctx &c, void *buf, size_t bytes, int root);
void sym_gemm_sharded(Ctx &c, GemmArgs g);
// R1 (optional): Out (r1->rows x N, ld r1->rows) = (A'B)[i, j] - u_i (A'B)[vrow, j]
struct R1 {
    int vrow;
    const double *u;   // nullptr: all ones
    int rows;
};
// a_col0: A points at column a_col0 of the logical K x M matrix (a rank's
// column slab of C: its shard's rows are the only ones it reads)
// int8-digit image of A's columns for the long-K products (tp_prod_i8.hip):
// columns [col0, col0 + cols) of the logical A, digit s of local column i at
// d + s slice + i Kp, its scale 2^(e - 54) at rs[i]
struct ProdDigits {
    const int8_t *d = nullptr;
    const double *rs = nullptr;
    size_t slice = 0;
    int Kp = 0, col0 = 0, cols = 0;
    int pending = 0;   // > 0: columns [pending, cols) not digitised yet (prod_digits_finish)
};
bool prod_i8_ok(int K, int N);
int prod_i8_pairs();   // digit pairs one int8 product sums (27 with six digits of A)
int prod_i8_adig();    // digits of A the image stores
// cm != nullptr: only columns [0, ncm) now, with their means (k_colmean's bits)
// into cm; the rest after the caller has written them, by prod_digits_finish
void prod_digits_build(Ctx &c, const double *A, int lda, int K, int cols, int col0, ProdDigits &pd,
                       double *cm = nullptr, int ncm = 0);
void prod_digits_finish(Ctx &c, const double *A, int lda, int K, ProdDigits &pd);
bool prod_digits_means_ok(int K);
// host -> device through the context's pinned ring (tp_upload.hip); counts:
// blocks of exact 16-bit counts travel packed.  Returns the bytes sent packed.
size_t upload_host(Ctx &c, const void *host, size_t bytes, void *d_dst, int nthreads, bool counts);
int prod_i8_partials(Ctx &c, const ProdDigits &pd, int r0, int M, const double *B, int ldb, int N, int K,
                     DevBuf &work, double **part);
// pd (optional): A's digit image; the product then runs on the int8 MFMA
// (same k chunks for every shard) when prod_i8_ok(K, N)
void rows_gemm_sharded(Ctx &c, const double *A, int lda, int M, const double *B, int ldb, int N, int K,
                       double *Out, int splitk_plain, int tag = 0, const R1 *r1 = nullptr, int a_col0 = 0,
                       const ProdDigits *pd = nullptr);

// exact X'X on int8 matrix cores for integer counts (tp_xtx.hip)
extern std::atomic<int> g_kprof_fine;   // 0: no per-launch Krylov product events (they open gaps on the stream)
int xtx_int_slices(Ctx &c, const double *d_X, int n);   // 0 = not integer counts (fp64 path)
const int8_t *xtx_slices(Ctx &c, const double *d_X, int n, int ns);
void xtx_int8_tiles(Ctx &c, const int8_t *sl, int n, int ns, double *d_S, int tc0, int tc1);   // 64-col tiles
// cm / csd given: the correlation epilogue in the store (d_S receives cor)
void xtx_int8_tiles128(Ctx &c, const int8_t *sl, int n, int ns, double *d_S, int tc0, int tc1,
                       const double *cm = nullptr, const double *csd = nullptr);
// columns [c0, c1) only, into d_slab (ld n, column c0 first): the C5 row-sharded C
void xtx_int8_slab128(Ctx &c, const int8_t *sl, int n, int ns, double *d_slab, int c0, int c1,
                      const double *cm = nullptr, const double *csd = nullptr);
int xtx_kp(int n);
// executed MACs of the context's last whole-triangle k_xtx_i8_w launch: out[0]
// executed int8 MACs, out[1] the slice-0 MACs, out[2] high-slice k-blocks
// summed over the tiles, out[3] tiles, out[4] k-blocks a tile (false: none)
bool xtx_w_exec(Ctx &c, double *out);
int8_t *xtx_slice_buf(Ctx &c, int n, int ns);
int xtx_int_slices_cols(Ctx &c, const double *d_cmax, const int *d_cbad, int n);
// sparse_cor in one call (R/TADpole.R:94-100,449): C = cor(X) with NaN -> 0, and
// C's column means into d_cmean when given.  Exact int8 X'X with the epilogue in
// the store when the gather's statistics say X holds counts < 2^14 (and its
// slices are already built), else X'X into d_S and the separate epilogue.
struct GatherStats {
    const double *cmax;
    const int *cbad;
    const long long *css;
    bool slices2;   // the gather wrote the 2-slice int8 image
    // the gather's source, for X on demand (the gather skipped writing it):
    // cor_product runs k_gather_colmean into S_X when the fp64 product is needed
    const double *M = nullptr;
    int n0 = 0;
    const int *good = nullptr;
};
// C5 row-sharded C (one matrix over R ranks on the Krylov path): shard r owns
// columns [rb[r], rb[r+1]) of [C | m | 1] (rb: rows_gemm_sharded's row plan
// over n + 2); narrow: d_C holds only this rank's columns (column rb[rank]
// first), else all of them (virtual shards)
struct CorSlab {
    int ns = 0;
    std::vector<int> rb;
    bool narrow = false;
};
// cm_defer (in/out): true asks to leave d_cmean for the PCA's digit pass
// (pca_dev's cm_pending) where C comes from the int8 X'X epilogue; it stays
// true only if the means were left out
void cor_product(Ctx &c, const double *d_X, int n, const double *d_m, const GatherStats *gs, double *d_S,
                 double *d_C, double *d_sd, double *d_cmean, const CorSlab *slab = nullptr, bool *cm_defer = nullptr);
// S = X'X by the exact int8 path when possible, sharded like sym_gemm_sharded
void xtx_product(Ctx &c, const double *d_X, int n, double *d_S);

struct PcaStats {
    int iters = 0; double resid = 0; double rate = 0; int block = 0; int blocks = 0;
    int krylov_steps = 0, krylov_dim = 0;   // block Krylov path (0: G formed)
    int prod_pairs = 0;                     // int8 digit pairs of the products with C (0: fp64 products)
    const double *d_theta = nullptr;        // device copy of h_theta (valid until the next small problem)
};
// the top k eigenpairs of a D x D projected matrix (tp_pca.hip)
// band_p > 0: T is block tridiagonal with band_p x band_p blocks (products
// with it skip the zero blocks when cfg_pca_band)
void small_topk_T(Ctx &c, double *Tm, int D, int k, double *Vs, std::vector<double> &h_theta, PcaStats &sst,
                  int band_p = 0);
// false: an orthogonalisation pass broke down (the caller takes the G path)
bool krylov_c_topk(Ctx &c, double *C, int c_col0, const double *mext, int n, int k, double *V, double *P,
                   std::vector<double> &h_theta, PcaStats &st, const ProdDigits *pd = nullptr);
// d_C: n x n, with room for 2n more doubles after it (the Krylov path writes
// m = colMeans(C) and a column of ones there); d_cmean: C's column means if the
// caller already has them (may be d_C + n n), else computed here
inline size_t pca_c_doubles(int n) { return (size_t)n * n + 2 * (size_t)n; }
// c_col0 / c_col1: d_C holds only columns [c_col0, c_col1) of [C | m | 1] (a
// C5 rank's slab, Krylov path; -1: all of them, with room for the two extra).
// cm_pending: d_cmean is the buffer for C's means, not filled yet (formed in
// A's digit pass on the int8 Krylov path, else by k_colmean: the same bits)
PcaStats pca_dev(Ctx &c, double *d_C, int n, int k, double *d_P, double *d_Pt,
                 double *h_sdev, const double *d_cmean = nullptr, int c_col0 = 0, int c_col1 = -1,
                 bool cm_pending = false);

}  // namespace tp
