/*
 * tadpole_hip.h — C ABI of libtadpole_hip.so, the MI355X (gfx950) engine for
 * TADpole's per-matrix hot path.
 *
 * The reference (3DGenomes/TADpole, R) has no FFI of its own: its seam is the R
 * function body R/TADpole.R:444-460, which these entry points replace
 *
 *   load_mat mask        R/TADpole.R:19-20,35-37,88-89   -> tp_mask
 *   sparse_cor + NaN->0  R/TADpole.R:94-100,448-449       -> tp_cor
 *   prcomp(cor, rank.)   R/TADpole.R:452-453              -> tp_pca
 *   find_params          R/TADpole.R:102-140,456          -> tp_sweep
 *   chclust(dist(pcs))   R/TADpole.R:108,459-460          -> tp_coniss
 *   dist(pcs)            R/TADpole.R:108,460              -> tp_dist
 *   calinhara(x, cutree) R/TADpole.R:117-120              -> tp_ch
 *   the whole seam       R/TADpole.R:348-349,444-468      -> tp_pipeline
 *   cutree/rle coords    R/TADpole.R:470-488              -> tp_level_coords
 *
 * Calling convention (so R's .C() can bind every entry without R headers, and
 * Python ctypes in the tests): every argument is a pointer; matrices are
 * column-major unless a layout flag says otherwise; logical = int; the caller
 * allocates every output; 1-based indices only where R would see them (merge
 * matrix, n_pcs, n_clusters).  NA in double outputs is R's NA_real_ bit
 * pattern (0x7FF00000000007A2), so R reads NA, not NaN.
 *
 * Status: every entry writes *status (0 = TP_OK).  On failure the message is
 * available from tp_last_error / tp_last_error_r (per thread).  A missing GPU
 * or HIP runtime is an error (TP_ERR_HIP): there is no CPU fallback.
 *
 * Device pointers: the *_dev variants take device-resident inputs (e.g. from a
 * torch tensor) and a hipStream_t (as void*, NULL = the library stream of that
 * device); their outputs are host pointers unless named d_*.
 */
#ifndef TADPOLE_HIP_H
#define TADPOLE_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

enum {
    TP_OK = 0,
    TP_ERR_ARG = 1,         /* bad sizes / arguments                              */
    TP_ERR_HIP = 2,         /* HIP runtime / device failure                       */
    TP_ERR_NO_BSTICK = 3,   /* a tree has no broken-stick level: R errors in
                               rep(NA, n_cluster) at R/TADpole.R:115            */
    TP_ERR_CAPACITY = 4,    /* an output array is too small (see *_cap args)     */
    TP_ERR_NUMERIC = 5,     /* PCA did not converge / non-finite scores          */
    TP_ERR_UNSUPPORTED = 6, /* size beyond what this build handles               */
    TP_ERR_INTERNAL = 7     /* an internal invariant failed (a library bug); in
                               a sharded call it aborts the communicator        */
};

/* flags for tp_pipeline / tp_mask */
#define TP_FLAG_ROW_MAJOR   1   /* input matrix buffer is row-major (numpy C order) */
#define TP_FLAG_CLEAN       2   /* input is already NA-free and symmetric          */
#define TP_FLAG_NO_MASK     4   /* keep every bin: the per-arm matrices of
                                   R/TADpole.R:362 are correlated as given        */
#define TP_FLAG_SHARDED     8   /* tp_pipeline_dev: split this matrix's products
                                   over the ranks of the device's communicator
                                   (tp_comm_init); every rank passes the same
                                   matrix and gets the same results            */
#define TP_FLAG_SUBSET     16   /* tp_pipeline(_dev): run on the principal
                                   submatrix good_idx[0 .. *n_good) names (input:
                                   1-based, strictly ascending; implies NO_MASK;
                                   bad[] is not written).  The centromere arms
                                   (R/TADpole.R:362) read straight from the
                                   cleaned whole matrix, never copied out      */
#define TP_FLAG_LDS_LEAN   32   /* tuning hint: another pipeline runs on this
                                   device at the same time; the CONISS sweep of
                                   a matrix too large for LDS keeps half its
                                   link data there (2 bytes a bin) so a tree of
                                   each pipeline fits on one CU.  Results are
                                   the same bits either way                    */

/* ---------------------------------------------------------------- runtime */
int  tp_version(void);                          /* ABI version, 2 (see below)    */
int  tp_device_count(void);                     /* HIP devices visible (>=0)     */
void tp_shutdown(void);                         /* free every device context     */
/* Free the scratch (device memory, pinned staging) of the context the library
 * keeps for a caller-supplied stream (*_dev entries with a non-NULL stream: one
 * context per stream, each holding ~N^2-sized scratch).  A call still running
 * on that stream keeps its context until it returns; the next call on the
 * stream makes a new one.  NULL stream: TP_ERR_ARG (tp_shutdown frees the
 * library's own stream).  Every entry locks the context it uses for the whole
 * call, so concurrent callers of one stream (or of the library stream)
 * serialise.  ABI 2: timings_ms of tp_pipeline / tp_pipeline_dev holds 32
 * doubles (ABI 1: 16) -- a caller built against version 1 must pass NULL
 * timings or a 32-double buffer. */
void tp_release_stream(const int *device, void *stream, int *status);
/* Context bookkeeping of `device`: live = caller-stream contexts kept now,
 * created = contexts (the library stream's included) made since the library
 * was loaded.  A caller that reuses its streams creates none after the first
 * call on each (tadpole_amd.genome's persistent stream pool is tested so). */
void tp_context_stats(const int *device, int *live, int *created, int *status);
/* Size the contexts of `nstreams` caller streams alike: each of their scratch
 * buffers grows to the largest size that buffer has in any of them (no data
 * kept; stream-ordered, synchronised before returning).  For a pool of streams
 * that any matrix of a workload may land on (tadpole_amd.genome): once every
 * matrix has run on one stream of the pool, no call regrows scratch. */
void tp_reserve_streams(const int *device, void *const *streams, const int *nstreams, int *status);
/* Attach a host word to the context of (device, stream) (NULL detaches):
 * every later tp_pipeline / tp_pipeline_dev on that context stores its stage
 * there as it goes -- 0 started, 1 mask read back, 2 correlation queued,
 * 3 PCA finished and the sweep about to be queued, 4 returned (success or
 * failure) -- with release ordering, so another host thread can poll it to
 * overlap work with this pipeline's later stages (the centromere arms: one
 * arm's correlation and PCA under the other arm's CONISS sweep). */
void tp_progress_attach(const int *device, void *stream, int *progress, int *status);
int  tp_last_error(char *buf, int len);         /* ctypes form                   */
void tp_last_error_r(char **buf, int *len);     /* R .C form                     */

/* -------------------------------------------------------------- multi-GPU */
/* One matrix over several GPUs (chr1 @5kb arms of ~24k bins;
 * the reference has no multi-GPU path -- it forks over PC prefixes,
 * R/TADpole.R:104).  One process (or host thread) per GPU.  Rank 0 calls
 * tp_comm_unique_id, the host distributes the 128 bytes (torch.distributed,
 * MPI, a file...), every rank calls tp_comm_init on its device, then
 * tp_pipeline_dev(..., flags | TP_FLAG_SHARDED) with the same matrix: X'X and
 * Xc'Xc are split by column tiles, G Q and Xc V by rows, the sweep by PC
 * prefixes, all gathered over RCCL (xGMI).  Results are bit-identical for any
 * rank count.  RCCL (librccl.so.1) is loaded at tp_comm_init.
 * tp_set_virtual_shards: test hook running the sharded schedule as nvirt
 * shards on one device (no communicator).  tp_shard_plan (host only): the
 * split, kind 0 = tile columns of the symmetric products, 1 = rows (64-row
 * blocks), 2 = trees; bounds[nranks + 1]. */
void tp_comm_unique_id(char *id /* 128 bytes */, int *status);
void tp_comm_init(const char *id, const int *nranks, const int *rank,
                  const int *device, int *status);
void tp_comm_destroy(const int *device);
void tp_set_virtual_shards(const int *device, const int *nvirt, int *status);
void tp_shard_plan(const int *n, const int *nranks, const int *kind,
                   int *bounds, int *status);

/* --------------------------------------------------------------- load_mat */
/* bigmemory::read.big.matrix(mat_file, type='double', sep='\t') (R/TADpole.R:17,
 * :160) natively: a memory-mapped, multi-threaded parse of the headerless
 * tab-separated matrix.  path: char** (the R .C string convention).
 * tp_tsv_dims: rows (lines) and columns (fields of the first line).
 * tp_read_tsv: fills out (nrow x ncol, column-major, or row-major with
 * TP_FLAG_ROW_MAJOR); NA/NaN/empty/non-numeric -> NaN, short lines NaN-padded,
 * long lines TP_ERR_ARG.  nthreads <= 0: all hardware threads.  Host only. */
void tp_tsv_dims(const char **path, int *nrow, int *ncol, int *status);
void tp_read_tsv(const char **path, const int *nrow, const int *ncol,
                 const int *nthreads, const int *flags, double *out, int *status);
/* The same parse straight into device memory: d_out (nrow x ncol, row-major,
 * on `device`) filled through the library's pinned staging in row blocks, each
 * block's copy queued on `stream` while the next block is parsed (the upload
 * hides under the parse).  Returns once the copies are complete. */
void tp_read_tsv_dev(const char **path, const int *nrow, const int *ncol,
                     const int *nthreads, const int *device, void *stream,
                     double *d_out, int *status);

/* Host -> device copy of `bytes` bytes of a pageable host buffer into d_dst
 * (device memory of `device`), queued on `stream` (hipStream_t, NULL: the
 * library's) through that stream's context's pinned staging: 16 MB blocks in
 * a ring of three, each block's host copy (nthreads threads, 0 = 1) overlapped
 * with the previous blocks' DMAs; returns when the data is on the device.
 * Stands where R's .C/ctypes caller would hand tp_pipeline a host matrix but
 * wants tp_pipeline_dev's stream (concurrent pipelines per GPU). */
void tp_upload_dev(const void *host, const long long *bytes, void *d_dst, const int *nthreads,
                   const int *device, void *stream, int *status);

/* The same for a float64 matrix of `count` values: 16 MB blocks whose every
 * value is an exact integer in [0, 65535] (Hi-C counts; no -0.0, NaN or
 * fraction) travel as 16-bit integers and are widened on the device to the
 * same doubles, any other block as float64.  *packed (may be NULL): bytes of
 * float64 that travelled packed.  tp_pipeline's host matrix takes this path. */
void tp_upload_counts_dev(const double *host, const long long *count, double *d_dst, const int *nthreads,
                          const int *device, void *stream, long long *packed, int *status);

/* ------------------------------------------------------------------- mask */
/* R/TADpole.R:19-20 (NA->0, forceSymmetric(uplo='U')), :35-37 (rowMeans, diag==0,
 * quantile type 7 at bad_frac), :88-89 (subset).  M: n0 x n0.  Outputs:
 * bad[n0] (logical), rowmean[n0] (may be NULL), *n_good, good_idx[n0] (1-based
 * original indices of kept bins, first *n_good entries valid). */
void tp_mask(const double *M, const int *n0, const double *bad_frac,
             const int *flags, const int *device, int *bad, double *rowmean,
             int *n_good, int *good_idx, int *status);
/* Same on a device-resident d_M (n0 x n0), work queued on `stream`; unless
 * TP_FLAG_CLEAN, d_M is cleaned and symmetrised IN PLACE (R/TADpole.R:19-20). */
void tp_mask_dev(double *d_M, const int *n0, const double *bad_frac,
                 const int *flags, const int *device, void *stream, int *bad,
                 double *rowmean, int *n_good, int *good_idx, int *status);

/* -------------------------------------------------------------------- cor */
/* sparse_cor(x)$cor with NaN -> 0 (R/TADpole.R:94-100,449).  X: n x n
 * symmetric (column-major), cor: n x n. */
void tp_cor(const double *X, const int *n, const int *device, double *cor,
            int *status);

/* -------------------------------------------------------------------- pca */
/* prcomp(C, rank. = k)$x (R/TADpole.R:452-453): P = (C - 1 colMeans(C)') V_k,
 * V_k the top-k right singular vectors.  C: n x n symmetric.  P: n x k.
 * sdev (length k, may be NULL) = singular values / sqrt(n-1) as prcomp. */
void tp_pca(const double *C, const int *n, const int *k, const int *device,
            double *P, double *sdev, int *status);

/* ------------------------------------------------------------------ sweep */
/* find_params (R/TADpole.R:102-140) on scores P (n x k, column-major):
 * for i = 1..k: CONISS on P[,1:i], broken stick -> n_cluster[i-1], CH on all k
 * columns for n = min(min_clusters, n_cluster)..n_cluster.
 * scores: k x w_cap column-major (NA where R has NA), *w = max n_cluster,
 * *n_pcs / *n_clusters = which.max(rowMeans(scores, na.rm=TRUE)) / which.max
 * of that row (1-based).  merge (2 x (n-1) ints, R merge matrix column-major)
 * and height (n-1) describe the tree of n_pcs (the dendrogram R re-computes
 * at R/TADpole.R:459-460); either may be NULL. */
void tp_sweep(const double *P, const int *n, const int *k,
              const int *min_clusters, const int *device, const int *w_cap,
              int *n_cluster, double *scores, int *w, int *n_pcs,
              int *n_clusters, int *merge, double *height, int *status);

/* ----------------------------------------------------------------- coniss */
/* rioja::chclust(dist(P), method="coniss") (R/TADpole.R:108): P n x ncols.
 * merge: (n-1) x 2 column-major hclust encoding (negative = singleton),
 * height (n-1): cumulative total within-cluster dispersion.
 * boundary (n-1, may be NULL): 1-based index of the first bin of the right
 * cluster of each merge (the boundary it removes). */
void tp_coniss(const double *P, const int *n, const int *ncols,
               const int *device, int *merge, double *height, int *boundary,
               int *status);

/* ------------------------------------------------------------------- dist */
/* stats::dist(P) euclidean, R's accumulation order: d has n(n-1)/2 entries,
 * lower triangle by columns (the R "dist" vector). */
void tp_dist(const double *P, const int *n, const int *ncols,
             const int *device, double *d, int *status);

/* --------------------------------------------------------------------- ch */
/* fpc::calinhara(P, labels, cn) (R/TADpole.R:119) for contiguous labels
 * 1..cn (as cutree gives on a constrained tree).  P n x k. */
void tp_ch(const double *P, const int *n, const int *k, const int *labels,
           const int *cn, const int *device, double *ch, int *status);

/* --------------------------------------------------------------- pipeline */
/* The whole seam: mask -> cor -> pca -> sweep -> tree of n_pcs.
 * M: n0 x n0 raw matrix (NA allowed unless TP_FLAG_CLEAN).
 * Outputs (caller-allocated):
 *   bad[n0], *n_good, good_idx[n0] (1-based original indices)
 *   *k = min(max_pcs, n_good), n_cluster[k_cap], scores[k_cap * w_cap]
 *   (k x w column-major, leading dimension *k), *w
 *   *n_pcs, *n_clusters (1-based), merge[2*(n0-1)] and height[n0-1] of the
 *   final tree (first n_good-1 rows valid), boundary[n0-1] (1-based, may be
 *   NULL), timings_ms[32] (may be NULL; when given, HIP events time:
 *   [0] mask+subset [1] cor [2] pca [3] sweep [4] total (ms), kernels
 *   [5] X'X GEMM [6] Xc'Xc GEMM (0 on the block Krylov path) [7] sum of
 *   the products with G (G*Q, or the Krylov steps' Xc'(Xc K_t)) [8] their
 *   count [9] CONISS [10] CH, and [11] PCA Chebyshev degrees [12] block
 *   [13] residual [14] n_good [15] k [16] Krylov steps (0: G formed)
 *   [17] Krylov dimension D [18] int8 slices of the exact X'X
 *   product (0: fp64 MFMA product) [19] int8 digit pairs of each Krylov
 *   product with C (0: fp64 MFMA products); [20..31] reserved, written 0). */
void tp_pipeline(const double *M, const int *n0, const int *max_pcs,
                 const int *min_clusters, const double *bad_frac,
                 const int *flags, const int *device, const int *k_cap,
                 const int *w_cap, int *bad, int *n_good, int *good_idx,
                 int *k, int *n_cluster, double *scores, int *w, int *n_pcs,
                 int *n_clusters, int *merge, double *height, int *boundary,
                 double *timings_ms, int *status);

/* Same, input already on the device (d_M, n0 x n0, may be overwritten when
 * TP_FLAG_CLEAN is not set) and work queued on `stream` (hipStream_t). */
void tp_pipeline_dev(const double *d_M, const int *n0, const int *max_pcs,
                     const int *min_clusters, const double *bad_frac,
                     const int *flags, const int *device, void *stream,
                     const int *k_cap, const int *w_cap, int *bad,
                     int *n_good, int *good_idx, int *k, int *n_cluster,
                     double *scores, int *w, int *n_pcs, int *n_clusters,
                     int *merge, double *height, int *boundary,
                     double *timings_ms, int *status);

/* ------------------------------------------------------------ tad coords */
/* The TAD start/end coordinates of several cut levels of the final tree at
 * once: R/TADpole.R:470-488 (cutree(dendro, kk) per significant level, the
 * labels placed on c(good, bad) order, rle runs -> rows (start, end)).
 * boundary[n-1]: as tp_pipeline returns it (first n_good-1 entries, n =
 * n_good), pos[n]: the 1-based coordinate of each kept bin in the full
 * matrix, levels[nlev]: each in 1..n.  out: sum(levels) rows of two ints
 * (start, end), row-major, level after level in `levels` order.  Host only
 * (R: .C("tp_level_coords", boundary, n, levels, nlev, pos, out = integer(2 *
 * sum(levels)), status = integer(1))). */
void tp_level_coords(const int *boundary, const int *n, const int *levels,
                     const int *nlev, const int *pos, int *out, int *status);

/* Device-resident stage entry points for tests and benches (d_* = device). */
void tp_sweep_dev(const double *d_P, const int *n, const int *k,
                  const int *min_clusters, const int *device, void *stream,
                  const int *w_cap, int *n_cluster, double *scores, int *w,
                  int *mrg_a_all, int *mrg_b_all, double *cost_all,
                  double *height_all, int *status);

#ifdef __cplusplus
}
#endif
#endif /* TADPOLE_HIP_H */
