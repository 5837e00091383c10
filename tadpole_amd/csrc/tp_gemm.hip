// fp64 GEMM on the CDNA4 matrix cores (v_mfma_f64_16x16x4_f64).
//
// Used for every O(N^3) / O(N^2 k) product of the path:
//   S = X'X            crossprod in sparse_cor        R/TADpole.R:96   (sym_upper)
//   G = Xc'Xc          normal matrix of prcomp's SVD  R/TADpole.R:453  (sym_upper)
//   Z = G Q            PCA subspace iteration
//   P = Xc V_k         prcomp scores x %*% rotation   R/TADpole.R:453
//
// Tile: 64x64 per workgroup, BK = 16, 256 threads = 4 waves in a 2x2 grid, each
// wave 32x32 = 2x2 MFMA tiles.  Operands are staged k-contiguous in LDS
// ([row][BK+1]: GPAD below), next tile prefetched into registers during the
// MFMAs.
// fp64 MFMA layout (cdna_hip_programming.md §3): A lane l = A[l&15][k=l>>4],
// B lane l = B[k=l>>4][l&15], D lane l reg r = D[(l>>4) + 4r][l&15].
#include "tp_common.cuh"
#include "tp_internal.h"

#include <algorithm>

namespace tp {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64, BN = 64, BK = 16;
// LDS row pad (doubles) of every operand tile here.  The fragment reads fuse
// into ds_read2_b64 (two k steps a read), which serves 16 contiguous lanes a
// cycle on banks (a/4) mod 32: rows fr = 0..15 of a 2-word span must land on
// distinct banks, i.e. a row stride of 2 mod 4 words.  A +2 pad (18 or 34
// doubles = 36 / 68 words) put two rows on each bank pair (rocprof: 40-45 % of
// the LDS cycles of k_gemm_f64 / _panel were conflict cycles); +1 (17 / 33
// doubles) is conflict-free for those reads and for the i-contiguous A stores.
#ifndef TP_GEMM_PAD
#define TP_GEMM_PAD 1
#endif
constexpr int GPAD = TP_GEMM_PAD;

// KB = k depth of one LDS stage (16 or 32): per thread KB/4 elements of each
// operand; rows stored k-contiguous with a GPAD pad (conflict-free fragment reads)
template <bool TA, int KB>
__device__ __forceinline__ void load_a(double (&ra)[KB / 4], const double *A, int lda, int M, int K, int i0, int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < KB / 4; ++p) {
        int idx = t + 256 * p;
        int row, kk;
        if (TA) { row = idx / KB; kk = idx % KB; }   // k contiguous in memory
        else    { kk = idx >> 6; row = idx & 63; }   // i contiguous in memory
        int i = i0 + row, k = k0 + kk;
        ra[p] = (i < M && k < K) ? (TA ? A[(size_t)k + (size_t)i * lda] : A[(size_t)i + (size_t)k * lda]) : 0.0;
    }
}
template <bool TA, int KB>
__device__ __forceinline__ void store_a(double (*As)[KB + GPAD], const double (&ra)[KB / 4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < KB / 4; ++p) {
        int idx = t + 256 * p;
        int row, kk;
        if (TA) { row = idx / KB; kk = idx % KB; }
        else    { kk = idx >> 6; row = idx & 63; }
        As[row][kk] = ra[p];
    }
}
template <int KB>
__device__ __forceinline__ void load_b(double (&rb)[KB / 4], const double *B, int ldb, int N, int K, int j0, int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < KB / 4; ++p) {
        int idx = t + 256 * p;
        int col = idx / KB, kk = idx % KB;
        int j = j0 + col, k = k0 + kk;
        rb[p] = (j < N && k < K) ? B[(size_t)k + (size_t)j * ldb] : 0.0;
    }
}
template <int KB>
__device__ __forceinline__ void store_b(double (*Bs)[KB + GPAD], const double (&rb)[KB / 4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < KB / 4; ++p) {
        int idx = t + 256 * p;
        Bs[idx / KB][idx % KB] = rb[p];
    }
}

// TAG only names the symbol (1 = the PCA's G Y products), so profiles can
// attribute launches; the code is the same.
template <bool TA, int KB, int TAG = 0>
__global__ void __launch_bounds__(256) k_gemm_f64(int M, int N, int K, const double *__restrict__ A, int lda,
                                                  const double *__restrict__ B, int ldb, double *C,
                                                  int ldc, int store_t, int sym, int tcol0, int kchunk,
                                                  size_t part_stride, int g_xcd_order,
                                                  const double *C0 = nullptr) {   // C0 may alias C (no restrict)
    __shared__ double As[2][BM][KB + GPAD];
    __shared__ double Bs[2][BN][KB + GPAD];
    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (each
    // with its own L2), so the logical tile index Lg makes consecutive
    // workgroups of one XCD neighbours -- the tiles of one A row panel (all
    // column tiles, same k chunk) run together and share it in that L2.
    const int total = (int)gridDim.x;   // tiles x k chunks
    const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
    const int Lg = g_xcd_order ? xcd * (total >> 3) + min(xcd, total & 7) + slot : (int)blockIdx.x;
    int bm, bn, z;
    if (sym) {  // linear id -> upper tile (bm <= bn), column by column from tile column tcol0
        const int nt = total / ((K + kchunk - 1) / kchunk);   // tiles (total / k chunks)
        int id = Lg % nt;
        z = Lg / nt;
        bn = tcol0;
        while (id > bn) { id -= bn + 1; ++bn; }
        bm = id;
    } else {
        const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
        bn = Lg % tn;
        bm = (Lg / tn) % tm;
        z = Lg / (tn * tm);
    }
    const int i0 = bm * BM, j0 = bn * BN;
    const int kbeg = z * kchunk;
    const int kend = min(K, kbeg + kchunk);
    C += part_stride * z;

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
    const int fr = lane & 15, fk = lane >> 4;

    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};

    double ra[KB / 4], rb[KB / 4];
    int buf = 0;
    if (kbeg < kend) {
        load_a<TA, KB>(ra, A, lda, M, kend, i0, kbeg);
        load_b<KB>(rb, B, ldb, N, kend, j0, kbeg);
        store_a<TA, KB>(As[0], ra);
        store_b<KB>(Bs[0], rb);
    }
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += KB) {
        const bool more = k0 + KB < kend;
        if (more) {
            load_a<TA, KB>(ra, A, lda, M, kend, i0, k0 + KB);
            load_b<KB>(rb, B, ldb, N, kend, j0, k0 + KB);
        }
#pragma unroll
        for (int kk = 0; kk < KB; kk += 4) {
            double af[2], bf[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                af[t] = As[buf][wm + t * 16 + fr][kk + fk];
                bf[t] = Bs[buf][wn + t * 16 + fr][kk + fk];
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        if (more) {
            store_a<TA, KB>(As[buf ^ 1], ra);
            store_b<KB>(Bs[buf ^ 1], rb);
        }
        __syncthreads();
        buf ^= 1;
    }
    // epilogue
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int i = i0 + wm + a * 16 + fk + 4 * r;
                int j = j0 + wn + b * 16 + fr;
                if (i >= M || j >= N) continue;
                double v = acc[a][b][r];
                if (sym) {
                    if (i > j) continue;
                    C[(size_t)i + (size_t)j * ldc] = v;
                    C[(size_t)j + (size_t)i * ldc] = v;
                } else if (store_t) {
                    C[(size_t)j + (size_t)i * ldc] = v;
                } else {
                    const size_t ci = (size_t)i + (size_t)j * ldc;
                    C[ci] = C0 ? C0[ci] - v : v;   // C0: C = C0 - A'B (one rounding, as a separate subtraction)
                }
            }
}
thread_local int g_gemm_kb = 16;   // k depth of the 64 x 64 kernel's LDS stages (16 / 32; same bits; 32 measured no faster)

// ---------------------------------------------------------------------------
// Large products: 128 x 128 output tile per 256-thread workgroup, each wave a
// 64 x 64 quadrant (4 x 4 MFMA tiles, 64 accumulators of f64), BK = 16 staged
// k-contiguous in LDS (+2 pad) and double-buffered, next block prefetched into
// registers during the MFMAs.  Half the L2 -> LDS traffic per flop of the
// 64 x 64 kernel and 4x the MFMAs per LDS fragment read.  Every output element
// sees the same k order (blocks of 16, steps of 4) as k_gemm_f64, so the two
// kernels give identical bits and can be mixed freely (also across shards).
constexpr int GB = 128, GBK = 16, GLD = GBK + GPAD;
template <bool TA>
__global__ void __launch_bounds__(256, 2) k_gemm_f64_big(int M, int N, int K, const double *__restrict__ A, int lda,
                                                         const double *__restrict__ B, int ldb,
                                                         double *__restrict__ C, int ldc, int store_t, int sym,
                                                         int tcol0) {
    __shared__ double As[2][GB][GLD];
    __shared__ double Bs[2][GB][GLD];
    int bm, bn;
    if (sym) {
        int id = blockIdx.x;
        bn = tcol0;
        while (id > bn) { id -= bn + 1; ++bn; }
        bm = id;
    } else {
        const int tm = (M + GB - 1) / GB;
        bm = blockIdx.x % tm;
        bn = blockIdx.x / tm;
    }
    const int i0 = bm * GB, j0 = bn * GB;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = (w & 1) * 64, wn = (w >> 1) * 64;
    const int fr = lane & 15, fk = lane >> 4;
    d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
    double ra[8], rb[8];
    auto load = [&](int k0) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int idx = t + 256 * p;
            int row, kk;
            if (TA) { row = idx >> 4; kk = idx & 15; }
            else    { kk = idx >> 7; row = idx & 127; }
            const int i = i0 + row, k = k0 + kk;
            ra[p] = (i < M && k < K) ? (TA ? A[(size_t)k + (size_t)i * lda] : A[(size_t)i + (size_t)k * lda]) : 0.0;
            const int col = idx >> 4, kb = idx & 15;
            const int j = j0 + col, k2 = k0 + kb;
            rb[p] = (j < N && k2 < K) ? B[(size_t)k2 + (size_t)j * ldb] : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int idx = t + 256 * p;
            int row, kk;
            if (TA) { row = idx >> 4; kk = idx & 15; }
            else    { kk = idx >> 7; row = idx & 127; }
            As[buf][row][kk] = ra[p];
            Bs[buf][idx >> 4][idx & 15] = rb[p];
        }
    };
    load(0);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int k0 = 0; k0 < K; k0 += GBK) {
        const bool more = k0 + GBK < K;
        if (more) load(k0 + GBK);
#pragma unroll
        for (int kk = 0; kk < GBK; kk += 4) {
            double af[4], bf[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                af[u] = As[buf][wm + u * 16 + fr][kk + fk];
                bf[u] = Bs[buf][wn + u * 16 + fr][kk + fk];
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wm + a * 16 + fk + 4 * r;
                const int j = j0 + wn + b * 16 + fr;
                if (i >= M || j >= N) continue;
                const double v = acc[a][b][r];
                if (sym) {
                    if (i > j) continue;
                    C[(size_t)i + (size_t)j * ldc] = v;
                    C[(size_t)j + (size_t)i * ldc] = v;
                } else if (store_t) {
                    C[(size_t)j + (size_t)i * ldc] = v;
                } else {
                    C[(size_t)i + (size_t)j * ldc] = v;
                }
            }
}

// ---------------------------------------------------------------------------
// Tall-skinny products (Z = G Q, P = Xc V, Q X: M ~ n, N = b <= 256): a
// 32 x 64 output tile per 256-thread workgroup, the 4 waves in a 2 x 2 grid,
// each 16 x 32 (two MFMA tiles), full K in every workgroup.  At n = 2000,
// b = 256 that is 62 x 4 = 248 workgroups -- one per CU -- where the 64 x 64
// kernel has 124 tiles.  Used for short K (the Ritz rotation Q X, K = b),
// where the 64 x 64 policy takes no split either.  BK = 32 per LDS stage (one barrier per 16 MFMAs a wave).  The
// k order of every output element is that of k_gemm_f64 (steps of 4 within
// blocks of 16; a 32-block is two 16-blocks back to back), so all three
// kernels give identical bits.
constexpr int PM = 32, PN = 64, PK = 32, PLD = PK + GPAD, PSETS = 3;
// Global loads run PSETS - 1 stages ahead of the MFMAs (register sets rotate):
// a stage is only ~1k MFMA cycles a wave, less than an HBM/MALL round trip.
template <bool TA>
__global__ void __launch_bounds__(256) k_gemm_f64_panel(int M, int N, int K, const double *__restrict__ A, int lda,
                                                        const double *__restrict__ B, int ldb,
                                                        double *C, int ldc, int store_t,
                                                        const double *C0) {   // C0 may alias C (no restrict)
    __shared__ double As[2][PM][PLD];
    __shared__ double Bs[2][PN][PLD];
    const int tm = (M + PM - 1) / PM;
    const int bm = blockIdx.x % tm, bn = blockIdx.x / tm;
    const int i0 = bm * PM, j0 = bn * PN;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = (w & 1) * 16, wn = (w >> 1) * 32;
    const int fr = lane & 15, fk = lane >> 4;
    d4 acc[2];
    acc[0] = (d4){0.0, 0.0, 0.0, 0.0};
    acc[1] = (d4){0.0, 0.0, 0.0, 0.0};
    // per stage: A tile PM x PK (4 per thread) + B tile PN x PK (8 per thread)
    double r[PSETS][12];
    auto load = [&](double (&x)[12], int k0) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int idx = t + 256 * p;
            int row, kk;
            if (TA) { row = idx >> 5; kk = idx & 31; }
            else    { kk = idx >> 5; row = idx & 31; }
            const int i = i0 + row, k = k0 + kk;
            x[p] = (i < M && k < K) ? (TA ? A[(size_t)k + (size_t)i * lda] : A[(size_t)i + (size_t)k * lda]) : 0.0;
        }
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int idx = t + 256 * p;
            const int col = idx >> 5, kb = idx & 31;
            const int j = j0 + col, k = k0 + kb;
            x[4 + p] = (j < N && k < K) ? B[(size_t)k + (size_t)j * ldb] : 0.0;
        }
    };
    auto store = [&](const double (&x)[12], int buf) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int idx = t + 256 * p;
            int row, kk;
            if (TA) { row = idx >> 5; kk = idx & 31; }
            else    { kk = idx >> 5; row = idx & 31; }
            As[buf][row][kk] = x[p];
        }
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int idx = t + 256 * p;
            Bs[buf][idx >> 5][idx & 31] = x[4 + p];
        }
    };
    const int S = (K + PK - 1) / PK;
#pragma unroll
    for (int u = 0; u < PSETS - 1; ++u)
        if (u < S) load(r[u], u * PK);
    if (S > 0) store(r[0], 0);
    __syncthreads();
    for (int s0 = 0; s0 < S; s0 += PSETS) {
#pragma unroll
        for (int u = 0; u < PSETS; ++u) {
            const int st = s0 + u;
            if (st >= S) break;
            // stage st is in LDS buffer st & 1; r[(u+1)%PSETS] holds stage st+1;
            // r[(u+PSETS-1)%PSETS] (stage st-1, already in LDS) takes stage st+PSETS-1
            if (st + PSETS - 1 < S) load(r[(u + PSETS - 1) % PSETS], (st + PSETS - 1) * PK);
            const int buf = st & 1;
#pragma unroll
            for (int kk = 0; kk < PK; kk += 4) {
                const double af = As[buf][wm + fr][kk + fk];
                const double b0 = Bs[buf][wn + fr][kk + fk];
                const double b1 = Bs[buf][wn + 16 + fr][kk + fk];
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, b0, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, b1, acc[1], 0, 0, 0);
            }
            if (st + 1 < S) store(r[(u + 1) % PSETS], buf ^ 1);
            __syncthreads();
        }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = i0 + wm + fk + 4 * q;
            const int j = j0 + wn + b * 16 + fr;
            if (i >= M || j >= N) continue;
            if (store_t) {
                C[(size_t)j + (size_t)i * ldc] = acc[b][q];
            } else {
                const size_t ci = (size_t)i + (size_t)j * ldc;
                C[ci] = C0 ? C0[ci] - acc[b][q] : acc[b][q];
            }
        }
}
thread_local int g_gemm_panel = 1;   // 0: tall-skinny products take the split-K 64 x 64 path (A/B tests)

// ---------------------------------------------------------------------------
// Long-K tall-skinny products C = A'B with A k-contiguous (the PCA's Xc K_t,
// Xc'(Xc K_t) and the scores Xc V: M = n, N = 64..256, K = n): a 128 x 64
// output tile per 256-thread workgroup, wave w owning rows 32w..32w+31 of it
// across all 64 columns -- 2 x 4 MFMA tiles, 8 accumulators, 6 LDS fragment
// reads per 8 MFMAs (the 64 x 64 kernel: 4 per 4).  BK = 16 double-buffered
// in LDS (+2 pad, 55 KB: two workgroups a CU), next stage prefetched into
// registers during the MFMAs, split-K chunks for a grid of ~2 workgroups a
// CU.  Same k order as k_gemm_f64 (steps of 4 within blocks of 16): for the
// same chunking the bits are those of the 64 x 64 kernel.
// TN = 32 (the C-Krylov blocks): a 128 x 32 tile, each wave 32 x 32 (2 x 2
// accumulators); same k order, so the bits of a column do not depend on TN.
constexpr int TSM = 128, TSN = 64, TSK = 16, TSLD = TSK + GPAD;
template <int TAG, int TN = TSN>
__global__ void __launch_bounds__(256, 2) k_gemm_ts(int M, int N, int K, const double *__restrict__ A, int lda,
                                                    const double *__restrict__ B, int ldb, double *__restrict__ C,
                                                    int ldc, int store_t, int kchunk, size_t part_stride) {
    constexpr int NB = TN / 16;   // accumulator columns per wave
    __shared__ double As[2][TSM][TSLD];
    __shared__ double Bs[2][TN][TSLD];
    const int tm = (M + TSM - 1) / TSM, tn = (N + TN - 1) / TN;
    // XCD-aware order (see k_gemm_f64): the column tiles of one row panel and
    // its neighbours run on one XCD and share the A panel in its L2
    const int total = (int)gridDim.x;
    const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
    const int Lg = xcd * (total >> 3) + min(xcd, total & 7) + slot;
    const int bn = Lg % tn, bm = (Lg / tn) % tm, z = Lg / (tn * tm);
    const int i0 = bm * TSM, j0 = bn * TN;
    const int kbeg = z * kchunk, kend = min(K, kbeg + kchunk);
    C += part_stride * z;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = 32 * w;
    const int fr = lane & 15, fk = lane >> 4;
    d4 acc[2][NB];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
    double ra[8], rb[NB];
    // thread t loads k = t & 15 of rows (t >> 4) + 16 p: 16 lanes read 128
    // contiguous bytes of one row
    const int lk = t & 15, lr = t >> 4;
    auto load = [&](int k0) {
        const int k = k0 + lk;
        const bool kin = k < kend;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int i = i0 + lr + 16 * p;
            ra[p] = (kin && i < M) ? A[(size_t)k + (size_t)i * lda] : 0.0;
        }
#pragma unroll
        for (int p = 0; p < NB; ++p) {
            const int j = j0 + lr + 16 * p;
            rb[p] = (kin && j < N) ? B[(size_t)k + (size_t)j * ldb] : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int p = 0; p < 8; ++p) As[buf][lr + 16 * p][lk] = ra[p];
#pragma unroll
        for (int p = 0; p < NB; ++p) Bs[buf][lr + 16 * p][lk] = rb[p];
    };
    auto mfma_stage = [&](int buf) {
#pragma unroll
        for (int kk = 0; kk < TSK; kk += 4) {
            double af[2], bf[NB];
#pragma unroll
            for (int a = 0; a < 2; ++a) af[a] = As[buf][wm + 16 * a + fr][kk + fk];
#pragma unroll
            for (int b = 0; b < NB; ++b) bf[b] = Bs[buf][16 * b + fr][kk + fk];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
    };
    if (kbeg < kend) {
        load(kbeg);
        store(0);
    }
    __syncthreads();
    int buf = 0;
    for (int k0 = kbeg; k0 < kend; k0 += TSK) {
        const bool more = k0 + TSK < kend;
        if (more) load(k0 + TSK);
        mfma_stage(buf);
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wm + 16 * a + fk + 4 * r;
                const int j = j0 + 16 * b + fr;
                if (i >= M || j >= N) continue;
                if (store_t) C[(size_t)j + (size_t)i * ldc] = acc[a][b][r];
                else C[(size_t)i + (size_t)j * ldc] = acc[a][b][r];
            }
}

// Fixed-order split-K reduction: C = sum_{z=0..S-1} part[z] (column-major M x N),
// z ascending; loads issued 8 at a time (S is a runtime count: one dependent
// load per partial otherwise).
template <int TAG = 0>
__global__ void __launch_bounds__(256) k_splitk_reduce(const double *part, size_t stride, int S, int M, int N,
                                                       double *C, int ldc, int store_t, const double *C0) {
    size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)M * N) return;
    int i = (int)(idx % M), j = (int)(idx / M);
    double v = part[idx];
    int z = 1;
    for (; z + 8 <= S; z += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = part[idx + (size_t)(z + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) v = v + t[u];
    }
    for (; z < S; ++z) v = v + part[idx + (size_t)z * stride];
    if (store_t) {
        C[(size_t)j + (size_t)i * ldc] = v;
    } else {
        const size_t ci = (size_t)i + (size_t)j * ldc;
        C[ci] = C0 ? C0[ci] - v : v;
    }
}

// The same fixed-order reduction with the rank-1 epilogue of GemmArgs::r1_*:
// rows [0, rows) of C (ldc) = sum(i, j) - u_i sum(vrow, j), where sum(vrow, j)
// is the value the plain reduction would store for that row (same order)
template <int TAG = 0>
__global__ void __launch_bounds__(256) k_splitk_reduce_r1(const double *part, size_t stride, int S, int M, int N,
                                                          int rows, int vrow, const double *u, double *C, int ldc) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)rows * N) return;
    const int i = (int)(idx % rows), j = (int)(idx / rows);
    auto red = [&](size_t e) {
        double v = part[e];
        int z = 1;
        for (; z + 8 <= S; z += 8) {
            double t[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) t[q] = part[e + (size_t)(z + q) * stride];
#pragma unroll
            for (int q = 0; q < 8; ++q) v = v + t[q];
        }
        for (; z < S; ++z) v = v + part[e + (size_t)z * stride];
        return v;
    };
    const double v = red((size_t)i + (size_t)j * M);
    const double w = red((size_t)vrow + (size_t)j * M);
    C[(size_t)i + (size_t)j * ldc] = v - (u ? u[i] * w : w);
}

// Out (rows x N, ld rows) = T(i, j) - u_i T(vrow, j), T(i, j) = T[i rs + j cs]:
// the rank-1 epilogue on a stored product (a gathered row-major one in the
// sharded path, rs = N, cs = 1; a column-major one, rs = 1, cs = M); same
// arithmetic as k_splitk_reduce_r1
__global__ void __launch_bounds__(256) k_r1_apply(const double *T, size_t rs, size_t cs, int N, int rows, int vrow,
                                                  const double *u, double *Out) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)rows * N) return;
    const int i = (int)(idx % rows), j = (int)(idx / rows);
    const double v = T[(size_t)i * rs + (size_t)j * cs], w = T[(size_t)vrow * rs + (size_t)j * cs];
    Out[idx] = v - (u ? u[i] * w : w);
}
void launch_r1_apply(const double *T, size_t rs, size_t cs, int N, int rows, int vrow, const double *u, double *Out,
                     hipStream_t s) {
    const size_t tot = (size_t)rows * N;
    hipLaunchKernelGGL(k_r1_apply, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, T, rs, cs, N, rows, vrow, u,
                       Out);
    TP_HIP(hipGetLastError());
}

// The two reductions above for partials made elsewhere (the int8-digit
// products, tp_prod_i8.hip): the same kernels and summation order
void launch_splitk_reduce_r1(const double *part, size_t stride, int S, int M, int N, int rows, int vrow,
                             const double *u, double *C, int ldc, hipStream_t s) {
    const size_t tot = (size_t)rows * N;
    hipLaunchKernelGGL(k_splitk_reduce_r1<1>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, part, stride, S, M,
                       N, rows, vrow, u, C, ldc);
    TP_HIP(hipGetLastError());
}
void launch_splitk_reduce(const double *part, size_t stride, int S, int M, int N, double *C, int ldc, int store_t,
                          hipStream_t s) {
    const size_t tot = (size_t)M * N;
    hipLaunchKernelGGL(k_splitk_reduce<1>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, part, stride, S, M, N,
                       C, ldc, store_t, (const double *)nullptr);
    TP_HIP(hipGetLastError());
}

// The fixed-order reduction with the affine epilogue of GemmArgs::affine:
// C = a sum + b Y [+ c Z] (the Chebyshev step; Y, Z share C's layout)
__global__ void __launch_bounds__(256) k_splitk_reduce_af(const double *part, size_t stride, int S, int M, int N,
                                                          double *C, int ldc, double a, double b, double c,
                                                          const double *Y, const double *Z) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)M * N) return;
    const int i = (int)(idx % M), j = (int)(idx / M);
    double v = part[idx];
    int z = 1;
    for (; z + 8 <= S; z += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = part[idx + (size_t)(z + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) v = v + t[u];
    }
    for (; z < S; ++z) v = v + part[idx + (size_t)z * stride];
    const size_t ci = (size_t)i + (size_t)j * ldc;
    double w = a * v + b * Y[ci];
    if (Z) w = w + c * Z[ci];
    C[ci] = w;
}
// in place on a stored product (S = 1): same arithmetic
__global__ void __launch_bounds__(256) k_affine_inplace(int M, int N, double *C, int ldc, double a, double b, double c,
                                                        const double *Y, const double *Z) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)M * N) return;
    const size_t ci = (size_t)(idx % M) + (size_t)(idx / M) * ldc;
    double w = a * C[ci] + b * Y[ci];
    if (Z) w = w + c * Z[ci];
    C[ci] = w;
}

// Many partials of a small output (Gram matrices of CholQR, K'W of the Krylov
// re-orthogonalisation): 64 outputs per workgroup, the partials of each split
// over the 4 waves (wave w: z = w, w + 4, ...: ascending), the four group sums
// combined in wave order.  Fixed order for a given S.
__global__ void __launch_bounds__(256) k_splitk_reduce4(const double *part, size_t stride, int S, int M, int N,
                                                        double *C, int ldc, int store_t, const double *C0) {
    __shared__ double red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t idx = (size_t)blockIdx.x * 64 + lane;
    const bool live = idx < (size_t)M * N;
    const size_t src = live ? idx : 0;
    double v = 0.0;
    int z = w;
    for (; z + 28 < S; z += 32) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = part[src + (size_t)(z + 4 * u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) v = v + t[u];
    }
    for (; z < S; z += 4) v = v + part[src + (size_t)z * stride];
    red[w][lane] = v;
    __syncthreads();
    if (w == 0 && live) {
        const double r = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
        const int i = (int)(idx % M), j = (int)(idx / M);
        if (store_t) {
            C[(size_t)j + (size_t)i * ldc] = r;
        } else {
            const size_t ci = (size_t)i + (size_t)j * ldc;
            C[ci] = C0 ? C0[ci] - r : r;
        }
    }
}

// Split-K plan of the 64 x 64 kernel.
static void split_plan(const GemmArgs &g, long nblk, int &S, int &kchunk) {
    S = g.splitk;
    if (S < 1) {
        // auto: fill the 256 CUs when the output has few tiles and K is long
        S = 1;
        if (nblk < 192 && g.K >= 512) S = (int)std::min<long>(8, std::max<long>(1, (384 + nblk - 1) / nblk));
        S = std::min(S, std::max(1, g.K / 128));
        if (cfg_gemm_splitk && nblk <= 64 && g.K >= 512) {
            // few output tiles, long K (Gram matrices Z'Z, the Krylov K'W, T Y):
            // one k-chunk is otherwise a long chain of dependent stages on a
            // quarter of the chip.  ~1024 workgroups, chunks of >= 8 stages
            // (>= 4 for a single tile), partials bounded by ~1/64 of the
            // operand bytes the product streams.
            const int kmin = nblk <= 4 ? 64 : 128;
            long s2 = std::min<long>(g.K / kmin, (1024 + nblk - 1) / nblk);
            const double outb = 8.0 * g.M * g.N;
            const double budget = std::max(16.0e6, 8.0 * g.M * (double)g.N * g.K / 64.0);
            s2 = std::min<long>(s2, (long)(budget / outb));
            s2 = std::min<long>(s2, 128);
            if (s2 > S) S = (int)s2;
        }
    }
    kchunk = ((g.K + S - 1) / S + BK - 1) / BK * BK;   // multiple of 16 for either stage depth
    if (kchunk < BK) kchunk = BK;
    S = (g.K + kchunk - 1) / kchunk;
    if (S < 1) S = 1;
}

void gemm_f64(const GemmArgs &g, DevBuf &work, hipStream_t s) {
    if (g.M <= 0 || g.N <= 0) return;
    if (g.sub_from && (g.sym_upper || g.store_t || g.rows))
        fail(TP_ERR_ARG, "gemm_f64: C = C0 - A'B only for plain column-major outputs");
    if (g.r1_vrow >= 0 && (g.store_t || !g.rows || g.r1_rows > g.M || g.r1_vrow >= g.M ||
                           !(rows_ts(g.K, g.N) && g.trans_a && !g.sym_upper && g.splitk <= 1)))
        fail(TP_ERR_ARG, "gemm_f64: the rank-1 epilogue is for plain long-K row-shardable products");
    if (g.sym_upper && g.M != g.N) fail(TP_ERR_ARG, "sym_upper GEMM needs a square output");
    if (g.affine && (g.sym_upper || g.store_t || g.sub_from || g.rows || g.r1_vrow >= 0 || !g.af_y ||
                     g.af_y == g.C || g.af_z == g.C))
        fail(TP_ERR_ARG, "gemm_f64: the affine epilogue is for plain column-major products into a separate C");
    const int tm = (g.M + BM - 1) / BM, tn = (g.N + BN - 1) / BN;
    // sym_upper: upper tiles of tile columns [tc0, tc1) (a column shard)
    const int tc0 = g.sym_upper ? std::max(0, g.tcol0) : 0;
    const int tc1 = g.sym_upper ? (g.tcol1 < 0 ? tn : std::min(tn, g.tcol1)) : 0;
    if (g.sym_upper && tc1 <= tc0) return;
    long nblk = g.sym_upper ? (long)tc1 * (tc1 + 1) / 2 - (long)tc0 * (tc0 + 1) / 2 : (long)tm * tn;
    // long-K tall-skinny A'B (Xc products of the PCA): 128 x 64 tiles, before
    // any other choice -- a row shard must take the same kernel and k chunks
    if (g.rows && rows_ts(g.K, g.N) && g.trans_a && !g.sym_upper && (g.splitk <= 0 || g.splitk == 1)) {
        const int tnw = g.N <= 32 ? 32 : TSN;   // tile width: 32 for the C-Krylov blocks
        const long tiles = (long)((g.M + TSM - 1) / TSM) * ((g.N + tnw - 1) / tnw);
        // the k chunks depend on K alone (not on M): a row shard of the
        // product (tp_shard.hip) then sums every element in the same order
        int S = 1;
        if (g.splitk <= 0) S = std::max(1, std::min(tnw == 32 ? cfg_gemm_ts32 : cfg_gemm_ts, g.K / 256));
        int kchunk = ((g.K + S - 1) / S + TSK - 1) / TSK * TSK;
        S = (g.K + kchunk - 1) / kchunk;
        double *out = g.C;
        int ldo = g.ldc, st = g.store_t;
        size_t pstride = 0;
        const bool r1 = g.r1_vrow >= 0;
        if (S > 1 || r1) {   // the rank-1 epilogue runs in the reduction (S = 1: a one-partial reduction)
            pstride = (size_t)g.M * g.N;
            out = work.as<double>(pstride * S);
            ldo = g.M;
            st = 0;
        }
        const dim3 grid((unsigned)(tiles * S));
        if (tnw == 32)
            hipLaunchKernelGGL((k_gemm_ts<1, 32>), grid, dim3(256), 0, s, g.M, g.N, g.K, g.A, g.lda, g.B, g.ldb, out,
                               ldo, st, kchunk, pstride);
        else if (g.tag == 1)
            hipLaunchKernelGGL(k_gemm_ts<1>, grid, dim3(256), 0, s, g.M, g.N, g.K, g.A, g.lda, g.B, g.ldb, out, ldo, st,
                               kchunk, pstride);
        else
            hipLaunchKernelGGL(k_gemm_ts<0>, grid, dim3(256), 0, s, g.M, g.N, g.K, g.A, g.lda, g.B, g.ldb, out, ldo, st,
                               kchunk, pstride);
        TP_HIP(hipGetLastError());
        if (r1) {
            const size_t tot = (size_t)g.r1_rows * g.N;
            const dim3 rg((unsigned)((tot + 255) / 256));
            if (g.tag == 1)
                hipLaunchKernelGGL(k_splitk_reduce_r1<1>, rg, dim3(256), 0, s, out, pstride, S, g.M, g.N, g.r1_rows,
                                   g.r1_vrow, g.r1_u, g.C, g.ldc);
            else
                hipLaunchKernelGGL(k_splitk_reduce_r1<0>, rg, dim3(256), 0, s, out, pstride, S, g.M, g.N, g.r1_rows,
                                   g.r1_vrow, g.r1_u, g.C, g.ldc);
            TP_HIP(hipGetLastError());
        } else if (S > 1) {
            const size_t tot = (size_t)g.M * g.N;
            const dim3 rg((unsigned)((tot + 255) / 256));
            if (g.tag == 1)
                hipLaunchKernelGGL(k_splitk_reduce<1>, rg, dim3(256), 0, s, out, pstride, S, g.M, g.N, g.C, g.ldc,
                                   (int)g.store_t, (const double *)nullptr);
            else
                hipLaunchKernelGGL(k_splitk_reduce<0>, rg, dim3(256), 0, s, out, pstride, S, g.M, g.N, g.C, g.ldc,
                                   (int)g.store_t, (const double *)nullptr);
            TP_HIP(hipGetLastError());
        }
        return;
    }
    // 128 x 128 kernel: no split-K, enough tiles to fill the chip, and (sym) a
    // tile-column range in 128-column units (g.big_cols)
    {
        const int tm2 = (g.M + 127) / 128, tn2 = (g.N + 127) / 128;
        const int c0 = g.sym_upper ? std::max(0, g.tcol0) : 0;
        const int c1 = g.sym_upper ? (g.tcol1 < 0 ? tn2 : std::min(tn2, g.tcol1)) : 0;
        const long nb2 = g.sym_upper ? (long)c1 * (c1 + 1) / 2 - (long)c0 * (c0 + 1) / 2 : (long)tm2 * tn2;
        // non-symmetric: >= 240 tiles of 128 means >= 960 of 64, where the auto
        // split-K policy below picks no split either (same bits)
        const bool want = g.sym_upper ? g.big_cols : (g.splitk <= 1 && nb2 >= 240 && g.K >= 512);
        if (want && !g.sub_from && !g.affine) {
            if (g.sym_upper && c1 <= c0) return;
            if (g.trans_a)
                hipLaunchKernelGGL(k_gemm_f64_big<true>, dim3((unsigned)nb2), dim3(256), 0, s, g.M, g.N, g.K, g.A,
                                   g.lda, g.B, g.ldb, g.C, g.ldc, (int)g.store_t, (int)g.sym_upper, c0);
            else
                hipLaunchKernelGGL(k_gemm_f64_big<false>, dim3((unsigned)nb2), dim3(256), 0, s, g.M, g.N, g.K, g.A,
                                   g.lda, g.B, g.ldb, g.C, g.ldc, (int)g.store_t, (int)g.sym_upper, c0);
            TP_HIP(hipGetLastError());
            return;
        }
    }
    // tall-skinny, not symmetric: 32 x 64 tiles, full K, when the 64 x 64 grid
    // is too small to fill the chip without a split (or a split is allowed)
    // (K < 512 only: with full K a wave per SIMD issues an f64 MFMA every ~150
    // cycles at best -- tools/mfma_rate.hip -- and the split-K 64 x 64 grid
    // with two workgroups a CU is faster)
    if (g_gemm_panel && !g.sym_upper && !g.affine && g.splitk <= 1 && nblk < 192 && g.N <= 512 && g.K < 512) {
        const long np = (long)((g.M + PM - 1) / PM) * ((g.N + PN - 1) / PN);
        if (np >= 128) {
            if (g.trans_a)
                hipLaunchKernelGGL(k_gemm_f64_panel<true>, dim3((unsigned)np), dim3(256), 0, s, g.M, g.N, g.K, g.A,
                                   g.lda, g.B, g.ldb, g.C, g.ldc, (int)g.store_t, g.sub_from);
            else
                hipLaunchKernelGGL(k_gemm_f64_panel<false>, dim3((unsigned)np), dim3(256), 0, s, g.M, g.N, g.K, g.A,
                                   g.lda, g.B, g.ldb, g.C, g.ldc, (int)g.store_t, g.sub_from);
            TP_HIP(hipGetLastError());
            return;
        }
    }
    int S = 0, kchunk = 0;
    split_plan(g, nblk, S, kchunk);
    // 1-D grid of tiles x k chunks (the kernel maps it XCD-aware)
    dim3 grid((unsigned)(nblk * S), 1, 1);
    double *out = g.C;
    int ldo = g.ldc;
    int st = g.store_t;
    size_t pstride = 0;
    if (S > 1) {
        pstride = (size_t)g.M * g.N;
        out = work.as<double>(pstride * S);
        ldo = g.M;
        st = 0;
    }
    if (g_gemm_kb == 32) {
        if (g.trans_a)
            hipLaunchKernelGGL((k_gemm_f64<true, 32>), grid, dim3(256), 0, s, g.M, g.N, g.K, g.A, g.lda, g.B, g.ldb,
                               out, ldo, st, (int)g.sym_upper, tc0, kchunk, pstride, cfg_gemm_xcd, S == 1 ? g.sub_from : nullptr);
        else
            hipLaunchKernelGGL((k_gemm_f64<false, 32>), grid, dim3(256), 0, s, g.M, g.N, g.K, g.A, g.lda, g.B, g.ldb,
                               out, ldo, st, (int)g.sym_upper, tc0, kchunk, pstride, cfg_gemm_xcd, S == 1 ? g.sub_from : nullptr);
    } else if (g.trans_a && g.tag == 1) {
        hipLaunchKernelGGL((k_gemm_f64<true, 16, 1>), grid, dim3(256), 0, s, g.M, g.N, g.K, g.A, g.lda, g.B, g.ldb,
                           out, ldo, st, (int)g.sym_upper, tc0, kchunk, pstride, cfg_gemm_xcd, S == 1 ? g.sub_from : nullptr);
    } else if (g.trans_a) {
        hipLaunchKernelGGL((k_gemm_f64<true, 16>), grid, dim3(256), 0, s, g.M, g.N, g.K, g.A, g.lda, g.B, g.ldb,
                           out, ldo, st, (int)g.sym_upper, tc0, kchunk, pstride, cfg_gemm_xcd, S == 1 ? g.sub_from : nullptr);
    } else {
        hipLaunchKernelGGL((k_gemm_f64<false, 16>), grid, dim3(256), 0, s, g.M, g.N, g.K, g.A, g.lda, g.B, g.ldb,
                           out, ldo, st, (int)g.sym_upper, tc0, kchunk, pstride, cfg_gemm_xcd, S == 1 ? g.sub_from : nullptr);
    }
    TP_HIP(hipGetLastError());
    if (g.affine) {
        const size_t tot = (size_t)g.M * g.N;
        const dim3 rg((unsigned)((tot + 255) / 256));
        if (S > 1)
            hipLaunchKernelGGL(k_splitk_reduce_af, rg, dim3(256), 0, s, out, pstride, S, g.M, g.N, g.C, g.ldc, g.af_a,
                               g.af_b, g.af_c, g.af_y, g.af_z);
        else
            hipLaunchKernelGGL(k_affine_inplace, rg, dim3(256), 0, s, g.M, g.N, g.C, g.ldc, g.af_a, g.af_b, g.af_c,
                               g.af_y, g.af_z);
        TP_HIP(hipGetLastError());
    } else if (S > 1) {
        size_t tot = (size_t)g.M * g.N;
        const dim3 rg((unsigned)((tot + 255) / 256));
        if (S >= 16 && tot <= ((size_t)1 << 18))
            hipLaunchKernelGGL(k_splitk_reduce4, dim3((unsigned)((tot + 63) / 64)), dim3(256), 0, s, out, pstride, S,
                               g.M, g.N, g.C, g.ldc, (int)g.store_t, g.sub_from);
        else if (g.tag == 1)
            hipLaunchKernelGGL(k_splitk_reduce<1>, rg, dim3(256), 0, s, out, pstride, S, g.M, g.N, g.C, g.ldc,
                               (int)g.store_t, g.sub_from);
        else
            hipLaunchKernelGGL(k_splitk_reduce<0>, rg, dim3(256), 0, s, out, pstride, S, g.M, g.N, g.C, g.ldc,
                               (int)g.store_t, g.sub_from);
        TP_HIP(hipGetLastError());
    }
}



}  // namespace tp
