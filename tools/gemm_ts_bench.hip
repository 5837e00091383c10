// Microbenchmark of the Krylov product C = A'B (A k-contiguous, M = n + 2,
// N = 64, K = n; the C3 shape by default): the library's k_gemm_ts tile
// (128 x 64, 4 waves of 32 x 64, BK 16) against variants.  Partials only (the
// split-K reduction is timed separately in the library).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/gemm_ts_bench.hip -o tools/gemm_ts_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int TSM = 128, TSN = 64;

__device__ __forceinline__ int xcd_order(int total) {
    const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
    return xcd * (total >> 3) + min(xcd, total & 7) + slot;
}

// ---- V0: the library kernel (k_gemm_ts)
template <int TSK>
__global__ void __launch_bounds__(256, 2) k_v0(int M, int N, int K, const double *__restrict__ A, int lda,
                                               const double *__restrict__ B, int ldb, double *__restrict__ C, int ldc,
                                               int kchunk, size_t part_stride) {
    constexpr int TSLD = TSK + 2;
    __shared__ double As[2][TSM][TSLD];
    __shared__ double Bs[2][TSN][TSLD];
    const int tm = (M + TSM - 1) / TSM, tn = (N + TSN - 1) / TSN;
    const int Lg = xcd_order((int)gridDim.x);
    const int bn = Lg % tn, bm = (Lg / tn) % tm, z = Lg / (tn * tm);
    const int i0 = bm * TSM, j0 = bn * TSN;
    const int kbeg = z * kchunk, kend = min(K, kbeg + kchunk);
    C += part_stride * z;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = 32 * w;
    const int fr = lane & 15, fk = lane >> 4;
    d4 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
    constexpr int PA = TSM * TSK / 256, PB = TSN * TSK / 256;
    double ra[PA], rb[PB];
    const int lk = t % TSK, lr = t / TSK;
    constexpr int RS = 256 / TSK;
    auto load = [&](int k0) {
        const int k = k0 + lk;
        const bool kin = k < kend;
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int i = i0 + lr + RS * p;
            ra[p] = (kin && i < M) ? A[(size_t)k + (size_t)i * lda] : 0.0;
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int j = j0 + lr + RS * p;
            rb[p] = (kin && j < N) ? B[(size_t)k + (size_t)j * ldb] : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int p = 0; p < PA; ++p) As[buf][lr + RS * p][lk] = ra[p];
#pragma unroll
        for (int p = 0; p < PB; ++p) Bs[buf][lr + RS * p][lk] = rb[p];
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
#pragma unroll
        for (int kk = 0; kk < TSK; kk += 4) {
            double af[2], bf[4];
#pragma unroll
            for (int a = 0; a < 2; ++a) af[a] = As[buf][wm + 16 * a + fr][kk + fk];
#pragma unroll
            for (int b = 0; b < 4; ++b) bf[b] = Bs[buf][16 * b + fr][kk + fk];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wm + 16 * a + fk + 4 * r;
                const int j = j0 + 16 * b + fr;
                if (i < M && j < N) C[(size_t)i + (size_t)j * ldc] = acc[a][b][r];
            }
}

// ---- V1: k sliced over the waves: every wave owns the whole 128 x 64 tile
// (8 x 4 accumulators) for one 4-deep MFMA step of each BK-deep stage (wave w:
// k = k0 + 4 w' .. for w' = w, w + 4, ...); 12 fragment reads per 32 MFMAs.
// The four waves' partials are summed in wave order at the end through LDS.
template <int TSK>
__global__ void __launch_bounds__(256, 2) k_v1(int M, int N, int K, const double *__restrict__ A, int lda,
                                               const double *__restrict__ B, int ldb, double *__restrict__ C, int ldc,
                                               int kchunk, size_t part_stride) {
    constexpr int TSLD = TSK + 2;
    __shared__ double As[2][TSM][TSLD];
    __shared__ double Bs[2][TSN][TSLD];
    const int tm = (M + TSM - 1) / TSM, tn = (N + TSN - 1) / TSN;
    const int Lg = xcd_order((int)gridDim.x);
    const int bn = Lg % tn, bm = (Lg / tn) % tm, z = Lg / (tn * tm);
    const int i0 = bm * TSM, j0 = bn * TSN;
    const int kbeg = z * kchunk, kend = min(K, kbeg + kchunk);
    C += part_stride * z;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int fr = lane & 15, fk = lane >> 4;
    d4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
    constexpr int PA = TSM * TSK / 256, PB = TSN * TSK / 256;
    double ra[PA], rb[PB];
    const int lk = t % TSK, lr = t / TSK;
    constexpr int RS = 256 / TSK;
    auto load = [&](int k0) {
        const int k = k0 + lk;
        const bool kin = k < kend;
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int i = i0 + lr + RS * p;
            ra[p] = (kin && i < M) ? A[(size_t)k + (size_t)i * lda] : 0.0;
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int j = j0 + lr + RS * p;
            rb[p] = (kin && j < N) ? B[(size_t)k + (size_t)j * ldb] : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int p = 0; p < PA; ++p) As[buf][lr + RS * p][lk] = ra[p];
#pragma unroll
        for (int p = 0; p < PB; ++p) Bs[buf][lr + RS * p][lk] = rb[p];
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
#pragma unroll
        for (int ks = 0; ks < TSK / 16; ++ks) {
            const int kk = 16 * ks + 4 * w + fk;
            double bf[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) bf[b] = Bs[buf][16 * b + fr][kk];
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                const double af = As[buf][16 * a + fr][kk];
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf[b], acc[a][b], 0, 0, 0);
            }
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    // wave-order sum of the four partial tiles, 4 accumulator rows a pass
    double *red = &As[0][0][0];   // 4 waves x 4 x 4 tiles x 256 doubles = 128 KiB?  no: pass of one a-row
#pragma unroll
    for (int a = 0; a < 8; ++a) {
        // red[w][b][r][lane] : 4 x 4 x 4 x 64 doubles = 32 KiB
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[((w * 4 + b) * 4 + r) * 64 + lane] = acc[a][b][r];
        __syncthreads();
        // wave w sums accumulator column b = w of this a-row
        {
            const int b = w;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double v = red[((0 * 4 + b) * 4 + r) * 64 + lane];
                v = v + red[((1 * 4 + b) * 4 + r) * 64 + lane];
                v = v + red[((2 * 4 + b) * 4 + r) * 64 + lane];
                v = v + red[((3 * 4 + b) * 4 + r) * 64 + lane];
                const int i = i0 + 16 * a + fk + 4 * r;
                const int j = j0 + 16 * b + fr;
                if (i < M && j < N) C[(size_t)i + (size_t)j * ldc] = v;
            }
        }
        __syncthreads();
    }
}


// ---- V2: 4 waves as 2 (M halves of 64 rows) x 2 (k slices): wave w owns rows
// 64 (w & 1) .. + 63 of the tile with 4 x 4 accumulators for the MFMA k-steps
// 2 (w >> 1), 2 (w >> 1) + 1 of each 16-deep stage: 16 fragment reads per 32
// MFMAs; the two k-slice partials are summed (slice 0 first) through LDS.
template <int TSK>
__global__ void __launch_bounds__(256, 2) k_v2(int M, int N, int K, const double *__restrict__ A, int lda,
                                               const double *__restrict__ B, int ldb, double *__restrict__ C, int ldc,
                                               int kchunk, size_t part_stride) {
    constexpr int TSLD = TSK + 2;
    __shared__ double As[2][TSM][TSLD];
    __shared__ double Bs[2][TSN][TSLD];
    const int tm = (M + TSM - 1) / TSM, tn = (N + TSN - 1) / TSN;
    const int Lg = xcd_order((int)gridDim.x);
    const int bn = Lg % tn, bm = (Lg / tn) % tm, z = Lg / (tn * tm);
    const int i0 = bm * TSM, j0 = bn * TSN;
    const int kbeg = z * kchunk, kend = min(K, kbeg + kchunk);
    C += part_stride * z;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = 64 * (w & 1), ksl = w >> 1;
    const int fr = lane & 15, fk = lane >> 4;
    d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
    constexpr int PA = TSM * TSK / 256, PB = TSN * TSK / 256;
    double ra[PA], rb[PB];
    const int lk = t % TSK, lr = t / TSK;
    constexpr int RS = 256 / TSK;
    auto load = [&](int k0) {
        const int k = k0 + lk;
        const bool kin = k < kend;
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int i = i0 + lr + RS * p;
            ra[p] = (kin && i < M) ? A[(size_t)k + (size_t)i * lda] : 0.0;
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int j = j0 + lr + RS * p;
            rb[p] = (kin && j < N) ? B[(size_t)k + (size_t)j * ldb] : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int p = 0; p < PA; ++p) As[buf][lr + RS * p][lk] = ra[p];
#pragma unroll
        for (int p = 0; p < PB; ++p) Bs[buf][lr + RS * p][lk] = rb[p];
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
#pragma unroll
        for (int ks = 0; ks < TSK / 8; ++ks) {
            const int kk = 8 * ks + 4 * ksl + fk;
            double af[4], bf[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) af[a] = As[buf][wm + 16 * a + fr][kk];
#pragma unroll
            for (int b = 0; b < 4; ++b) bf[b] = Bs[buf][16 * b + fr][kk];
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
    // slice 1 hands its partials to slice 0 through LDS (4 x 4 x 4 x 64 doubles per M half)
    double *red = &As[0][0][0];
    if (ksl == 1) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) red[(((w & 1) * 16 + a * 4 + b) * 4 + r) * 64 + lane] = acc[a][b][r];
    }
    __syncthreads();
    if (ksl == 0) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double v = acc[a][b][r] + red[(((w & 1) * 16 + a * 4 + b) * 4 + r) * 64 + lane];
                    const int i = i0 + wm + 16 * a + fk + 4 * r;
                    const int j = j0 + 16 * b + fr;
                    if (i < M && j < N) C[(size_t)i + (size_t)j * ldc] = v;
                }
    }
}


// ---- V3: v0 with 16-byte global loads (two consecutive k of a row per lane:
// 8 lanes cover a row's 128 B, a wave 8 rows) and 16-byte LDS stores
template <int TSK>
__global__ void __launch_bounds__(256, 2) k_v3(int M, int N, int K, const double *__restrict__ A, int lda,
                                               const double *__restrict__ B, int ldb, double *__restrict__ C, int ldc,
                                               int kchunk, size_t part_stride) {
    constexpr int TSLD = TSK + 2;
    __shared__ double As[2][TSM][TSLD];
    __shared__ double Bs[2][TSN][TSLD];
    const int tm = (M + TSM - 1) / TSM, tn = (N + TSN - 1) / TSN;
    const int Lg = xcd_order((int)gridDim.x);
    const int bn = Lg % tn, bm = (Lg / tn) % tm, z = Lg / (tn * tm);
    const int i0 = bm * TSM, j0 = bn * TSN;
    const int kbeg = z * kchunk, kend = min(K, kbeg + kchunk);
    C += part_stride * z;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = 32 * w;
    const int fr = lane & 15, fk = lane >> 4;
    d4 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
    constexpr int KP = TSK / 2;                 // k pairs per row
    constexpr int RS = 256 / KP;                // rows per pass
    constexpr int PA = TSM / RS, PB = TSN / RS;
    double2 ra[PA], rb[PB];
    const int lk = t % KP, lr = t / KP;
    auto load = [&](int k0) {
        const int k = k0 + 2 * lk;
        const bool kin = k < kend;   // kend even (K chunks are multiples of 16; K even checked by the host)
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int i = i0 + lr + RS * p;
            ra[p] = (kin && i < M) ? *(const double2 *)(A + (size_t)k + (size_t)i * lda) : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int j = j0 + lr + RS * p;
            rb[p] = (kin && j < N) ? *(const double2 *)(B + (size_t)k + (size_t)j * ldb) : make_double2(0.0, 0.0);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int p = 0; p < PA; ++p) *(double2 *)&As[buf][lr + RS * p][2 * lk] = ra[p];
#pragma unroll
        for (int p = 0; p < PB; ++p) *(double2 *)&Bs[buf][lr + RS * p][2 * lk] = rb[p];
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
#pragma unroll
        for (int kk = 0; kk < TSK; kk += 4) {
            double af[2], bf[4];
#pragma unroll
            for (int a = 0; a < 2; ++a) af[a] = As[buf][wm + 16 * a + fr][kk + fk];
#pragma unroll
            for (int b = 0; b < 4; ++b) bf[b] = Bs[buf][16 * b + fr][kk + fk];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wm + 16 * a + fk + 4 * r;
                const int j = j0 + 16 * b + fr;
                if (i < M && j < N) C[(size_t)i + (size_t)j * ldc] = acc[a][b][r];
            }
}

// ---- V5: parametrised: TM rows per workgroup (4 waves of TM/4 rows x 64
// columns), BK-deep stages, NBUF LDS buffers (1: register prefetch, two
// barriers a stage), OCC workgroups a CU (launch bounds)
template <int TM, int BK, int NBUF, int OCC, int TN = TSN>
__global__ void __launch_bounds__(256, OCC) k_v5(int M, int N, int K, const double *__restrict__ A, int lda,
                                                 const double *__restrict__ B, int ldb, double *__restrict__ C,
                                                 int ldc, int kchunk, size_t part_stride) {
    constexpr int LD = BK + 2;
    constexpr int WA = TM / 64;   // 16-row accumulator tiles per wave
    constexpr int NBF = TN / 16;
    __shared__ double As[NBUF][TM][LD];
    __shared__ double Bs[NBUF][TN][LD];
    const int tm = (M + TM - 1) / TM, tn = (N + TN - 1) / TN;
    const int Lg = xcd_order((int)gridDim.x);
    const int bn = Lg % tn, bm = (Lg / tn) % tm, z = Lg / (tn * tm);
    const int i0 = bm * TM, j0 = bn * TN;
    const int kbeg = z * kchunk, kend = min(K, kbeg + kchunk);
    C += part_stride * z;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = (TM / 4) * w;
    const int fr = lane & 15, fk = lane >> 4;
    d4 acc[WA][NBF];
#pragma unroll
    for (int a = 0; a < WA; ++a)
#pragma unroll
        for (int b = 0; b < NBF; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
    constexpr int PA = TM * BK / 256, PB = TN * BK / 256;
    double ra[PA], rb[PB];
    const int lk = t % BK, lr = t / BK;
    constexpr int RS = 256 / BK;
    auto load = [&](int k0) {
        const int k = k0 + lk;
        const bool kin = k < kend;
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int i = i0 + lr + RS * p;
            ra[p] = (kin && i < M) ? A[(size_t)k + (size_t)i * lda] : 0.0;
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int j = j0 + lr + RS * p;
            rb[p] = (kin && j < N) ? B[(size_t)k + (size_t)j * ldb] : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int p = 0; p < PA; ++p) As[buf][lr + RS * p][lk] = ra[p];
#pragma unroll
        for (int p = 0; p < PB; ++p) Bs[buf][lr + RS * p][lk] = rb[p];
    };
    if (kbeg < kend) {
        load(kbeg);
        store(0);
    }
    __syncthreads();
    int buf = 0;
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        const bool more = k0 + BK < kend;
        if (more) load(k0 + BK);
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
            double af[WA], bf[NBF];
#pragma unroll
            for (int a = 0; a < WA; ++a) af[a] = As[buf][wm + 16 * a + fr][kk + fk];
#pragma unroll
            for (int b = 0; b < NBF; ++b) bf[b] = Bs[buf][16 * b + fr][kk + fk];
#pragma unroll
            for (int a = 0; a < WA; ++a)
#pragma unroll
                for (int b = 0; b < NBF; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        if (NBUF == 1) __syncthreads();
        if (more) store(NBUF == 1 ? 0 : buf ^ 1);
        __syncthreads();
        if (NBUF == 2) buf ^= 1;
    }
#pragma unroll
    for (int a = 0; a < WA; ++a)
#pragma unroll
        for (int b = 0; b < NBF; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wm + 16 * a + fk + 4 * r;
                const int j = j0 + 16 * b + fr;
                if (i < M && j < N) C[(size_t)i + (size_t)j * ldc] = acc[a][b][r];
            }
}

__global__ void k_rand(double *p, size_t n, unsigned long long seed) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long z = seed + 0x9E3779B97F4A7C15ULL * (i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    p[i] = ((double)(z >> 11) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 7729;
    const int N = argc > 2 ? atoi(argv[2]) : 64, M = n + 2, K = n;
    const int reps = 20;
    double *A, *B, *P0, *P1;
    CK(hipMalloc(&A, (size_t)M * K * 8));
    CK(hipMalloc(&B, (size_t)K * N * 8));
    const size_t pst = (size_t)M * N;
    const int SMAX = 32;
    CK(hipMalloc(&P0, pst * SMAX * 8));
    CK(hipMalloc(&P1, pst * SMAX * 8));
    hipLaunchKernelGGL(k_rand, dim3((unsigned)(((size_t)M * K + 255) / 256)), dim3(256), 0, 0, A, (size_t)M * K, 1ULL);
    hipLaunchKernelGGL(k_rand, dim3((unsigned)(((size_t)K * N + 255) / 256)), dim3(256), 0, 0, B, (size_t)K * N, 2ULL);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double flops = 2.0 * M * N * (double)K;
    auto run = [&](const char *name, auto kern, int TM, int S, double *out) {
        int kchunk = ((K + S - 1) / S + 15) / 16 * 16;
        const int SS = (K + kchunk - 1) / kchunk;
        const dim3 grid((unsigned)(((M + TM - 1) / TM) * SS));
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, M, N, K, A, n, B, n, out, M, kchunk, pst);
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, M, N, K, A, n, B, n, out, M, kchunk, pst);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf("%-34s S=%2d grid=%5u %8.1f us  %6.2f TF/s\n", name, SS, grid.x, us, flops / (us * 1e-6) / 1e12);
        fflush(stdout);
    };
    printf("M=%d N=%d K=%d\n", M, N, K);
    if (N == 64) {
        run("v0 k_gemm_ts BK16", k_v0<16>, 128, 8, P0);
        run("v5 TM128 BK16 NBUF2 OCC2", k_v5<128, 16, 2, 2>, 128, 8, P1);
        run("v5 TM128 BK32 NBUF1 OCC2", k_v5<128, 32, 1, 2>, 128, 8, P1);
        run("v5 TM64 BK16 NBUF2 OCC4", k_v5<64, 16, 2, 4>, 64, 8, P1);
        run("v0 k_gemm_ts BK16 (again)", k_v0<16>, 128, 8, P0);
    } else {
        run("v5 TM128 TN32 BK16 NBUF2 OCC2 (lib)", k_v5<128, 16, 2, 2, 32>, 128, 8, P0);
        run("v5 TM128 TN32 BK16 NBUF2 OCC3", k_v5<128, 16, 2, 3, 32>, 128, 8, P1);
        run("v5 TM256 TN32 BK16 NBUF2 OCC2", k_v5<256, 16, 2, 2, 32>, 256, 8, P1);
        run("v5 TM256 TN32 BK16 NBUF2 OCC2", k_v5<256, 16, 2, 2, 32>, 256, 16, P1);
        run("v5 TM256 TN32 BK8 NBUF2 OCC2", k_v5<256, 8, 2, 2, 32>, 256, 16, P1);
        run("v5 TM256 TN32 BK32 NBUF1 OCC2", k_v5<256, 32, 1, 2, 32>, 256, 8, P1);
        run("v5 TM128 TN32 BK32 NBUF2 OCC2", k_v5<128, 32, 2, 2, 32>, 128, 8, P1);
        run("v5 TM128 TN32 BK16 NBUF2 OCC2 (lib, again)", k_v5<128, 16, 2, 2, 32>, 128, 8, P0);
    }
    return 0;
}
