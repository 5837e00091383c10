// The PCA's long-K products Out = A'B (A = [C | m | 1], K = n rows, M = n + 2
// columns; B = an n x 64 Krylov block of the G-space path) on the int8 MFMA
// instead of the fp64 one (R/TADpole.R:453, prcomp's products; tp_pca.hip).
//
// Every column of A and of B is cut into seven balanced base-256 digits of a
// 54-bit fixed-point image scaled by a power of two per column:
//   x = 2^(e - 54) sum_{s=0..6} d_s 256^(6 - s),  d_s in [-128, 127],
// |x| < 2^e (e from the column's largest |x|), so the image differs from x by
// at most 2^(e - 55) -- below half an fp64 ulp of the column's largest entry.
// A'B is then sum over digit pairs (s, t) of 256^(12 - s - t) D_s'E_t, each
// D_s'E_t an exact int32 MFMA product (|sum| <= kchunk 2^14 per pair).  Pairs
// with s + t <= 6 are kept, grouped by u = s + t into seven int32
// accumulators (<= 7 pairs each: kchunk <= 16384 keeps them below 2^31); the
// dropped pairs weigh <= 256^-7 of the leading one.  The product reads
// TP_PD_ADIG of A's digits: 7 (28 pairs) is within ~5e-17 of sum |A_ki||B_kj|,
// the rounding level of the fp64 product; 6 (27 pairs, the default) drops the
// (6, 0) pair and A's last 8 bits, ~1e-15.  The seven sums are combined in
// fp64 (smallest weight first) and scaled by the two columns' powers of two.
// 27 int8 MFMAs of 16 x 16 x 64 (2^20 ops, 16 cycles each) produce what 16
// fp64 16 x 16 x 4 MFMAs (2^11 flops each) do at 64 cycles: 2.4x less MFMA
// time for the same output.
//
// A's digits are formed once per PCA (A is fixed over all ~32 products); B's
// per product.  The product kernel writes fp64 split-K partials that the
// fp64 path's fixed-order reductions (with the rank-1 centring epilogue) sum:
// k chunks depend on K alone, so a row shard computes every element with the
// same bits as the whole product.
#include <algorithm>
#include <cmath>

#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

// knob 36: the int8-digit products in the G-space Krylov path (0: the fp64
// k_gemm_ts; 1: k_pd_prod, 64-row tiles; 5: k_pd_prodA, 128-row tiles).  Within ~1e-15 of sum |A||B|
// (test_prod_i8_digit_product); the 32 C3 products 4.6 ms against 6.3
// 

constexpr int PD_DIG = 7;   // digits per value
#ifndef TP_PD_ADIG
// digits of A the product reads, and the digits A's image stores.  6: the
// (6, 0) pair and A's least significant digit dropped.  Dropping a balanced
// digit (|d_6| <= 128 at weight 2^(e - 54)) leaves A's image within 2^(e - 47)
// of A, 2^-46..2^-47 of the column's largest |x| -- a fixed perturbation of C
// shared by every product of the PCA, not per-product rounding (~7e-15 on C's
// entries; errors 3e-17 -> 5e-16..9e-16 of sum |A||B|; C3 products 6.63 ->
// 6.12 ms with the first layout)
#define TP_PD_ADIG 6
#endif
constexpr int PD_ADIG = TP_PD_ADIG;
typedef int pd_i32x4 __attribute__((ext_vector_type(4)));

// Digit image layout (both operands): 64 columns x 64 k bytes per block, the
// ND digit blocks of one (column tile, k step) contiguous (ND = PD_ADIG for
// A, whose last digit the product never reads; PD_DIG for the blocks) --
//   ((c / 64) nsteps + k / 64) ND 4096 + s 4096 + (c % 64) 64 + k % 64
// -- so a workgroup's k step of A (64 rows, six digits) is one contiguous 24 KB
// read (DRAM pages streamed, not 64-byte pieces of 384 columns).
constexpr int PD_BLK = 4096;
template <int ND>
__device__ __forceinline__ size_t pd_off(int c, int k, int nsteps) {
    return ((size_t)(c >> 6) * nsteps + (k >> 6)) * (ND * PD_BLK) + (size_t)(c & 63) * 64 + (k & 63);
}

// 2^(54 - e) and 2^(e - 54) for a column with largest |x| < 2^e, e clamped
// at -968 so the scale stays finite (columns below 2^-968 lose their low bits)
__device__ __forceinline__ int pd_exp(double mx) {
    int e = 0;
    if (mx > 0.0 && isfinite(mx)) (void)frexp(mx, &e);
    return max(e, -968);
}

// Digits of x[k0..k0+3] (zero past K or when !ok): one 4-byte word per digit,
// digit s < ND at d + s PD_BLK (d = the image at pd_off<ND>(c, k0)); all seven
// are formed, the first ND stored.  The balanced digits (least significant
// first: d = the signed low byte of r, r = (r - d) / 256) are the bytes of
// u = q + 0x808080808080 -- the six low digits offset by 128 (xor 0x80), the
// top digit byte 6 as is -- so no carry loop: one 64-bit add, then byte
// permutes gather digit s of the four values into one word.
template <int ND>
__device__ __forceinline__ void pd_digits4(const double *__restrict__ x, int K, int k0, bool ok, double sc,
                                           int8_t *__restrict__ d) {
    unsigned lo[4], hi[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int k = k0 + u;
        const double v = (ok && k < K) ? x[k] : 0.0;
        const unsigned long long uq = (unsigned long long)llrint(v * sc) + 0x808080808080ULL;   // |q| <= 2^54
        lo[u] = (unsigned)uq ^ 0x80808080u;
        hi[u] = (unsigned)(uq >> 32) ^ 0x8080u;
    }
    // byte b of a[0..3] -> bytes 0..3 of one word (v_perm_b32: selector 0..3 the
    // second operand's bytes, 4..7 the first's, 12 a zero byte)
    auto gather = [](const unsigned (&a)[4], unsigned b) {
        const unsigned sel = 0x0C0C0000u | ((4u + b) << 8) | b;
        const unsigned t01 = __builtin_amdgcn_perm(a[1], a[0], sel);
        const unsigned t23 = __builtin_amdgcn_perm(a[3], a[2], sel);
        return __builtin_amdgcn_perm(t23, t01, 0x05040100u);
    };
    const unsigned w[PD_DIG] = {gather(hi, 2), gather(hi, 1), gather(hi, 0), gather(lo, 3),
                                gather(lo, 2), gather(lo, 1), gather(lo, 0)};
#pragma unroll
    for (int s = 0; s < ND; ++s) *(unsigned *)(d + (size_t)s * PD_BLK) = w[s];
}

// Digits of one column per workgroup: column c of X (K values, ld ldx) ->
// the image at pd_off(c, k) (k < Kp; zero past K and for c >= cols), the column
// scale 2^(e - 54) into scale[c] (NaN for a non-finite column, so the product
// is NaN as the fp64 one would be).
template <int ND>
__global__ void __launch_bounds__(256) k_pd_digits(const double *__restrict__ X, int ldx, int K, int cols, int Kp,
                                                   int8_t *__restrict__ D, double *__restrict__ scale) {
    __shared__ double red[4];
    const int c = blockIdx.x;
    const int t = threadIdx.x;
    const double *x = X + (size_t)c * ldx;
    const bool live = c < cols;
    double mx = 0.0;
    if (live)
        for (int k = t; k < K; k += 256) mx = fmax(mx, fabs(x[k]));
    // NaN-propagating max: fmax drops NaN, so flag non-finite values apart
    bool bad = false;
    if (live)
        for (int k = t; k < K; k += 256) bad |= !isfinite(x[k]);
    mx = bad ? INFINITY : mx;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    const int e = pd_exp(mx);   // mx < 2^e
    const double sc = ldexp(1.0, 54 - e);
    if (t == 0) scale[c] = !live ? 0.0 : (isfinite(mx) ? ldexp(1.0, e - 54) : NAN);
    const int nsteps = Kp / 64;
    for (int k0 = 4 * t; k0 < Kp; k0 += 1024)
        pd_digits4<ND>(x, K, k0, live && isfinite(mx), sc, D + pd_off<ND>(c, k0, nsteps));
}

// The same, for K <= 1024 IT: the column is read once (values kept in
// registers across the max and the digits), thread t holding k = 1024 i + 4 t
// .. + 3 -- one HBM pass over C instead of two (the second pass of k_pd_digits
// misses L2 at C3: 1.87 GB moved for 0.9 GB of data)
// TB threads a column (256; 1024 for the long columns of the C-space path:
// 24 300 bins with IT = 6 instead of k_pd_digits' three passes over C)
template <int IT, int ND, int TB = 256>
__global__ void __launch_bounds__(TB) k_pd_digits_reg(const double *__restrict__ X, int ldx, int K, int cols, int Kp,
                                                      int8_t *__restrict__ D, double *__restrict__ scale) {
    constexpr int NW = TB / 64;
    __shared__ double red[NW];
    // adjacent columns on one XCD (workgroups are dealt round-robin over the 8):
    // columns c and c + 1 fill the two halves of each 128-byte line of the image
    // in the same L2 (gridDim.x is a multiple of 64)
    const int c = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
    const int t = threadIdx.x;
    const double *x = X + (size_t)c * ldx;
    const bool live = c < cols;
    double v[IT][4];
    double mx = 0.0;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < IT; ++i)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = 4 * TB * i + 4 * t + u;
            v[i][u] = (live && k < K) ? x[k] : 0.0;
            mx = fmax(mx, fabs(v[i][u]));
            bad |= !isfinite(v[i][u]);
        }
    mx = bad ? INFINITY : mx;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    mx = red[0];
#pragma unroll
    for (int q = 1; q < NW; ++q) mx = fmax(mx, red[q]);
    const int e = pd_exp(mx);   // mx < 2^e
    const double sc = ldexp(1.0, 54 - e);
    if (t == 0) scale[c] = !live ? 0.0 : (isfinite(mx) ? ldexp(1.0, e - 54) : NAN);
    const bool ok = live && isfinite(mx);
    const int nsteps = Kp / 64;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const int k0 = 4 * TB * i + 4 * t;
        if (k0 < Kp) pd_digits4<ND>(v[i], 4, 0, ok, sc, D + pd_off<ND>(c, k0, nsteps));
    }
}
constexpr int PD_REG_IT = 8;   // register path up to K = 8192

// A's digit image and C's column means in one pass over C: two adjacent
// columns (c0, c0 + 1) a workgroup of ten waves.
//   waves 0..7 (digits): thread t = 32 g + 16 h + j holds column c0 + h, rows
//     64 (g + 16 i) + 4 j .. + 3 (i < 8, K <= 8192) in registers; column maxima
//     by a 16-lane-row butterfly and LDS (fmax: k_pd_digits_reg's scale bits);
//     then each digit word store of a wave covers whole 128-byte lines of the
//     image (the two columns' 64-byte halves side by side: one workgroup per
//     column wrote half lines, ~3 TB/s);
//   waves 8, 9 (means, c < ncm): column c0 + w - 8 streamed in k_colmean's
//     order -- lane l sums rows l, l + 64, ... in double-double, then the wave
//     butterfly -- from L2 (the digit waves read the same lines at the same
//     time), so the means carry k_colmean's bits.
// Columns [c_begin, c_end) (live below `cols`, zero digits above).  Replaces
// k_colmean (124 us at C3) and the digit pass (~315 us).
constexpr int PD_CM_W = 10;
template <int ND>
__global__ void __launch_bounds__(64 * PD_CM_W) k_pd_digits_cm(const double *__restrict__ X, int ldx, int K, int c_begin,
                                                             int c_end, int cols, int Kp, int8_t *__restrict__ D,
                                                             double *__restrict__ scale, double *__restrict__ cm,
                                                             int ncm) {
    __shared__ double red[8][2];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int c0 = c_begin + 2 * (int)blockIdx.x;
    if (w >= 8) {   // ---- means
        const int c = c0 + (w - 8);
        __syncthreads();   // the digit waves' one barrier
        if (c >= c_end || c >= ncm || c >= cols) return;
        const double *x = X + (size_t)c * ldx;
        double hs = 0.0, ls = 0.0;
        constexpr int U = 16;   // two batches of U loads a lane in flight around the chain
        double va[U], vb[U];
        auto load = [&](double (&v)[U], int r) {
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = r + 64 * u < K ? x[r + 64 * u] : 0.0;
        };
        auto take = [&](const double (&v)[U], int r) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (r + 64 * u < K) dd_add_d(hs, ls, v[u]);
        };
        int r = lane;
        load(va, r);
        for (; r < K; r += 128 * U) {
            load(vb, r + 64 * U);
            take(va, r);
            load(va, r + 128 * U);
            take(vb, r + 64 * U);
        }
        wave_dd_sum(hs, ls);
        if (lane == 0) cm[c] = dd_div_d(hs, ls, (double)K);
        return;
    }
    // ---- digits
    const int g = t >> 5, h = (t >> 4) & 1, j = t & 15;
    const int c = c0 + h;
    const bool inr = c < c_end;                 // this launch writes column c
    const bool live = inr && c < cols;
    const double *x = X + (size_t)min(c, c_end - 1) * ldx;
    double v[8][4];
    double mx = 0.0;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = 64 * (g + 16 * i) + 4 * j + u;
            v[i][u] = (live && k < K) ? x[k] : 0.0;
            mx = fmax(mx, fabs(v[i][u]));
            bad |= !isfinite(v[i][u]);
        }
    mx = bad ? INFINITY : mx;
#pragma unroll
    for (int o = 1; o <= 32; o <<= 1)   // lanes of the same column: bit 4 (16) fixed
        if (o != 16) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if ((lane & 47) == 0) red[w][h] = mx;   // lanes 0 and 16
    __syncthreads();
    mx = red[0][h];
#pragma unroll
    for (int q = 1; q < 8; ++q) mx = fmax(mx, red[q][h]);
    if (!inr) return;
    const int e = pd_exp(mx);   // mx < 2^e
    const double sc = ldexp(1.0, 54 - e);
    if (g == 0 && j == 0) scale[c] = !live ? 0.0 : (isfinite(mx) ? ldexp(1.0, e - 54) : NAN);
    const bool ok = live && isfinite(mx);
    const int nsteps = Kp / 64;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int k0 = 64 * (g + 16 * i) + 4 * j;
        if (k0 < Kp) pd_digits4<ND>(v[i], 4, 0, ok, sc, D + pd_off<ND>(c, k0, nsteps));
    }
}

// A Krylov block's digits (N = 64 columns): one workgroup per (column, 1024-row
// slice), N x Kp / 1024 of them instead of N.  Each forms its column's largest
// |x| from the whole column (the same loads and fmax as k_pd_digits_reg, so
// the same scale bits) and digitises only its slice: the 64-workgroup form ran
// its 32 k-rows of digit work a thread on a quarter of the chip.  Work item q
// = slice * N + column, dealt XCD-contiguously so columns c and c + 1 of a
// slice (the two halves of each 128-byte line of the image) share an L2.
#ifndef TP_PD_SPW
#define TP_PD_SPW 4   // 1024-row slices a k_pd_digits_blk workgroup digitises (each reads its whole column
                      // for the scale): C3 products with digits 3.49 -> 3.35 ms against 1 (2: 3.39)
#endif
template <int IT, int SPW = 1>
__global__ void __launch_bounds__(256) k_pd_digits_blk(const double *__restrict__ X, int ldx, int K, int N, int Kp,
                                                       int8_t *__restrict__ D, double *__restrict__ scale) {
    __shared__ double red[4];
    const int G = (int)gridDim.x;
    const int q = (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3);
    const int c = q % N, sg = q / N;   // slices SPW sg .. SPW sg + SPW - 1
    const int t = threadIdx.x;
    const double *x = X + (size_t)c * ldx;
    double mx = 0.0;
    bool bad = false;
    double v[SPW][4];
#pragma unroll
    for (int i = 0; i < IT; ++i)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = 1024 * i + 4 * t + u;
            const double y = k < K ? x[k] : 0.0;
            mx = fmax(mx, fabs(y));
            bad |= !isfinite(y);
            if (i / SPW == sg) v[i % SPW][u] = y;
        }
    mx = bad ? INFINITY : mx;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    const int e = pd_exp(mx);   // mx < 2^e
    if (sg == 0 && t == 0) scale[c] = isfinite(mx) ? ldexp(1.0, e - 54) : NAN;
#pragma unroll
    for (int h = 0; h < SPW; ++h) {
        const int k0 = 1024 * (SPW * sg + h) + 4 * t;
        if (k0 < Kp)
            pd_digits4<PD_DIG>(v[h], 4, 0, isfinite(mx), ldexp(1.0, 54 - e), D + pd_off<PD_DIG>(c, k0, Kp / 64));
    }
}

// The same digits for a few columns (a Krylov block, N = 64): the column's
// largest |x| from per-1024-row partial maxima (k_pd_colmax), one workgroup
// per 1024 rows of a column -- 64 x (Kp / 1024) workgroups instead of 64.
__global__ void __launch_bounds__(256) k_pd_colmax(const double *__restrict__ X, int ldx, int K, int SL,
                                                   double *__restrict__ pmax) {
    __shared__ double red[4];
    const int c = blockIdx.x / SL, sl = blockIdx.x % SL;
    const int t = threadIdx.x;
    const double *x = X + (size_t)c * ldx;
    double mx = 0.0;
    bool bad = false;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int k = sl * 1024 + 4 * t + u;
        if (k < K) {
            const double v = x[k];
            mx = fmax(mx, fabs(v));
            bad |= !isfinite(v);
        }
    }
    mx = bad ? INFINITY : mx;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    if (t == 0) pmax[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}
__global__ void __launch_bounds__(256) k_pd_digits_sl(const double *__restrict__ X, int ldx, int K, int Kp, int SL,
                                                      const double *__restrict__ pmax, int8_t *__restrict__ D,
                                                      double *__restrict__ scale) {
    const int c = blockIdx.x / SL, sl = blockIdx.x % SL;
    const int t = threadIdx.x;
    double mx = 0.0;
    for (int q = 0; q < SL; ++q) mx = fmax(mx, pmax[c * SL + q]);
    const int e = pd_exp(mx);
    if (sl == 0 && t == 0) scale[c] = isfinite(mx) ? ldexp(1.0, e - 54) : NAN;
    const int k0 = sl * 1024 + 4 * t;
    if (k0 < Kp)
        pd_digits4<PD_DIG>(X + (size_t)c * ldx, K, k0, isfinite(mx), ldexp(1.0, 54 - e), D + pd_off<PD_DIG>(c, k0, Kp / 64));
}

// Out partials: rows [0, M) of A'B from the digit images Da (A's column tiles
// from row 0 of Out on) and Db (the block's 64 columns), both in the pd_off
// layout.  4 waves in 2 x 2, wave w a 32 x 32 output block (2 x 2 MFMA tiles,
// seven accumulators each): 64 rows x 64 columns a workgroup; blockIdx ->
// (row tile, k chunk) dealt XCD-contiguously.  Each 64-byte k step of both
// images (PD_ADIG x 4 KB of A, 7 x 4 KB of B, each a contiguous run) is
// staged through registers into LDS (96-byte rows: conflict-free b128 fragment
// reads and staging writes, PD_LD).
// NB = 1 (the default): one LDS buffer of 78 KB (PD_BUF), the next step's
// loads in registers while this step's MFMAs run, two barriers a step, two
// workgroups a CU (each one's MFMAs run under the other's waits).
// NB = 2: two LDS buffers (156 KB, one workgroup a CU), two k steps of loads
// in flight in two register sets, one barrier a step (measured slower; no
// longer dispatched since round 6, kept as the template's second form).
// LDS row stride (bytes).  The 16-lane groups of ds_read_b128 ({0-3,12-15,
// 20-27}, ...: banks (a/4) mod 64) read fragment rows l & 15 at byte 16 (l >> 4):
// with 96-byte rows the 16 lanes of every group land on 16 distinct 4-bank
// blocks ((6 m + q) mod 16 all distinct); the 80-byte rows of round 4 put two
// lanes on each busy block (rocprof: SQ_LDS_BANK_CONFLICT = 50 % of the LDS
// cycles of k_pd_prod<1>).  Two 78 KB buffers still fit one CU (two
// workgroups of NB = 1, one of NB = 2).
#ifndef TP_PD_LD
#define TP_PD_LD 96
#endif
constexpr int PD_LD = TP_PD_LD;
constexpr int PD_ASZ = PD_ADIG * 64 * PD_LD, PD_BUF = PD_ASZ + PD_DIG * 64 * PD_LD;
static_assert(2 * PD_BUF <= 160 * 1024, "two k_pd_prod buffers must fit the CU's LDS");
// Staging: thread t moves one 16-byte piece of every 4 KB digit block -- row
// pd_srow(t), k quarter t % 4.  The 8-lane groups of ds_write_b128 (banks
// (a/4) mod 32) then hold rows r and r + 2 ((6 r + j) mod 8 distinct at 96-byte
// rows); a wave's global load is still one contiguous 1 KB (rows 16 w ..
// 16 w + 15, permuted within it).
__device__ __forceinline__ int pd_srow(int t) {
    return PD_LD == 96 ? 4 * (t >> 4) + ((t >> 3) & 1) + 2 * ((t >> 2) & 1) : t >> 2;
}
template <int NB>
__global__ void __launch_bounds__(256, 3 - NB) k_pd_prod(const int8_t *__restrict__ Da, int Kp, int M,
                                                    const int8_t *__restrict__ Db, const double *__restrict__ rs,
                                                    const double *__restrict__ cs, double *__restrict__ part,
                                                    size_t pstride, int kchunk) {
    extern __shared__ __attribute__((aligned(16))) int8_t pd_lds[];
    const int tm = (M + 63) / 64;
    const int total = (int)gridDim.x;
    const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
    const int Lg = xcd * (total >> 3) + min(xcd, total & 7) + slot;
    const int bm = Lg % tm, z = Lg / tm;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1;
    const int fr = lane & 15, fk = (lane >> 4) * 16;
    const int kbeg = z * kchunk, kend = min(Kp, kbeg + kchunk);
    const int nsteps = Kp / 64;
    TP_DASSERT(Kp % 64 == 0 && kchunk % 64 == 0 && kend - kbeg >= 64);
    pd_i32x4 acc[PD_DIG][2][2];
#pragma unroll
    for (int u = 0; u < PD_DIG; ++u)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[u][a][b] = pd_i32x4{0, 0, 0, 0};
    // staging: thread t moves row sr, k quarter t % 4 of every 4 KB digit block
    // of the step (pd_srow)
    const int sr = pd_srow(t), sk = (t & 3) * 16;
    const int8_t *ga = Da + (size_t)bm * nsteps * (PD_ADIG * PD_BLK) + 64 * sr + sk;
    const int8_t *gb = Db + 64 * sr + sk;
    const int T = (kend - kbeg) / 64, st0 = kbeg / 64;
    pd_i32x4 ra[PD_DIG], rb[PD_DIG], xa[PD_DIG], xb[PD_DIG];
    // loads past the chunk re-read its last step (clamped, unconditional: the
    // compiler counts them) and land in the buffer no later step reads
    auto gload = [&](pd_i32x4 (&ta)[PD_DIG], pd_i32x4 (&tb)[PD_DIG], int st) {
        const int sk = st0 + min(st, T - 1);
        const size_t oa = (size_t)sk * (PD_ADIG * PD_BLK), ob = (size_t)sk * (PD_DIG * PD_BLK);
#pragma unroll
        for (int s = 0; s < PD_DIG; ++s) {
            if (s < PD_ADIG) ta[s] = *(const pd_i32x4 *)(ga + oa + s * PD_BLK);
            tb[s] = *(const pd_i32x4 *)(gb + ob + s * PD_BLK);
        }
    };
    auto lstore = [&](const pd_i32x4 (&ta)[PD_DIG], const pd_i32x4 (&tb)[PD_DIG], int bf) {
        int8_t *L = pd_lds + bf * PD_BUF;
#pragma unroll
        for (int s = 0; s < PD_DIG; ++s) {
            if (s < PD_ADIG) *(pd_i32x4 *)(L + (s * 64 + sr) * PD_LD + sk) = ta[s];
            *(pd_i32x4 *)(L + PD_ASZ + (s * 64 + sr) * PD_LD + sk) = tb[s];
        }
    };
    auto mstep = [&](int bf) {
        const int8_t *L = pd_lds + bf * PD_BUF;
        pd_i32x4 fb[PD_DIG][2];
#pragma unroll
        for (int tt = 0; tt < PD_DIG; ++tt)
#pragma unroll
            for (int b = 0; b < 2; ++b)
                fb[tt][b] = *(const pd_i32x4 *)(L + PD_ASZ + (tt * 64 + 32 * wc + 16 * b + fr) * PD_LD + fk);
#pragma unroll
        for (int s0 = 0; s0 < PD_ADIG; ++s0) {
            pd_i32x4 fa[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) fa[a] = *(const pd_i32x4 *)(L + (s0 * 64 + 32 * wr + 16 * a + fr) * PD_LD + fk);
#pragma unroll
            for (int tt = 0; tt + s0 < PD_DIG; ++tt)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc[s0 + tt][a][b] =
                            __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[a], fb[tt][b], acc[s0 + tt][a][b], 0, 0, 0);
        }
    };
    if constexpr (NB == 1) {
        (void)xa;
        (void)xb;
        gload(ra, rb, 0);
        lstore(ra, rb, 0);
        __syncthreads();
        for (int st = 0; st < T; ++st) {
            gload(ra, rb, st + 1);
#ifndef TP_PD_NO_SCHED_PIN
            // the next step's loads issue before this step's MFMAs (left alone,
            // the scheduler sinks them three quarters of the way down the MFMA
            // block and their HBM latency is exposed every step)
            __builtin_amdgcn_sched_barrier(0);
#endif
            mstep(0);
            __syncthreads();
            lstore(ra, rb, 0);
            __syncthreads();
        }
    } else {
        gload(ra, rb, 0);
        lstore(ra, rb, 0);
        gload(ra, rb, 1);
        gload(xa, xb, 2);
        __syncthreads();
        for (int st = 0;; st += 2) {
            mstep(0);                // step st
            lstore(ra, rb, 1);       // step st + 1
            __syncthreads();
            gload(ra, rb, st + 3);
            if (st + 1 >= T) break;
            mstep(1);                // step st + 1
            lstore(xa, xb, 0);       // step st + 2
            __syncthreads();
            gload(xa, xb, st + 4);
            if (st + 2 >= T) break;
        }
    }
    const int i0 = bm * 64 + 32 * wr, j0 = 32 * wc;
    double *P = part + pstride * z;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + 16 * a + (lane >> 4) * 4 + r;
                const int j = j0 + 16 * b + fr;
                if (i >= M) continue;
                // weight of u: 256^(12 - u) 2^-108 -> 2^(-12 - 8u), times the scales
                double v = 0.0;
#pragma unroll
                for (int u = PD_DIG - 1; u >= 0; --u) v += (double)acc[u][a][b][r] * ldexp(1.0, 96 - 8 * u);
                P[(size_t)i + (size_t)j * M] = (v * rs[i]) * cs[j];
            }
}

// k_pd_prodA (knob 36 = 5): the same products, pairs, int32 sums and combine
// (the bits of k_pd_prod) for 128-row tiles, built on the per-CU fill rate
// (tools/ubench_fill.hip: ~20 GB/s a CU from HBM, ~35 from L2, registers and
// LDS-DMA alike).  k_pd_prod moves A's 48 KB (HBM) and the block's 56 KB (L2,
// re-read by every 64-row workgroup) per two workgroups a step: 4.0 us
// predicted, 4.06 measured.  Here each of 8 waves owns 16 rows x 64 columns
// (seven int32 sums x 4 tiles, 112 registers), so A's fragments are
// wave-private: loaded straight into registers (1 KiB per digit, 2 steps
// ahead in 3 register sets), never through LDS; only the block (28 KB a step)
// is staged, by LDS-DMA into a 3-stage ring with the bank swizzle on the
// source (k_xtx_i8_glds's).  A step moves 76 KB for 128 x 64 outputs.
constexpr int PA_ST = 3;   // block ring stages
__device__ __forceinline__ void pd_glds16(const void *g, void *l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}
// s_waitcnt vmcnt(N) as an instruction the compiler's wait insertion sees
template <int N>
__device__ __forceinline__ void pd_wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}
__device__ __forceinline__ void pd_wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// RB 16-row A fragments and CB 16-column block fragments a wave (seven int32
// sums x RB x CB tiles: 112 registers for 1 x 4); 8 waves, so a workgroup
// covers 128 RB rows of A and N = 16 CB columns (1 x 4: the G-space blocks of
// 64 columns; 1 x 2: the C-space blocks of 32).
template <int RB, int CB>
__global__ void __launch_bounds__(512, 1) k_pd_prodA(const int8_t *__restrict__ Da, int Kp, int M,
                                                     const int8_t *__restrict__ Db, const double *__restrict__ rs,
                                                     const double *__restrict__ cs, double *__restrict__ part,
                                                     size_t pstride, int kchunk) {
    static_assert(RB * CB <= 4, "tile shapes");
    constexpr int NCH = PD_DIG * CB;            // block chunks (1 KiB) a stage
    constexpr int DW = (NCH + 7) / 8;           // DMAs a wave a stage
    constexpr int ROWS = 128 * RB;
    __shared__ __attribute__((aligned(16))) int8_t L[PA_ST * NCH * 1024];
    const int tm = (M + ROWS - 1) / ROWS, tm64 = (M + 63) / 64;
    const int total = (int)gridDim.x;
    const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
    const int Lg = xcd * (total >> 3) + min(xcd, total & 7) + slot;
    const int bm = Lg % tm, z = Lg / tm;
    const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int fr = lane & 15, kc = lane >> 4;
    const int kbeg = z * kchunk, kend = min(Kp, kbeg + kchunk);
    const int nsteps = Kp / 64;
    TP_DASSERT(Kp % 64 == 0 && kchunk % 64 == 0 && kend - kbeg >= 64);
    const int T = (kend - kbeg) / 64, st0 = kbeg / 64;
    // A: wave w's 16 RB rows start at row0 (inside one 64-column tile of the
    // image; a tile past the image -- odd tile count -- re-reads the last one:
    // its rows are past M and never stored); lane (fr, kc) of fragment a loads
    // row 16 a + fr, k bytes 16 kc ..
    const int row0 = bm * ROWS + 16 * RB * w;
    const int8_t *ga = Da + (size_t)min(row0 >> 6, tm64 - 1) * nsteps * (PD_ADIG * PD_BLK) +
                       ((row0 & 63) + fr) * 64 + 16 * kc;
    // the block: chunk c (< NCH) = digit c / CB, columns 16 (c % CB) ..; lane p
    // loads column p >> 2, k quarter (p & 3) ^ ((p >> 4) & 2)
    const int8_t *gb = Db + ((lane >> 2) * 64 + 16 * ((lane & 3) ^ ((lane >> 4) & 2)));
    auto aload = [&](pd_i32x4 (&ra)[PD_ADIG][RB], int st) {
        const size_t o = (size_t)(st0 + min(st, T - 1)) * (PD_ADIG * PD_BLK);
#pragma unroll
        for (int s = 0; s < PD_ADIG; ++s)
#pragma unroll
            for (int a = 0; a < RB; ++a) ra[s][a] = *(const pd_i32x4 *)(ga + o + s * PD_BLK + a * 1024);
    };
    auto bissue = [&](int st) {   // stage st of the block into ring slot st % PA_ST
        const size_t o = (size_t)(st0 + min(st, T - 1)) * (PD_DIG * PD_BLK);
        int8_t *dst = L + (st % PA_ST) * (NCH * 1024);
#pragma unroll
        for (int i = 0; i < DW; ++i) {
            // past the last chunk a wave repeats its previous one (same bytes to
            // the same LDS place): DW DMAs a wave, one wait count, no branch (a
            // branch around a DMA -- e.g. a small dummy one -- makes the
            // compiler wait vmcnt(0) before the next MFMAs)
            const int c = w + 8 * i < NCH ? w + 8 * i : w + 8 * (i - 1);
            pd_glds16(gb + o + (c / CB) * PD_BLK + (c % CB) * 1024, dst + c * 1024);
        }
    };
    pd_i32x4 acc[PD_DIG][RB][CB];
#pragma unroll
    for (int u = 0; u < PD_DIG; ++u)
#pragma unroll
        for (int a = 0; a < RB; ++a)
#pragma unroll
            for (int b = 0; b < CB; ++b) acc[u][a][b] = pd_i32x4{0, 0, 0, 0};
    const int roff = (4 * fr + (kc ^ ((fr >> 2) & 2))) * 16;
    auto mstep = [&](const pd_i32x4 (&ra)[PD_ADIG][RB], int st) {
        const int8_t *Lb = L + (st % PA_ST) * (NCH * 1024) + roff;
#pragma unroll
        for (int q = 0; q < PD_DIG; ++q) {
            pd_i32x4 fb[CB];
#pragma unroll
            for (int b = 0; b < CB; ++b) fb[b] = *(const pd_i32x4 *)(Lb + (CB * q + b) * 1024);
#pragma unroll
            for (int s0 = 0; s0 + q < PD_DIG && s0 < PD_ADIG; ++s0)
#pragma unroll
                for (int a = 0; a < RB; ++a)
#pragma unroll
                    for (int b = 0; b < CB; ++b)
                        acc[s0 + q][a][b] =
                            __builtin_amdgcn_mfma_i32_16x16x64_i8(ra[s0][a], fb[b], acc[s0 + q][a][b], 0, 0, 0);
        }
    };
    // step st, after the wait and the barrier: block stage st everywhere and
    // stage st - 1's slot free; A(st + 2) loaded into the set step st - 1 used
    // and block stage st + 2 issued (ring of 3).  (A one-step form with two
    // register sets gets compiler waits of vmcnt(0) before its MFMAs: the
    // compiler's count ignores the DMAs issued after the A loads.)
    pd_i32x4 r0[PD_ADIG][RB], r1[PD_ADIG][RB], r2[PD_ADIG][RB];
    aload(r0, 0);
    bissue(0);
    aload(r1, 1);
    bissue(1);
    auto step = [&](pd_i32x4 (&cur)[PD_ADIG][RB], pd_i32x4 (&nxt)[PD_ADIG][RB], int st) {
        pd_wait_vm<PD_ADIG * RB + DW>();   // A(st + 1) and stage st + 1 may stay in flight
        pd_wait_lgkm0();
        __builtin_amdgcn_s_barrier();
        aload(nxt, st + 2);
        bissue(st + 2);
        mstep(cur, st);
    };
    int st = 0;
    for (; st + 2 < T; st += 3) {
        step(r0, r2, st);
        step(r1, r0, st + 1);
        step(r2, r1, st + 2);
    }
    if (st < T) step(r0, r2, st);
    if (st + 1 < T) step(r1, r0, st + 1);
    pd_wait_vm<0>();   // the redundant tail loads and DMAs land before the workgroup ends
#pragma unroll
    for (int a = 0; a < RB; ++a)
#pragma unroll
        for (int b = 0; b < CB; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = row0 + 16 * a + 4 * kc + r;
                const int j = 16 * b + fr;
                if (i >= M) continue;
                double v = 0.0;
#pragma unroll
                for (int u = PD_DIG - 1; u >= 0; --u) v += (double)acc[u][a][b][r] * ldexp(1.0, 96 - 8 * u);
                (part + pstride * z)[(size_t)i + (size_t)j * M] = (v * rs[i]) * cs[j];
            }
}

// k chunks from K alone (shards agree); <= 16384 rows a chunk (accumulator range)
#ifndef TP_PD_KDIV
#define TP_PD_KDIV 1920  // C3: 4 k chunks, 244 k_pd_prodA workgroups (one round of one a CU): the 32
                         // products with digits and reductions 3.97 -> 3.45 ms against 8 chunks
                         // (3 chunks: 3.94, 2: 4.97 -- fewer workgroups than CUs); 24.3k (C space,
                         // 12 chunks): 33.2 -> ~31 ms
#endif
static int pd_kchunk(int Kp) {
    const int S = std::max(1, std::min(16, Kp / TP_PD_KDIV));
    int kc = ((Kp + S - 1) / S + 63) / 64 * 64;
    return std::min(kc, 16384);
}

int prod_i8_adig() { return PD_ADIG; }

int prod_i8_pairs() {
    int n = 0;
    for (int a = 0; a < PD_ADIG; ++a) n += PD_DIG - a;
    return n;
}

// N = 64 (the G-space Krylov blocks; the kernel's workgroup is 64 x 64)
// N = 64: the G-space blocks (knob 36's kernel); N = 32: the C-space blocks
// (k_pd_prodA<1, 2>, knob 45)
bool prod_i8_ok(int K, int N) { return (N == 64 || N == 32) && K >= 64; }

static void launch_digits_cm(const double *A, int lda, int K, int c_begin, int c_end, int cols, ProdDigits &pd,
                             double *cm, int ncm, hipStream_t s) {
    if (c_end <= c_begin) return;
    hipLaunchKernelGGL(k_pd_digits_cm<PD_ADIG>, dim3((unsigned)((c_end - c_begin + 1) / 2)), dim3(64 * PD_CM_W), 0, s,
                       A, lda, K, c_begin, c_end, cols, pd.Kp, (int8_t *)pd.d, (double *)pd.rs, cm, ncm);
    TP_HIP(hipGetLastError());
}


bool prod_digits_means_ok(int K) { return cfg_pd_cm && K >= 64 && (K + 63) / 64 * 64 <= 8192; }

void prod_digits_build(Ctx &c, const double *A, int lda, int K, int cols, int col0, ProdDigits &pd, double *cm,
                       int ncm) {
    hipStream_t s = c.cur;
    pd.Kp = (K + 63) / 64 * 64;
    pd.col0 = col0;
    pd.cols = cols;
    // whole 64-column tiles (zero past cols); a product's row tiles start on a
    // tile (prod_i8_partials)
    const int cp = (cols + 63) / 64 * 64;
    pd.slice = (size_t)cp * pd.Kp;   // bytes of one digit over the image
    // A's image keeps the PD_ADIG digits the product reads (the
    // seventh was written and never read, n^2 bytes a PCA)
    char *base = c.buf[S_PDIGA].as<char>(PD_ADIG * pd.slice + (size_t)cp * sizeof(double) + 256);
    pd.d = (int8_t *)base;
    pd.rs = (double *)(base + (PD_ADIG * pd.slice + 255) / 256 * 256);
    pd.pending = 0;
    if (cm) {
        // columns [0, ncm) with their means now; [ncm, cp) by prod_digits_finish
        // once the caller has written those columns (m and 1 come from the means)
        if (!prod_digits_means_ok(K) || ncm < 1 || ncm > cols || col0 != 0)
            fail(TP_ERR_INTERNAL, "prod_digits_build: means only over the leading columns of a whole image (K >= 64)");
        launch_digits_cm(A, lda, K, 0, ncm, cols, pd, cm, ncm, s);
        pd.pending = ncm;
        return;
    }
    if (pd.Kp <= 1024 * PD_REG_IT)
        hipLaunchKernelGGL((k_pd_digits_reg<PD_REG_IT, PD_ADIG>), dim3((unsigned)cp), dim3(256), 0, s, A, lda, K, cols,
                           pd.Kp, (int8_t *)pd.d, (double *)pd.rs);
    else if (pd.Kp <= 4096 * 6 && cfg_pd_digits_big)   // one read of each long column (1024 threads)
        hipLaunchKernelGGL((k_pd_digits_reg<6, PD_ADIG, 1024>), dim3((unsigned)cp), dim3(1024), 0, s, A, lda, K, cols,
                           pd.Kp, (int8_t *)pd.d, (double *)pd.rs);
    else
        hipLaunchKernelGGL(k_pd_digits<PD_ADIG>, dim3((unsigned)cp), dim3(256), 0, s, A, lda, K, cols, pd.Kp,
                           (int8_t *)pd.d, (double *)pd.rs);
    TP_HIP(hipGetLastError());
}

void prod_digits_finish(Ctx &c, const double *A, int lda, int K, ProdDigits &pd) {
    if (pd.pending <= 0) return;
    const int cp = (pd.cols + 63) / 64 * 64;
    launch_digits_cm(A, lda, K, pd.pending, cp, pd.cols, pd, nullptr, 0, c.cur);
    pd.pending = 0;
}

// partials of rows [r0, r0 + M) (global column indices of A) of A'B into
// `work`: returns the chunk count; pstride = M N
int prod_i8_partials(Ctx &c, const ProdDigits &pd, int r0, int M, const double *B, int ldb, int N, int K,
                     DevBuf &work, double **part) {
    hipStream_t s = c.cur;
    if (!prod_i8_ok(K, N) || (K + 63) / 64 * 64 != pd.Kp || r0 < pd.col0 || r0 + M > pd.col0 + pd.cols ||
        (r0 - pd.col0) % 64 || pd.pending)
        fail(TP_ERR_INTERNAL, "prod_i8: rows outside the digit image or off its 64-column tiles, or an unsupported block");
    const size_t slb = (size_t)64 * pd.Kp;   // the image spaces k steps by whole 64-column tiles
    char *bb = c.buf[S_PDIGB].as<char>(PD_DIG * slb + 256 + 512 * sizeof(double) +
                                        (size_t)N * ((pd.Kp + 1023) / 1024) * sizeof(double));
    int8_t *Db = (int8_t *)bb;
    double *cs = (double *)(bb + (PD_DIG * slb + 255) / 256 * 256);
    const int SL = (pd.Kp + 1023) / 1024;
    double *pmax = (double *)(bb + (PD_DIG * slb + 255) / 256 * 256 + 512 * sizeof(double));
    if (pd.Kp <= 1024 * PD_REG_IT && cfg_pd_digits_blk) {   // one launch, a workgroup per (column, slice)
        hipLaunchKernelGGL((k_pd_digits_blk<PD_REG_IT, TP_PD_SPW>), dim3((unsigned)(N * ((SL + TP_PD_SPW - 1) / TP_PD_SPW))),
                           dim3(256), 0, s, B, ldb, K, N, pd.Kp, Db, cs);
    } else if (pd.Kp <= 1024 * PD_REG_IT) {   // one launch, the block read once
        hipLaunchKernelGGL((k_pd_digits_reg<PD_REG_IT, PD_DIG>), dim3((unsigned)N), dim3(256), 0, s, B, ldb, K, N, pd.Kp,
                           Db, cs);
    } else {
        hipLaunchKernelGGL(k_pd_colmax, dim3((unsigned)(N * SL)), dim3(256), 0, s, B, ldb, K, SL, pmax);
        hipLaunchKernelGGL(k_pd_digits_sl, dim3((unsigned)(N * SL)), dim3(256), 0, s, B, ldb, K, pd.Kp, SL, pmax, Db,
                           cs);
    }
    const int kc = pd_kchunk(pd.Kp);
    const int S = (pd.Kp + kc - 1) / kc;
    const size_t pstride = (size_t)M * N;
    *part = work.as<double>(pstride * S);
    const int8_t *Da = pd.d + (size_t)(r0 - pd.col0) * pd.Kp * PD_ADIG;   // whole tiles: 64 columns x Kp x PD_ADIG
    const double *rs = pd.rs + (r0 - pd.col0);
    const int tm = (M + 63) / 64;
    // one LDS buffer, two workgroups a CU (the double-buffered one-workgroup
    // form, the 128-row tiles and the LDS-DMA ring measured slower and were
    // removed in round 6)
    const dim3 ga((unsigned)((M + 127) / 128 * S));
    if (N == 32)
        hipLaunchKernelGGL((k_pd_prodA<1, 2>), ga, dim3(512), 0, s, Da, pd.Kp, M, Db, rs, cs, *part, pstride, kc);
    else if (t_knob.prod_i8 == 5)
        hipLaunchKernelGGL((k_pd_prodA<1, 4>), ga, dim3(512), 0, s, Da, pd.Kp, M, Db, rs, cs, *part, pstride, kc);
    else
        hipLaunchKernelGGL(k_pd_prod<1>, dim3((unsigned)(tm * S)), dim3(256), (size_t)PD_BUF, s, Da, pd.Kp, M, Db, rs,
                           cs, *part, pstride, kc);
    TP_HIP(hipGetLastError());
    return S;
}

}  // namespace tp
