// Symmetric eigendecomposition of the small b x b Rayleigh-Ritz matrix of the
// PCA (H = Q'GQ, b = block size, <= 1280: k <= 1024), the library's own
// kernels only (a rocSOLVER dsyevd spent hundreds of tiny launches in latrd).
//
//   k_sytrd_l   one 1024-thread workgroup reduces H to tridiagonal T = Q_H' H Q_H
//               (Householder, LAPACK dsytd2 'L' conventions: reflector j has
//               u[j+1] = 1, u[r] = A[r][j] for r >= j+2, stored in place).  The
//               rank-2 update of step j is applied lazily inside step j+1's pass
//               over the trailing lower triangle, fused with the product
//               p = A22 v of step j+1: one read + one write of the trailing
//               matrix per step (L2-resident), column dots by wave reductions,
//               row dots in per-lane registers (lane owns rows r = 64q + lane).
//   k_sytrd32   the same with the matrix in registers as 32 x 32 tiles (b <= 256).
//   k_bisect / k_invit  eigenpairs of T (Sturm bisection, inverse iteration).
//   k_ormtr_l   C <- Q_H C: one wave per column of C, reflectors applied in
//               reverse order with the column held in registers.
#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

constexpr int EIG_BMAX = 1280;   // b = k + oversampling for k <= 1024
constexpr int SY_WAVES = 16;

// QM = rows per lane (b <= 64 QM).  NPR rows of per-wave partials in LDS: 16
// (one per wave) up to QM = 10; for QM = 20 (b <= 1280) 8, the waves of the
// upper half adding theirs to the lower half's rows in a second round.
template <int QM, bool ST = false>
__global__ void __launch_bounds__(1024) k_sytrd_l(double *A, int b, double *d, double *e, double *tau,
                                                  long long *stamps = nullptr) {
    constexpr int BM = 64 * QM;
    constexpr int NPR = QM > 10 ? 8 : SY_WAVES;
    long long sacc[4] = {0, 0, 0, 0};
    long long st0 = ST ? (long long)__builtin_amdgcn_s_memtime() : 0;
#define SY_STAMP(ph)                                                      \
    if (ST) {                                                             \
        long long _t = (long long)__builtin_amdgcn_s_memtime();           \
        sacc[ph] += _t - st0;                                             \
        st0 = _t;                                                         \
    }
    __shared__ double V[2][BM], W[2][BM], PC[BM];
    __shared__ double PRW[NPR][BM];
    __shared__ double RED[SY_WAVES + 8];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    double vold[QM], wold[QM], vnew[QM], prow[QM], nxt[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) vold[q] = wold[q] = nxt[q] = 0.0;
    for (int r = t; r < BM; r += 1024) V[1][r] = W[1][r] = V[0][r] = W[0][r] = 0.0;
    __syncthreads();

    for (int j = 0; j + 2 < b; ++j) {
        const int P = j & 1;
        // ---- (a)+(b) wave 0: column j with the pending update of step j-1,
        //      then the reflector of column j (dlarfg)
        if (wv == 0) {
            const double uj = V[P ^ 1][j], wj = W[P ^ 1][j];
            double cur[QM];
            double xs = 0.0, al = 0.0;
#pragma unroll
            for (int q = 0; q < QM; ++q) {
                const int r = 64 * q + lane;
                cur[q] = 0.0;
                if (r >= j && r < b) {
                    // column j as left by the previous pass (wave 0 kept it), or memory at j = 0
                    double a = j == 0 ? A[(size_t)j * b + r] : nxt[q];
                    a = fma(-vold[q], wj, fma(-wold[q], uj, a));
                    cur[q] = a;
                    if (r == j) d[j] = a;
                    if (r == j + 1) al = a;
                    if (r >= j + 2) xs = fma(a, a, xs);
                }
            }
            const double xnorm2 = wave_sum(xs);
            const double alpha = readlane_d(al, (j + 1) & 63);   // the lane owning row j+1
            double beta, tj, scale;
            if (xnorm2 == 0.0) {
                beta = alpha;
                tj = 0.0;
                scale = 0.0;
            } else {
                beta = -copysign(sqrt(fma(alpha, alpha, xnorm2)), alpha);
                tj = (beta - alpha) / beta;
                scale = 1.0 / (alpha - beta);
            }
#pragma unroll
            for (int q = 0; q < QM; ++q) {
                const int r = 64 * q + lane;
                if (r < b) {
                    double v = 0.0;
                    if (r == j + 1) v = 1.0;
                    else if (r >= j + 2) {
                        v = cur[q] * scale;
                        A[(size_t)j * b + r] = v;
                    }
                    V[P][r] = v;
                }
            }
            if (lane == 0) {
                e[j] = beta;
                tau[j] = tj;
                RED[SY_WAVES] = tj;
            }
        }
        __syncthreads();
        SY_STAMP(0);
        const double tj = RED[SY_WAVES];
        // ---- (c) pass over the trailing lower triangle, columns c >= j+1:
        //      apply update j-1, accumulate p = A22 v_j
#pragma unroll
        for (int q = 0; q < QM; ++q) {
            vnew[q] = V[P][64 * q + lane];
            prow[q] = 0.0;
        }
        // columns c = j+1+wv+16k, four per batch: all loads of a batch are in
        // flight together (the pass is L2-latency bound otherwise)
        constexpr int U = QM <= 4 ? 4 : 2;
        for (int cb = j + 1 + wv; cb < b; cb += SY_WAVES * U) {
            double a[U][QM];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c = cb + SY_WAVES * u;
#pragma unroll
                for (int q = 0; q < QM; ++q) {
                    const int r = 64 * q + lane;
                    a[u][q] = (c < b && r >= c && r < b) ? A[(size_t)c * b + r] : 0.0;
                }
            }
            double pc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c = cb + SY_WAVES * u;
                pc[u] = 0.0;
                if (c < b) {
                    const double uc = V[P ^ 1][c], wc = W[P ^ 1][c], vc = V[P][c];
                    double *col = A + (size_t)c * b;
#pragma unroll
                    for (int q = 0; q < QM; ++q) {
                        const int r = 64 * q + lane;
                        if (r >= c && r < b) {
                            double x = fma(-vold[q], wc, fma(-wold[q], uc, a[u][q]));
                            a[u][q] = x;
                            if (c != j + 1) col[r] = x;   // column j+1 stays in wave 0's registers
                            prow[q] = fma(x, vc, prow[q]);
                            if (r > c) pc[u] = fma(x, vnew[q], pc[u]);
                        }
                    }
                }
            }
            if (wv == 0 && cb == j + 1) {
#pragma unroll
                for (int q = 0; q < QM; ++q) nxt[q] = a[0][q];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c = cb + SY_WAVES * u;
                const double ps = wave_sum(pc[u]);
                if (lane == 0 && c < b) PC[c] = ps;
            }
        }
        if (NPR == SY_WAVES || wv < NPR) {
#pragma unroll
            for (int q = 0; q < QM; ++q) PRW[wv][64 * q + lane] = prow[q];
        }
        if (NPR < SY_WAVES) {
            __syncthreads();
            if (wv >= NPR) {
#pragma unroll
                for (int q = 0; q < QM; ++q) PRW[wv - NPR][64 * q + lane] += prow[q];
            }
        }
        __syncthreads();
        SY_STAMP(1);
        // ---- (d) p = tau A22 v, alpha2 = -tau/2 p'v, w = p + alpha2 v (rows
        //      t, t + 1024, ... of this thread)
        constexpr int RT = (BM + 1023) / 1024;
        double p[RT], pv = 0.0;
#pragma unroll
        for (int u = 0; u < RT; ++u) {
            const int rr = t + 1024 * u;
            p[u] = 0.0;
            if (rr < b && rr >= j + 1) {
                double s = PC[rr];
#pragma unroll
                for (int w = 0; w < NPR; ++w) s = s + PRW[w][rr];
                p[u] = tj * s;
                pv = fma(p[u], V[P][rr], pv);
            }
        }
        pv = wave_sum(pv);
        if (lane == 0) RED[wv] = pv;
        __syncthreads();
        double dot = 0.0;
#pragma unroll
        for (int w = 0; w < SY_WAVES; ++w) dot = dot + RED[w];
        const double alpha2 = -0.5 * tj * dot;
#pragma unroll
        for (int u = 0; u < RT; ++u) {
            const int rr = t + 1024 * u;
            if (rr < BM) W[P][rr] = (rr < b && rr >= j + 1) ? fma(alpha2, V[P][rr], p[u]) : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < QM; ++q) {
            vold[q] = V[P][64 * q + lane];
            wold[q] = W[P][64 * q + lane];
        }
        SY_STAMP(2);
    }
    if (ST && threadIdx.x == 0)
        for (int q = 0; q < 3; ++q) stamps[q] = sacc[q];
#undef SY_STAMP
    // ---- last 2 x 2 block with the pending update, T entries.  Column b-2 was
    //      left in wave 0's registers by the last pass: write it back first.
    if (wv == 0 && b >= 3) {
#pragma unroll
        for (int q = 0; q < QM; ++q) {
            const int r = 64 * q + lane;
            if (r >= b - 2 && r < b) A[(size_t)(b - 2) * b + r] = nxt[q];
        }
    }
    __syncthreads();
    if (t == 0) {
        if (b >= 2) {
            const int j = b - 2;
            const int P = (b - 3) & 1;   // parity of the last reflector step (if any)
            double a00 = A[(size_t)j * b + j], a10 = A[(size_t)j * b + j + 1], a11 = A[(size_t)(j + 1) * b + j + 1];
            if (b >= 3) {
                const double v0 = V[P][j], v1 = V[P][j + 1], w0 = W[P][j], w1 = W[P][j + 1];
                a00 = a00 - (v0 * w0 + w0 * v0);
                a10 = a10 - (v1 * w0 + w1 * v0);
                a11 = a11 - (v1 * w1 + w1 * v1);
            }
            d[j] = a00;
            d[j + 1] = a11;
            e[j] = a10;
            tau[j] = 0.0;
        } else {
            d[0] = A[0];
        }
    }
}

// ---------------------------------------------------------------------------
// Lane-exchange helpers of the register-resident tridiagonalisation (k_sytrd32).
__device__ __forceinline__ double xor16_sum(double v) {   // v[l] + v[l ^ 16]
    int lo = __double2loint(v), hi = __double2hiint(v);
    auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double xor32_sum(double v) {   // v[l] + v[l ^ 32]
    int lo = __double2loint(v), hi = __double2hiint(v);
    auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double row16_sum(double v) {   // sum over the 16 lanes of a row
    v = v + dpp_d<0xB1>(v);
    v = v + dpp_d<0x4E>(v);
    v = v + dpp_d<0x141>(v);
    v = v + dpp_d<0x140>(v);
    return v;
}
// Re-materialise a wave-uniform value at each use (keeps the derived masks and
// addresses of every slot from staying live across the loop: no spills).
__device__ __forceinline__ int sy_opaque(int v) {
    v = __builtin_amdgcn_readfirstlane(v);
    asm volatile("" : "+s"(v));
    return v;
}

typedef double sy_d4 __attribute__((ext_vector_type(4)));


// ---------------------------------------------------------------------------
// k_sytrd32: the same reduction and outputs (LAPACK dsytd2 'L'), b <= 256,
// with the upper triangle in registers as 32 x 32 tiles and three barriers a
// step.  Built to cut the per-step cost of k_sytrd_reg (removed in round 6; ~14 k cycles: the
// 16 x 16 tiles need a 16-lane reduction per tile row, and wave 0 alone forms
// the reflector and assembles p in long LDS chains while 15 waves wait).
//
// Lane l of a tile holds the 4 x 4 block rows 4 ra .. 4 ra + 3, columns
// 4 cb .. 4 cb + 3 (ra = l & 7, cb = l >> 3), so a tile's row partials of
// p = A v reduce over lane bits 3..5 (row_ror:8, permlane16/32 swaps) and
// its column partials over bits 0..2 (quad perms, one swizzle), each as a
// reduce-scatter: 4 values -> 1 over three levels, 4 exchanges instead of 12.
// The 36 tiles of b = 256 are dealt round-robin to 12 waves in the order
// (tile row descending, column ascending): at every step the live tiles
// (tile row >= j / 32) are a prefix of that order, so each wave's live tiles
// are a prefix of its slots and the work stays balanced as it shrinks.
// Step j:
//   1. every wave forms the reflector from row j (published in LDS) -- no
//      barrier between the reflector and the product; wave 0 stores it and v;
//   2. per live tile, row and column partials of A v          -> LDS, B1
//   3. waves 0..3 sum the partials of p (fixed order), tau, p'v -> LDS, B2
//   4. w = p - (tau/2)(p'v) v; every live tile A -= v w' + w v'; the owners
//      of row j + 1 publish it                                         B0
// ST: diagnostic build with s_memtime stamps (phases 1..4 of wave 0).
// ---------------------------------------------------------------------------
constexpr int S32_W = 12;      // waves
constexpr int S32_SL = 3;      // tiles a wave: 36 of b = 256 over 12 waves

__device__ __forceinline__ double swap16_sum(double a, double b) {   // even rows: a + a[l^16]; odd: b + b[l^16]
    auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
    auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double swap32_sum(double a, double b) {   // lanes < 32: a + a[l^32]; else b + b[l^32]
    auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
    auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double swz_xor4(double v) {   // v[l ^ 4] (ds_swizzle bitmask mode)
    const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), 0x101F);
    const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), 0x101F);
    return __hiloint2double(hi, lo);
}

// 1 / x by the hardware reciprocal and two Newton steps (within an ulp or
// two: a reflector's scale and tau need no correct rounding)
__device__ __forceinline__ double rcp_nr(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = r * fma(-x, r, 2.0);
    return r * fma(-x, r, 2.0);
}

template <bool ST>
__global__ void __launch_bounds__(64 * S32_W) k_sytrd32(double *A, int b, double *d, double *e, double *tau,
                                                         long long *stamps) {
    __shared__ double xrow[256], vs[256], ps[256];
    __shared__ double rowp[8][8][32];   // [I][K][row of block I]: row partials of tile (I, K)
    __shared__ double colp[8][8][32];   // [I][K][column of block K]: column partials of tile (I, K), I < K
    __shared__ double pvp[4], fin[2];
    long long sacc[4] = {0, 0, 0, 0};
    long long st0 = ST ? (long long)__builtin_amdgcn_s_memtime() : 0;
#define S32_STAMP(ph)                                                     \
    if (ST) {                                                             \
        long long _t = (long long)__builtin_amdgcn_s_memtime();           \
        sacc[ph] += _t - st0;                                             \
        st0 = _t;                                                         \
    }
    const int t = threadIdx.x, l = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int ra = l & 7, cb = l >> 3;
    const int bp = (b + 31) & ~31, T = bp >> 5;
    const int ntile = T * (T + 1) / 2;
    // slot s of wave w: list index s * S32_W + w, list = tile rows descending,
    // columns ascending; row I holds indices [N(I+1), N(I)), N(I) = (T-I)(T-I+1)/2
    int tI[S32_SL], tK[S32_SL];
#pragma unroll
    for (int s = 0; s < S32_SL; ++s) {
        int id = s * S32_W + w, I = T - 1, cnt = 1;
        if (id < ntile) {
            while (id >= cnt) {
                id -= cnt;
                --I;
                ++cnt;
            }
            tI[s] = __builtin_amdgcn_readfirstlane(I);
            tK[s] = __builtin_amdgcn_readfirstlane(I + id);
        } else {
            tI[s] = -1;
            tK[s] = -1;
        }
    }
    // re-materialised at each use: keeps per-slot addresses from being hoisted
    // out of the step loop (and spilled)
#define S32_I(s) sy_opaque(tI[s])
#define S32_K(s) sy_opaque(tK[s])
    for (int q = t; q < 256; q += 64 * S32_W) xrow[q] = vs[q] = ps[q] = 0.0;
    for (int q = t; q < 8 * 8 * 32; q += 64 * S32_W) (&rowp[0][0][0])[q] = (&colp[0][0][0])[q] = 0.0;
    __syncthreads();
    double x[S32_SL][4][4];
#pragma unroll
    for (int s = 0; s < S32_SL; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int R = 32 * tI[s] + 4 * ra + i, C = 32 * tK[s] + 4 * cb + k;
                x[s][i][k] = (tI[s] >= 0 && R < b && C < b) ? A[(size_t)min(R, C) * b + max(R, C)] : 0.0;
            }
    // row 0 -> LDS (tile row 0 = the tail of the list)
#pragma unroll
    for (int s = 0; s < S32_SL; ++s)
        if (tI[s] == 0 && ra == 0)
#pragma unroll
            for (int k = 0; k < 4; ++k) xrow[32 * tK[s] + 4 * cb + k] = x[s][0][k];
    __syncthreads();   // every load of A done before reflectors overwrite it
    const bool h0 = l & 1, h1 = l & 2, h3 = l & 8, h4 = l & 16;

    for (int j = 0; j + 2 < b; ++j) {
        const int J = j >> 5;
        const int nlive = (T - J) * (T - J + 1) / 2;
        // ---- 1. reflector (dlarfg) from row j, every wave: v for this lane's
        //      four positions -> LDS (every wave writes the same words; a wave
        //      then reads back its own writes, in order: no barrier)
        double xv[4];
        {
            const double2 a0 = *(const double2 *)&xrow[4 * l], a1 = *(const double2 *)&xrow[4 * l + 2];
            xv[0] = a0.x; xv[1] = a0.y; xv[2] = a1.x; xv[3] = a1.y;
        }
        const double alpha = xrow[j + 1];
        double sq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) sq[u] = (4 * l + u >= j + 2 && 4 * l + u < b) ? xv[u] * xv[u] : 0.0;
        const double xnorm2 = wave_sum((sq[0] + sq[1]) + (sq[2] + sq[3]));
        double beta, tj, scale;
        if (xnorm2 == 0.0) {
            beta = alpha;
            tj = 0.0;
            scale = 0.0;
        } else {
            beta = -copysign(sqrt(fma(alpha, alpha, xnorm2)), alpha);
            tj = (beta - alpha) * rcp_nr(beta);
            scale = rcp_nr(alpha - beta);
        }
        double vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = 4 * l + u;
            vv[u] = c == j + 1 ? 1.0 : ((c > j + 1 && c < b) ? xv[u] * scale : 0.0);
        }
        *(double2 *)&vs[4 * l] = make_double2(vv[0], vv[1]);
        *(double2 *)&vs[4 * l + 2] = make_double2(vv[2], vv[3]);
        if (w == 0) {
            // column j of A below the diagonal <- v (rows <= j + 1 get 0 / 1:
            // the reflector's implicit entries, never read back; every input
            // element was loaded before the loop)
            if (4 * l + 3 < b && (b & 1) == 0) {
                *(double2 *)&A[(size_t)j * b + 4 * l] = make_double2(vv[0], vv[1]);
                *(double2 *)&A[(size_t)j * b + 4 * l + 2] = make_double2(vv[2], vv[3]);
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (4 * l + u < b) A[(size_t)j * b + 4 * l + u] = vv[u];
            }
            if (l == 0) {
                d[j] = xrow[j];
                e[j] = beta;
                tau[j] = tj;
            }
        }
        S32_STAMP(0);
        // ---- 2. partials of A v over the live tiles
#pragma unroll
        for (int s = 0; s < S32_SL; ++s) {
            if (s * S32_W + w < nlive) {
                const int I = S32_I(s), K = S32_K(s);
                const int r0 = 32 * I + 4 * ra, c0 = 32 * K + 4 * cb;
                double vr[4], vc[4];
                {
                    const double2 a0 = *(const double2 *)&vs[r0], a1 = *(const double2 *)&vs[r0 + 2];
                    const double2 b0 = *(const double2 *)&vs[c0], b1 = *(const double2 *)&vs[c0 + 2];
                    vr[0] = a0.x; vr[1] = a0.y; vr[2] = a1.x; vr[3] = a1.y;
                    vc[0] = b0.x; vc[1] = b0.y; vc[2] = b1.x; vc[3] = b1.y;
                }
                double rp[4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    rp[i] = fma(x[s][i][3], vc[3], fma(x[s][i][2], vc[2], fma(x[s][i][1], vc[1], x[s][i][0] * vc[0])));
                {   // reduce-scatter over cb (lane bits 3, 4, 5)
                    const double s0 = h3 ? rp[0] : rp[2], s1 = h3 ? rp[1] : rp[3];
                    const double k0 = h3 ? rp[2] : rp[0], k1 = h3 ? rp[3] : rp[1];
                    const double t0 = k0 + dpp_d<0x128>(s0), t1 = k1 + dpp_d<0x128>(s1);
                    const double u = swap16_sum(t0, t1);
                    const double tot = swap32_sum(u, u);
                    if (l < 32) rowp[I][K][4 * ra + (h3 ? 2 : 0) + (h4 ? 1 : 0)] = tot;
                }
                if (I != K) {
                    double cp[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        cp[k] = fma(x[s][3][k], vr[3], fma(x[s][2][k], vr[2], fma(x[s][1][k], vr[1], x[s][0][k] * vr[0])));
                    // reduce-scatter over ra (lane bits 0, 1, 2)
                    const double s0 = h0 ? cp[0] : cp[2], s1 = h0 ? cp[1] : cp[3];
                    const double k0 = h0 ? cp[2] : cp[0], k1 = h0 ? cp[3] : cp[1];
                    const double t0 = k0 + dpp_d<0xB1>(s0), t1 = k1 + dpp_d<0xB1>(s1);
                    const double sx = h1 ? t0 : t1, kx = h1 ? t1 : t0;
                    const double u = kx + dpp_d<0x4E>(sx);
                    const double tot = u + swz_xor4(u);
                    if ((l & 4) == 0) colp[I][K][4 * cb + (h0 ? 2 : 0) + (h1 ? 1 : 0)] = tot;
                }
            }
        }
        lds_barrier();   // B1
        S32_STAMP(1);
        // ---- 3. p = tau A22 v (0 at c <= j), p'v: waves 0..3, one position a
        //      lane; the T - J terms of block m in a fixed order (row partials of
        //      tiles (m, m..T-1), then column partials of tiles (J..m-1, m)),
        //      all loads issued at once
        if (w < 4) {
            const int c = 64 * w + l, m = c >> 5, r = c & 31;
            double tv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int K = m + q, I = J + (q - (T - m));
                tv[q] = K < T ? rowp[m][K][r] : (I < m ? colp[I & 7][m][r] : 0.0);
            }
            const double sum = ((tv[0] + tv[1]) + (tv[2] + tv[3])) + ((tv[4] + tv[5]) + (tv[6] + tv[7]));
            const double p = (c > j && m >= J) ? tj * sum : 0.0;
            ps[c] = p;
            const double pv = wave_sum(p * vs[c]);
            if (l == 0) pvp[w] = pv;
        }
        lds_barrier();   // B2
        S32_STAMP(2);
        // ---- 4. w = p + alpha2 v; A -= v w' + w v' on the live tiles
        const double alpha2 = -0.5 * tj * (((pvp[0] + pvp[1]) + pvp[2]) + pvp[3]);
#pragma unroll
        for (int s = 0; s < S32_SL; ++s) {
            if (s * S32_W + w < nlive) {
                const int r0 = 32 * S32_I(s) + 4 * ra, c0 = 32 * S32_K(s) + 4 * cb;
                double vr[4], vc[4], wr[4], wc[4];
                {
                    const double2 a0 = *(const double2 *)&vs[r0], a1 = *(const double2 *)&vs[r0 + 2];
                    const double2 b0 = *(const double2 *)&vs[c0], b1 = *(const double2 *)&vs[c0 + 2];
                    const double2 p0 = *(const double2 *)&ps[r0], p1 = *(const double2 *)&ps[r0 + 2];
                    const double2 q0 = *(const double2 *)&ps[c0], q1 = *(const double2 *)&ps[c0 + 2];
                    vr[0] = a0.x; vr[1] = a0.y; vr[2] = a1.x; vr[3] = a1.y;
                    vc[0] = b0.x; vc[1] = b0.y; vc[2] = b1.x; vc[3] = b1.y;
                    wr[0] = fma(alpha2, vr[0], p0.x); wr[1] = fma(alpha2, vr[1], p0.y);
                    wr[2] = fma(alpha2, vr[2], p1.x); wr[3] = fma(alpha2, vr[3], p1.y);
                    wc[0] = fma(alpha2, vc[0], q0.x); wc[1] = fma(alpha2, vc[1], q0.y);
                    wc[2] = fma(alpha2, vc[2], q1.x); wc[3] = fma(alpha2, vc[3], q1.y);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int k = 0; k < 4; ++k) x[s][i][k] = fma(-vr[i], wc[k], fma(-wr[i], vc[k], x[s][i][k]));
            }
        }
        // ---- publish row j + 1 (its tile row's owners)
        {
            const int j1 = j + 1, J1 = j1 >> 5, rr = j1 & 31;
#pragma unroll
            for (int s = 0; s < S32_SL; ++s) {
                if (S32_I(s) == J1 && ra == (rr >> 2)) {
                    const int c0 = 32 * S32_K(s) + 4 * cb;
                    double y[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) y[k] = (rr & 3) == 0 ? x[s][0][k] : ((rr & 3) == 1 ? x[s][1][k] : ((rr & 3) == 2 ? x[s][2][k] : x[s][3][k]));
                    *(double2 *)&xrow[c0] = make_double2(y[0], y[1]);
                    *(double2 *)&xrow[c0 + 2] = make_double2(y[2], y[3]);
                }
            }
        }
        lds_barrier();   // B0
        S32_STAMP(3);
    }
    // ---- the last 2 x 2 block: row b-2 is in LDS, A[b-1][b-1] from its owner
    {
        const int rl = b - 1, I = rl >> 5, rr = rl & 31;
#pragma unroll
        for (int s = 0; s < S32_SL; ++s)
            if (tI[s] == I && tK[s] == I && ra == (rr >> 2) && cb == (rr >> 2))
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (i == (rr & 3)) fin[0] = x[s][i][i];
    }
    __syncthreads();
    if (t == 0) {
        if (b >= 2) {
            d[b - 2] = xrow[b - 2];
            d[b - 1] = fin[0];
            e[b - 2] = xrow[b - 1];
            tau[b - 2] = 0.0;
        } else {
            d[0] = xrow[0];
        }
    }
    if (ST && t == 0)
        for (int q = 0; q < 4; ++q) stamps[q] = sacc[q];
#undef S32_STAMP
#undef S32_I
#undef S32_K
}
bool sytrd32_supported(int b) { return b >= 3 && b <= 256; }

// C <- Q_H C, Q_H = H_0 H_1 ... H_{b-3}: one wave per column of C (b x b, ldc = b)
template <int QM>
__global__ void __launch_bounds__(256) k_ormtr_l(const double *A, const double *tau, int b, double *C) {
    const int lane = threadIdx.x & 63;
    const int col = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (col >= b) return;
    double x[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) {
        const int r = 64 * q + lane;
        x[q] = r < b ? C[(size_t)col * b + r] : 0.0;
    }
    // reflector j's vector is loaded one iteration ahead (latency hidden)
    auto load_u = [&](double (&u)[QM], int j) {
#pragma unroll
        for (int q = 0; q < QM; ++q) {
            const int r = 64 * q + lane;
            u[q] = (r == j + 1) ? 1.0 : ((r >= j + 2 && r < b) ? A[(size_t)j * b + r] : 0.0);
        }
    };
    double un[QM];
    double tn = 0.0;
    if (b >= 3) {
        load_u(un, b - 3);
        tn = tau[b - 3];
    }
    for (int j = b - 3; j >= 0; --j) {
        double u[QM];
#pragma unroll
        for (int q = 0; q < QM; ++q) u[q] = un[q];
        const double tj = tn;
        if (j > 0) {
            load_u(un, j - 1);
            tn = tau[j - 1];
        }
        if (tj == 0.0) continue;
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < QM; ++q) s = fma(u[q], x[q], s);
        s = wave_sum(s) * tj;
#pragma unroll
        for (int q = 0; q < QM; ++q) x[q] = fma(-s, u[q], x[q]);
    }
#pragma unroll
    for (int q = 0; q < QM; ++q) {
        const int r = 64 * q + lane;
        if (r < b) C[(size_t)col * b + r] = x[q];
    }
}

// ---------------------------------------------------------------------------
// Eigenpairs of the symmetric tridiagonal T (d, e) without rocSOLVER:
//   k_bisect: one wave per eigenvalue index, 64-section per step (each lane one
//     Sturm count, the first lane whose count exceeds the index brackets it):
//     6 bits per step, ~10 steps to 2 ulp.  Gershgorin interval, LAPACK pivmin.
//   k_invit: inverse iteration (LAPACK dstein scheme) one wave per vector:
//     LU with partial pivoting of T - sigma I and the solves by lane 0 in LDS,
//     2 iterations from a deterministic pseudo-random start (the shift is a
//     2-ulp eigenvalue: one solve already converges); eigenvalues
//     closer than ctol = 1e-7 ||T|| form a cluster whose first wave computes
//     all members, modified Gram-Schmidt against earlier members every
//     iteration.  theta = Rayleigh quotient of the final vector.
struct TriNorm {
    double lo, hi, tnorm, pivmin;
};

__device__ TriNorm tri_bounds(const double *d, const double *e, int b, double *sd, double *se, double *red) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, nw = blockDim.x >> 6;
    double lo = 1e308, hi = -1e308, em = 0.0;
    for (int i = t; i < b; i += blockDim.x) {
        const double di = d[i];
        const double el = i > 0 ? fabs(e[i - 1]) : 0.0, er = i + 1 < b ? fabs(e[i]) : 0.0;
        sd[i] = di;
        se[i] = i + 1 < b ? e[i] : 0.0;
        lo = fmin(lo, di - el - er);
        hi = fmax(hi, di + el + er);
        em = fmax(em, er * er);
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o, 64));
        hi = fmax(hi, __shfl_xor(hi, o, 64));
        em = fmax(em, __shfl_xor(em, o, 64));
    }
    if (lane == 0) {
        red[wv] = lo;
        red[8 + wv] = hi;
        red[16 + wv] = em;
    }
    __syncthreads();
    for (int w = 0; w < nw; ++w) {
        lo = fmin(lo, red[w]);
        hi = fmax(hi, red[8 + w]);
        em = fmax(em, red[16 + w]);
    }
    TriNorm r;
    r.tnorm = fmax(fabs(lo), fabs(hi));
    r.pivmin = 2.2250738585072014e-308 * fmax(1.0, em);
    const double fudge = 2.0 * 2.220446049250313e-16 * r.tnorm * (double)b + 4.0 * r.pivmin;
    r.lo = lo - fudge;
    r.hi = hi + fudge;
    return r;
}

// se2 = e^2.  1/q by the hardware reciprocal + two Newton steps (a Sturm count
// tolerates a last-bit error in the quotient: it is the count of a matrix a
// few ulps away, as LAPACK's own pivmin guard already assumes).
__device__ __forceinline__ int sturm_count(const double *sd, const double *se2, int b, double x, double pivmin) {
    int cnt = 0;
    double q = sd[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
#pragma unroll 4
    for (int i = 1; i < b; ++i) {
        double r = __builtin_amdgcn_rcp(q);
        r = r * fma(-q, r, 2.0);
        r = r * fma(-q, r, 2.0);
        q = (sd[i] - x) - se2[i - 1] * r;
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
    }
    return cnt;
}

// lam[idx] = idx-th smallest eigenvalue (midpoint of a ~2-ulp bracket);
// lam[b] = ||T|| bound (Gershgorin), written by block 0.
__global__ void __launch_bounds__(256) k_bisect(const double *d, const double *e, int b, double *lam) {
    __shared__ double sd[EIG_BMAX], se[EIG_BMAX], red[32];   // 20 KB at EIG_BMAX = 1280
    const TriNorm tn = tri_bounds(d, e, b, sd, se, red);
    for (int i = threadIdx.x; i + 1 < b; i += blockDim.x) se[i] = se[i] * se[i];   // e^2 for the counts
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (blockIdx.x == 0 && threadIdx.x == 0) lam[b] = tn.tnorm;
    if (idx >= b) return;
    double lo = tn.lo, hi = tn.hi;
    for (int it = 0; it < 40; ++it) {
        const double width = hi - lo;
        if (!(width > fmax(4.440892098500626e-16 * fmax(fabs(lo), fabs(hi)), 2.0 * tn.pivmin))) break;
        const double x = lo + width * ((double)(lane + 1) * (1.0 / 65.0));
        const int cnt = sturm_count(sd, se, b, x, tn.pivmin);
        const unsigned long long m = __ballot(cnt > idx);
        if (m == 0ULL) {
            lo = readlane_d(x, 63);
        } else {
            const int f = (int)__builtin_ctzll(m);
            const double xf = readlane_d(x, f);
            if (f > 0) lo = readlane_d(x, f - 1);
            hi = xf;
        }
    }
    if (lane == 0) lam[idx] = 0.5 * (lo + hi);
}

__device__ __forceinline__ double hash_unit(unsigned int m, unsigned int i) {
    uint64_t z = 0x9E3779B97F4A7C15ULL * ((uint64_t)m * 1000003ULL + i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

// Z (b x b, column m = eigenvector m), theta[m] = Rayleigh quotient.  dd holds
// the reciprocal pivots of U.  NV vectors (waves) per workgroup, b <= BM: 4 for
// b <= 640, 1 above (the LU factors of one vector take 5 BM doubles of LDS).
template <int BM, int NV>
__global__ void __launch_bounds__(64 * NV) k_invit(const double *d, const double *e, int b, const double *lam,
                                                   double *Z, double *theta) {
    __shared__ double sd[BM], se[BM];
    __shared__ double dd[NV][BM], du[NV][BM], du2[NV][BM], dl[NV][BM], xv[NV][BM];
    __shared__ unsigned char swp[NV][BM];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int i = t; i < b; i += 64 * NV) {
        sd[i] = d[i];
        se[i] = i + 1 < b ? e[i] : 0.0;
    }
    __syncthreads();
    const int idx = blockIdx.x * NV + wv;
    if (idx >= b) return;
    const double tnorm = lam[b];
    const double eps = 2.220446049250313e-16;
    const double ctol = 1e-7 * tnorm;
    if (idx > 0 && lam[idx] - lam[idx - 1] <= ctol) return;   // a member: its leader computes it
    int last = idx;
    while (last + 1 < b && lam[last + 1] - lam[last] <= ctol) ++last;
    double *x = xv[wv];
    double sig_prev = 0.0;
    for (int m = idx; m <= last; ++m) {
        double sig = lam[m];
        if (m > idx && sig - sig_prev < 10.0 * eps * fabs(sig)) sig = sig_prev + 10.0 * eps * fmax(fabs(sig), tnorm * eps);
        sig_prev = sig;
        // ---- LU with partial pivoting of T - sig I (dgttrf), lane 0
        if (lane == 0) {
            const double tiny = eps * tnorm + 1e-300;
            double cd = sd[0] - sig;                 // current diagonal
            double cu = b > 1 ? se[0] : 0.0;         // current superdiagonal
            for (int i = 0; i + 1 < b; ++i) {
                const double sub = se[i];            // T(i+1, i)
                const double nd = sd[i + 1] - sig;   // T(i+1, i+1)
                const double nu = i + 2 < b ? se[i + 1] : 0.0;   // T(i+1, i+2)
                if (fabs(cd) >= fabs(sub)) {
                    const double piv = cd != 0.0 ? cd : tiny;
                    const double f = sub / piv;
                    dd[wv][i] = 1.0 / piv;
                    du[wv][i] = cu;
                    du2[wv][i] = 0.0;
                    dl[wv][i] = f;
                    swp[wv][i] = 0;
                    cd = nd - f * cu;
                    cu = nu;
                } else {
                    const double f = cd / sub;
                    dd[wv][i] = 1.0 / sub;
                    du[wv][i] = nd;
                    du2[wv][i] = nu;
                    dl[wv][i] = f;
                    swp[wv][i] = 1;
                    cd = cu - f * nd;
                    cu = -f * nu;
                }
            }
            dd[wv][b - 1] = 1.0 / (cd != 0.0 ? cd : tiny);
        }
        // ---- start vector
        for (int i = lane; i < b; i += 64) x[i] = hash_unit((unsigned)m, (unsigned)i);
        for (int it = 0; it < 2; ++it) {
            // scale to max-norm 1, then solve L U x = y (lane 0)
            double mx = 0.0;
            for (int i = lane; i < b; i += 64) mx = fmax(mx, fabs(x[i]));
            for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
            const double inv = mx > 0.0 ? 1.0 / mx : 1.0;
            for (int i = lane; i < b; i += 64) x[i] *= inv;
            if (lane == 0) {
                for (int i = 0; i + 1 < b; ++i) {
                    double yi = x[i], yn = x[i + 1];
                    if (swp[wv][i]) {
                        const double tmp = yi;
                        yi = yn;
                        yn = tmp;
                        x[i] = yi;
                    }
                    x[i + 1] = yn - dl[wv][i] * yi;
                }
                double x2 = 0.0, x1 = x[b - 1] * dd[wv][b - 1];
                x[b - 1] = x1;
                for (int i = b - 2; i >= 0; --i) {
                    const double xi = (x[i] - du[wv][i] * x1 - du2[wv][i] * x2) * dd[wv][i];
                    x[i] = xi;
                    x2 = x1;
                    x1 = xi;
                }
            }
            // MGS against the earlier cluster members, then normalise
            for (int p = idx; p < m; ++p) {
                double s = 0.0;
                for (int i = lane; i < b; i += 64) s = fma(Z[(size_t)p * b + i], x[i], s);
                s = wave_sum(s);
                for (int i = lane; i < b; i += 64) x[i] = fma(-s, Z[(size_t)p * b + i], x[i]);
            }
            double nn = 0.0;
            for (int i = lane; i < b; i += 64) nn = fma(x[i], x[i], nn);
            nn = wave_sum(nn);
            const double rn = 1.0 / sqrt(nn);
            for (int i = lane; i < b; i += 64) x[i] *= rn;
        }
        // ---- store, Rayleigh quotient
        double rq = 0.0;
        for (int i = lane; i < b; i += 64) {
            const double xi = x[i];
            double tx = sd[i] * xi;
            if (i > 0) tx = fma(se[i - 1], x[i - 1], tx);
            if (i + 1 < b) tx = fma(se[i], x[i + 1], tx);
            rq = fma(xi, tx, rq);
            Z[(size_t)m * b + i] = xi;
        }
        rq = wave_sum(rq);
        if (lane == 0) theta[m] = rq;
    }
}

bool eig_sym_supported(int b) { return b >= 1 && b <= EIG_BMAX; }

// In place: A (b x b, lower triangle of a symmetric matrix) <- eigenvectors,
// theta <- eigenvalues ascending, b <= EIG_BMAX (1280: k <= 1024).  work: >=
// b*b + 4*b + 8 doubles.  Tridiagonalisation (register-resident for b <= 256 a
// multiple of 16, else L2-resident), Sturm bisection + inverse iteration,
// back-transformation -- the library's own kernels only (no rocSOLVER).
void eig_sym(double *A, int b, double *theta, double *work, hipStream_t s) {
    if (!eig_sym_supported(b)) fail(TP_ERR_UNSUPPORTED, "eig_sym: b > 1280 (EIG_BMAX)");
    double *C = work, *e = C + (size_t)b * b, *tau = e + b, *dg = tau + b, *lam = dg + b;   // lam: b + 1
    if (sytrd32_supported(b))
        hipLaunchKernelGGL((k_sytrd32<false>), dim3(1), dim3(64 * S32_W), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    else if (b <= 256)
        hipLaunchKernelGGL((k_sytrd_l<4, false>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    else if (b <= 512)
        hipLaunchKernelGGL((k_sytrd_l<8, false>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    else if (b <= 640)
        hipLaunchKernelGGL((k_sytrd_l<10, false>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    else
        hipLaunchKernelGGL((k_sytrd_l<20, false>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    TP_HIP(hipGetLastError());
    {
        const unsigned g = (unsigned)((b + 3) / 4);
        hipLaunchKernelGGL(k_bisect, dim3(g), dim3(256), 0, s, dg, e, b, lam);
        if (b <= 640)
            hipLaunchKernelGGL((k_invit<640, 4>), dim3(g), dim3(256), 0, s, dg, e, b, lam, C, theta);
        else
            hipLaunchKernelGGL((k_invit<EIG_BMAX, 1>), dim3((unsigned)b), dim3(64), 0, s, dg, e, b, lam, C, theta);
        TP_HIP(hipGetLastError());
    }
    if (b <= 256)
        hipLaunchKernelGGL(k_ormtr_l<4>, dim3((b + 3) / 4), dim3(256), 0, s, A, tau, b, C);
    else if (b <= 512)
        hipLaunchKernelGGL(k_ormtr_l<8>, dim3((b + 3) / 4), dim3(256), 0, s, A, tau, b, C);
    else if (b <= 640)
        hipLaunchKernelGGL(k_ormtr_l<10>, dim3((b + 3) / 4), dim3(256), 0, s, A, tau, b, C);
    else
        hipLaunchKernelGGL(k_ormtr_l<20>, dim3((b + 3) / 4), dim3(256), 0, s, A, tau, b, C);
    TP_HIP(hipGetLastError());
    TP_HIP(hipMemcpyAsync(A, C, (size_t)b * b * sizeof(double), hipMemcpyDeviceToDevice, s));
}

// diagnostic: one tridiagonalisation by either kernel (which: 0 k_sytrd_l, 2 k_sytrd32)
void sytrd_which(double *A, int b, double *work, int which, hipStream_t s, long long *d_stamps) {
    double *e = work, *tau = e + b, *dg = tau + b;
    (void)d_stamps;
    if (which == 2) {
        if (!sytrd32_supported(b)) fail(TP_ERR_ARG, "k_sytrd32: b must be 3..256");
        hipLaunchKernelGGL((k_sytrd32<false>), dim3(1), dim3(64 * S32_W), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    } else if (which == 1) {
        fail(TP_ERR_ARG, "k_sytrd_reg (which 1) was removed in round 6 (k_sytrd32 replaced it)");
    } else if (b <= 256) {
        hipLaunchKernelGGL((k_sytrd_l<4, false>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    } else if (b <= 512) {
        hipLaunchKernelGGL((k_sytrd_l<8, false>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    } else {
        hipLaunchKernelGGL((k_sytrd_l<10, false>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, (long long *)nullptr);
    }
    TP_HIP(hipGetLastError());
}
// diagnostic: the tridiagonalisation alone with per-phase cycle stamps
// (k_sytrd32 for b <= 256: 0 reflector, 1 partials + B1, 2 p + B2, 3 update +
// publish + B0; k_sytrd_l above: 0 reflector, 1 trailing pass, 2 p/w combine)
void sytrd_stamped(double *A, int b, double *work, long long *d_stamps, hipStream_t s) {
    double *e = work, *tau = e + b, *dg = tau + b;
    if (sytrd32_supported(b))
        hipLaunchKernelGGL((k_sytrd32<true>), dim3(1), dim3(64 * S32_W), 0, s, A, b, dg, e, tau, d_stamps);
    else if (b <= 256)
        hipLaunchKernelGGL((k_sytrd_l<4, true>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, d_stamps);
    else
        hipLaunchKernelGGL((k_sytrd_l<8, true>), dim3(1), dim3(1024), 0, s, A, b, dg, e, tau, d_stamps);
    TP_HIP(hipGetLastError());
}

}  // namespace tp
