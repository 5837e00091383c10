// Small dense kernels for the PCA's CholQR orthonormalisation Q = Z R^{-1}:
//   k_chol: one 512-thread workgroup computes U = chol(W + s I) (upper,
//     W = U'U) for b <= 480, blocked by 32: diagonal block factored by one wave
//     in LDS, panel solved in registers, trailing matrix updated in global
//     memory (L2-resident) by 64x64 macro tiles with 4x4 register micro tiles.
//     Also writes rdiag[j] = 1 / U_jj.  W is Jacobi-scaled to unit diagonal
//     first (so columns of very different norm -- a Chebyshev-filtered block --
//     factor as well as the normalised block), and the shift s = rel on that
//     unit diagonal keeps ill-conditioned blocks positive definite (shifted
//     CholQR).
//   k_trsm_ru: Q = Z U^{-1} (right, upper), one workgroup per 16 rows of Z,
//     16-column blocks of U staged in LDS; spreads the O(n b^2) solve over
//     n/16 workgroups.
// These replace potrf + trsm library calls whose dozens of tiny launches
// dominated the PCA.
#include <utility>

#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

constexpr int NB = 32;
constexpr int BMAX = 480;       // the panel in LDS
constexpr int BMAX_BIG = 1280;  // PG: the panel in global scratch (L2), b up to 1280 (k <= 1024)
constexpr int NT = 512;   // threads of k_chol: 8 waves, 256 VGPRs each

// PG: the 32-row panel lives in global scratch Pg (ld b + 8) instead of LDS
template <bool STAMPS, bool PG = false>
__global__ void __launch_bounds__(NT) k_chol_t(double *W, double *rdiag, int b, double rel, int *info,
                                               long long *stamps, double *Pg = nullptr) {
    long long st_acc[4] = {0, 0, 0, 0};
    long long st_t0 = STAMPS ? (long long)__builtin_amdgcn_s_memtime() : 0;
#define TP_STAMP(ph)                                                      \
    if (STAMPS) {                                                         \
        long long _t = (long long)__builtin_amdgcn_s_memtime();           \
        st_acc[ph] += _t - st_t0;                                         \
        st_t0 = _t;                                                       \
    }
    __shared__ double D[NB][NB + 1];       // factored diagonal block U_pp
    __shared__ double rd[NB];              // 1 / diag(U_pp)
    __shared__ double prow[NB];            // pivot row broadcast (wave 0)
    __shared__ double Psh[PG ? 1 : NB][PG ? 1 : BMAX + 8];   // panel U[o:o+32, o+32:b]
    __shared__ double scl[PG ? BMAX_BIG : BMAX];             // diag(W)^-1/2
    double *const Pp = PG ? Pg : &Psh[0][0];
    const int pld = PG ? b + 8 : BMAX + 8;
#define P(r, c) Pp[(size_t)(r) * pld + (c)]
    const int t = threadIdx.x;
    const int T = b / NB;
    // ---- Jacobi scaling (van der Sluis): factor W' = S W S, S = diag(W)^-1/2,
    //      so the filtered block's column-norm spread does not reach the pivots;
    //      shift s = rel on the unit diagonal.  U = U' S^-1 at the end.
    for (int j = t; j < b; j += NT) {
        const double dj = W[(size_t)j * b + j];
        scl[j] = dj > 0.0 ? 1.0 / sqrt(dj) : 1.0;
    }
    if (t == 0) *info = 0;
    __syncthreads();
    for (int col = t >> 6; col < b; col += NT / 64) {
        const double sc = scl[col];
        for (int r = t & 63; r <= col; r += 64) {
            double v = W[(size_t)col * b + r] * (scl[r] * sc);
            if (r == col) v += rel;
            W[(size_t)col * b + r] = v;
        }
    }
    __syncthreads();
    TP_STAMP(3);

    for (int p = 0; p < T; ++p) {
        const int o = p * NB;
        // (a) 32 x 32 diagonal block by wave 0: lane l owns row r = l & 31 at
        //     columns c = (l >> 5) + 2m, m < 16, in registers; the pivot row is
        //     broadcast through LDS (one wave barrier per step)
        if (t < 64) {
            const int r = t & 31, cp = t >> 5;
            double d[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int c = cp + 2 * m;
                d[m] = (c >= r) ? W[(size_t)(o + c) * b + o + r] : 0.0;
            }
            // Entries left of the diagonal (c < r) carry garbage after the
            // first steps; they are never read for c < j and never stored.
            for (int j = 0; j < NB; ++j) {
                if (r == j) {
#pragma unroll
                    for (int m = 0; m < 16; ++m) prow[cp + 2 * m] = d[m];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                double dj = prow[j];
                if (!(dj > 0.0)) {
                    if (t == 0) atomicOr(info, 1);
                    dj = 1e-300;
                }
                // 1/sqrt(dj): hardware estimate + one Newton step (<= 1-2 ulp:
                // fine for an orthonormalisation the next pass cleans up)
                double rp = __builtin_amdgcn_rsq(dj);
                rp = rp * fma(-0.5 * dj * rp, rp, 1.5);
                const double f = (r > j) ? prow[r] * (rp * rp) : 0.0;   // U(j,r) / piv, 0: no-op
                const double sc = (r == j) ? rp : 1.0;           // row j: D[j][c] / piv
#pragma unroll
                for (int m = 0; m < 16; ++m) d[m] = fma(-f, prow[cp + 2 * m], d[m]) * sc;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int c = cp + 2 * m;
                D[r][c] = (c >= r) ? d[m] : 0.0;
                if (c >= r) W[(size_t)(o + c) * b + o + r] = d[m];
                if (c == r) {
                    rd[r] = 1.0 / d[m];
                }
            }
        }
        __syncthreads();
        TP_STAMP(0);
        // (b) panel U_pj = U_pp^{-T} W_pj, one thread per column, in registers
        const int ncol = b - o - NB;
        for (int c = t; c < ncol; c += NT) {
            const int col = o + NB + c;
            double v[NB];
#pragma unroll
            for (int r = 0; r < NB; ++r) v[r] = W[(size_t)col * b + o + r];
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                v[q] = v[q] * rd[q];
#pragma unroll
                for (int r = q + 1; r < NB; ++r) v[r] = v[r] - D[q][r] * v[q];
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int r = 0; r < NB; ++r) {
                P(r, c) = v[r];
                W[(size_t)col * b + o + r] = v[r];
            }
        }
        __syncthreads();
        TP_STAMP(1);
        // (c) trailing update W[i, l] -= sum_r P[r][i] P[r][l] over the upper
        //     triangle, one 8x8 register tile per thread
        const int mt = (ncol + 7) / 8;
        const int ntile = mt * (mt + 1) / 2;
        for (int tile = t; tile < ntile; tile += NT) {
            int ti = 0, rem = tile;
            while (rem >= mt - ti) { rem -= mt - ti; ++ti; }
            const int tl = ti + rem;
            const int i0 = ti * 8, l0 = tl * 8;
            double acc[8][8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int v = 0; v < 8; ++v) acc[u][v] = 0.0;
            for (int r = 0; r < NB; ++r) {
                double ai[8], al[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    ai[u] = P(r, i0 + u);   // P padded: columns >= ncol read stale / zero, unused
                    al[u] = P(r, l0 + u);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
#pragma unroll
                    for (int v = 0; v < 8; ++v) acc[u][v] = fma(ai[u], al[v], acc[u][v]);
            }
            // RMW in two halves of 32 (clamped-address loads batched, then
            // predicated stores) to stay within the register budget
#pragma unroll
            for (int hv = 0; hv < 8; hv += 4) {
                double w[8][4];
#pragma unroll
                for (int v = 0; v < 4; ++v)
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int ll = min(l0 + hv + v, ncol - 1), ii = min(i0 + u, ncol - 1);
                        w[u][v] = W[(size_t)(o + NB + ll) * b + o + NB + ii];
                    }
#pragma unroll
                for (int v = 0; v < 4; ++v)
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int ll = l0 + hv + v, ii = i0 + u;
                        if (ll < ncol && ii <= ll)
                            W[(size_t)(o + NB + ll) * b + o + NB + ii] = w[u][v] - acc[u][hv + v];
                    }
            }
        }
        __syncthreads();
        TP_STAMP(2);
    }
    // ---- undo the scaling: U = U' S^-1, rdiag = 1 / diag(U)
    for (int col = t >> 6; col < b; col += NT / 64) {
        const double isc = 1.0 / scl[col];
        for (int r = t & 63; r <= col; r += 64) {
            const double v = W[(size_t)col * b + r] * isc;
            W[(size_t)col * b + r] = v;
            if (r == col) rdiag[col] = 1.0 / v;
        }
    }
    TP_STAMP(3);
    if (STAMPS && t == 0)
        for (int q = 0; q < 4; ++q) stamps[q] = st_acc[q];
#undef TP_STAMP
#undef P
}
template __global__ void k_chol_t<false>(double *, double *, int, double, int *, long long *, double *);
template __global__ void k_chol_t<true>(double *, double *, int, double, int *, long long *, double *);
template __global__ void k_chol_t<false, true>(double *, double *, int, double, int *, long long *, double *);

// Q = Z U^{-1}: Z, Q n x b column-major (ld n), U b x b upper (ld b),
// rdiag = 1 / diag(U).  Workgroup = 16 rows; thread (r, c) = (t & 15, t >> 4).
// TR rows a workgroup (16; 8 for b > 480, where 16 rows of Q and U's column
// block no longer fit the LDS together)
constexpr int TC = 16;
template <int TR, int BM>
__global__ void __launch_bounds__(TR * TC) k_trsm_ru(const double *Z, int n, int b, const double *U,
                                                     const double *rdiag, double *Q) {
    __shared__ double Qs[TR][BM + 1];
    __shared__ double Ub[TC][BM + 1];
    const int t = threadIdx.x;
    const int r = t % TR, c = t / TR;
    const int row0 = blockIdx.x * TR;
    const int row = row0 + r;
    const bool live = row < n;
    for (int o = 0; o < b; o += TC) {
        // stage U[0:o+TC, o:o+TC] as Ub[c][m] = U(m, o+c)
        for (int e = t; e < (o + TC) * TC; e += TR * TC) {
            const int m = e % (o + TC), cc = e / (o + TC);
            Ub[cc][m] = U[(size_t)(o + cc) * b + m];
        }
        __syncthreads();
        double acc = live ? Z[(size_t)(o + c) * n + row] : 0.0;
        int m = 0;
        for (; m + 3 < o; m += 4) {
            acc = acc - Qs[r][m] * Ub[c][m];
            acc = acc - Qs[r][m + 1] * Ub[c][m + 1];
            acc = acc - Qs[r][m + 2] * Ub[c][m + 2];
            acc = acc - Qs[r][m + 3] * Ub[c][m + 3];
        }
        for (; m < o; ++m) acc = acc - Qs[r][m] * Ub[c][m];
        Qs[r][o + c] = acc;
        __syncthreads();
        // triangular block: row r solved by thread (r, 0)
        if (c == 0) {
            double q[TC];
#pragma unroll
            for (int cc = 0; cc < TC; ++cc) {
                double v = Qs[r][o + cc];
#pragma unroll
                for (int c2 = 0; c2 < cc; ++c2) v = v - q[c2] * Ub[cc][o + c2];
                q[cc] = v * rdiag[o + cc];
            }
#pragma unroll
            for (int cc = 0; cc < TC; ++cc) Qs[r][o + cc] = q[cc];
        }
        __syncthreads();
    }
    if (live)
        for (int cc = c; cc < b; cc += TC) Q[(size_t)cc * n + row] = Qs[r][cc];
}

// b > 640: the same solve with U's column block staged in chunks of CH rows
// (Ub for a whole column block of U no longer fits the LDS beside Q's rows)
template <int TR, int BM, int CH>
__global__ void __launch_bounds__(TR * TC) k_trsm_ru_big(const double *Z, int n, int b, const double *U,
                                                         const double *rdiag, double *Q) {
    __shared__ double Qs[TR][BM + 1];
    __shared__ double Ub[TC][CH + 1];
    const int t = threadIdx.x;
    const int r = t % TR, c = t / TR;
    const int row = blockIdx.x * TR + r;
    const bool live = row < n;
    for (int o = 0; o < b; o += TC) {
        double acc = live ? Z[(size_t)(o + c) * n + row] : 0.0;
        for (int m0 = 0; m0 < o; m0 += CH) {   // rows m0 .. m0 + mlen - 1 of U's column block o
            const int mlen = min(CH, o - m0);
            __syncthreads();
            for (int e = t; e < mlen * TC; e += TR * TC) {
                const int mm = e % mlen, cc = e / mlen;
                Ub[cc][mm] = U[(size_t)(o + cc) * b + m0 + mm];
            }
            __syncthreads();
            for (int m = 0; m < mlen; ++m) acc = acc - Qs[r][m0 + m] * Ub[c][m];
        }
        __syncthreads();
        for (int e = t; e < TC * TC; e += TR * TC) {   // the diagonal block U[o:o+TC, o:o+TC]
            const int mm = e % TC, cc = e / TC;
            Ub[cc][mm] = U[(size_t)(o + cc) * b + o + mm];
        }
        Qs[r][o + c] = acc;
        __syncthreads();
        if (c == 0) {
            double q[TC];
#pragma unroll
            for (int cc = 0; cc < TC; ++cc) {
                double v = Qs[r][o + cc];
#pragma unroll
                for (int c2 = 0; c2 < cc; ++c2) v = v - q[c2] * Ub[cc][c2];
                q[cc] = v * rdiag[o + cc];
            }
#pragma unroll
            for (int cc = 0; cc < TC; ++cc) Qs[r][o + cc] = q[cc];
        }
        __syncthreads();
    }
    if (live)
        for (int cc = c; cc < b; cc += TC) Q[(size_t)cc * n + row] = Qs[r][cc];
}

size_t chol_panel_doubles(int b) { return b > BMAX ? (size_t)NB * (b + 8) : 0; }
void launch_chol(double *d_W, double *d_rdiag, int b, double rel, int *d_info, hipStream_t s, double *d_panel) {
    if (b % NB != 0 || b > BMAX_BIG) fail(TP_ERR_ARG, "chol: block size must be a multiple of 32, <= 1280");
    if (b > BMAX) {
        if (!d_panel) fail(TP_ERR_ARG, "chol: b > 480 needs panel scratch (chol_panel_doubles)");
        hipLaunchKernelGGL((k_chol_t<false, true>), dim3(1), dim3(NT), 0, s, d_W, d_rdiag, b, rel, d_info, nullptr,
                           d_panel);
    } else {
        hipLaunchKernelGGL((k_chol_t<false>), dim3(1), dim3(NT), 0, s, d_W, d_rdiag, b, rel, d_info, nullptr,
                           nullptr);
    }
    TP_HIP(hipGetLastError());
}

void launch_chol_stamped(double *d_W, double *d_rdiag, int b, double rel, int *d_info, long long *d_st,
                         hipStream_t s) {
    if (b % NB != 0 || b > BMAX) fail(TP_ERR_ARG, "chol (stamped): block size must be a multiple of 32, <= 480");
    hipLaunchKernelGGL((k_chol_t<true>), dim3(1), dim3(NT), 0, s, d_W, d_rdiag, b, rel, d_info, d_st, nullptr);
    TP_HIP(hipGetLastError());
}

void launch_trsm_ru(const double *d_Z, int n, int b, const double *d_U, const double *d_rdiag, double *d_Q,
                    hipStream_t s) {
    if (b % TC != 0 || b > BMAX_BIG) fail(TP_ERR_ARG, "trsm: block size must be a multiple of 16, <= 1280");
    if (b <= BMAX)
        hipLaunchKernelGGL((k_trsm_ru<16, BMAX>), dim3((n + 15) / 16), dim3(256), 0, s, d_Z, n, b, d_U, d_rdiag, d_Q);
    else if (b <= 640)
        hipLaunchKernelGGL((k_trsm_ru<8, 640>), dim3((n + 7) / 8), dim3(128), 0, s, d_Z, n, b, d_U, d_rdiag, d_Q);
    else
        hipLaunchKernelGGL((k_trsm_ru_big<8, BMAX_BIG, 256>), dim3((n + 7) / 8), dim3(128), 0, s, d_Z, n, b, d_U,
                           d_rdiag, d_Q);
    TP_HIP(hipGetLastError());
}


// ---------------------------------------------------------------------------
// k_chol_inv: U = chol(S W S + rel I) S^-1 and Y = U^-1 in ONE workgroup with
// the whole matrix resident in registers, for b <= 256 (b % 16 == 0).
//
// The b x b upper triangle is cut into 16 x 16 tiles (T = b/16, T(T+1)/2 <= 136
// tiles).  Each of the 16 waves owns up to 9 tiles as v_mfma_f64_16x16x4_f64
// accumulators (lane l, reg q = element (row (l>>4)+4q, col l&15)), dealt
// round-robin in the order (tile row descending, column ascending) so every
// step's active tiles split evenly over the waves.  Every tile product is four
// MFMAs whose operands are fragments in LDS laid out lane-for-lane, so the
// updates read LDS without bank conflicts and never move data between lanes:
//   * a tile X in accumulator layout is also the B operand of A*X and the A
//     operand of X'*B for chunk q = reg q;
//   * diagonal blocks are factored by their owner wave (16 pivot steps with a
//     wave barrier each), applying the same row operations to an identity, so
//     the step also yields E_p = U_pp^-T in A-operand layout.
// Factorisation (right-looking, p = 0..T-1):
//   panel    U_pj = E_p A_pj                      (owners of row p)
//   trailing A_ij -= U_pi' U_pj, i > p           (owner of (p+1,p+1) first,
//                                                  then it factors block p+1
//                                                  while the rest update)
// Inversion (Y = U^-1, p = T-1..0), B_ij accumulating in the freed registers:
//   Y_pj = E_p' B_pj (B_pp = I);  B_ij -= U_ip Y_pj for i < p <= j
// Jacobi scaling (van der Sluis) and the shift as in k_chol_t; Y = S Y'.
// Q = Z Y is then one MFMA GEMM instead of a row-block triangular solve.
// ---------------------------------------------------------------------------
typedef double tp_d4 __attribute__((ext_vector_type(4)));
constexpr int CI_BMAX = 256;

__device__ __forceinline__ tp_d4 mfma64(double a, double b, tp_d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Re-materialise a wave-uniform value at each use: stops the compiler from
// keeping every slot's derived masks and addresses live across the kernel.
__device__ __forceinline__ int ci_opaque(int v) {
    v = __builtin_amdgcn_readfirstlane(v);
    asm volatile("" : "+s"(v));
    return v;
}

// One pivot of the 16x16 diagonal factor.  Lane l holds row r = l & 15 at
// columns cp + 4m (cp = l >> 4) of the working block D and of E (the same row
// operations applied to I).  Pivot row J: a row_newbcast DPP of lane J of each
// 16-lane row; D[r][J] (= D[J][r] for r > J, the Schur complement is
// symmetric) by one bpermute; the pivot by readlane.  No LDS, no barrier.
template <int J>
__device__ __forceinline__ void ci_pivot(double (&d)[4], double (&e)[4], int l, bool &bad) {
    const int r = l & 15;
    double pd[4], pe[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        pd[m] = dpp_d<0x150 + J>(d[m]);
        pe[m] = dpp_d<0x150 + J>(e[m]);
    }
    double dj = readlane_d(d[J >> 2], J + 16 * (J & 3));
    if (!(dj > 0.0)) {
        bad = true;
        dj = 1e-300;
    }
    double rp = __builtin_amdgcn_rsq(dj);
    rp = rp * fma(-0.5 * dj * rp, rp, 1.5);   // one Newton step: <= 2 ulp
    const double drj = __shfl(d[J >> 2], r + 16 * (J & 3), 64);
    const double f = (r > J) ? drj * (rp * rp) : 0.0;
    const double sc = (r == J) ? rp : 1.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        d[m] = fma(-f, pd[m], d[m]) * sc;
        e[m] = fma(-f, pe[m], e[m]) * sc;
    }
}
template <int... J>
__device__ __forceinline__ void ci_pivots(double (&d)[4], double (&e)[4], int l, bool &bad,
                                          std::integer_sequence<int, J...>) {
    (ci_pivot<J>(d, e, l, bad), ...);
}

// Factor the symmetric 16x16 diagonal block v (accumulator layout == its
// transpose, being symmetric).  On return v holds U_pp' transposed (lane l,
// reg m = U[l & 15][(l >> 4) + 4m], upper part valid) and Eb holds
// E_p = U_pp'^-T in A-operand layout.
__device__ __forceinline__ void ci_diag(tp_d4 &v, int l, double *Eb, bool &bad) {
    const int r = l & 15, cp = l >> 4;
    double d[4], e[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        d[m] = v[m];
        e[m] = (r == cp + 4 * m) ? 1.0 : 0.0;
    }
    ci_pivots(d, e, l, bad, std::make_integer_sequence<int, 16>{});
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        Eb[m * 64 + l] = e[m];
        v[m] = d[m];
    }
}

// CI_W waves; TMAX: the largest tile count b / 16 the instance handles
template <int CI_W, int TMAX>
__global__ void __launch_bounds__(64 * CI_W) k_chol_inv(double *W, double *F, double *sc, double *rdiag, int b,
                                                        double rel, int *info, long long *stamps) {
    constexpr int CI_SLOTS = (TMAX * (TMAX + 1) / 2 + CI_W - 1) / CI_W;   // tiles per wave
    // stamps (diagnostics, may be NULL): [0] prologue [1] factorisation +
    // output cycles, [4] cycles inside diagonal factors
    __shared__ unsigned long long dcyc;
    __shared__ int sbad;
    long long tst = (long long)__builtin_amdgcn_s_memtime();
#define CI_STAMP(k)                                                          \
    if (stamps && threadIdx.x == 0) {                                        \
        const long long _n = (long long)__builtin_amdgcn_s_memtime();        \
        stamps[k] = _n - tst;                                                \
        tst = _n;                                                            \
    }
#define CI_DIAG(v)                                                           \
    {                                                                        \
        const long long _a = (long long)__builtin_amdgcn_s_memtime();        \
        bool _bad = false;                                                   \
        ci_diag(v, l, Eb[diag_p], _bad);                                     \
        if (_bad && l == 0) sbad = 1;                                        \
        if (stamps && l == 0)                                                \
            atomicAdd(&dcyc, (unsigned long long)((long long)__builtin_amdgcn_s_memtime() - _a)); \
    }
    __shared__ double Eb[TMAX][4 * 64];   // E_p fragments (A-operand layout)
    __shared__ double Pb[TMAX][4 * 64];   // row panel of U
    __shared__ double scl[16 * TMAX];
    const int t = threadIdx.x, l = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int T = b >> 4;
    const int ntiles = T * (T + 1) / 2;
    const int lr = l >> 4, lc = l & 15;
    // tile coordinates of each slot, wave-uniform, packed (row << 8 | col);
    // an empty slot gets row 255 / col 0 so no "row == p" test matches it
    int tc[CI_SLOTS];
#pragma unroll
    for (int s = 0; s < CI_SLOTS; ++s) {
        int id = s * CI_W + w;
        int v = 255 << 8;
        if (id < ntiles) {
            int i = T - 1, cnt = 1;
            while (id >= cnt) {
                id -= cnt;
                --i;
                ++cnt;
            }
            v = (i << 8) | (i + id);
        }
        tc[s] = __builtin_amdgcn_readfirstlane(v);
    }
#define TI(s) (ci_opaque(tc[s]) >> 8)
#define TJ(s) (ci_opaque(tc[s]) & 255)
#define LIVE(s) (TI(s) != 255)
    for (int j = t; j < b; j += 64 * CI_W) {
        const double dj = W[(size_t)j * b + j];
        scl[j] = dj > 0.0 ? 1.0 / sqrt(dj) : 1.0;
    }
    if (t == 0) {
        sbad = 0;
        dcyc = 0;
    }
    // branch-free loads (an empty slot reads W[0]) so all of them are in flight
    tp_d4 a[CI_SLOTS];
#pragma unroll
    for (int s = 0; s < CI_SLOTS; ++s) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // W is the full symmetric Gram matrix: read element (R, C) as
            // W[C][R] so the 16 lanes of a row segment read 128 contiguous bytes
            const int R = 16 * TI(s) + lr + 4 * q, C = 16 * TJ(s) + lc;
            a[s][q] = LIVE(s) ? W[(size_t)R * b + C] : 0.0;
        }
    }
    __syncthreads();   // scl ready; every load done before W is overwritten with U
#pragma unroll
    for (int s = 0; s < CI_SLOTS; ++s) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int R = 16 * TI(s) + lr + 4 * q, C = 16 * TJ(s) + lc;
            double v = 0.0;
            if (LIVE(s)) {
                v = a[s][q] * (scl[min(R, C)] * scl[max(R, C)]);
                if (R == C) v += rel;
            }
            a[s][q] = v;
        }
    }
    __syncthreads();
    CI_STAMP(0);
    // ---------------- factorisation.  Step p: the owner of (p, p) applies
    // step p-1's update to it and factors it while the other waves finish step
    // p-1's trailing update; then row p of U (the panel) is formed.
    for (int p = 0; p < T; ++p) {
        {
            tp_d4 dv = {0.0, 0.0, 0.0, 0.0};
            bool have = false;
#pragma unroll
            for (int s = 0; s < CI_SLOTS; ++s) {
                if (TI(s) == p && TJ(s) == p) {
                    if (p > 0) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) a[s] = mfma64(-Pb[p][q * 64 + l], Pb[p][q * 64 + l], a[s]);
                    }
                    dv = a[s];
                    have = true;
                }
            }
            if (have) {
                const int diag_p = p;
                CI_DIAG(dv);
            }
#pragma unroll
            for (int s = 0; s < CI_SLOTS; ++s)
                if (TI(s) == p && TJ(s) == p) a[s] = dv;
        }
        if (p > 0) {
#pragma unroll
            for (int s = 0; s < CI_SLOTS; ++s) {
                if (TI(s) >= p && !(TI(s) == p && TJ(s) == p)) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        a[s] = mfma64(-Pb[TI(s)][q * 64 + l], Pb[TJ(s)][q * 64 + l], a[s]);
                }
                __builtin_amdgcn_sched_barrier(0);   // bound the operands in flight
            }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < CI_SLOTS; ++s) {
            if (TI(s) == p && TJ(s) > p) {
                tp_d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int q = 0; q < 4; ++q) acc = mfma64(Eb[p][q * 64 + l], a[s][q], acc);
                a[s] = acc;
#pragma unroll
                for (int q = 0; q < 4; ++q) Pb[TJ(s)][q * 64 + l] = acc[q];
            }
        }
        __syncthreads();
    }
    // Outputs for k_trsm_frag: U' tiles (i < j) and E_p (at tile (p, p)) as
    // 2 KB operand fragments, F[(i T + j) 256 + q 64 + lane] (coalesced);
    // diag(U) = diag(U') / s into W's diagonal, rdiag = 1 / diag(U), sc = s.
#pragma unroll
    for (int s = 0; s < CI_SLOTS; ++s) {
        if (LIVE(s)) {
            double *f = F + (size_t)(TI(s) * T + TJ(s)) * 256;
            if (TI(s) == TJ(s)) {
                const int o = 16 * TI(s);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    f[q * 64 + l] = Eb[TI(s)][q * 64 + l];
                    if (lr + 4 * q == lc) {   // held transposed: (lc, lr + 4q)
                        const double u = a[s][q] / scl[o + lc];
                        W[(size_t)(o + lc) * b + o + lc] = u;
                        rdiag[o + lc] = 1.0 / u;
                    }
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) f[q * 64 + l] = a[s][q];
            }
        }
    }
    for (int j = t; j < b; j += 64 * CI_W) sc[j] = scl[j];
    if (t == 0) *info = sbad;
    CI_STAMP(1);
    if (stamps && t == 0) stamps[4] = (long long)dcyc;
#undef CI_STAMP
#undef CI_DIAG
}

template __global__ void k_chol_inv<8, 16>(double *, double *, double *, double *, int, double, int *, long long *);
template __global__ void k_chol_inv<16, 16>(double *, double *, double *, double *, int, double, int *, long long *);
template __global__ void k_chol_inv<4, 4>(double *, double *, double *, double *, int, double, int *, long long *);

thread_local int g_chol_inv_waves = 0;   // 0: 4 waves for b <= 64, else 16; 4 / 8 / 16 force (diagnostics switch)

// ---------------------------------------------------------------------------
// k_trsm_frag: Q = Z U^-1 = (Z S) U'^-1 from k_chol_inv's fragments, one
// 4-wave workgroup per 16 rows of Z.  With X_J = (Z S)_J' (the transposed
// block column J of the row block; wave J & 3 owns it), right-looking: for
// m = 0..T-1
//   X_m <- E_m X_m                       (owner; published through LDS)
//   X_J <- X_J - U'_mJ' X_m,  J > m      (every wave, its own columns)
// Accumulator layout of X' == B-operand layout of X', so X_m is used in place;
// A operands are 2 KB fragments read from global memory (L2-resident,
// coalesced), the next tile row's prefetched during the current one.
// ---------------------------------------------------------------------------
template <int T>
__global__ void __launch_bounds__(256) k_trsm_frag(const double *__restrict__ Z, int n, const double *__restrict__ F,
                                                   const double *__restrict__ sc, double *__restrict__ Q) {
    constexpr int S = (T + 3) / 4;   // columns per wave
    __shared__ double ys[2][4 * 64];
    const int t = threadIdx.x, l = t & 63, lr = l >> 4, lc = l & 15;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int row = blockIdx.x * 16 + lc;
    const bool live = row < n;
    tp_d4 x[S], fr[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int J = 4 * s + w;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = 16 * J + lr + 4 * q;   // x[s] = (Z S)_J' : D[c - 16J][row]
            x[s][q] = (live && J < T) ? Z[(size_t)c * n + row] * sc[c] : 0.0;
            fr[s][q] = (J < T) ? F[(size_t)J * 256 + q * 64 + l] : 0.0;   // tile row 0
        }
    }
    for (int m = 0; m < T; ++m) {
        tp_d4 nx[S];
        if (m + 1 < T) {
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int J = 4 * s + w;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    nx[s][q] = (J > m && J < T) ? F[(size_t)((m + 1) * T + J) * 256 + q * 64 + l] : 0.0;
            }
        }
        double *y = ys[m & 1];
        if ((m & 3) == w) {
#pragma unroll
            for (int s = 0; s < S; ++s) {
                if (4 * s + w == m) {
                    tp_d4 v = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int q = 0; q < 4; ++q) v = mfma64(fr[s][q], x[s][q], v);
                    x[s] = v;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        y[q * 64 + l] = v[q];
                        if (live) Q[(size_t)(16 * m + lr + 4 * q) * n + row] = v[q];
                    }
                }
            }
        }
        lds_barrier();
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int J = 4 * s + w;
            if (J > m && J < T) {
#pragma unroll
                for (int q = 0; q < 4; ++q) x[s] = mfma64(-fr[s][q], y[q * 64 + l], x[s]);
            }
        }
        if (m + 1 < T) {
#pragma unroll
            for (int s = 0; s < S; ++s) fr[s] = nx[s];
        }
    }
}

void launch_chol_inv(double *d_W, double *d_F, double *d_sc, double *d_rdiag, int b, double rel, int *d_info,
                     hipStream_t s, long long *d_stamps) {
    if (b % 16 != 0 || b > CI_BMAX || b < 16) fail(TP_ERR_ARG, "chol_inv: block size must be a multiple of 16, <= 256");
    const int w = g_chol_inv_waves ? g_chol_inv_waves : (b <= 64 ? 4 : 16);
    if (w == 4 && b <= 64)
        hipLaunchKernelGGL((k_chol_inv<4, 4>), dim3(1), dim3(256), 0, s, d_W, d_F, d_sc, d_rdiag, b, rel, d_info,
                           d_stamps);
    else if (w == 8)
        hipLaunchKernelGGL((k_chol_inv<8, 16>), dim3(1), dim3(512), 0, s, d_W, d_F, d_sc, d_rdiag, b, rel, d_info,
                           d_stamps);
    else
        hipLaunchKernelGGL((k_chol_inv<16, 16>), dim3(1), dim3(1024), 0, s, d_W, d_F, d_sc, d_rdiag, b, rel, d_info,
                           d_stamps);
    TP_HIP(hipGetLastError());
}

template <int T>
static void trsm_frag_t(const double *Z, int n, const double *F, const double *sc, double *Q, hipStream_t s) {
    hipLaunchKernelGGL(k_trsm_frag<T>, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, s, Z, n, F, sc, Q);
}

void launch_trsm_frag(const double *d_Z, int n, int b, const double *d_F, const double *d_sc, double *d_Q,
                      hipStream_t s) {
    switch (b / 16) {
#define TP_T(k) case k: trsm_frag_t<k>(d_Z, n, d_F, d_sc, d_Q, s); break;
        TP_T(1) TP_T(2) TP_T(3) TP_T(4) TP_T(5) TP_T(6) TP_T(7) TP_T(8)
        TP_T(9) TP_T(10) TP_T(11) TP_T(12) TP_T(13) TP_T(14) TP_T(15) TP_T(16)
#undef TP_T
        default: fail(TP_ERR_ARG, "trsm_frag: block size must be a multiple of 16, <= 256");
    }
    TP_HIP(hipGetLastError());
}

}  // namespace tp
