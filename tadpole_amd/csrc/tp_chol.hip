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
#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

constexpr int NB = 32;
constexpr int BMAX = 480;
constexpr int NT = 512;   // threads of k_chol: 8 waves, 256 VGPRs each

template <bool STAMPS>
__global__ void __launch_bounds__(NT) k_chol_t(double *W, double *rdiag, int b, double rel, int *info,
                                               long long *stamps) {
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
    __shared__ double P[NB][BMAX + 8];     // panel U[o:o+32, o+32:b]
    __shared__ double scl[BMAX];           // diag(W)^-1/2
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
                P[r][c] = v[r];
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
                    ai[u] = P[r][i0 + u];   // P padded: columns >= ncol read stale / zero, unused
                    al[u] = P[r][l0 + u];
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
}
template __global__ void k_chol_t<false>(double *, double *, int, double, int *, long long *);
template __global__ void k_chol_t<true>(double *, double *, int, double, int *, long long *);

// Q = Z U^{-1}: Z, Q n x b column-major (ld n), U b x b upper (ld b),
// rdiag = 1 / diag(U).  Workgroup = 16 rows; thread (r, c) = (t & 15, t >> 4).
constexpr int TR = 16, TC = 16;
__global__ void __launch_bounds__(256) k_trsm_ru(const double *Z, int n, int b, const double *U,
                                                 const double *rdiag, double *Q) {
    __shared__ double Qs[TR][BMAX + 1];
    __shared__ double Ub[TC][BMAX + 1];
    const int t = threadIdx.x;
    const int r = t & 15, c = t >> 4;
    const int row0 = blockIdx.x * TR;
    const int row = row0 + r;
    const bool live = row < n;
    for (int o = 0; o < b; o += TC) {
        // stage U[0:o+TC, o:o+TC] as Ub[c][m] = U(m, o+c)
        for (int e = t; e < (o + TC) * TC; e += 256) {
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

void launch_chol(double *d_W, double *d_rdiag, int b, double rel, int *d_info, hipStream_t s) {
    if (b % NB != 0 || b > BMAX) fail(TP_ERR_ARG, "chol: block size must be a multiple of 32, <= 480");
    hipLaunchKernelGGL(k_chol_t<false>, dim3(1), dim3(NT), 0, s, d_W, d_rdiag, b, rel, d_info, nullptr);
    TP_HIP(hipGetLastError());
}

void launch_chol_stamped(double *d_W, double *d_rdiag, int b, double rel, int *d_info, long long *d_st,
                         hipStream_t s) {
    hipLaunchKernelGGL(k_chol_t<true>, dim3(1), dim3(NT), 0, s, d_W, d_rdiag, b, rel, d_info, d_st);
    TP_HIP(hipGetLastError());
}

void launch_trsm_ru(const double *d_Z, int n, int b, const double *d_U, const double *d_rdiag, double *d_Q,
                    hipStream_t s) {
    if (b % TC != 0 || b > BMAX) fail(TP_ERR_ARG, "trsm: block size must be a multiple of 16, <= 480");
    hipLaunchKernelGGL(k_trsm_ru, dim3((n + TR - 1) / TR), dim3(256), 0, s, d_Z, n, b, d_U, d_rdiag, d_Q);
    TP_HIP(hipGetLastError());
}

}  // namespace tp
