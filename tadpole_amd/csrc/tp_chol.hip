// Small dense kernels for the PCA's CholQR orthonormalisation Q = Z R^{-1}:
//   k_chol: one 512-thread workgroup computes U = chol(W + s I) (upper,
//     W = U'U) for b <= 480, blocked by 32: diagonal block factored by one wave
//     in LDS, panel solved in registers, trailing matrix updated in global
//     memory (L2-resident) by 64x64 macro tiles with 4x4 register micro tiles.
//     Also writes rdiag[j] = 1 / U_jj.  The shift s = rel * max(diag) keeps
//     ill-conditioned blocks positive definite (shifted CholQR).
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
    __shared__ double D[NB][NB + 1];       // diagonal block
    __shared__ double P[NB][BMAX + 1];     // panel U[o:o+32, o+32:b]
    __shared__ double red[32];
    const int t = threadIdx.x;
    const int T = b / NB;
    // ---- shift: s = rel * max diag
    double mx = 0.0;
    for (int j = t; j < b; j += NT) mx = fmax(mx, W[(size_t)j * b + j]);
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    if (t == 0) {
        double m = 0.0;
        for (int q = 0; q < NT / 64; ++q) m = fmax(m, red[q]);
        red[0] = m;
        *info = 0;
    }
    __syncthreads();
    const double shift = rel * red[0];
    for (int j = t; j < b; j += NT) W[(size_t)j * b + j] += shift;
    __syncthreads();

    TP_STAMP(3);
    for (int p = 0; p < T; ++p) {
        const int o = p * NB;
        // (a) diagonal block -> LDS, unblocked upper Cholesky by wave 0
        for (int e = t; e < NB * NB; e += NT) {
            const int r = e & 31, c = e >> 5;
            D[r][c] = (r <= c) ? W[(size_t)(o + c) * b + o + r] : 0.0;
        }
        __syncthreads();
        if (t < 64) {
            for (int j = 0; j < NB; ++j) {
                double d = D[j][j];
                if (!(d > 0.0)) {
                    if (t == 0) atomicOr(info, 1);
                    d = 1e-300;
                }
                const double piv = sqrt(d);
                // scale row j (one division per lane), then the trailing update
                if (t >= j && t < NB) D[j][t] = (t == j) ? piv : D[j][t] / piv;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                {
                    const int r = t & 31;            // fixed per lane
                    const double djr = D[j][r];
                    double dv[16], djc[16];
#pragma unroll
                    for (int m = 0; m < 16; ++m) {   // c = (t >> 5) + 2m
                        const int c = (t >> 5) + 2 * m;
                        dv[m] = D[r][c];
                        djc[m] = D[j][c];
                    }
#pragma unroll
                    for (int m = 0; m < 16; ++m) {
                        const int c = (t >> 5) + 2 * m;
                        if (r > j && c >= r) D[r][c] = dv[m] - djr * djc[m];
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        __syncthreads();
        for (int e = t; e < NB * NB; e += NT) {
            const int r = e & 31, c = e >> 5;
            if (r <= c) W[(size_t)(o + c) * b + o + r] = D[r][c];
        }
        if (t < NB) rdiag[o + t] = 1.0 / D[t][t];
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
                v[q] = v[q] / D[q][q];
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
        // (c) trailing update W[i, l] -= sum_r P[r][i] P[r][l], i, l < ncol,
        //     64x64 macro tiles on and above the diagonal, 4x4 per thread
        const int mt = ncol / 64 + ((ncol & 63) ? 1 : 0);
        const int ngrp = NT / 256, grp = t >> 8, lt = t & 255, tx = lt & 15, ty = lt >> 4;
        int tile = 0;
        for (int ti = 0; ti < mt; ++ti)
            for (int tl = ti; tl < mt; ++tl, ++tile) {
                if ((tile % ngrp) != grp) continue;
                const int i0 = ti * 64, l0 = tl * 64;
                double acc[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc[u][v] = 0.0;
                for (int r = 0; r < NB; ++r) {
                    double ai[4], al[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        int ii = i0 + tx + 16 * u, ll = l0 + ty + 16 * u;
                        ai[u] = ii < ncol ? P[r][ii] : 0.0;
                        al[u] = ll < ncol ? P[r][ll] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int v = 0; v < 4; ++v) acc[u][v] = fma(ai[u], al[v], acc[u][v]);
                }
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int ll = l0 + ty + 16 * v;
                    if (ll >= ncol) continue;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int ii = i0 + tx + 16 * u;
                        if (ii >= ncol) continue;
                        size_t idx = (size_t)(o + NB + ll) * b + o + NB + ii;
                        W[idx] = W[idx] - acc[u][v];
                    }
                }
            }
        __syncthreads();
        TP_STAMP(2);
    }
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
