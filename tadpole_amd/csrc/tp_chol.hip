// Small dense kernels for the PCA's CholQR orthonormalisation (b <= 512):
//   k_chol_inv: one 1024-thread workgroup computes U = chol(W + s I) (upper,
//   W = U'U) and X = U^{-1}, blocked by 32 with the panel in LDS and the
//   trailing matrix in global memory (L2-resident: 512 KB at b = 256).  The
//   caller then forms Q = Z X with the MFMA GEMM.  Replaces LAPACK-style
//   potrf + trsm library calls whose dozens of tiny launches dominated the
//   PCA.  Numerics: plain right-looking Cholesky; the shift s = rel*max(diag)
//   keeps it positive definite for ill-conditioned blocks (shifted CholQR).
#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

constexpr int NB = 32;

// W: b x b column-major (only the upper triangle is read), overwritten with U
// in its upper triangle.  X: b x b column-major, receives U^{-1} (upper,
// zero below).  b must be a multiple of 32 (the caller pads).
__global__ void __launch_bounds__(1024) k_chol_inv(double *W, double *X, int b, double rel, int *info) {
    __shared__ double D[NB][NB + 1];      // diagonal block / its inverse
    __shared__ double P[NB][512 + 1];     // panel row block U[p, :]
    __shared__ double red[32];
    const int t = threadIdx.x;
    const int T = b / NB;
    // ---- shift: s = rel * max diag
    double mx = 0.0;
    for (int j = t; j < b; j += blockDim.x) mx = fmax(mx, W[(size_t)j * b + j]);
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    if (t == 0) {
        double m = 0.0;
        for (int q = 0; q < (int)(blockDim.x >> 6); ++q) m = fmax(m, red[q]);
        red[0] = m;
        *info = 0;
    }
    __syncthreads();
    const double shift = rel * red[0];
    __syncthreads();
    for (int j = t; j < b; j += blockDim.x) W[(size_t)j * b + j] += shift;
    __syncthreads();

    for (int p = 0; p < T; ++p) {
        const int o = p * NB;
        // (a) diagonal block -> LDS, unblocked upper Cholesky
        {
            int r = t & 31, c = t >> 5;   // 1024 threads = 32 x 32
            D[r][c] = (r <= c) ? W[(size_t)(o + c) * b + o + r] : 0.0;
        }
        __syncthreads();
        for (int j = 0; j < NB; ++j) {
            if (t == 0) {
                double d = D[j][j];
                if (!(d > 0.0)) { atomicOr(info, 1); d = 1e-300; }
                D[j][j] = sqrt(d);
            }
            __syncthreads();
            const double piv = D[j][j];
            if (t > j && t < NB) D[j][t] = D[j][t] / piv;
            __syncthreads();
            {
                int r = t & 31, c = t >> 5;
                if (r > j && c >= r) D[r][c] = D[r][c] - D[j][r] * D[j][c];
            }
            __syncthreads();
        }
        // write U_pp back
        {
            int r = t & 31, c = t >> 5;
            if (r <= c) W[(size_t)(o + c) * b + o + r] = D[r][c];
        }
        __syncthreads();
        // (b) panel U_pj = U_pp^{-T} W_pj for columns o+NB .. b-1 (forward
        //     substitution per column, one thread per column)
        const int ncol = b - o - NB;
        for (int c = t; c < ncol; c += blockDim.x) {
            const int col = o + NB + c;
            for (int r = 0; r < NB; ++r) {
                double s = W[(size_t)col * b + o + r];
                for (int q = 0; q < r; ++q) s = s - D[q][r] * P[q][NB + c];
                double v = s / D[r][r];
                P[r][NB + c] = v;          // this thread's column only
                W[(size_t)col * b + o + r] = v;
            }
        }
        __syncthreads();
        // (c) trailing update W_il -= sum_r U(o+r, i) U(o+r, l), o+NB <= i <= l
        const int m = ncol;
        const size_t tot = (size_t)m * m;
        for (size_t e = t; e < tot; e += blockDim.x) {
            int i = (int)(e % m), l = (int)(e / m);
            if (i > l) continue;
            double s = 0.0;
#pragma unroll 8
            for (int r = 0; r < NB; ++r) s = fma(P[r][NB + i], P[r][NB + l], s);
            size_t idx = (size_t)(o + NB + l) * b + o + NB + i;
            W[idx] = W[idx] - s;
        }
        __syncthreads();
    }
    // ---- X = U^{-1}: diagonal blocks inverted in LDS, then block columns
    //      X[0:o, j] = - X[0:o, 0:o] U[0:o, j] X_jj
    for (size_t e = t; e < (size_t)b * b; e += blockDim.x) X[e] = 0.0;
    __syncthreads();
    for (int p = 0; p < T; ++p) {
        const int o = p * NB;
        {
            int r = t & 31, c = t >> 5;
            D[r][c] = (r <= c) ? W[(size_t)(o + c) * b + o + r] : 0.0;
        }
        __syncthreads();
        // invert upper triangular D in place, column by column (thread = column)
        if (t < NB) {
            const int c = t;                 // column c of inv(D), kept in P[:, c]
            for (int r = NB - 1; r >= 0; --r) {
                double x = 0.0;
                if (r == c) x = 1.0 / D[c][c];
                else if (r < c) {
                    double s = 0.0;
                    for (int q = r + 1; q <= c; ++q) s = s + D[r][q] * P[q][c];
                    x = -s / D[r][r];
                }
                P[r][c] = x;
            }
        }
        __syncthreads();
        {
            int r = t & 31, c = t >> 5;
            X[(size_t)(o + c) * b + o + r] = (r <= c) ? P[r][c] : 0.0;
        }
        // Y = U[0:o, o:o+NB] X_jj  -> P[:, NB + ...] is too small for o rows;
        // compute X[0:o, col] row by row: thread per (row, col)
        __syncthreads();
        if (o > 0) {
            // Y(i, c) = sum_q U(i, o+q) X_jj(q, c), i < o
            for (int e = t; e < o * NB; e += blockDim.x) {
                int i = e % o, c = e / o;
                double s = 0.0;
                for (int q = 0; q <= c; ++q) s = fma(W[(size_t)(o + q) * b + i], P[q][c], s);
                X[(size_t)(o + c) * b + i] = s;   // temporary: Y
            }
            __syncthreads();
            // X(i, o+c) = - sum_{m=i}^{o-1} X(i, m) Y(m, c)   (X upper on 0:o)
            // rows are independent; read Y column into LDS first
            for (int c = 0; c < NB; ++c) {
                for (int i = t; i < o; i += blockDim.x) P[0][NB + i] = X[(size_t)(o + c) * b + i];
                __syncthreads();
                for (int i = t; i < o; i += blockDim.x) {
                    double s = 0.0;
                    for (int mm = i; mm < o; ++mm) s = fma(X[(size_t)mm * b + i], P[0][NB + mm], s);
                    X[(size_t)(o + c) * b + i] = -s;
                }
                __syncthreads();
            }
        }
        __syncthreads();
    }
}

void launch_chol_inv(double *d_W, double *d_X, int b, double rel, int *d_info, hipStream_t s) {
    if (b % NB != 0 || b > 512) fail(TP_ERR_ARG, "chol_inv: block size must be a multiple of 32, <= 512");
    hipLaunchKernelGGL(k_chol_inv, dim3(1), dim3(1024), 0, s, d_W, d_X, b, rel, d_info);
    TP_HIP(hipGetLastError());
}

}  // namespace tp
