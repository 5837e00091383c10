// Kernels of the C-Krylov orthogonalisation (BCGS-PIP passes), shared by
// tp_krylov.hip and the microbenchmark tools/pip_bench.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "tp_common.cuh"

namespace tp {

typedef double d4k __attribute__((ext_vector_type(4)));
constexpr int KP = 32;   // Krylov block width of this path

// ---- Z partials: part[c] = A(rows of chunk c)' W(rows of chunk c), A = [K | W]
// (D + KP columns: K's D columns, then W's), output (D + KP) x KP col-major,
// ld = D + KP.  Tile: 64 A-columns x 32, wave w = A-columns 16w..16w+15;
// 16-row stages with three stages of register prefetch in flight (the loads
// are L2 / MALL latency-bound, not bandwidth-bound).
constexpr int PZ_COLS = 64;
// Local passes: the first Dh columns come from K, the remaining D - Dh from
// Kt (Dh < 0: all D from K).
__global__ void __launch_bounds__(256) k_pipz(const double *__restrict__ K, int D, const double *__restrict__ W, int n,
                                              int chunk, double *__restrict__ part, size_t pstride,
                                              const double *__restrict__ Kt = nullptr, int Dh = -1) {
    __shared__ double As[2][PZ_COLS][18];
    __shared__ double Bs[2][KP][18];
    const int ldz = D + KP;
    const int dt = (ldz + PZ_COLS - 1) / PZ_COLS;
    const int c0 = (blockIdx.x % dt) * PZ_COLS, z = blockIdx.x / dt;
    const int r0 = z * chunk, r1 = min(n, r0 + chunk);
    double *out = part + pstride * z;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int fr = lane & 15, fk = lane >> 4;
    const int lk = t & 15, lc = t >> 4;   // k row within the stage, column group
    const int dh = Dh < 0 ? D : Dh;
    auto colp = [&](int col) -> const double * {
        return col < dh ? K + (size_t)col * n
                        : (col < D ? Kt + (size_t)(col - dh) * n : (col < ldz ? W + (size_t)(col - D) * n : nullptr));
    };
    const double *pa[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) pa[p] = colp(c0 + lc + 16 * p);
    const double *pb[2] = {W + (size_t)lc * n, W + (size_t)(lc + 16) * n};
    double ra[3][4], rb[3][2];
    auto load = [&](int q, int k0) {
        const int k = k0 + lk;
        const bool in = k < r1;
#pragma unroll
        for (int p = 0; p < 4; ++p) ra[q][p] = (in && pa[p]) ? pa[p][k] : 0.0;
#pragma unroll
        for (int p = 0; p < 2; ++p) rb[q][p] = in ? pb[p][k] : 0.0;
    };
    auto store = [&](int q, int buf) {
#pragma unroll
        for (int p = 0; p < 4; ++p) As[buf][lc + 16 * p][lk] = ra[q][p];
#pragma unroll
        for (int p = 0; p < 2; ++p) Bs[buf][lc + 16 * p][lk] = rb[q][p];
    };
    d4k acc[2];
    acc[0] = acc[1] = (d4k){0.0, 0.0, 0.0, 0.0};
    auto compute = [&](int buf) {
#pragma unroll
        for (int kk = 0; kk < 16; kk += 4) {
            const double af = As[buf][16 * w + fr][kk + fk];
            const double b0 = Bs[buf][fr][kk + fk], b1 = Bs[buf][16 + fr][kk + fk];
            acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, b0, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, b1, acc[1], 0, 0, 0);
        }
    };
    const int nst = (r1 - r0 + 15) / 16;
    if (nst > 0) load(0, r0);
    if (nst > 1) load(1, r0 + 16);
    if (nst > 2) load(2, r0 + 32);
    if (nst > 0) store(0, 0);
    __syncthreads();
    // stage s: compute from LDS buffer s & 1; register set s % 3 is free after
    // its store (at s - 1), so it takes stage s + 3
    for (int s0 = 0; s0 < nst; s0 += 3) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int st = s0 + u;
            if (st < nst) {   // uniform
                compute(st & 1);
                if (st + 1 < nst) store((u + 1) % 3, (st + 1) & 1);
                if (st + 3 < nst) load(u, r0 + 16 * (st + 3));
                __syncthreads();
            }
        }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = c0 + 16 * w + fk + 4 * r, j = 16 * b + fr;
            if (i < ldz) out[(size_t)i + (size_t)j * ldz] = acc[b][r];
        }
}

// ---- reduce the Z partials (ascending chunk order) for a 64-row slice, and
// the slice's share of H'H (H = rows < D of Z): hh[s] (32 x 32, col-major)
constexpr int PR = 64;   // rows per reduce slice
constexpr int PR_TB = 1024;   // threads: two entries each, 16 partials of each in flight
__global__ void __launch_bounds__(PR_TB) k_pipr(const double *__restrict__ part, size_t pstride, int S, int D,
                                                double *__restrict__ Z, double *__restrict__ hh) {
    __shared__ double Hs[PR][KP + 1];
    const int ldz = D + KP;
    const int r0 = blockIdx.x * PR;
    const int t = threadIdx.x;
    constexpr int NE = PR * KP / PR_TB;   // entries per thread
    constexpr int G = 16;                 // partials of an entry in flight
    size_t idx[NE];
    bool in[NE];
    double v[NE];
#pragma unroll
    for (int h = 0; h < NE; ++h) {
        const int e = t + PR_TB * h;
        const int row = r0 + (e & (PR - 1)), col = e / PR;
        in[h] = row < ldz;
        idx[h] = in[h] ? (size_t)row + (size_t)col * ldz : 0;
        v[h] = part[idx[h]];
    }
    // summed in ascending chunk order (the bits of a sequential sum)
    int z = 1;
    for (; z + G <= S; z += G) {
        double q[NE][G];
#pragma unroll
        for (int h = 0; h < NE; ++h)
#pragma unroll
            for (int u = 0; u < G; ++u) q[h][u] = part[idx[h] + (size_t)(z + u) * pstride];
#pragma unroll
        for (int h = 0; h < NE; ++h)
#pragma unroll
            for (int u = 0; u < G; ++u) v[h] = v[h] + q[h][u];
    }
    for (; z < S; ++z) {
#pragma unroll
        for (int h = 0; h < NE; ++h) v[h] = v[h] + part[idx[h] + (size_t)z * pstride];
    }
#pragma unroll
    for (int h = 0; h < NE; ++h) {
        const int e = t + PR_TB * h;
        const int row = r0 + (e & (PR - 1)), col = e / PR;
        if (in[h]) Z[idx[h]] = v[h];
        Hs[e & (PR - 1)][col] = row < D ? v[h] : 0.0;
    }
    if (r0 >= D) return;   // uniform: no H rows in this slice
    __syncthreads();
    double *o = hh + (size_t)blockIdx.x * KP * KP;
#pragma unroll
    for (int h = 0; h < KP * KP / PR_TB; ++h) {
        const int e = t + PR_TB * h;
        const int a = e & 31, b = e >> 5;
        double acc = 0.0;
#pragma unroll 16
        for (int r = 0; r < PR; ++r) acc = fma(Hs[r][a], Hs[r][b], acc);
        o[a + KP * b] = acc;
    }
}

// ---- the small step: S = Z_w - H'H (symmetrised), Jacobi scaling d, shifted
// Cholesky S/(d d') + shift I = R'^T R' by row reduction of [S/(d d') | I]
// (the right block ends as R'^-T), Ri = R^-1 = D^-1 R'^-1 (upper, col-major ld
// KP).  512 threads hold the 32 x 64 augmented matrix in registers (thread:
// row t >> 4, columns t & 15 + 16 q); step j reads the pivot row and column
// from LDS (double-buffered by parity), one barrier a step.
// lowdin (the second pass, where S = I + E with |E| ~ 1e-13): Ri = I - E/2
// (the symmetric (I + E)^-1/2 to O(E^2)) when max|E| <= 1e-6, else the
// Cholesky as above.  info: 1 on a non-positive pivot.
// STOP (microbenchmark only, tools/pip_bench.hip): 1 = the sums only, 3 = all
template <int STOP = 3>
__global__ void __launch_bounds__(512) k_pips(const double *__restrict__ Z, int D, const double *__restrict__ hh,
                                              int nh, double shift, double *__restrict__ Ri, int *info, int lowdin) {
    __shared__ double Ss[KP][KP + 1];
    __shared__ double dsc[KP];
    __shared__ double rowb[2][2 * KP], colb[2][KP];
    __shared__ int big, badf;
    const int ldz = D + KP;
    const int t = threadIdx.x;
    if (t == 0) {
        big = 0;
        badf = 0;
    }
    {
        double v[2] = {0.0, 0.0};
        int s0 = 0;
        for (; s0 + 4 <= nh; s0 += 4) {
            double q[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int u = 0; u < 4; ++u) q[h][u] = hh[(size_t)(s0 + u) * KP * KP + t + 512 * h];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int u = 0; u < 4; ++u) v[h] = v[h] + q[h][u];
        }
        for (; s0 < nh; ++s0) {
#pragma unroll
            for (int h = 0; h < 2; ++h) v[h] = v[h] + hh[(size_t)s0 * KP * KP + t + 512 * h];
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int e = t + 512 * h, a = e & 31, b = e >> 5;
            Ss[a][b] = Z[(size_t)(D + a) + (size_t)b * ldz] - v[h];
        }
    }
    __syncthreads();
    if (STOP == 1) {
        if (t < KP) Ri[t] = Ss[t][t];
        return;
    }
    if (lowdin) {
        bool far = false;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int e = t + 512 * h, a = e & 31, b = e >> 5;
            far |= !(fabs(Ss[a][b] - (a == b ? 1.0 : 0.0)) <= 1e-6);
        }
        if (far) big = 1;
        __syncthreads();
        if (!big) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = t + 512 * h, a = e & 31, b = e >> 5;
                const double eab = 0.5 * (Ss[a][b] + Ss[b][a]) - (a == b ? 1.0 : 0.0);
                Ri[a + KP * b] = (a == b ? 1.0 : 0.0) - 0.5 * eab;
            }
            return;
        }
    }
    if (t < KP) {
        const double dd = sqrt(Ss[t][t]);
        if (!(dd > 0.0)) badf = 1;
        dsc[t] = dd > 0.0 ? dd : 1.0;
    }
    __syncthreads();
    const int ar = t >> 4, cl = t & 15;
    double A[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = cl + 16 * q;
        A[q] = q < 2 ? 0.5 * (Ss[ar][col] + Ss[col][ar]) / (dsc[ar] * dsc[col]) + (ar == col ? shift : 0.0)
                     : (col - KP == ar ? 1.0 : 0.0);
    }
    if (ar == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) rowb[0][cl + 16 * q] = A[q];
    }
    if (cl == 0) colb[0][ar] = A[0];
    __syncthreads();
    bool bad = false;
    for (int j = 0; j < KP; ++j) {
        const int buf = j & 1;
        const double p = rowb[buf][j];
        bad |= !(p > 0.0);
        const double pp = p > 0.0 ? p : 1e-300;
        double sc = __builtin_amdgcn_rsq(pp);               // ~1 ulp, then one Newton step
        sc = sc * fma(-0.5 * pp * sc, sc, 1.5);
        const double la = colb[buf][ar] * sc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int col = cl + 16 * q;
            const double rc = rowb[buf][col] * sc;   // R'(j, col) / E(j, col - KP)
            if (ar == j) A[q] = (col >= j) ? rc : 0.0;
            else if (ar > j) A[q] = fma(-la, rc, A[q]);
        }
        if (j + 1 < KP) {
            if (ar == j + 1) {
#pragma unroll
                for (int q = 0; q < 4; ++q) rowb[buf ^ 1][cl + 16 * q] = A[q];
            }
            if (cl == ((j + 1) & 15)) colb[buf ^ 1][ar] = ((j + 1) >> 4) ? A[1] : A[0];
        }
        __syncthreads();
    }
    // right block row ar = E(ar, .) = R'^-T(ar, .):  Ri(a, ar) = E(ar, a) / d_a
#pragma unroll
    for (int q = 2; q < 4; ++q) {
        const int a = cl + 16 * (q - 2);
        Ri[a + KP * ar] = a <= ar ? A[q] / dsc[a] : 0.0;
    }
    if (bad) badf = 1;
    __syncthreads();
    if (t == 0 && badf) *info = 1;
}

// ---- apply, part 1: partial K H of a 64-row tile over a quarter of the D
// columns of K (workgroup = (row tile, split z)); H = Z rows < D (ld D + KP)
// staged through LDS in 32-deep chunks, K fragments straight from global
// memory.  part: [tile][z] 64 x 32 row-major.
constexpr int PA_ROWS = 64, PA_SPLIT = 4, PA_KC = 32;
// (Kt, Dh: as k_pipz; Dh a multiple of PA_KC)
__global__ void __launch_bounds__(256) k_pipa(const double *__restrict__ K, int D, int n, const double *__restrict__ Z,
                                              double *__restrict__ part, const double *__restrict__ Kt = nullptr,
                                              int Dh = -1) {
    __shared__ double Hs[2][KP][PA_KC + 2];
    const int ldz = D + KP;
    const int tile = blockIdx.x / PA_SPLIT, z = blockIdx.x % PA_SPLIT;
    const int i0 = tile * PA_ROWS;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int fr = lane & 15, fk = lane >> 4;
    const int nk = (D + PA_KC - 1) / PA_KC;   // chunks of 32 columns of K
    const int c0 = (int)((long)nk * z / PA_SPLIT), c1 = (int)((long)nk * (z + 1) / PA_SPLIT);
    const int row = min(i0 + 16 * w + fr, n - 1);   // clamped: rows past n are not stored
    d4k acc[2];
    acc[0] = acc[1] = (d4k){0.0, 0.0, 0.0, 0.0};
    // H chunk: thread t loads column t >> 3, k (t & 7) * 4 + u
    const int hc = t >> 3, hk = (t & 7) * 4;
    double rh[4], ra[8];
    const int dh = Dh < 0 ? D : Dh;
    auto load = [&](int ch) {
        const int k0 = ch * PA_KC;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + hk + u;
            rh[u] = k < D ? Z[(size_t)k + (size_t)hc * ldz] : 0.0;
        }
        const double *Kc = k0 < dh ? K + (size_t)k0 * n : Kt + (size_t)(k0 - dh) * n;   // uniform per chunk
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) {
            const int k = k0 + 4 * s2 + fk;
            ra[s2] = k < D ? Kc[(size_t)row + (size_t)(4 * s2 + fk) * n] : 0.0;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int u = 0; u < 4; ++u) Hs[buf][hc][hk + u] = rh[u];
    };
    if (c0 < c1) {
        load(c0);
        store(0);
    }
    __syncthreads();
    int buf = 0;
    for (int ch = c0; ch < c1; ++ch) {
        double fa[8];
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) fa[s2] = ra[s2];
        const bool more = ch + 1 < c1;
        if (more) load(ch + 1);
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) {
            const double b0 = Hs[buf][fr][4 * s2 + fk], b1 = Hs[buf][16 + fr][4 * s2 + fk];
            acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[s2], b0, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[s2], b1, acc[1], 0, 0, 0);
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    double *pp = part + ((size_t)tile * PA_SPLIT + z) * PA_ROWS * KP;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) pp[(16 * w + fk + 4 * r) * KP + 16 * b + fr] = acc[b][r];
}

// ---- apply, part 2: out = (W0 - sum_z part[z]) Ri on a 64-row tile (the
// splits summed in order; U Ri on the matrix cores, wave w = rows 16w..).
// out may alias W0 (the workgroup reads its rows before its barrier and
// writes them after).
__global__ void __launch_bounds__(256) k_pipc(const double *__restrict__ part, const double *__restrict__ Ri, int n,
                                              const double *W0, double *out) {
    __shared__ double Us[PA_ROWS][KP + 2];
    __shared__ double Rs[KP][KP + 2];   // Rs[col][k] = Ri(k, col): B fragments k-contiguous
    const int tile = blockIdx.x, i0 = tile * PA_ROWS, t = threadIdx.x;
    const int lane = t & 63, w = t >> 6, fr = lane & 15, fk = lane >> 4;
    for (int e = t; e < KP * KP; e += 256) Rs[e >> 5][e & 31] = Ri[e];
    const double *pt = part + (size_t)tile * PA_SPLIT * PA_ROWS * KP;
    // the splits' sums read along their rows (row-major 64 x 32: consecutive
    // lanes, consecutive columns -- the earlier row-fastest order put each lane
    // on its own 256-byte row), then W0 down its columns; the same kh and W0 - kh
#pragma unroll
    for (int h = 0; h < PA_ROWS * KP / 256; ++h) {
        const int e = t + 256 * h, il = e >> 5, j = e & 31;
        const size_t o = (size_t)il * KP + j;
        Us[il][j] = ((pt[o] + pt[o + PA_ROWS * KP]) + pt[o + 2 * PA_ROWS * KP]) + pt[o + 3 * PA_ROWS * KP];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < PA_ROWS * KP / 256; ++h) {
        const int e = t + 256 * h, il = e & 63, j = e >> 6, i = i0 + il;
        Us[il][j] = i < n ? W0[(size_t)i + (size_t)j * n] - Us[il][j] : 0.0;
    }
    __syncthreads();
    d4k acc[2];
    acc[0] = acc[1] = (d4k){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < KP; kk += 4) {
        const double af = Us[16 * w + fr][kk + fk];
        acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, Rs[fr][kk + fk], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, Rs[16 + fr][kk + fk], acc[1], 0, 0, 0);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + 16 * w + fk + 4 * r, j = 16 * b + fr;
            if (i < n) out[(size_t)i + (size_t)j * n] = acc[b][r];
        }
}

}  // namespace tp
