// prcomp(cor, rank. = k)$x  (R/TADpole.R:452-453) on the GPU.
//
// R computes a FULL thin SVD of the column-centred N x N matrix (LAPACK gesdd)
// and keeps k = min(max_pcs, N) right singular vectors, i.e. the top-k
// eigenvectors of G = Xc' Xc, Xc = C - 1 colMeans(C)' (centring, tp_prep.hip).
// Two ways to the same eigenvectors (only span(V_1..V_i) matters downstream:
// distances and CH are invariant to sign and to rotations inside a prefix):
//
//  * small N (N < t_knob.pca_krylov_min): G = Xc'Xc on the fp64 MFMA (N^3), then
//    Chebyshev-filtered block subspace iteration on G (block b = k +
//    oversampling, CholQR orthonormalisation, Rayleigh-Ritz at the end);
//  * large N: G is never formed.  A block Krylov space of G (block p, s steps,
//    D = s p columns) is built with two skinny products per step, W = Xc'(Xc Q)
//    (2 x 2 N^2 p flops instead of N^3 + 2 N^2 b per subspace-iteration degree),
//    every block re-orthogonalised twice against all earlier ones (CGS2) and
//    orthonormalised by CholQR2.  The projected T = K'GK (D x D) is then solved
//    for its top k eigenpairs by the same subspace iteration (products with T
//    are D x D, not N x N), and V = K Y.  Block Krylov needs ~10x fewer products
//    with G than subspace iteration (C3: D = 1024 columns vs 27 x 256).
//
// Either way the iteration stops when every Ritz pair j <= k has
// ||G v - theta v|| <= tol * theta_1 (checked in the N-dimensional space), and
// the scores are P = Xc V_k (fp64 MFMA GEMM).  When N <= b the Ritz problem is
// G itself (exact full eigendecomposition).
#include <algorithm>
#include <cmath>
#include <functional>
#include <vector>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {


// deterministic pseudo-random start block, uniform in (-1, 1)
__global__ void k_rand_block(double *Q, int n, int b, uint64_t seed) {
    size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)n * b) return;
    uint64_t z = seed + 0x9E3779B97F4A7C15ULL * (idx + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    Q[idx] = ((double)(z >> 11) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
}

// Wk[:, j] = W[:, b-1-j], j < k  (eigenvectors in descending eigenvalue order)
__global__ void k_select_rev(const double *W, int b, int k, double *Wk) {
    size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)b * k) return;
    int i = (int)(idx % b), j = (int)(idx / b);
    Wk[idx] = W[(size_t)(b - 1 - j) * b + i];
}

// resid[j] = || Y[:, j] - theta_j V[:, j] ||_2: one 256-thread workgroup per
// column, four loads in flight a thread (one wave per column was a 121-step
// dependent chain at n = 7729: 39 us for k = 200 columns)
__global__ void __launch_bounds__(256) k_resid(const double *Y, const double *V, const double *theta_asc, int n, int b,
                                               int k, double *resid) {
    __shared__ double red[4];
    const int j = blockIdx.x, t = threadIdx.x;
    if (j >= k) return;
    const double th = theta_asc[b - 1 - j];
    const double *y = Y + (size_t)j * n, *v = V + (size_t)j * n;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    int a = t;
    for (; a + 768 < n; a += 1024) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double r = y[a + 256 * u] - th * v[a + 256 * u];
            acc[u] = fma(r, r, acc[u]);
        }
    }
    for (; a < n; a += 256) {
        const double r = y[a] - th * v[a];
        acc[0] = fma(r, r, acc[0]);
    }
    double tot = wave_sum((acc[0] + acc[1]) + (acc[2] + acc[3]));
    if ((t & 63) == 0) red[t >> 6] = tot;
    __syncthreads();
    if (t == 0) resid[j] = sqrt(((red[0] + red[1]) + red[2]) + red[3]);
}

// Q = orth(Z): W = Z'Z (symmetric GEMM), U = chol(W + s I) (one workgroup),
// Q = Z U^{-1} (row-block TRSM).  `passes` CholQR passes.  X holds 1/diag(U).
// For b <= 256 the factor comes from one register-resident MFMA kernel and
// Q = Z U^{-1} from an all-register MFMA solve; Y (b x b) holds the factor's
// operand fragments, X (b x b) 1/diag(U) and the Jacobi scaling.
static void orth_cholqr(Ctx &c, double *Z, double *Qout, double *Tmp, int n, int b, double *W, double *X,
                        double *Y, int *d_info, int passes, double shift) {
    double *src = Z;
    for (int p = 0; p < passes; ++p) {
        GemmArgs g{b, b, n, src, n, true, src, n, W, b};
        g.sym_upper = true;
        g.splitk = 0;   // auto: deep split for few-tile Gram matrices (tp_gemm.hip)
        gemm_f64(g, c.buf[S_PARTIAL], c.cur);
        double *dst = ((passes - 1 - p) % 2 == 0) ? Qout : Tmp;   // last pass lands in Qout
        if (b <= kCholInvMax && b % 16 == 0) {
            launch_chol_inv(W, Y, X + b, X, b, p == 0 ? shift : 0.0, d_info, c.cur);
            launch_trsm_frag(src, n, b, Y, X + b, dst, c.cur);
        } else {
            double *panel = b > 480 ? c.buf[S_CHOLP].as<double>(chol_panel_doubles(b)) : nullptr;
            launch_chol(W, X, b, p == 0 ? shift : 0.0, d_info, c.cur, panel);
            launch_trsm_ru(src, n, b, W, X, dst, c.cur);
        }
        src = dst;
    }
}

// Chebyshev three-term step: Y = alpha * GY + beta * Yc + gamma * Yp (n x b)
__global__ void k_cheb(double *Y, const double *GY, const double *Yc, const double *Yp, size_t cnt, double alpha,
                       double beta, double gamma) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    double v = alpha * GY[t] + beta * Yc[t];
    if (Yp) v = v + gamma * Yp[t];
    Y[t] = v;
}

typedef double d4b __attribute__((ext_vector_type(4)));

// Out = a (T Y) + bc Yc [+ cc Yp] (AFF) or T Y, for T symmetric and block
// tridiagonal with P x P blocks (the block Krylov projection, D x D, ld D),
// Y, Out, Yc, Yp D x b (ld D).  One workgroup per (block row, 16 columns):
// 3 x P / 16 waves, wave (kb, rw) a 16 x 16 tile of rows rw over T's block
// column ib - 1 + kb, all of its loads issued at once (one memory latency per
// product, not one per k step); the three partial tiles are summed in LDS in
// a fixed order and the epilogue reads and writes whole column segments.
// 2 D (3P) b flops instead of 2 D^2 b.
template <bool AFF, int P>
__global__ void __launch_bounds__(12 * P) k_band_ty(const double *__restrict__ T, const double *__restrict__ Y,
                                                     double *Out, int D, double a, double bc, const double *Yc,
                                                     double cc, const double *Yp) {
    constexpr int NRW = P / 16;   // row waves per block column
    __shared__ double tile[3][P][17];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, fr = l & 15, fk = l >> 4;
    const int rw = w % NRW, kb = w / NRW;
    const int ib = blockIdx.x, c0 = blockIdx.y * 16;
    const int r0 = ib * P + 16 * rw;
    const int kc = ib - 1 + kb;   // T's block column
    d4b acc = (d4b){0.0, 0.0, 0.0, 0.0};
    if (kc >= 0 && kc * P < D) {
        const double *tp = T + (size_t)(r0 + fr) + (size_t)(kc * P + fk) * D;   // T[r0 + fr][k + fk]
        const double *yp = Y + (size_t)(kc * P + fk) + (size_t)(c0 + fr) * D;   // Y[k + fk][c0 + fr]
        double af[P / 4], bf[P / 4];
#pragma unroll
        for (int u = 0; u < P / 4; ++u) {
            af[u] = tp[(size_t)(4 * u) * D];
            bf[u] = yp[4 * u];
        }
#pragma unroll
        for (int u = 0; u < P / 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(af[u], bf[u], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) tile[kb][16 * rw + fk + 4 * r][fr] = acc[r];
    __syncthreads();
    if (threadIdx.x >= 4 * P) return;
    // column c0 + j, rows ib P + q + e P / 4 (16 consecutive lanes a 128-byte
    // column segment)
    const int j = threadIdx.x / (P / 4), q = threadIdx.x % (P / 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int rl = q + e * (P / 4);
        const size_t idx = (size_t)(ib * P + rl) + (size_t)(c0 + j) * D;
        double v = (tile[0][rl][j] + tile[1][rl][j]) + tile[2][rl][j];
        if (AFF) {
            v = a * v + bc * Yc[idx];
            if (Yp) v = v + cc * Yp[idx];
        }
        Out[idx] = v;
    }
}

// T (D x D, ld D) from the Krylov CGS2 coefficients H1 + H2 (ld Dm): block
// (bi, bj) with bi < bj from column block bj, mirrored below the diagonal,
// diagonal blocks symmetrised, blocks off the tridiagonal band zero
__global__ void k_assemble_T(const double *H1, const double *H2, int Dm, int D, int p, double *T) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)D * D) return;
    const int i = (int)(t % D), j = (int)(t / D);
    const int bi = i / p, bj = j / p;
    const size_t a = (size_t)i + (size_t)j * Dm, b = (size_t)j + (size_t)i * Dm;
    double v;
    if (bi + 1 < bj || bj + 1 < bi) v = 0.0;   // K_i'G K_j = 0 for |i - j| > 1 (rounding left out)
    else if (bi < bj) v = H1[a] + H2[a];
    else if (bi > bj) v = H1[b] + H2[b];
    else v = 0.5 * ((H1[a] + H2[a]) + (H1[b] + H2[b]));
    T[t] = v;
}

__global__ void k_fill_const(double *p, int n, double v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// |U_jj| of the last Cholesky (upper triangle of W) -> host, ascending index j
__global__ void k_diag(const double *W, int b, double *d) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < b) d[j] = fabs(W[(size_t)j * b + j]);
}


using Prod = std::function<void(const double *, double *)>;
// Out = a (A Y) + b Yc [+ c Yp]: the product with the Chebyshev step in its
// epilogue (same arithmetic as k_cheb on a stored A Y)
using ProdAff = std::function<void(const double *Y, double *Out, double a, double b, const double *Yc, double c,
                                   const double *Yp)>;

// Top-k eigenpairs of a symmetric n x n operator by Chebyshev-filtered block
// subspace iteration.  prod(Y, Out): Out = A Y (n x b, ld n).  A (n x n, ld n)
// is read only when b >= n (exact eigendecomposition).  V (n x k): the Ritz
// vectors, descending; h_theta: ascending Ritz values of the last Rayleigh-Ritz
// problem.  Scratch: S_Q S_Z S_SWEEP S_SWEEP2 S_SMALL S_MISC (+ S_PARTIAL).
static void subspace_topk(Ctx &c, const double *A, int n, int k, const Prod &prod, double *V,
                          std::vector<double> &h_theta, PcaStats &st, uint64_t seed, int margin = 0,
                          const ProdAff *paff = nullptr) {
    hipStream_t s = c.cur;
    const int over = cfg_pca_over > 0 ? cfg_pca_over : std::max(32, k / 4);
    const int rnd = cfg_pca_over > 0 ? 16 : 32;
    int b = std::min(n, ((k + over + rnd - 1) / rnd) * rnd);
    st.block = b;
    if (b >= n) {
        // exact: eigendecomposition of A itself (small n)
        b = n;
        int *d_info = c.buf[S_MISC].as<int>(64);
        double *theta = c.buf[S_SMALL].as<double>((size_t)n + 64);
        double *E = c.buf[S_Z].as<double>((size_t)n * n);
        TP_HIP(hipMemcpyAsync(E, A, (size_t)n * n * sizeof(double), hipMemcpyDeviceToDevice, s));
        (void)d_info;
        eig_sym(E, n, theta, c.buf[S_PARTIAL].as<double>((size_t)n * n + 4 * n + 64), s);   // n <= b <= 1280
        size_t tot = (size_t)n * k;
        hipLaunchKernelGGL(k_select_rev, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, E, n, k, V);
        TP_HIP(hipGetLastError());
        h_theta.resize(n);
        double *pn = (double *)c.pinned((size_t)n * sizeof(double));
        TP_HIP(hipMemcpyAsync(pn, theta, n * sizeof(double), hipMemcpyDeviceToHost, s));
        stream_sync(c, s);
        memcpy(h_theta.data(), pn, n * sizeof(double));
        st.d_theta = theta;
        trace_mark(s, "pca: exact eig");
        st.iters = 0;
        st.resid = 0.0;
        return;
    }
    double *Q = c.buf[S_Q].as<double>((size_t)n * b);
    double *Z = c.buf[S_Z].as<double>((size_t)n * b);
    double *T = c.buf[S_SWEEP].as<double>((size_t)n * b);
    double *Wsm = c.buf[S_SMALL].as<double>((size_t)3 * b * b + 2 * b + 64);
    double *Xinv = Wsm + (size_t)b * b;
    double *theta = Xinv + (size_t)b * b;
    double *offd = theta + b;
    double *Yinv = offd + b;   // b x b, U^{-1} of the last CholQR
    double *resid = c.buf[S_MISC].as<double>(64 + k + b) + 64;
    int *d_info = c.buf[S_MISC].as<int>(64);
    const size_t nb = (size_t)n * b;
    // random start block (well conditioned: the first iteration's CholQR
    // orthonormalises A Q0 directly)
    hipLaunchKernelGGL(k_rand_block, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, Q, n, b, seed);
    TP_HIP(hipGetLastError());
    double *Yb = c.buf[S_SWEEP2].as<double>((size_t)n * b);   // 4th block buffer (sweep scratch later)
    auto iterate = [&](int count) {   // plain subspace iteration
        for (int it = 0; it < count; ++it) {
            prod(Q, Z);
            orth_cholqr(c, Z, Q, T, n, b, Wsm, Xinv, Yinv, d_info, 1, 1e-14);
        }
    };
    // Chebyshev filter of degree m on [0, cut]: Q <- orth(T_m((A - e)/h) Q),
    // e = h = cut / 2 (scaled three-term recurrence), then CholQR
    auto cheb_block = [&](int m, double cut) {
        const double e = 0.5 * cut, hh = 0.5 * cut;
        const size_t cnt = (size_t)n * b;
        const unsigned grid = (unsigned)((cnt + 255) / 256);
        double *prev = Q, *cur = T, *gy = Z, *nxt = Yb;
        if (paff) {
            (*paff)(Q, cur, 1.0 / hh, -e / hh, Q, 0.0, nullptr);
        } else {
            prod(Q, gy);
            hipLaunchKernelGGL(k_cheb, dim3(grid), dim3(256), 0, s, cur, gy, Q, (const double *)nullptr, cnt,
                               1.0 / hh, -e / hh, 0.0);
        }
        for (int j = 1; j < m; ++j) {
            if (paff) {
                (*paff)(cur, nxt, 2.0 / hh, -2.0 * e / hh, cur, -1.0, prev);
            } else {
                prod(cur, gy);
                hipLaunchKernelGGL(k_cheb, dim3(grid), dim3(256), 0, s, nxt, gy, cur, prev, cnt, 2.0 / hh,
                                   -2.0 * e / hh, -1.0);
            }
            double *old = prev;
            prev = cur;
            cur = nxt;
            nxt = old;
        }
        TP_HIP(hipGetLastError());
        // cur holds Y_m; orthonormalise into Q (the CholQR temp must differ)
        double *tmp = (cur == T) ? Yb : T;
        if (cur == Q) {   // never: Q is Y_0 and m >= 1, but keep the buffers distinct
            TP_HIP(hipMemcpyAsync(tmp, cur, cnt * sizeof(double), hipMemcpyDeviceToDevice, s));
            cur = tmp;
            tmp = (cur == T) ? Yb : T;
        }
        orth_cholqr(c, cur, Q, tmp, n, b, Wsm, Xinv, Yinv, d_info, 1, 1e-14);
    };
    const double target = 1e-12;
    const int max_deg = 600;
    // phase 1: four plain iterations as two squared ones (Z = A (A Q), one
    // CholQR each), then read the spectrum estimate off the Cholesky
    // diagonal (|U_jj| -> lambda_j^2 in orthogonal iteration on A^2)
    int done = 4;
    for (int it = 0; it < 2; ++it) {
        prod(Q, T);
        prod(T, Z);
        orth_cholqr(c, Z, Q, T, n, b, Wsm, Xinv, Yinv, d_info, 1, 1e-14);
    }
    double cut = 0.0, gk = 2.0, g1cap = 10.0;
    int mdeg = 1;
    {
        std::vector<double> dg(b);
        hipLaunchKernelGGL(k_diag, dim3((b + 255) / 256), dim3(256), 0, s, Wsm, b, resid);
        double *pn = (double *)c.pinned((size_t)b * sizeof(double));
        TP_HIP(hipMemcpyAsync(pn, resid, b * sizeof(double), hipMemcpyDeviceToHost, s));
        stream_sync(c, s);
        memcpy(dg.data(), pn, b * sizeof(double));
        for (double &x : dg) x = std::sqrt(x);
        const double l1 = dg[0], lk = dg[k - 1], lb = dg[b - 1];
        cut = lb;
        if (cut > 0 && lk > cut && l1 >= lk) {
            const double x1 = 2.0 * l1 / cut - 1.0, xk = 2.0 * lk / cut - 1.0;
            const double g1 = x1 + std::sqrt(x1 * x1 - 1.0);
            gk = xk + std::sqrt(xk * xk - 1.0);
            g1cap = g1;
            // keep the filtered block CholQR-conditionable: (g1/gk)^m <= 1e6
            mdeg = (int)std::floor(std::log(1e6) / std::log(std::max(g1 / gk, 1.0001)));
            mdeg = std::max(1, std::min(8, mdeg));
        } else {
            cut = 0.0;
        }
        st.rate = gk > 1 ? 1.0 / gk : 0.9;
        int need = (int)std::ceil(std::log(1.0 / target) / std::log(std::max(gk, 1.0005))) + cfg_pca_margin + margin;
        need = std::min(need, max_deg);
        if (cut > 0) {
            // Block degrees double: after total degree D the j-th column's
            // components along the larger eigenvectors l < j have shrunk
            // by (g_j/g_l)^D, so a block of degree D + mdeg amplifies them
            // no more than the first block of degree mdeg did.  Capped so
            // T_m(lambda_1) stays far from overflow in the Gram matrix.
            const int mcap = std::max(1, std::min(24, (int)std::floor(100.0 / std::log10(std::max(g1cap, 10.0)))));
            // The span of a filtered block is accurate only to ~kappa eps, kappa
            // ~ the block's amplification ratio (g1/gk)^m: a schedule ending on a
            // long block stalls near 1e-10 (C3's small problem: planned 31
            // degrees, 8.9e-11 after 37).  The last `tail` degrees (a factor
            // 1e3 at the rate gk) therefore go in blocks of at most 2.
            const int tail = std::min(need, (int)std::ceil(std::log(1e3) / std::log(std::max(gk, 1.0005))));
            int deg = 0;
            while (deg < need) {
                int m = std::min({need - deg, std::max(mdeg, deg + mdeg), mcap});
                if (need - deg <= tail) m = std::min(m, std::min(2, mdeg));
                else m = std::min(m, need - tail - deg);
                cheb_block(m, cut);
                deg += m;
                ++st.blocks;
            }
            done += need;
        } else {
            iterate(need);
            done += need;
        }
    }
    std::vector<double> h_res(k);
    h_theta.resize(b);
    for (int round = 0; round < 6; ++round) {
        // Rayleigh-Ritz: orthonormalise tightly, H = Q'AQ, eigen-decompose, rotate
        // Q is orthonormal to ~kappa^2 eps after the last one-pass CholQR:
        // one more pass on Q itself restores eps-orthonormality
        orth_cholqr(c, Q, Z, T, n, b, Wsm, Xinv, Yinv, d_info, 1, 1e-14);
        std::swap(Q, Z);
        prod(Q, Z);
        GemmArgs hq{b, b, n, Q, n, true, Z, n, Wsm, b};
        hq.sym_upper = true;
        hq.splitk = std::max(1, std::min(32, n / 128));
        gemm_f64(hq, c.buf[S_PARTIAL], s);
        eig_sym(Wsm, b, theta, c.buf[S_PARTIAL].as<double>((size_t)b * b + 4 * b + 64), s);
        size_t tot = (size_t)b * b;
        hipLaunchKernelGGL(k_select_rev, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, Wsm, b, b, Xinv);
        // rotate: V = Q X (into T); A V = (A Q) X = Z X for the residuals of
        // the top k Ritz pairs, ||A v - theta v||, without another product
        // with A (into Yb)
        GemmArgs rq{n, b, b, Q, n, false, Xinv, b, T, n};
        rq.splitk = 0;
        gemm_f64(rq, c.buf[S_PARTIAL], s);
        GemmArgs gv{n, k, b, Z, n, false, Xinv, b, Yb, n};
        gv.splitk = 0;
        gemm_f64(gv, c.buf[S_PARTIAL], s);
        std::swap(Q, T);
        hipLaunchKernelGGL(k_resid, dim3(k), dim3(256), 0, s, Yb, Q, theta, n, b, k, resid);
        TP_HIP(hipGetLastError());
        {
            // one pinned staging, one sync (pageable read-backs each stage
            // and synchronise on their own)
            double *pn = (double *)c.pinned((size_t)(k + b) * sizeof(double));
            TP_HIP(hipMemcpyAsync(pn, resid, k * sizeof(double), hipMemcpyDeviceToHost, s));
            TP_HIP(hipMemcpyAsync(pn + k, theta, b * sizeof(double), hipMemcpyDeviceToHost, s));
            stream_sync(c, s);
            memcpy(h_res.data(), pn, k * sizeof(double));
            memcpy(h_theta.data(), pn + k, b * sizeof(double));
        }
        st.d_theta = theta;
        const double th1 = std::fabs(h_theta[b - 1]);
        double worst = 0.0;
        for (int j = 0; j < k; ++j) worst = std::max(worst, h_res[j] / (th1 > 0 ? th1 : 1.0));
        st.resid = worst;
        const double thk = h_theta[b - k], thb = h_theta[0];
        const double rho = (thk > 0 && thb > 0) ? std::min(0.98, std::max(1e-3, thb / thk)) : 0.9;
        st.rate = rho;
        if (getenv("TP_TRACE_PCA"))
            fprintf(stderr, "[pca] n=%d round %d degree %d worst %.2e thk/thb %.3f cut %.3e gk %.3f mdeg %d\n", n,
                    round, done, worst, thb > 0 ? thk / thb : 0.0, cut, gk, mdeg);
        if (!(worst > target * 10) || done >= max_deg) break;
        int more;
        if (cut > 0) {
            // Ritz values bound the spectrum better now: cut at theta_b and
            // take the Chebyshev growth at theta_k per degree for the
            // factor worst / target still to remove
            cut = std::max(cut, thb);
            double g = 1.0005;
            if (thk > cut) {
                const double x = 2.0 * thk / cut - 1.0;
                g = std::max(g, x + std::sqrt(x * x - 1.0));
            }
            const int need = (int)std::ceil(std::log(worst / target) / std::log(g)) + 1;
            more = std::max(1, std::min(max_deg - done, need));
            for (int deg = 0; deg < more; deg += mdeg) cheb_block(std::min(mdeg, more - deg), cut);
        } else {
            const int need = (int)std::ceil(std::log(target / worst) / std::log(rho)) + 2;
            more = std::max(2, std::min(max_deg - done, need));
            iterate(more);
        }
        done += more;
    }
    st.iters = done;
    if (!(st.resid <= 1e-8)) fail(TP_ERR_NUMERIC, "PCA subspace iteration did not converge");
    TP_HIP(hipMemcpyAsync(V, Q, (size_t)n * k * sizeof(double), hipMemcpyDeviceToDevice, s));
}

// The projected problem of the Krylov paths: the top k eigenpairs of T (D x
// D, symmetric, ld D) by the subspace iteration above (products with T are
// D x D GEMMs, the Chebyshev step in their split-K reduction).  Vs: D x k.

static void band_ty(const double *T, const double *Y, double *Out, int D, int b, int p, bool aff, double a, double bc,
                    const double *Yc, double cc, const double *Yp, hipStream_t s) {
    if (p % 32 || p > 64 || D % p || b % 16) fail(TP_ERR_ARG, "band_ty: p must be 32 or 64, D a multiple of p, b of 16");
    const dim3 grid(D / p, b / 16), blk(12 * p);
    if (p == 64) {
        if (aff) hipLaunchKernelGGL((k_band_ty<true, 64>), grid, blk, 0, s, T, Y, Out, D, a, bc, Yc, cc, Yp);
        else hipLaunchKernelGGL((k_band_ty<false, 64>), grid, blk, 0, s, T, Y, Out, D, 0.0, 0.0, nullptr, 0.0, nullptr);
    } else {
        if (aff) hipLaunchKernelGGL((k_band_ty<true, 32>), grid, blk, 0, s, T, Y, Out, D, a, bc, Yc, cc, Yp);
        else hipLaunchKernelGGL((k_band_ty<false, 32>), grid, blk, 0, s, T, Y, Out, D, 0.0, 0.0, nullptr, 0.0, nullptr);
    }
    TP_HIP(hipGetLastError());
}

void small_topk_T(Ctx &c, double *Tm, int D, int k, double *Vs, std::vector<double> &h_theta, PcaStats &sst, int band_p) {
    hipStream_t s = c.cur;
    const bool band = band_p > 0 && cfg_pca_band;
    Prod tprod = [&](const double *Y, double *Out) {
        if (band) {
            band_ty(Tm, Y, Out, D, sst.block, band_p, false, 0, 0, nullptr, 0, nullptr, s);
            return;
        }
        GemmArgs g{D, sst.block, D, Tm, D, true, Y, D, Out, D};
        g.splitk = 0;
        gemm_f64(g, c.buf[S_PARTIAL], s);
    };
    ProdAff taff = [&](const double *Y, double *Out, double a, double b, const double *Yc, double cc,
                       const double *Yp) {
        if (band) {
            band_ty(Tm, Y, Out, D, sst.block, band_p, true, a, b, Yc, cc, Yp, s);
            return;
        }
        GemmArgs g{D, sst.block, D, Tm, D, true, Y, D, Out, D};
        g.splitk = 0;
        g.affine = true;
        g.af_a = a;
        g.af_b = b;
        g.af_y = Yc;
        g.af_c = cc;
        g.af_z = Yp;
        gemm_f64(g, c.buf[S_PARTIAL], s);
    };
    // +2 planned degrees: a product with T costs ~1.5 % of a Rayleigh-Ritz
    // round (one-workgroup tridiagonalisation) that a near miss of the
    // residual check would add
    subspace_topk(c, Tm, D, k, tprod, Vs, h_theta, sst, 0x5EEDULL + (uint64_t)D, 2, cfg_pca_cheb_fused ? &taff : nullptr);
}

// Block Krylov path (see the file comment): V (n x k) = top-k eigenvectors of
// G = Xc'Xc without forming G, or Xc: C is symmetric, so with m = colMeans(C)
// Xc K = C K - 1 (m'K) and Xc'Y = C Y - m (1'Y) -- both products stream C
// itself and the centring is two rank-1 corrections of an n x p block.
// Blocks K_t (n x p) in S_KRY, G K_t in S_KRYG, T = K'GK in S_KRYT, the small
// problem's vectors in S_KRYV.
static int krylov_block(int k) { return cfg_pca_krylov_block > 0 ? cfg_pca_krylov_block : (k >= 128 ? 64 : 32); }

static void krylov_topk(Ctx &c, double *C, int c_col0, const double *mext, int n, int k, double *V, double *P,
                        std::vector<double> &h_theta, PcaStats &st, const ProdDigits *pd) {
    hipStream_t s = c.cur;
    const int p = krylov_block(k);
    // D ~ 5k columns; denser spectra of larger matrices need more (C5 arms:
    // +4 steps at 24k bins)
    int steps = (5 * k + p - 1) / p;
    if (n > 12000) steps += 2 * (int)std::ceil(std::log2((double)n / 12000.0));
    if (cfg_pca_krylov_steps > 0) steps = cfg_pca_krylov_steps;
    const int smax = std::max(steps, std::min(steps + 24, (n / 2) / p));
    steps = std::min(steps, smax);
    double *K = c.buf[S_KRY].as<double>((size_t)n * p * smax);
    double *GK = c.buf[S_KRYG].as<double>((size_t)n * p * smax);
    double *XK = c.buf[S_KRYX].as<double>((size_t)n * p * smax);   // Xc K_t: the scores come from it
    const size_t np = (size_t)n * p;
    const unsigned g1 = (unsigned)((np + 255) / 256);
    // The CGS2 coefficients of both passes, H1 and H2 (Dm x Dm each, ld Dm):
    // column block t - 1 holds K'(G K_{t-1}) and K'W1 of step t, so their sum
    // is T's column block t - 1 above and on the diagonal (G K_{t-1} = K (H1 +
    // H2) + K_t R with K_t orthogonal to K): T = K'GK without its own product
    const int Dm = p * smax;
    double *H1 = c.buf[S_KRYH].as<double>(2 * (size_t)Dm * Dm);
    double *H2 = H1 + (size_t)Dm * Dm;
    // per-step scratch; re-fetched by every extend() because the small
    // problem (subspace_topk) grows and reallocates the same slots
    double *W, *Zt, *Wsm, *Xinv, *Yinv;
    int *d_info;
    auto scratch = [&]() {
        W = c.buf[S_Q].as<double>(np);
        Zt = c.buf[S_Z].as<double>(np);
        Wsm = c.buf[S_SMALL].as<double>((size_t)3 * p * p + 2 * p + 64);
        Xinv = Wsm + (size_t)p * p;
        Yinv = Xinv + (size_t)p * p;
        d_info = c.buf[S_MISC].as<int>(64);
    };
    scratch();
    hipLaunchKernelGGL(k_rand_block, dim3(g1), dim3(256), 0, s, W, n, p, 0x5EEDULL + (uint64_t)n);
    TP_HIP(hipGetLastError());
    orth_cholqr(c, W, K, Zt, n, p, Wsm, Xinv, Yinv, d_info, 2, 1e-14);
    const double target = 1e-12;
    int built = 0;   // blocks with G K_t computed
    int kdone = 1;   // blocks K_t available
    auto extend = [&](int upto) {
        scratch();
        for (int t = built; t < upto; ++t) {
            if (t >= kdone) {
                // K_t: G K_{t-1} re-orthogonalised twice against K_0..K_{t-1} (CGS2), CholQR2.
                // W = src - K (K'src) in the product's epilogue (src = G K_{t-1}, then W)
                const int D = t * p;
                // Pass 0 against the last two blocks only (knob 28): G K_{t-1}
                // lies in span(K_{t-2}, K_{t-1}, K_t) in exact arithmetic, so
                // the older blocks' coefficients are rounding-level, and pass
                // 1 (against every block) removes them -- local
                // orthogonalisation + full reorthogonalisation, half the
                // streaming of K.  T's band needs only those two blocks of H1.
                for (int pass = 0; pass < 2; ++pass) {
                    const double *src = pass == 0 ? GK + (size_t)(t - 1) * np : W;
                    const int D0 = (pass == 0 && cfg_krylov_local) ? std::max(0, (t - 2) * p) : 0;
                    double *Hc = (pass == 0 ? H1 : H2) + (size_t)(t - 1) * p * Dm + D0;   // column block t - 1
                    const double *Kc = K + (size_t)D0 * n;
                    GemmArgs pr{D - D0, p, n, Kc, n, true, src, n, Hc, Dm};   // K'src
                    pr.splitk = 0;
                    gemm_f64(pr, c.buf[S_PARTIAL], s);
                    GemmArgs up{n, p, D - D0, Kc, n, false, Hc, Dm, W, n};   // W = src - K (K'src)
                    up.splitk = 0;
                    up.sub_from = src;
                    gemm_f64(up, c.buf[S_PARTIAL], s);
                }
                orth_cholqr(c, W, K + (size_t)t * np, Zt, n, p, Wsm, Xinv, Yinv, d_info, 2, 1e-14);
                kdone = t + 1;
            }
            double *Kt = K + (size_t)t * np;
            double *GKt = GK + (size_t)t * np;
            double *XKt = XK + (size_t)t * np;
            // [C | m | 1]' B: rows n and n + 1 of the product are m'B and 1'B,
            // so each centring correction rides in the product's reduction
            kprof_begin(c, K_GQ_GEMM);
            const R1 r_xk{n, nullptr, n};        // Xc K_t = C K_t - 1 (m'K_t)
            rows_gemm_sharded(c, C, n, n + 2, Kt, n, p, n, XKt, 0, 1, &r_xk, c_col0, pd);
            kprof_end(c, K_GQ_GEMM);
            kprof_begin(c, K_GQ_GEMM);
            const R1 r_gk{n + 1, mext, n};   // Xc'(Xc K_t) = C (Xc K_t) - m (1'Xc K_t)
            rows_gemm_sharded(c, C, n, n + 2, XKt, n, p, n, GKt, 0, 1, &r_gk, c_col0, pd);
            kprof_end(c, K_GQ_GEMM);
        }
        built = std::max(built, upto);
    };
    std::vector<double> h_res(k);
    for (;;) {
        extend(steps);
        const int D = steps * p;
        trace_mark(s, "pca: krylov");
        // T = K'GK from the CGS2 coefficients; the last column block (no
        // step after it) by one K'(G K_{s-1}) product
        {
            GemmArgs lg{D, p, n, K, n, true, GK + (size_t)(steps - 1) * np, n, H1 + (size_t)(steps - 1) * p * Dm, Dm};
            lg.splitk = 0;
            gemm_f64(lg, c.buf[S_PARTIAL], s);
            TP_HIP(hipMemset2DAsync(H2 + (size_t)(steps - 1) * p * Dm, (size_t)Dm * sizeof(double), 0,
                                    (size_t)D * sizeof(double), p, s));
        }
        double *Tm = c.buf[S_KRYT].as<double>((size_t)D * D);
        {
            const size_t cnt = (size_t)D * D;
            hipLaunchKernelGGL(k_assemble_T, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, H1, H2, Dm, D, p, Tm);
            TP_HIP(hipGetLastError());
        }
        double *Vs = c.buf[S_KRYV].as<double>((size_t)D * k);
        PcaStats sst;
        small_topk_T(c, Tm, D, k, Vs, h_theta, sst, p);
        // V = K Y, G V = (G K) Y; residuals in the n-dimensional space
        GemmArgs vg{n, k, D, K, n, false, Vs, D, V, n};
        vg.splitk = 0;
        gemm_f64(vg, c.buf[S_PARTIAL], s);
        double *GV = c.buf[S_Q].as<double>((size_t)n * k);
        GemmArgs gg{n, k, D, GK, n, false, Vs, D, GV, n};
        gg.splitk = 0;
        gemm_f64(gg, c.buf[S_PARTIAL], s);
        const int bs = (int)h_theta.size();
        // the small problem's Ritz values are still on the device (S_SMALL)
        double *resid = c.buf[S_MISC].as<double>(64 + 2 * (size_t)bs + k) + 64 + bs;
        hipLaunchKernelGGL(k_resid, dim3(k), dim3(256), 0, s, GV, V, sst.d_theta, n, bs, k, resid);
        TP_HIP(hipGetLastError());
        double *pn = (double *)c.pinned((size_t)k * sizeof(double));
        TP_HIP(hipMemcpyAsync(pn, resid, k * sizeof(double), hipMemcpyDeviceToHost, s));
        event_mark(c, s);
        // scores P = Xc V = (Xc K) Y: an n x D by D x k product instead of
        // another pass over Xc (2 n D k flops, not 2 n^2 k), queued behind the
        // residual read-back so the device has work while the host checks it
        // (recomputed if the check extends the space); the host waits for the
        // read-back only, and queues the sweep while the product runs
        GemmArgs pg{n, k, D, XK, n, false, Vs, D, P, n};
        pg.splitk = 0;
        gemm_f64(pg, c.buf[S_PARTIAL], s);
        event_sync(c);
        memcpy(h_res.data(), pn, k * sizeof(double));
        const double th1 = std::fabs(h_theta[bs - 1]);
        double worst = 0.0;
        for (int j = 0; j < k; ++j) worst = std::max(worst, h_res[j] / (th1 > 0 ? th1 : 1.0));
        st.resid = worst;
        st.iters = sst.iters;
        st.block = sst.block;
        st.blocks = sst.blocks;
        st.krylov_steps = steps;
        st.krylov_dim = D;
        if (getenv("TP_TRACE_PCA"))
            fprintf(stderr, "[pca] krylov n=%d p=%d steps=%d D=%d small: degree %d resid %.2e | n-space worst %.2e\n",
                    n, p, steps, D, sst.iters, sst.resid, worst);
        if (!(worst > target * 10) || steps >= smax) break;
        steps = std::min(smax, steps + 4);
    }
    if (!(st.resid <= 1e-8)) fail(TP_ERR_NUMERIC, "PCA block Krylov iteration did not converge");
}

PcaStats pca_dev(Ctx &c, double *d_C, int n, int k, double *d_P, double *d_Pt, double *h_sdev,
                 const double *d_cmean, int c_col0, int c_col1, bool cm_pending) {
    PcaStats st;
    hipStream_t s = c.cur;
    const double *mean = d_cmean;
    const int b_est = std::min(n, ((k + std::max(32, k / 4) + 31) / 32) * 32);
    const bool krylov = n >= t_knob.pca_krylov_min && b_est < n;
    const bool cspace = t_knob.pca_ckrylov > 0 || (t_knob.pca_ckrylov < 0 && n >= cfg_ckry_min);
    const int cend = c_col1 < 0 ? n + 2 : c_col1;
    // the int8-digit products: the G-space blocks of krylov_block(k) columns, the
    // C-space blocks of 32 (knob 45)
    const bool i8 = krylov && t_knob.prod_i8 > 0 &&
                    (cspace ? t_knob.pd_cspace != 0 && prod_i8_ok(n, 32) : prod_i8_ok(n, krylov_block(k)));
    // cm_pending: d_cmean is where C's column means go; with the int8 products
    // over all of [C | m | 1] they come out of A's digit pass (k_colmean's bits)
    const bool cm_fused = cm_pending && i8 && c_col0 == 0 && cend == n + 2 && prod_digits_means_ok(n);
    if (cm_pending && !d_cmean) fail(TP_ERR_INTERNAL, "pca_dev: pending means need their buffer");
    if (cm_pending && !cm_fused) launch_colmean(d_C, n, n, const_cast<double *>(d_cmean), s);
    if (!mean) {
        double *cm = c.buf[S_COLMEAN].as<double>(n);
        launch_colmean(d_C, n, n, cm, s);
        mean = cm;
    }
    double *V = c.buf[S_W].as<double>((size_t)n * k);       // n x k, descending
    std::vector<double> h_theta;
    double *Xc = nullptr, *XcT = nullptr;
    if (c_col0 != 0 && !krylov) fail(TP_ERR_ARG, "pca_dev: a column slab of C needs the Krylov path");
    if (krylov) {
        // the int8-digit image of this rank's columns of [C | m | 1] for the
        // ~32 products with it (tp_prod_i8.hip); with fused means its first n
        // columns now, m and 1 once they are written below
        ProdDigits pdg;
        const ProdDigits *pd = nullptr;
        if (cm_fused) prod_digits_build(c, d_C, n, n, n + 2, 0, pdg, const_cast<double *>(d_cmean), n);
        // [m | 1] (the centring's rank-1 terms) for every rank, and as columns
        // n, n + 1 of [C | m | 1] (the products' extra rows m'B, 1'B) where
        // this rank holds them (all of C, or the last rank's slab)
        double *mext = c.buf[S_MEXT].as<double>(2 * (size_t)n);
        if (mean != mext) TP_HIP(hipMemcpyAsync(mext, mean, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(k_fill_const, dim3((n + 255) / 256), dim3(256), 0, s, mext + n, n, 1.0);
        TP_HIP(hipGetLastError());
        if (c_col0 <= n && cend >= n + 2)
            TP_HIP(hipMemcpyAsync(d_C + (size_t)(n - c_col0) * n, mext, 2 * (size_t)n * sizeof(double),
                                  hipMemcpyDeviceToDevice, s));
        // neither Xc nor XcT is formed; the Krylov space of C (tp_krylov.hip),
        // or of G when an orthogonalisation pass of that path breaks down
        if (cm_fused) {
            prod_digits_finish(c, d_C, n, n, pdg);
            pd = &pdg;
        } else if (i8) {
            prod_digits_build(c, d_C, n, n, cend - c_col0, c_col0, pdg);
            pd = &pdg;
        }
        if (!cspace || !krylov_c_topk(c, d_C, c_col0, mext, n, k, V, d_P, h_theta, st, pd)) {
            h_theta.clear();
            st = PcaStats{};
            krylov_topk(c, d_C, c_col0, mext, n, k, V, d_P, h_theta, st, pd);
            st.prod_pairs = pd ? prod_i8_pairs() : 0;
        }
    } else {
        Xc = c.buf[S_XC].as<double>((size_t)n * n);
        XcT = c.buf[S_XCT].as<double>((size_t)n * n);
        launch_center(d_C, mean, n, Xc, XcT, s);
        double *G = c.buf[S_G].as<double>((size_t)n * n);
        {
            GemmArgs g{n, n, n, Xc, n, true, Xc, n, G, n};
            g.sym_upper = true;
            kprof_begin(c, K_G_GEMM);
            sym_gemm_sharded(c, g);
            kprof_end(c, K_G_GEMM);
        }
        trace_mark(s, "pca: G");
        Prod gq = [&](const double *Yin, double *Out) {   // Out = G Yin (row-sharded)
            kprof_begin(c, K_GQ_GEMM);
            rows_gemm_sharded(c, G, n, n, Yin, n, st.block, n, Out, 0, 1);
            kprof_end(c, K_GQ_GEMM);
        };
        subspace_topk(c, G, n, k, gq, V, h_theta, st, 0x5EEDULL + (uint64_t)n);
    }
    // scores P = Xc V  (= XcT' V): n x k column-major; Pt row-major (the
    // Krylov path formed them from its stored Xc K_t)
    if (!krylov) rows_gemm_sharded(c, XcT, n, n, V, n, k, n, d_P, 0);
    if (d_Pt) launch_transpose(d_P, n, k, n, d_Pt, k, s);
    if (h_sdev) {
        // prcomp sdev = d / sqrt(max(1, n-1)), d = singular values of Xc = sqrt(eig(G))
        int bb = (int)h_theta.size();
        for (int j = 0; j < k; ++j) {
            double e = h_theta[bb - 1 - j];
            h_sdev[j] = std::sqrt(std::max(0.0, e)) / std::sqrt((double)std::max(1, n - 1));
        }
    }
    return st;
}

}  // namespace tp
