// prcomp(cor, rank. = k)$x  (R/TADpole.R:452-453) on the GPU.
//
// R computes a FULL thin SVD of the column-centred N x N matrix (LAPACK gesdd)
// and keeps k = min(max_pcs, N) right singular vectors.  Here:
//   Xc = C - 1 colMeans(C)'                       (centring, tp_prep.hip)
//   G  = Xc' Xc                                   (fp64 MFMA GEMM, symmetric)
//   block subspace iteration on G, block b = k + oversampling, CholQR2
//   orthonormalisation, Rayleigh-Ritz at the end (b x b eigensolve)
//   P  = Xc V_k                                   (fp64 MFMA GEMM)
// Only span(V_1..V_i) matters downstream (distances and CH are invariant to
// sign and to rotations inside the top-i space), and the iteration stops when
// every Ritz pair j <= k has ||G v - theta v|| <= tol * theta_1.
// When N <= b the Ritz problem is G itself (exact full eigendecomposition).
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include <cstdio>
#include <cstdlib>

#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

static void rb_check(rocblas_status st, const char *what) {
    if (st != rocblas_status_success) fail(TP_ERR_HIP, std::string("rocBLAS/rocSOLVER failure in ") + what);
}

static rocblas_handle blas_for(Ctx &c) {
    if (!c.blas) {
        rocblas_handle h;
        rb_check(rocblas_create_handle(&h), "rocblas_create_handle");
        c.blas = h;
    }
    rocblas_handle h = (rocblas_handle)c.blas;
    rb_check(rocblas_set_stream(h, c.cur), "rocblas_set_stream");
    return h;
}

void blas_shutdown_all() {}   // handles are per context (freed with it)

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

// resid[j] = || Y[:, j] - theta_j V[:, j] ||_2  (one wave per column)
__global__ void __launch_bounds__(256) k_resid(const double *Y, const double *V, const double *theta_asc, int n, int b,
                                               int k, double *resid) {
    int lane = threadIdx.x & 63;
    int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= k) return;
    double th = theta_asc[b - 1 - j];
    double acc = 0.0;
    for (int a = lane; a < n; a += 64) {
        double r = Y[(size_t)j * n + a] - th * V[(size_t)j * n + a];
        acc = fma(r, r, acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) resid[j] = sqrt(acc);
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
        g.splitk = std::max(1, std::min(32, n / 128));
        gemm_f64(g, c.buf[S_PARTIAL], c.cur);
        double *dst = ((passes - 1 - p) % 2 == 0) ? Qout : Tmp;   // last pass lands in Qout
        if (b <= kCholInvMax && b % 16 == 0) {
            launch_chol_inv(W, Y, X + b, X, b, p == 0 ? shift : 0.0, d_info, c.cur);
            launch_trsm_frag(src, n, b, Y, X + b, dst, c.cur);
        } else {
            launch_chol(W, X, b, p == 0 ? shift : 0.0, d_info, c.cur);
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

// |U_jj| of the last Cholesky (upper triangle of W) -> host, ascending index j
__global__ void k_diag(const double *W, int b, double *d) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < b) d[j] = fabs(W[(size_t)j * b + j]);
}

int g_pca_margin = 0;   // extra Chebyshev degrees over the planned count (the residual check adds more when needed; tools/pca_margin.py)

PcaStats pca_dev(Ctx &c, const double *d_C, int n, int k, double *d_P, double *d_Pt, double *h_sdev) {
    PcaStats st;
    hipStream_t s = c.cur;
    double *mean = c.buf[S_COLMEAN].as<double>(n);
    double *Xc = c.buf[S_XC].as<double>((size_t)n * n);
    double *XcT = c.buf[S_XCT].as<double>((size_t)n * n);
    double *G = c.buf[S_G].as<double>((size_t)n * n);
    launch_colmean(d_C, n, n, mean, s);
    launch_center(d_C, mean, n, Xc, XcT, s);
    {
        GemmArgs g{n, n, n, Xc, n, true, Xc, n, G, n};
        g.sym_upper = true;
        kprof_begin(c, K_G_GEMM);
        sym_gemm_sharded(c, g);
        kprof_end(c, K_G_GEMM);
    }
    trace_mark(s, "pca: G");
    const int over = std::max(32, k / 4);
    int b = std::min(n, ((k + over + 31) / 32) * 32);
    st.block = b;
    double *V = c.buf[S_W].as<double>((size_t)n * k);       // n x k, descending
    std::vector<double> h_theta;
    if (b >= n) {
        // exact: eigendecomposition of G itself (small n)
        rocblas_handle h = blas_for(c);
        b = n;
        int *d_info = c.buf[S_MISC].as<int>(64);
        double *theta = c.buf[S_SMALL].as<double>((size_t)n + 64);
        double *E = c.buf[S_Z].as<double>((size_t)n * n);
        TP_HIP(hipMemcpyAsync(E, G, (size_t)n * n * sizeof(double), hipMemcpyDeviceToDevice, s));
        double *offbuf = c.buf[S_Q].as<double>((size_t)n + 64);
        if (eig_sym_supported(n))
            eig_sym(h, E, n, theta, c.buf[S_PARTIAL].as<double>((size_t)n * n + 4 * n + 64), d_info, s);
        else
            rb_check(rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_upper, n, E, n, theta, offbuf,
                                      d_info),
                     "dsyevd");
        size_t tot = (size_t)n * k;
        hipLaunchKernelGGL(k_select_rev, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, E, n, k, V);
        TP_HIP(hipGetLastError());
        h_theta.resize(n);
        TP_HIP(hipMemcpyAsync(h_theta.data(), theta, n * sizeof(double), hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
        trace_mark(s, "pca: exact eig");
        st.iters = 0;
    } else {
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
        // orthonormalises G Q0 directly)
        hipLaunchKernelGGL(k_rand_block, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, Q, n, b,
                           0x5EEDULL + (uint64_t)n);
        TP_HIP(hipGetLastError());
        double *Yb = c.buf[S_SWEEP2].as<double>((size_t)n * b);   // 4th block buffer (sweep scratch later)
        auto gemm_gq = [&](const double *Yin, double *Out) {   // Out = G Yin (row-sharded)
            kprof_begin(c, K_GQ_GEMM);
            rows_gemm_sharded(c, G, n, n, Yin, n, b, n, Out, 0, 1);
            kprof_end(c, K_GQ_GEMM);
        };
        auto iterate = [&](int count) {   // plain subspace iteration
            for (int it = 0; it < count; ++it) {
                gemm_gq(Q, Z);
                orth_cholqr(c, Z, Q, T, n, b, Wsm, Xinv, Yinv, d_info, 1, 1e-14);
            }
        };
        // Chebyshev filter of degree m on [0, cut]: Q <- orth(T_m((G - e)/h) Q),
        // e = h = cut / 2 (scaled three-term recurrence), then CholQR
        auto cheb_block = [&](int m, double cut) {
            const double e = 0.5 * cut, hh = 0.5 * cut;
            const size_t cnt = (size_t)n * b;
            const unsigned grid = (unsigned)((cnt + 255) / 256);
            double *prev = Q, *cur = T, *gy = Z, *nxt = Yb;
            gemm_gq(Q, gy);
            hipLaunchKernelGGL(k_cheb, dim3(grid), dim3(256), 0, s, cur, gy, Q, (const double *)nullptr, cnt,
                               1.0 / hh, -e / hh, 0.0);
            for (int j = 1; j < m; ++j) {
                gemm_gq(cur, gy);
                hipLaunchKernelGGL(k_cheb, dim3(grid), dim3(256), 0, s, nxt, gy, cur, prev, cnt, 2.0 / hh,
                                   -2.0 * e / hh, -1.0);
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
        // phase 1: four plain iterations as two squared ones (Z = G (G Q), one
        // CholQR each), then read the spectrum estimate off the Cholesky
        // diagonal (|U_jj| -> lambda_j^2 in orthogonal iteration on G^2)
        int done = 4;
        for (int it = 0; it < 2; ++it) {
            gemm_gq(Q, T);
            gemm_gq(T, Z);
            orth_cholqr(c, Z, Q, T, n, b, Wsm, Xinv, Yinv, d_info, 1, 1e-14);
        }
        double cut = 0.0, gk = 2.0, g1cap = 10.0;
        int mdeg = 1;
        {
            std::vector<double> dg(b);
            hipLaunchKernelGGL(k_diag, dim3((b + 255) / 256), dim3(256), 0, s, Wsm, b, resid);
            TP_HIP(hipMemcpyAsync(dg.data(), resid, b * sizeof(double), hipMemcpyDeviceToHost, s));
            TP_HIP(hipStreamSynchronize(s));
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
            int need = (int)std::ceil(std::log(1.0 / target) / std::log(std::max(gk, 1.0005))) + g_pca_margin;
            need = std::min(need, max_deg);
            if (cut > 0) {
                // Block degrees double: after total degree D the j-th column's
                // components along the larger eigenvectors l < j have shrunk
                // by (g_j/g_l)^D, so a block of degree D + mdeg amplifies them
                // no more than the first block of degree mdeg did.  Capped so
                // T_m(lambda_1) stays far from overflow in the Gram matrix.
                const int mcap = std::max(1, std::min(24, (int)std::floor(100.0 / std::log10(std::max(g1cap, 10.0)))));
                int deg = 0;
                while (deg < need) {
                    const int m = std::min({need - deg, std::max(mdeg, deg + mdeg), mcap});
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
        rocblas_handle h = blas_for(c);
        for (int round = 0; round < 6; ++round) {
            // Rayleigh-Ritz: orthonormalise tightly, H = Q'GQ, eigen-decompose, rotate
            // Q is orthonormal to ~kappa^2 eps after the last one-pass CholQR:
            // one more pass on Q itself restores eps-orthonormality
            orth_cholqr(c, Q, Z, T, n, b, Wsm, Xinv, Yinv, d_info, 1, 1e-14);
            std::swap(Q, Z);
            rows_gemm_sharded(c, G, n, n, Q, n, b, n, Z, 0);
            GemmArgs hq{b, b, n, Q, n, true, Z, n, Wsm, b};
            hq.sym_upper = true;
            hq.splitk = std::max(1, std::min(32, n / 128));
            gemm_f64(hq, c.buf[S_PARTIAL], s);
            if (eig_sym_supported(b))
                eig_sym(h, Wsm, b, theta, c.buf[S_PARTIAL].as<double>((size_t)b * b + 4 * b + 64), d_info, s);
            else
                rb_check(rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_upper, b, Wsm, b, theta, offd,
                                          d_info),
                         "dsyevd(RR)");
            size_t tot = (size_t)b * b;
            hipLaunchKernelGGL(k_select_rev, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, Wsm, b, b, Xinv);
            // rotate: V = Q X (into T); G V = (G Q) X = Z X for the residuals of
            // the top k Ritz pairs, ||G v - theta v||, without another product
            // with G (into Yb)
            GemmArgs rq{n, b, b, Q, n, false, Xinv, b, T, n};
            rq.splitk = 0;
            gemm_f64(rq, c.buf[S_PARTIAL], s);
            GemmArgs gv{n, k, b, Z, n, false, Xinv, b, Yb, n};
            gv.splitk = 0;
            gemm_f64(gv, c.buf[S_PARTIAL], s);
            std::swap(Q, T);
            hipLaunchKernelGGL(k_resid, dim3((k + 3) / 4), dim3(256), 0, s, Yb, Q, theta, n, b, k, resid);
            TP_HIP(hipGetLastError());
            TP_HIP(hipMemcpyAsync(h_res.data(), resid, k * sizeof(double), hipMemcpyDeviceToHost, s));
            TP_HIP(hipMemcpyAsync(h_theta.data(), theta, b * sizeof(double), hipMemcpyDeviceToHost, s));
            TP_HIP(hipStreamSynchronize(s));
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
    // scores P = Xc V  (= XcT' V): n x k column-major; Pt row-major
    rows_gemm_sharded(c, XcT, n, n, V, n, k, n, d_P, 0);
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
