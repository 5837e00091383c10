// prcomp(cor, rank. = k) (R/TADpole.R:452-453) by block Krylov in C itself.
//
// G = Xc'Xc with Xc = C - 1 m' (m = colMeans(C), C symmetric), so Xc = Pc C
// and G = C Pc C.  A Krylov space of C whose start block holds the vector 1
// contains the Krylov space of G of half the depth, and it grows by one
// product with C per block instead of two: for PSD C the degree-2s polynomial
// in C is also the better filter (T_2s(x) on [0, a] against T_s(2x^2 - 1) on
// [0, a^2]).  Measured on the C3 / 10k matrices (tools/krylov_c_model.py):
// blocks of 32 columns, 33 blocks give Ritz residuals 3-4e-13 with 34
// products of 32 columns, against 1.1e-12 for 32 products of 64 columns on G.
//
//   K_0 = orth([1 | random]);  P_t = Xc K_t = C K_t - 1 (m'K_t)  (one pass
//   over C, the rank-1 term in the split-K reduction);  K_{t+1} = P_t made
//   orthogonal to K_0..K_t by BCGS-PIP2: per pass Z = [K W]'W, R = chol(Z_w -
//   H'H) (H = K'W), W <- (W - K H) R^-1 -- two passes.
//   T = P'P = K'GK (the exact Rayleigh quotient of G on span K), its top-k
//   pairs by the subspace iteration of tp_pca.hip, V = K Y, scores Xc V = P Y.
//   Residual without a product with a k-column block: Xc v lies in
//   span(K_0..K_s), so G v = Xc'Q (Q' Xc v) with Q = [K_0..K_s] and
//   Xc'Q = P_Q + 1 (m'Q) - m (1'Q) -- one more block, then small products.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "tp_common.cuh"
#include "tp_internal.h"
#include "tp_krylov_kernels.cuh"

namespace tp {

// resid[j] = || GV_j + a_j 1 - b_j m - theta_j V_j ||, ab = [a_j; b_j] (2 x k)
__global__ void __launch_bounds__(256) k_resid_c(const double *GV, const double *V, const double *ab, const double *m,
                                                 const double *theta_asc, int n, int bs, int k, double *resid) {
    __shared__ double red[4];
    const int j = blockIdx.x;
    const int t = threadIdx.x;
    const double th = theta_asc[bs - 1 - j], a = ab[2 * j], b = ab[2 * j + 1];
    double acc = 0.0;
    for (int i = t; i < n; i += 256) {
        const double r = GV[(size_t)j * n + i] + a - b * m[i] - th * V[(size_t)j * n + i];
        acc = fma(r, r, acc);
    }
    acc = wave_sum(acc);
    if ((t & 63) == 0) red[t >> 6] = acc;
    __syncthreads();
    if (t == 0) resid[j] = sqrt(((red[0] + red[1]) + red[2]) + red[3]);
}

// deterministic start block [1 | uniform(-1, 1)] (n x KP)
__global__ void k_start_block(double *Q, int n, uint64_t seed) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)n * KP) return;
    if (idx < (size_t)n) {
        Q[idx] = 1.0;
        return;
    }
    uint64_t z = seed + 0x9E3779B97F4A7C15ULL * (idx + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    Q[idx] = ((double)(z >> 11) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
}

// Default off: at C3 the 34 products of 32 columns take 4.7 ms against 6.3 ms
// for the G path's 32 of 64, but the 66 orthogonalisation passes (each a
// split-K reduction over n, its reduce, the small step and the apply: ~75 us,
// latency-bound) cost 5.1 ms against the G path's 3.3 ms: PCA 14.9 vs 14.1 ms
// (profiles/r03b_*).  Kept, tested, behind knob 20.
// 1: Krylov in C (this file), 0: Krylov in G (tp_pca.hip), -1: C from
// cfg_ckry_min bins on.  Measured (round 4, MI355X, PCA ms G vs C): 10k bins
// 18.3 vs 18.1, 24.3k bins 96.0 vs 77.3 -- the C space halves the product
// flops, and above ~10k bins that outweighs its costlier orthogonalisation
// (at C3, 7.7k bins, the G space is ~0.8 ms faster)

// One BCGS-PIP pass of block slot `D / KP` (columns D..D+KP-1 of Kb, n x KP):
// W0 is the block to orthonormalise against Kb's first D columns (W0 may be
// the slot itself); the result lands in the slot.
struct PipScratch {
    double *part, *Z, *hh, *Ri, *apart;
    int *info;
};
// local >= 4: the pass runs against K_0 and the two blocks before slot `local`
// only (a local first pass, see krylov_c_topk); the result still lands in
// slot D / KP = local.
// Rows per Z partial: ~1024 workgroups of k_pipz (dt column tiles x n /
// chunk row chunks), 512 to 1024 rows (fewer partials for k_pipr to sum; 24.3k
// bins, PCA: fixed 256 rows 74.5 ms, 512 73.4, 768 73.3, 1024 73.7)
static int pip_chunk(int n, int dt) {
    if (cfg_ckry_chunk > 0) return std::max(64, cfg_ckry_chunk);
    const long want = ((long)n * dt / 1024 + 63) / 64 * 64;
    return (int)std::max<long>(512, std::min<long>(1024, want));
}
static void pip_pass(Ctx &c, double *Kb, int n, int D, const double *W0, const PipScratch &ps, double shift,
                     int lowdin = 0, int local = 0) {
    hipStream_t s = c.cur;
    double *out = Kb + (size_t)D * n;
    const double *Kt = nullptr;
    int Dh = -1;
    if (local >= 4) {
        Kt = Kb + (size_t)(local - 2) * KP * n;
        Dh = KP;
        D = 3 * KP;
    }
    const int ldz = D + KP;
    const int dt = (ldz + PZ_COLS - 1) / PZ_COLS;
    const int chunk = pip_chunk(n, dt);
    const int S = (n + chunk - 1) / chunk;
    const size_t pstride = (size_t)ldz * KP;
    hipLaunchKernelGGL(k_pipz, dim3((unsigned)(dt * S)), dim3(256), 0, s, Kb, D, W0, n, chunk, ps.part, pstride, Kt,
                       Dh);
    const int nsl = (ldz + PR - 1) / PR, nh = (D + PR - 1) / PR;
    hipLaunchKernelGGL(k_pipr, dim3((unsigned)nsl), dim3(PR_TB), 0, s, ps.part, pstride, S, D, ps.Z, ps.hh);
    hipLaunchKernelGGL(k_pips<3>, dim3(1), dim3(512), 0, s, ps.Z, D, ps.hh, nh, shift, ps.Ri, ps.info, lowdin);
    const int tiles = (n + PA_ROWS - 1) / PA_ROWS;
    if (D > 0)
        hipLaunchKernelGGL(k_pipa, dim3((unsigned)(tiles * PA_SPLIT)), dim3(256), 0, s, Kb, D, n, ps.Z, ps.apart, Kt,
                           Dh);
    else
        TP_HIP(hipMemsetAsync(ps.apart, 0, (size_t)tiles * PA_SPLIT * PA_ROWS * KP * 8, s));
    hipLaunchKernelGGL(k_pipc, dim3((unsigned)tiles), dim3(256), 0, s, ps.apart, ps.Ri, n, W0, out);
    TP_HIP(hipGetLastError());
}

size_t ckry_partial_doubles(int n, int dmax) {
    // the most partials any pass needs: the smallest chunk is the floor's
    const int chunk = cfg_ckry_chunk > 0 ? std::max(64, cfg_ckry_chunk) : 512;
    return (size_t)((n + chunk - 1) / chunk) * (size_t)(dmax + KP) * KP;
}

// the small problem and the n-space check (tp_pca.hip)

bool krylov_c_topk(Ctx &c, double *C, int c_col0, const double *mext, int n, int k, double *V, double *P,
                   std::vector<double> &h_theta, PcaStats &st, const ProdDigits *pd) {
    hipStream_t s = c.cur;
    // blocks before the first check: D ~ 5.28 k (C3 / 10k: 33 blocks of 32 for
    // k = 200), more for the denser spectra of larger matrices
    int steps = (int)std::ceil(5.28 * k / KP);
    if (n > 12000) steps += (int)std::ceil(12.0 * std::log2((double)n / 12000.0));   // 24k: 45 (44 measured)
    if (cfg_ckry_steps > 0) steps = cfg_ckry_steps;
    steps = std::max(1, steps);
    // T = K'GK is block pentadiagonal in the 32-column blocks (G = C Pc C,
    // C K_t in span K_{t-1..t+1}, the rank-1 centring term in K_0, K_1): with
    // an even block count it is block TRIdiagonal in 64-column blocks, so the
    // small problem's products with T are banded (k_band_ty, as the G path)
    if (cfg_pca_band) steps += steps & 1;
    const int smax = std::max(steps, std::min(steps + 48, (n / 2) / KP));
    steps = std::min(steps, smax);
    const size_t np = (size_t)n * KP;
    // K: smax + 1 blocks (the residual block), P the same
    double *K = c.buf[S_KRY].as<double>(np * (smax + 1));
    double *Pb = c.buf[S_KRYX].as<double>(np * (smax + 1));
    const int dmax = (smax + 1) * KP;
    PipScratch ps;
    auto scratch = [&]() {
        ps.part = c.buf[S_KRYG].as<double>(ckry_partial_doubles(n, dmax));
        char *sm = c.buf[S_SMALL2].as<char>((size_t)(dmax + KP) * KP * 8 + (size_t)((dmax + PR - 1) / PR) * KP * KP * 8 +
                                            (size_t)KP * KP * 8 + 256);
        ps.Z = (double *)sm;
        ps.hh = ps.Z + (size_t)(dmax + KP) * KP;
        ps.Ri = ps.hh + (size_t)((dmax + PR - 1) / PR) * KP * KP;
        ps.info = (int *)(ps.Ri + KP * KP);
        const int tiles = (n + PA_ROWS - 1) / PA_ROWS;
        ps.apart = c.buf[S_KRYA].as<double>((size_t)tiles * PA_SPLIT * PA_ROWS * KP);
    };
    scratch();
    TP_HIP(hipMemsetAsync(ps.info, 0, sizeof(int), s));
    hipLaunchKernelGGL(k_start_block, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, K, n,
                       0x5EEDULL + (uint64_t)n);
    TP_HIP(hipGetLastError());
    pip_pass(c, K, n, 0, K, ps, 1e-14);   // CholQR2 of the start block
    pip_pass(c, K, n, 0, K, ps, 0.0);
    int nprod = 0;   // P_0..P_{nprod-1} computed (K_0..K_{nprod-1} formed)
    auto extend = [&](int upto) {   // P_0..P_upto; K_t formed from P_{t-1} just before its product
        scratch();
        for (int t = nprod; t <= upto; ++t) {
            if (t >= 1) {
                const int D = t * KP;
                // Xc K_{t-1} = C K_{t-1} - 1 (m'K_{t-1}) lies in span(K_0, K_{t-2},
                // K_{t-1}, K_t) in exact arithmetic (C symmetric: the block
                // Lanczos recurrence; 1 is in span K_0), so the first pass runs
                // against those blocks only and the second, against every block,
                // removes the rounding-level rest (knob 33)
                pip_pass(c, K, n, D, Pb + (size_t)(t - 1) * np, ps, 1e-14, 0, cfg_ckry_local ? t : 0);
                pip_pass(c, K, n, D, K + (size_t)D * n, ps, 0.0, 1);   // Gram ~ I + 1e-13: Lowdin
            }
            double *Kt = K + (size_t)t * np, *Pt = Pb + (size_t)t * np;
            kprof_begin(c, K_GQ_GEMM);
            const R1 r_xk{n, nullptr, n};   // Xc K_t = C K_t - 1 (m'K_t)
            rows_gemm_sharded(c, C, n, n + 2, Kt, n, KP, n, Pt, 0, 1, &r_xk, c_col0, pd);
            kprof_end(c, K_GQ_GEMM);
        }
        nprod = std::max(nprod, upto + 1);
    };
    // the check with s = steps uses T from P_0..P_{s-1} and the residual block K_s, P_s
    std::vector<double> h_res(k);
    for (;;) {
        extend(steps);
        const int D = steps * KP;
        const int DQ = D + KP;
        trace_mark(s, "pca: c-krylov");
        double *Tm = c.buf[S_KRYT].as<double>((size_t)D * D);
        GemmArgs tg{D, D, n, Pb, n, true, Pb, n, Tm, D};   // T = P'P
        tg.sym_upper = true;
        {
            // a few hundred 64 x 64 upper tiles over K = n: split K so ~1000
            // workgroups run (one k chunk a tile ran 2.2 ms at 24.3k bins, D 1472)
            const long nt = (long)((D + 63) / 64) * ((D + 63) / 64 + 1) / 2;
            tg.splitk = n >= 4096 ? (int)std::max<long>(1, std::min<long>(8, (1024 + nt - 1) / nt)) : 0;
        }
        gemm_f64(tg, c.buf[S_PARTIAL], s);
        double *Vs = c.buf[S_KRYV].as<double>((size_t)D * k);
        PcaStats sst;
        // banded products when T is block tridiagonal in 64-column blocks (its
        // entries off the band are rounding-level and are not read)
        small_topk_T(c, Tm, D, k, Vs, h_theta, sst, (cfg_pca_band && D % 64 == 0) ? 64 : 0);
        // V = K Y, scores Xc V = P Y
        GemmArgs vg{n, k, D, K, n, false, Vs, D, V, n};
        vg.splitk = 0;
        gemm_f64(vg, c.buf[S_PARTIAL], s);
        GemmArgs sg{n, k, D, Pb, n, false, Vs, D, P, n};
        sg.splitk = 0;
        gemm_f64(sg, c.buf[S_PARTIAL], s);
        // residual: z = Q'(Xc V) (DQ x k), ab = [m 1]'Q z (2 x k), G V = P_Q z + 1 a' - m b'
        double *z = c.buf[S_SWEEP].as<double>((size_t)DQ * k + 4 * (size_t)DQ + 4 * (size_t)k + 64);
        double *mq = z + (size_t)DQ * k;
        double *ab = mq + 2 * (size_t)DQ;
        GemmArgs zg{DQ, k, n, K, n, true, P, n, z, DQ};
        zg.splitk = 0;
        gemm_f64(zg, c.buf[S_PARTIAL], s);
        GemmArgs mg{2, DQ, n, mext, n, true, K, n, mq, 2};
        mg.splitk = 0;
        gemm_f64(mg, c.buf[S_PARTIAL], s);
        GemmArgs ag{2, k, DQ, mq, 2, false, z, DQ, ab, 2};
        ag.splitk = 1;
        gemm_f64(ag, c.buf[S_PARTIAL], s);
        double *GV = c.buf[S_Q].as<double>((size_t)n * k);
        GemmArgs gg{n, k, DQ, Pb, n, false, z, DQ, GV, n};
        gg.splitk = 0;
        gemm_f64(gg, c.buf[S_PARTIAL], s);
        const int bs = (int)h_theta.size();
        // the small problem's Ritz values are still on the device (S_SMALL)
        double *resid = c.buf[S_MISC].as<double>(64 + 2 * (size_t)bs + k) + 64 + bs;
        hipLaunchKernelGGL(k_resid_c, dim3(k), dim3(256), 0, s, GV, V, ab, mext, sst.d_theta, n, bs, k, resid);
        TP_HIP(hipGetLastError());
        int hinfo = 0;
        {
            char *pin = (char *)c.pinned((size_t)k * sizeof(double) + 16);
            TP_HIP(hipMemcpyAsync(pin, resid, k * sizeof(double), hipMemcpyDeviceToHost, s));
            TP_HIP(hipMemcpyAsync(pin + (size_t)k * sizeof(double), ps.info, sizeof(int), hipMemcpyDeviceToHost, s));
            stream_sync(c, s);
            memcpy(h_res.data(), pin, k * sizeof(double));
            memcpy(&hinfo, pin + (size_t)k * sizeof(double), sizeof(int));
        }
        if (hinfo) return false;   // an orthogonalisation pass broke down: the caller takes the G path
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
            fprintf(stderr, "[pca] c-krylov n=%d p=%d steps=%d D=%d small: degree %d resid %.2e | n-space worst %.2e\n",
                    n, KP, steps, D, sst.iters, sst.resid, worst);
        if (!(worst > 1e-11) || steps >= smax) break;
        steps = std::min(smax, steps + 8);
    }
    if (!(st.resid <= 1e-8)) fail(TP_ERR_NUMERIC, "PCA block Krylov (C) iteration did not converge");
    return true;
}

}  // namespace tp
