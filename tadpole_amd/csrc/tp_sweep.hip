// The find_params sweep (R/TADpole.R:102-140) on the GPU.
//
// k_coniss: one wave per tree i (PC prefix 1..i).  CONISS (rioja::chclust,
//   R/TADpole.R:108) in Ward/centroid form: adjacent-pair merge costs live in
//   LDS, a 64-ary min tree (block minima in LDS) gives the leftmost smallest
//   pair, cluster column sums live in HBM (one N x i slab per tree).  Each of
//   the N-1 merges touches O(i) sums and two costs: the dist() matrix of
//   R/TADpole.R:108 is never formed.  The broken stick (rioja bstick.chclust,
//   R/TADpole.R:111-113) runs in the same launch on the tree's heights.
// k_ch: one 256-thread workgroup per tree.  fpc::calinhara (R/TADpole.R:119)
//   for every cut from n_cluster down to min_clusters: segment SS of the finest
//   cut by two passes over rows, then each coarser cut adds the Ward increment
//   of the two segments its merge joins (nested cuts of one tree).
//
// Floating-point order is the canonical one of oracle/tp_oracle.c (64-lane
// strided partials + xor butterfly, explicit fma), so results are bit-identical
// to the oracle for the same PC scores.
#include "tp_common.cuh"
#include "tp_internal.h"

#include <cstring>

namespace tp {

constexpr int KMAXSLOT = 4;   // columns per lane: k <= 256

__device__ __forceinline__ bool key_less(double v1, int i1, double v2, int i2) {
    return v1 < v2 || (v1 == v2 && i1 < i2);
}
__device__ __forceinline__ void wave_argmin(double &v, int &idx) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        double v2 = __shfl_xor(v, m, 64);
        int i2 = __shfl_xor(idx, m, 64);
        if (key_less(v2, i2, v, idx)) { v = v2; idx = i2; }
    }
}

// pairwise tree over 64 leaves = the xor butterfly's summation tree
template <int W> struct PTree {
    template <class F> __device__ static __forceinline__ double run(const F &f, int m0) {
        return PTree<W / 2>::run(f, m0) + PTree<W / 2>::run(f, m0 + W / 2);
    }
};
template <> struct PTree<1> {
    template <class F> __device__ static __forceinline__ double run(const F &f, int m0) { return f(m0); }
};

// tree i (1-based) keeps an n x i slab; trees tree0+1..tree0+ntrees are packed
static __host__ __device__ inline size_t sums_off(int n, int tree0, int i) {
    return (size_t)n * ((size_t)i * (i - 1) / 2 - (size_t)(tree0 + 1) * tree0 / 2);
}
size_t sweep_sums_doubles(int n, int tree0, int ntrees) { return sums_off(n, tree0, tree0 + ntrees + 1); }

__device__ __forceinline__ double nan2inf(double x) { return isnan(x) ? __longlong_as_double(0x7FF0000000000000LL) : x; }

__global__ void __launch_bounds__(64) k_coniss(SweepDev sd) {
    extern __shared__ double lds[];
    const int n = sd.n, ldp = sd.ldp;
    const int ti = blockIdx.x;                 // tree slot
    const int i = sd.tree0 + ti + 1;           // PC prefix length
    const int lane = threadIdx.x;
    const int nbk = (n + 63) / 64;
    const double INF = __longlong_as_double(0x7FF0000000000000LL);
    const double QNAN = __longlong_as_double(0x7FF8000000000000LL);
    double *cost = lds;                      // n
    double *bmv = cost + n;                  // nbk
    int *bmi = (int *)(bmv + nbk);           // nbk
    int *link = bmi + nbk + (nbk & 1);       // n
    const double *Pt = sd.Pt;
    double *S = sd.sums + sums_off(n, sd.tree0, i);
    int *mrg_a = sd.mrg_a + (size_t)ti * (n - 1);
    int *mrg_b = sd.mrg_b + (size_t)ti * (n - 1);
    double *mcost = sd.cost + (size_t)ti * (n - 1);
    double *height = sd.height + (size_t)ti * (n - 1);

    // ---- initial adjacent costs (singletons: weight 1/2), lane-serial canonical tree
    for (int p = lane; p < n; p += 64) {
        link[p] = p;
        if (p < n - 1) {
            const double *x = Pt + (size_t)p * ldp;
            const double *y = x + ldp;
            auto leaf = [&](int m) {
                double acc = 0.0;
#pragma unroll
                for (int t = 0; t < KMAXSLOT; ++t) {
                    int j = m + 64 * t;
                    if (j < i) {
                        double d = x[j] - y[j];
                        acc = fma(d, d, acc);
                    }
                }
                return acc;
            };
            double tot = PTree<64>::run(leaf, 0);
            cost[p] = nan2inf(0.5 * tot);
        } else {
            cost[p] = QNAN;   // no right neighbour: not a candidate
        }
    }
    __syncthreads();
    for (int b = 0; b < nbk; ++b) {
        int p = b * 64 + lane;
        double v = INF;
        int idx = p + n;
        if (p < n && !isnan(cost[p])) { v = cost[p]; idx = p; }
        wave_argmin(v, idx);
        if (lane == 0) { bmv[b] = v; bmi[b] = idx; }
    }
    __syncthreads();

    double h = 0.0;
    for (int s = 0; s < n - 1; ++s) {
        // ---- global argmin over block minima
        double v = INF;
        int idx = 0x7FFFFFFF;
        for (int b = lane; b < nbk; b += 64)
            if (key_less(bmv[b], bmi[b], v, idx)) { v = bmv[b]; idx = bmi[b]; }
        wave_argmin(v, idx);
        const int a = idx;                // a candidate always exists here
        const int ea = link[a];
        const int b = ea + 1;
        const int eb = link[b];
        const int ls = a > 0 ? link[a - 1] : -1;
        const int r = eb + 1 < n ? eb + 1 : -1;
        const int er = r >= 0 ? link[r] : -1;
        const double c = cost[a];
        const int na = ea - a + 1, nbb = eb - b + 1, nm = na + nbb;
        const int nl = ls >= 0 ? a - ls : 0, nr = r >= 0 ? er - r + 1 : 0;
        // ---- cluster sums (singletons straight from the scores)
        double sa[KMAXSLOT], sb[KMAXSLOT], sl[KMAXSLOT], sr[KMAXSLOT];
#pragma unroll
        for (int t = 0; t < KMAXSLOT; ++t) {
            int j = lane + 64 * t;
            sa[t] = sb[t] = sl[t] = sr[t] = 0.0;
            if (j < i) {
                sa[t] = na == 1 ? Pt[(size_t)a * ldp + j] : S[(size_t)a * i + j];
                sb[t] = nbb == 1 ? Pt[(size_t)b * ldp + j] : S[(size_t)b * i + j];
                if (ls >= 0) sl[t] = nl == 1 ? Pt[(size_t)ls * ldp + j] : S[(size_t)ls * i + j];
                if (r >= 0) sr[t] = nr == 1 ? Pt[(size_t)r * ldp + j] : S[(size_t)r * i + j];
            }
        }
        double sm[KMAXSLOT];
#pragma unroll
        for (int t = 0; t < KMAXSLOT; ++t) {
            sm[t] = sa[t] + sb[t];
            int j = lane + 64 * t;
            if (j < i) S[(size_t)a * i + j] = sm[t];
        }
        // ---- the two new adjacent costs
        const double fm = (double)nm;
        double cl = QNAN, cr = QNAN;
        if (ls >= 0) {
            const double fl = (double)nl;
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < KMAXSLOT; ++t)
                if (lane + 64 * t < i) {
                    double d = sl[t] / fl - sm[t] / fm;
                    acc = fma(d, d, acc);
                }
            double tot = wave_sum(acc);
            cl = nan2inf(((fl * fm) / (fl + fm)) * tot);
        }
        if (r >= 0) {
            const double fr = (double)nr;
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < KMAXSLOT; ++t)
                if (lane + 64 * t < i) {
                    double d = sm[t] / fm - sr[t] / fr;
                    acc = fma(d, d, acc);
                }
            double tot = wave_sum(acc);
            cr = nan2inf(((fm * fr) / (fm + fr)) * tot);
        }
        h = h + c;
        if (lane == 0) {
            mrg_a[s] = a;
            mrg_b[s] = b;
            mcost[s] = c;
            height[s] = h;
            link[a] = eb;
            link[eb] = a;
            cost[b] = QNAN;
            cost[a] = cr;                 // QNAN when there is no right neighbour
            if (ls >= 0) cost[ls] = cl;
        }
        __syncthreads();
        // ---- refresh the block minima that changed
        const int b1 = a >> 6, b2 = b >> 6, b3 = ls >= 0 ? (ls >> 6) : b1;
        int blks[3] = {b1, b2 != b1 ? b2 : -1, (b3 != b1 && b3 != b2) ? b3 : -1};
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int bk = blks[q];
            if (bk < 0) continue;
            int p = bk * 64 + lane;
            double vv = INF;
            int ii = p + n;
            if (p < n) {
                double cp = cost[p];
                if (!isnan(cp)) { vv = cp; ii = p; }
            }
            wave_argmin(vv, ii);
            if (lane == 0) { bmv[bk] = vv; bmi[bk] = ii; }
        }
        __syncthreads();
    }

    // ---- broken stick (rioja bstick.chclust, vegan bstick.default) on heights
    if (lane == 0) {
        const int nobj = n - 1;
        int ncl = -1;
        if (nobj >= 2) {
            const double tot = height[nobj - 1];
            double *cs = cost;   // reuse: cs[t], t = 1..nobj  (n entries)
            double hi = 0.0, lo = 0.0;
            for (int t = 1; t <= nobj; ++t) {
                dd_add_d(hi, lo, tot / (double)(nobj - t + 1));
                cs[t - 1] = hi + lo;
            }
            int run = 0;
            bool started = false;
            for (int j = 1; j <= nobj - 1; ++j) {
                double disp = fabs(height[nobj - 1 - j] - height[nobj - j]);
                double bs = cs[nobj - j] / (double)nobj;
                if (disp > bs) { started = true; ++run; }
                else if (started) break;
            }
            ncl = started ? run : -1;
        }
        sd.n_cluster[ti] = ncl;
    }
}

// ------------------------------------------------------------ CH over cuts
// canonical segment statistics of rows s..e, by one wave (see tpo_seg_ss)
__device__ double seg_ss_wave(const double *Pt, int ldp, int k, int s, int e, double *sumout, int lane) {
    const double fn = (double)(e - s + 1);
    double part = 0.0;
#pragma unroll
    for (int t = 0; t < KMAXSLOT; ++t) {
        int j = lane + 64 * t;
        if (j >= k) break;
        double sj = 0.0;
        for (int a = s; a <= e; ++a) sj = sj + Pt[(size_t)a * ldp + j];
        if (sumout) sumout[j] = sj;
        double mj = sj / fn;
        double ss = 0.0;
        for (int a = s; a <= e; ++a) {
            double d = Pt[(size_t)a * ldp + j] - mj;
            ss = fma(d, d, ss);
        }
        part = part + ss;
    }
    return wave_sum(part);
}

__global__ void __launch_bounds__(64) k_trS(const double *Pt, int n, int ldp, int k, double *out) {
    double v = seg_ss_wave(Pt, ldp, k, 0, n - 1, nullptr, threadIdx.x);
    if (threadIdx.x == 0) *out = v;
}

__global__ void __launch_bounds__(256) k_ch(SweepDev sd) {
    const int n = sd.n, k = sd.k, ldp = sd.ldp;
    const int ti = blockIdx.x;
    const int nc = sd.n_cluster[ti];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (nc < 1) return;
    if (nc > sd.w_cap || nc > sd.seg_cap) {
        if (threadIdx.x == 0) atomicOr(sd.err, 1);
        return;
    }
    const int ldsc = sd.ntrees;
    double *score_row = sd.scores + ti;            // element n -> score_row[(n-1)*ldsc]
    if (nc == 1) {
        if (threadIdx.x == 0) score_row[0] = r_nan();
        return;
    }
    const int m = sd.min_clusters < nc ? sd.min_clusters : nc;
    const int *mb = sd.mrg_b + (size_t)ti * (n - 1);
    // per-tree scratch (global; this workgroup only)
    double *seg = sd.seg + (size_t)ti * sd.seg_cap * (k + 1);   // seg_cap x k sums
    double *ssg = seg + (size_t)sd.seg_cap * k;                        // seg_cap
    int *segs = sd.iseg + (size_t)ti * (2 * sd.seg_cap + 2);     // nc + 1
    int *alive = segs + sd.seg_cap + 1;                                // nc
    // finest cut: the boundaries removed by the last nc-1 merges, ascending
    for (int t = threadIdx.x; t < nc - 1; t += blockDim.x) {
        int bt = mb[n - 2 - t];
        int rank = 0;
        for (int u = 0; u < nc - 1; ++u) rank += mb[n - 2 - u] < bt;
        segs[rank + 1] = bt;
    }
    if (threadIdx.x == 0) { segs[0] = 0; segs[nc] = n; }
    __syncthreads();
    for (int g = w; g < nc; g += 4) {
        double ss = seg_ss_wave(sd.Pt, ldp, k, segs[g], segs[g + 1] - 1, seg + (size_t)g * k, lane);
        if (lane == 0) { ssg[g] = ss; alive[g] = 1; }
    }
    __syncthreads();
    if (w != 0) return;
    // wave 0 only from here: every lane keeps its own copy of the state it
    // reads back (alive flags written by all lanes, sums by their own lane)
    const double trS = *sd.trS;
    double trW = 0.0;
    for (int g = 0; g < nc; ++g) trW = trW + ssg[g];
    if (lane == 0)
        score_row[(size_t)(nc - 1) * ldsc] = ((double)(n - nc) * (trS - trW)) / ((double)(nc - 1) * trW);
    for (int lev = nc - 1; lev >= m && lev >= 1; --lev) {
        const int b = mb[n - lev - 1];
        int gb = -1;
        for (int g = lane; g < nc; g += 64)
            if (alive[g] && segs[g] == b) gb = g;
        for (int o = 1; o < 64; o <<= 1) gb = max(gb, __shfl_xor(gb, o, 64));
        int ga = gb - 1;
        while (ga >= 0 && !alive[ga]) --ga;
        int nx = gb + 1;
        while (nx < nc && !alive[nx]) ++nx;
        const int na = b - segs[ga];
        const int nbb = (nx < nc ? segs[nx] : n) - b;
        const double fa = (double)na, fb = (double)nbb;
        double *SA = seg + (size_t)ga * k, *SB = seg + (size_t)gb * k;
        double acc = 0.0;
#pragma unroll
        for (int t = 0; t < KMAXSLOT; ++t) {
            int j = lane + 64 * t;
            if (j < k) {
                double d = SA[j] / fa - SB[j] / fb;
                acc = fma(d, d, acc);
            }
        }
        double tot = wave_sum(acc);
        trW = trW + ((fa * fb) / (fa + fb)) * tot;
#pragma unroll
        for (int t = 0; t < KMAXSLOT; ++t) {
            int j = lane + 64 * t;
            if (j < k) SA[j] = SA[j] + SB[j];
        }
        alive[gb] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0)
            score_row[(size_t)(lev - 1) * ldsc] =
                lev == 1 ? r_nan() : ((double)(n - lev) * (trS - trW)) / ((double)(lev - 1) * trW);
    }
}

__global__ void k_fill(double *p, size_t cnt, double v) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < cnt) p[t] = v;
}

static size_t coniss_lds_bytes(int n) {
    int nbk = (n + 63) / 64;
    return (size_t)n * 8 + (size_t)nbk * 12 + 8 + (size_t)n * 4 + 16;
}

void launch_sweep(const SweepDev &sd, hipStream_t s, Ctx *prof) {
    if (sd.k > 64 * KMAXSLOT) fail(TP_ERR_UNSUPPORTED, "max_pcs > 256 is not supported by this build");
    if (sd.n < 3) fail(TP_ERR_NO_BSTICK, "fewer than 3 good bins: no broken-stick level");
    size_t lds = coniss_lds_bytes(sd.n);
    if (lds > 160 * 1024) fail(TP_ERR_UNSUPPORTED, "matrix too large for the LDS-resident CONISS (n > ~13000)");
    TP_HIP(hipFuncSetAttribute((const void *)k_coniss, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (sd.ntrees < 1 || sd.tree0 < 0 || sd.tree0 + sd.ntrees > sd.k) fail(TP_ERR_ARG, "bad tree range");
    size_t cnt = (size_t)sd.ntrees * sd.w_cap;
    double na;
    {
        uint64_t u = kRNaBits;
        memcpy(&na, &u, 8);
    }
    hipLaunchKernelGGL(k_fill, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, sd.scores, cnt, na);
    TP_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_trS, dim3(1), dim3(64), 0, s, sd.Pt, sd.n, sd.ldp, sd.k, sd.trS);
    TP_HIP(hipGetLastError());
    if (prof) kprof_begin(*prof, K_CONISS);
    hipLaunchKernelGGL(k_coniss, dim3(sd.ntrees), dim3(64), lds, s, sd);
    TP_HIP(hipGetLastError());
    if (prof) kprof_end(*prof, K_CONISS);
    if (prof) kprof_begin(*prof, K_CH);
    hipLaunchKernelGGL(k_ch, dim3(sd.ntrees), dim3(256), 0, s, sd);
    TP_HIP(hipGetLastError());
    if (prof) kprof_end(*prof, K_CH);
}

void launch_coniss_only(const SweepDev &sd, hipStream_t s) {
    if (sd.tree0 + sd.ntrees > 64 * KMAXSLOT) fail(TP_ERR_UNSUPPORTED, "more than 256 columns");
    size_t lds = coniss_lds_bytes(sd.n);
    if (lds > 160 * 1024) fail(TP_ERR_UNSUPPORTED, "matrix too large for the LDS-resident CONISS (n > ~13000)");
    TP_HIP(hipFuncSetAttribute((const void *)k_coniss, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_coniss, dim3(sd.ntrees), dim3(64), lds, s, sd);
    TP_HIP(hipGetLastError());
}

// ------------------------------------------- single calinhara (tp_ch entry)
__global__ void __launch_bounds__(256) k_ch_single(const double *Pt, int n, int ldp, int k, const int *bnd, int cn,
                                                   double *ssg, double *trS_out, double *out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int g = w; g < cn + 1; g += 4) {
        // g == cn: the whole matrix (tr S)
        int s0 = g == cn ? 0 : bnd[g], e0 = g == cn ? n - 1 : bnd[g + 1] - 1;
        double ss = seg_ss_wave(Pt, ldp, k, s0, e0, nullptr, lane);
        if (lane == 0) ssg[g] = ss;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double trW = 0.0;
        for (int g = 0; g < cn; ++g) trW = trW + ssg[g];
        double trS = ssg[cn];
        *trS_out = trS;
        *out = cn == 1 ? r_nan() : ((double)(n - cn) * (trS - trW)) / ((double)(cn - 1) * trW);
    }
}

void launch_ch_only(const double *d_Pt, int n, int ldp, int k, const int *d_bnd, int cn, double *d_seg,
                    double *d_out, hipStream_t s) {
    hipLaunchKernelGGL(k_ch_single, dim3(1), dim3(256), 0, s, d_Pt, n, ldp, k, d_bnd, cn, d_seg, d_seg + cn + 1,
                       d_out);
    TP_HIP(hipGetLastError());
}

// ---------------------------------------------------------- stats::dist
// R distance.c R_euclidean: dist += dev*dev sequentially over columns, then
// sqrt; no contraction.  P column-major n x ncols.  d in R's "dist" order.
__global__ void __launch_bounds__(256) k_dist(const double *P, int n, int ldp, int ncols, double *d) {
    const int j = blockIdx.y;                                  // column of the pair (i > j)
    const int i = j + 1 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double dist = 0.0;
    for (int c = 0; c < ncols; ++c) {
        double dev = P[i + (size_t)c * ldp] - P[j + (size_t)c * ldp];
        dist = dist + dev * dev;
    }
    size_t ij = (size_t)j * n - (size_t)j * (j + 1) / 2 + (size_t)(i - j - 1);
    d[ij] = sqrt(dist);
}

void launch_dist(const double *d_P, int n, int ldp, int ncols, double *d_d, hipStream_t s) {
    if (n < 2) return;
    dim3 g((n + 255) / 256, n - 1);
    hipLaunchKernelGGL(k_dist, g, dim3(256), 0, s, d_P, n, ldp, ncols, d_d);
    TP_HIP(hipGetLastError());
}

}  // namespace tp
