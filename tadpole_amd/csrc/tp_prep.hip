// Pre-processing kernels: load_mat cleaning + bad-column mask + subset
// (R/TADpole.R:19-20,35-37,88-89), the sparse_cor epilogue
// (R/TADpole.R:94-100,449) and prcomp's column centring (R/TADpole.R:453).
// All of these are HBM-streaming passes over an N x N fp64 matrix.
#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

// ------------------------------------------------ NA -> 0, forceSymmetric(U)
// Treat the buffer as column-major B(r,c) = buf[r + c*n0].  The matrix's upper
// triangle is B's upper triangle for column-major input, B's lower for
// row-major input (src_upper = false).  One 64x64 tile pair per workgroup: the
// source tile is read once, its mirror written whole, and the source itself
// written back only where it held a NaN (was: rewritten whole, 30 of the 20
// necessary GB at the 49 851-bin C5 matrix, 9.2 ms).
// T x T tiles, T * T / 16 threads (16 elements each): T = 64 (256 threads, 33 KB
// of LDS) or 128 (1024 threads, 132 KB: 1 KB contiguous runs on both the read
// and the mirrored write instead of 512 B)
template <int T>
__global__ void __launch_bounds__(T * T / 16) k_clean_symmetrize(double *M, int n0, int nb, bool src_upper) {
    constexpr int NT = T / 16;   // rows of threads
    __shared__ double t[T][T + 1];
    // linear block id -> (bi <= bj): row bi starts at S(bi) = bi nb - bi (bi - 1) / 2
    // (closed form, then an exact integer fix-up; was a loop over up to nb rows)
    const long long id = blockIdx.x;
    auto row_start = [&](long long r) { return r * nb - r * (r - 1) / 2; };
    const double tb = 2.0 * nb + 1.0;
    int bi = (int)((tb - sqrt(tb * tb - 8.0 * (double)id)) * 0.5);
    bi = bi < 0 ? 0 : (bi >= nb ? nb - 1 : bi);
    while (bi > 0 && row_start(bi) > id) --bi;
    while (bi + 1 < nb && row_start(bi + 1) <= id) ++bi;
    const int bj = bi + (int)(id - row_start(bi));
    const int tx = threadIdx.x % T, ty = threadIdx.x / T;
    // source tile rows/cols (buffer coordinates)
    int sr0 = src_upper ? bi * T : bj * T;
    int sc0 = src_upper ? bj * T : bi * T;
    unsigned nanm = 0;   // bit u: this thread's element (tx, ty + NT u) was NaN
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int r = sr0 + tx, c = sc0 + ty + NT * u;
        v[u] = (r < n0 && c < n0) ? M[(size_t)r + (size_t)c * n0] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const bool bad = isnan(v[u]);
        nanm |= bad ? 1u << u : 0u;
        t[tx][ty + NT * u] = bad ? 0.0 : v[u];
    }
    __syncthreads();
    if (bi != bj) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int y = ty + NT * u;
            int r = sr0 + tx, c = sc0 + y;
            if ((nanm >> u & 1u) && r < n0 && c < n0) M[(size_t)r + (size_t)c * n0] = 0.0;
            // mirrored tile: B(sc0 + tx, sr0 + y) = t[y][tx]
            int r2 = sc0 + tx, c2 = sr0 + y;
            if (r2 < n0 && c2 < n0) M[(size_t)r2 + (size_t)c2 * n0] = t[y][tx];
        }
    } else {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int y = ty + NT * u;
            int r = sr0 + tx, c = sc0 + y;
            bool from_here = src_upper ? (tx <= y) : (tx >= y);
            if (r < n0 && c < n0 && (!from_here || (nanm >> u & 1u)))
                M[(size_t)r + (size_t)c * n0] = from_here ? 0.0 : t[y][tx];
        }
    }
}

// knob 50: k_clean_symmetrize tile edge -- 0 (default): 128 from 16 384 bins
// (49 851: 6.18 -> 5.36 ms), 64 below (7 808, Infinity-Cache resident: 93 vs
// 100 us); 64 / 128 force one

void launch_clean_symmetrize(double *d_M, int n0, bool src_upper, hipStream_t s) {
    if (cfg_clean_tile == 128 || (cfg_clean_tile == 0 && n0 >= 16384)) {
        int nb = (n0 + 127) / 128;
        long nblk = (long)nb * (nb + 1) / 2;
        hipLaunchKernelGGL(k_clean_symmetrize<128>, dim3((unsigned)nblk), dim3(1024), 0, s, d_M, n0, nb, src_upper);
    } else {
        int nb = (n0 + 63) / 64;
        long nblk = (long)nb * (nb + 1) / 2;
        hipLaunchKernelGGL(k_clean_symmetrize<64>, dim3((unsigned)nblk), dim3(256), 0, s, d_M, n0, nb, src_upper);
    }
    TP_HIP(hipGetLastError());
}

// Lane-strided double-double sum of a column (rows lane, lane + 64, ...), U
// loads in flight per lane; the accumulation order is the sequential one.
template <int U>
__device__ __forceinline__ void dd_col_acc(const double *src, int n, int lane, double &hi, double &lo) {
    int r = lane;
    for (; r + 64 * (U - 1) < n; r += 64 * U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[r + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) dd_add_d(hi, lo, v[u]);
    }
    for (; r < n; r += 64) dd_add_d(hi, lo, src[r]);
}

// ------------------------------------------ rowMeans (long double in R) + diag
// The matrix is symmetric here, so row a is column a (contiguous).  One wave
// per column; double-double accumulation stands in for R's LDOUBLE.
__global__ void __launch_bounds__(256) k_rowmean_diag(const double *M, int n0, double *rm, double *dg) {
    int lane = threadIdx.x & 63;
    int a = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (a >= n0) return;
    const double *col = M + (size_t)a * n0;
    double hi = 0.0, lo = 0.0;
    dd_col_acc<8>(col, n0, lane, hi, lo);
    wave_dd_sum(hi, lo);
    if (lane == 0) {
        rm[a] = dd_div_d(hi, lo, (double)n0);
        if (dg) dg[a] = col[a];
    }
}

void launch_rowmean_diag(const double *d_M, int n0, double *d_rowmean, double *d_diag, hipStream_t s) {
    hipLaunchKernelGGL(k_rowmean_diag, dim3((n0 + 3) / 4), dim3(256), 0, s, d_M, n0, d_rowmean, d_diag);
    TP_HIP(hipGetLastError());
}

// ------------------------------------- quantile type 7 + bad mask + compaction
// One 1024-thread workgroup.  Order statistics by MSB-first radix select on
// order-preserving 64-bit keys, then R's type-7 interpolation, then the mask
// bad = diag == 0 | r < q and an order-preserving compaction of good bins.
__device__ uint64_t radix_select(const double *r, int n, int rank, unsigned *hist, uint64_t *bcast) {
    uint64_t prefix = 0, pmask = 0;
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            uint64_t key = dkey(r[i]);
            if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            // the digit d holding rank: wave 0 scans the histogram, four bins a
            // lane (a serial 256-bin loop on one thread was ~10 us a pass)
            const int l = threadIdx.x;
            const unsigned h0 = hist[4 * l], h1 = hist[4 * l + 1], h2 = hist[4 * l + 2], h3 = hist[4 * l + 3];
            unsigned incl = h0 + h1 + h2 + h3;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned y = __shfl_up(incl, o, 64);
                if (l >= o) incl += y;
            }
            const unsigned ex = incl - (h0 + h1 + h2 + h3);   // bins below 4 l
            const unsigned rk = (unsigned)rank;
            // the bin holding rank lies in the first lane whose inclusive sum exceeds it
            const unsigned long long m = __ballot(incl > rk);
            // m != 0 while rank < the count of matching keys; if that invariant
            // ever broke, lane 63 (the last bin) answers, so the pass writes a
            // defined prefix instead of leaving stale values (TP_DASSERT traps
            // it in checked builds)
            TP_DASSERT(m != 0ull);
            const int L = m ? (int)__builtin_ctzll(m) : 63;
            if (l == L) {
                unsigned cum = ex;
                int d = 4 * l;
                if (cum + h0 <= rk) {
                    cum += h0;
                    ++d;
                    if (cum + h1 <= rk) {
                        cum += h1;
                        ++d;
                        if (cum + h2 <= rk) {
                            cum += h2;
                            ++d;
                        }
                    }
                }
                bcast[0] = prefix | ((uint64_t)d << shift);
                bcast[1] = (uint64_t)(rank - (int)cum);
            }
        }
        __syncthreads();
        prefix = bcast[0];
        rank = (int)bcast[1];
        pmask |= (uint64_t)255 << shift;
        __syncthreads();
    }
    return prefix;
}

__global__ void __launch_bounds__(1024) k_mask_select(const double *r, const double *dg, int n0, double bad_frac,
                                                      double qindex, int *bad, int *good, int *ngood) {
    __shared__ unsigned hist[256];
    __shared__ uint64_t bcast[2];
    __shared__ unsigned long long umin;
    __shared__ unsigned cnt_le;
    __shared__ int scan[1024];
    __shared__ double qsh;
    const bool use_q = bad_frac != 0.0;
    if (use_q) {
        int lo = (int)floor(qindex), hi = (int)ceil(qindex);
        uint64_t klo = radix_select(r, n0, lo - 1, hist, bcast);
        double xlo = dkey_inv(klo), xhi = xlo;
        if (hi != lo) {
            if (threadIdx.x == 0) { umin = ~0ULL; cnt_le = 0; }
            __syncthreads();
            unsigned c = 0;
            unsigned long long mn = ~0ULL;
            for (int i = threadIdx.x; i < n0; i += blockDim.x) {
                uint64_t key = dkey(r[i]);
                if (key <= klo) ++c;
                else if (key < mn) mn = key;
            }
            atomicAdd(&cnt_le, c);
            atomicMin(&umin, mn);
            __syncthreads();
            if (cnt_le <= (unsigned)(hi - 1)) xhi = dkey_inv(umin);
        }
        if (threadIdx.x == 0) {
            double q = xlo;
            if (qindex > (double)lo && xhi != q) {
                double h = qindex - (double)lo;
                q = (1.0 - h) * q + h * xhi;
            }
            qsh = q;
        }
        __syncthreads();
    }
    const double q = use_q ? qsh : 0.0;
    // chunked, order-preserving compaction
    const int T = blockDim.x;
    const int chunk = (n0 + T - 1) / T;
    const int b0 = threadIdx.x * chunk, b1 = min(n0, b0 + chunk);
    int c = 0;
    for (int a = b0; a < b1; ++a) {
        int isbad = (dg[a] == 0.0) || (use_q && r[a] < q);
        bad[a] = isbad;
        c += !isbad;
    }
    scan[threadIdx.x] = c;
    __syncthreads();
    for (int off = 1; off < T; off <<= 1) {
        int v = threadIdx.x >= off ? scan[threadIdx.x - off] : 0;
        __syncthreads();
        scan[threadIdx.x] += v;
        __syncthreads();
    }
    int pos = scan[threadIdx.x] - c;
    for (int a = b0; a < b1; ++a)
        if (!bad[a]) good[pos++] = a;
    if (threadIdx.x == T - 1) *ngood = scan[T - 1];
}

void launch_mask_select(const double *d_rowmean, const double *d_diag, int n0, double bad_frac, double qindex,
                        int *d_bad, int *d_good, int *d_ngood, hipStream_t s) {
    hipLaunchKernelGGL(k_mask_select, dim3(1), dim3(1024), 0, s, d_rowmean, d_diag, n0, bad_frac, qindex, d_bad,
                       d_good, d_ngood);
    TP_HIP(hipGetLastError());
}

// --------------------------------------- X = M[good, good] + colMeans(X) (dd)
__global__ void __launch_bounds__(256) k_gather_colmean(const double *M, int n0, const int *good, int n, double *X,
                                                        double *cm) {
    int lane = threadIdx.x & 63;
    int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= n) return;
    const double *src = M + (size_t)good[j] * n0;
    double *dst = X + (size_t)j * n;
    double hi = 0.0, lo = 0.0;
    constexpr int U = 8;   // gathers in flight per lane (same accumulation order)
    int a = lane;
    for (; a + 64 * (U - 1) < n; a += 64 * U) {
        int gi[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) gi[u] = good[a + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[gi[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            dst[a + 64 * u] = v[u];
            dd_add_d(hi, lo, v[u]);
        }
    }
    for (; a < n; a += 64) {
        double v = src[good[a]];
        dst[a] = v;
        dd_add_d(hi, lo, v);
    }
    wave_dd_sum(hi, lo);
    if (lane == 0 && cm) cm[j] = dd_div_d(hi, lo, (double)n);
}

void launch_gather_colmean(const double *d_M, int n0, const int *d_good, int n, double *d_X, double *d_colmean,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_gather_colmean, dim3((n + 3) / 4), dim3(256), 0, s, d_M, n0, d_good, n, d_X, d_colmean);
    TP_HIP(hipGetLastError());
}

// The same gather and column means, plus what the exact int8 X'X needs, in
// the same pass over X (instead of two more passes over it: the integrality
// scan and the slicing): per column the maximum, a flag for entries that are
// not non-negative integers, the exact sum of squares (int64: S_jj of X'X, for
// sd), and -- speculatively, for counts below 2^14 -- the two 7-bit int8
// slices (column j of slice s at sl + s Np Kp + j Kp, rows zero-padded to Kp;
// grid over Np columns: the padding columns get zero slices).  X may be null:
// the int8 X'X never reads it, so the pipeline writes X only if the counts turn
// out not to be integers (k_gather_colmean, same column means).
__global__ void __launch_bounds__(256) k_gather_prep(const double *M, int n0, const int *good, int n, double *X,
                                                     double *cm, double *cmax, int *cbad, long long *css,
                                                     int8_t *sl, int Kp, int Np) {
    int lane = threadIdx.x & 63;
    int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= Np) return;
    const size_t slice = (size_t)Np * Kp;
    if (j >= n) {   // padding column: zero slices
        for (int k = lane * 4; k < Kp; k += 256) {
            *(unsigned *)(sl + (size_t)j * Kp + k) = 0u;
            *(unsigned *)(sl + slice + (size_t)j * Kp + k) = 0u;
        }
        return;
    }
    const double *src = M + (size_t)good[j] * n0;
    double *dst = X ? X + (size_t)j * n : nullptr;   // X == nullptr: not written (int8 path)
    int8_t *s0 = sl + (size_t)j * Kp, *s1 = s0 + slice;
    double hi = 0.0, lo = 0.0, mx = 0.0;
    long long ss = 0;
    bool bad = false;
    auto take = [&](int a, double v) {
        if (dst) dst[a] = v;
        dd_add_d(hi, lo, v);
        const bool ok = v >= 0.0 && v == floor(v) && v < 2147483648.0;
        bad |= !ok;
        mx = fmax(mx, v);
        const long long iv = ok ? (long long)v : 0;
        ss += iv * iv;
        s0[a] = (int8_t)(iv & 127);
        s1[a] = (int8_t)((iv >> 7) & 127);
    };
    constexpr int U = 8;   // gathers in flight per lane (same accumulation order as k_gather_colmean)
    int a = lane;
    for (; a + 64 * (U - 1) < n; a += 64 * U) {
        int gi[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) gi[u] = good[a + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[gi[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) take(a + 64 * u, v[u]);
    }
    for (; a < n; a += 64) take(a, src[good[a]]);
    for (int k = n + lane; k < Kp; k += 64) {   // zero rows past n
        s0[k] = 0;
        s1[k] = 0;
    }
    wave_dd_sum(hi, lo);
    for (int o = 32; o > 0; o >>= 1) {
        mx = fmax(mx, __shfl_xor(mx, o, 64));
        ss += __shfl_xor(ss, o, 64);
    }
    const bool anyb = __ballot(bad) != 0ULL;
    if (lane == 0) {
        if (cm) cm[j] = dd_div_d(hi, lo, (double)n);
        cmax[j] = mx;
        cbad[j] = anyb ? 1 : 0;
        css[j] = ss;
    }
}

void launch_gather_prep(const double *d_M, int n0, const int *d_good, int n, double *d_X, double *d_colmean,
                        double *d_cmax, int *d_cbad, long long *d_css, int8_t *d_sl, int Kp, int Np, hipStream_t s) {
    hipLaunchKernelGGL(k_gather_prep, dim3((Np + 3) / 4), dim3(256), 0, s, d_M, n0, d_good, n, d_X, d_colmean, d_cmax,
                       d_cbad, d_css, d_sl, Kp, Np);
    TP_HIP(hipGetLastError());
}

// sd[j] = sqrt(cov_jj) from the exact S_jj = sum_i x_ij^2 (k_cor_sd's expression;
// S_jj < 2^53 is exact in a double, the value X'X's diagonal holds)
__global__ void __launch_bounds__(256) k_cor_sd_ss(const long long *css, const double *m, int n, double *sd) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const double fn = (double)n, fn1 = (double)(n - 1);
    sd[j] = sqrt(((double)css[j] - fn * (m[j] * m[j])) / fn1);
}
void launch_cor_sd_ss(const long long *d_css, const double *d_m, int n, double *d_sd, hipStream_t s) {
    hipLaunchKernelGGL(k_cor_sd_ss, dim3((n + 255) / 256), dim3(256), 0, s, d_css, d_m, n, d_sd);
    TP_HIP(hipGetLastError());
}

__global__ void __launch_bounds__(256) k_colmean(const double *A, int n, int ncols, int ld, double *cm) {
    int lane = threadIdx.x & 63;
    int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= ncols) return;
    const double *src = A + (size_t)j * ld;
    double hi = 0.0, lo = 0.0;
    dd_col_acc<8>(src, n, lane, hi, lo);
    wave_dd_sum(hi, lo);
    if (lane == 0) cm[j] = dd_div_d(hi, lo, (double)n);
}

void launch_colmean(const double *d_A, int n, int ld, double *d_mean, hipStream_t s) {
    launch_colmean_cols(d_A, n, n, ld, d_mean, s);
}
// means of ncols columns of n rows (a column slab of C): the same per-column bits
void launch_colmean_cols(const double *d_A, int n, int ncols, int ld, double *d_mean, hipStream_t s) {
    if (ncols <= 0) return;
    hipLaunchKernelGGL(k_colmean, dim3((ncols + 3) / 4), dim3(256), 0, s, d_A, n, ncols, ld, d_mean);
    TP_HIP(hipGetLastError());
}

// ------------------------------------------------- sparse_cor epilogue (R order)
// cov = (S - n * (m m')) / (n - 1); cor = cov / (sd sd'), sd = sqrt(diag(cov));
// NaN -> 0 (R/TADpole.R:96-98,449).  Rounding order as R evaluates it.
// sd[j] = sqrt(cov_jj) (the expression of the per-element form, once per column)
__global__ void __launch_bounds__(256) k_cor_sd(const double *S, const double *m, int n, double *sd) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const double fn = (double)n, fn1 = (double)(n - 1);
    sd[j] = sqrt((S[(size_t)j * n + j] - fn * (m[j] * m[j])) / fn1);
}

// one column per blockIdx.y, rows over the threads (no 64-bit index division:
// two divmods per element made this pass run at 3 TB/s)
__global__ void __launch_bounds__(256) k_cor_epilogue(const double *S, const double *m, const double *sd, int n,
                                                      double *C) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double fn = (double)n, fn1 = (double)(n - 1);
    for (int j = blockIdx.y; j < n; j += gridDim.y) {   // gridDim.y <= 65535
        const size_t id = (size_t)j * n + i;
        const double cij = (S[id] - fn * (m[i] * m[j])) / fn1;
        double v = cij / (sd[i] * sd[j]);
        if (isnan(v)) v = 0.0;
        C[id] = v;
    }
}


// The same elements, one wave per column j, with C's column mean formed in the same
// pass: the lane-strided double-double order of k_colmean (rows lane, lane + 64, ...,
// then the wave sum), so cm[j] has k_colmean's bits and C is not read again for it.
template <int U>
__global__ void __launch_bounds__(256) k_cor_epilogue_mean(const double *S, const double *m, const double *sd, int n,
                                                           double *C, double *cm) {
    const int lane = threadIdx.x & 63;
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= n) return;
    const double fn = (double)n, fn1 = (double)(n - 1), mj = m[j], sdj = sd[j];
    const double *Sj = S + (size_t)j * n;
    double *Cj = C + (size_t)j * n;
    double hi = 0.0, lo = 0.0;
    auto elem = [&](int i, double sij) {
        const double cij = (sij - fn * (m[i] * mj)) / fn1;
        double v = cij / (sd[i] * sdj);
        if (isnan(v)) v = 0.0;
        Cj[i] = v;
        dd_add_d(hi, lo, v);
    };
    int r = lane;
    for (; r + 64 * (U - 1) < n; r += 64 * U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = Sj[r + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) elem(r + 64 * u, v[u]);
    }
    for (; r < n; r += 64) elem(r, Sj[r]);
    wave_dd_sum(hi, lo);
    if (lane == 0) cm[j] = dd_div_d(hi, lo, fn);
}

void launch_cor_epilogue(const double *d_S, const double *d_m, int n, double *d_C, double *d_sd, hipStream_t s,
                         double *d_cmean) {
    hipLaunchKernelGGL(k_cor_sd, dim3((n + 255) / 256), dim3(256), 0, s, d_S, d_m, n, d_sd);
    if (d_cmean)
        hipLaunchKernelGGL(k_cor_epilogue_mean<8>, dim3((n + 3) / 4), dim3(256), 0, s, d_S, d_m, d_sd, n, d_C,
                           d_cmean);
    else
        hipLaunchKernelGGL(k_cor_epilogue, dim3((unsigned)((n + 255) / 256), (unsigned)std::min(n, 65535)), dim3(256),
                           0, s, d_S, d_m, d_sd, n, d_C);
    TP_HIP(hipGetLastError());
}

// ------------------------------------------------ prcomp centring (scale(x, TRUE))
// Xc = C - 1 mean'  and its transpose XcT = C - mean 1' (C symmetric).
__global__ void __launch_bounds__(256) k_center(const double *C, const double *mean, int n, double *Xc, double *XcT) {
    const int a = blockIdx.x * blockDim.x + threadIdx.x;   // row a of column i
    if (a >= n) return;
    for (int i = blockIdx.y; i < n; i += gridDim.y) {   // gridDim.y <= 65535
        const size_t idx = (size_t)i * n + a;
        double c = C[idx];
        Xc[idx] = c - mean[i];
        if (XcT) XcT[idx] = c - mean[a];
    }
}

void launch_center(const double *d_C, const double *d_mean, int n, double *d_Xc, double *d_XcT, hipStream_t s) {
    hipLaunchKernelGGL(k_center, dim3((unsigned)((n + 255) / 256), (unsigned)std::min(n, 65535)), dim3(256), 0, s, d_C,
                       d_mean, n, d_Xc, d_XcT);
    TP_HIP(hipGetLastError());
}

// --------------------------------------------------------------- transpose
__global__ void __launch_bounds__(256) k_transpose(const double *A, int rows, int cols, int lda, double *T, int ldt) {
    __shared__ double t[32][33];
    int r0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
    int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int y = ty; y < 32; y += 8) {
        int r = r0 + tx, c = c0 + y;
        t[y][tx] = (r < rows && c < cols) ? A[(size_t)r + (size_t)c * lda] : 0.0;
    }
    __syncthreads();
    for (int y = ty; y < 32; y += 8) {
        int c = c0 + tx, r = r0 + y;
        if (r < rows && c < cols) T[(size_t)c + (size_t)r * ldt] = t[tx][y];
    }
}

void launch_transpose(const double *d_A, int rows, int cols, int lda, double *d_T, int ldt, hipStream_t s) {
    dim3 g((rows + 31) / 32, (cols + 31) / 32);
    hipLaunchKernelGGL(k_transpose, g, dim3(256), 0, s, d_A, rows, cols, lda, d_T, ldt);
    TP_HIP(hipGetLastError());
}

}  // namespace tp
