// S = X'X (crossprod in sparse_cor, R/TADpole.R:96) EXACTLY on the int8 matrix
// cores when X holds non-negative integer counts (raw Hi-C contact matrices).
//
// Each count x < 2^(7 ns) is split into ns 7-bit slices x = sum_s 2^(7s) x_s,
// x_s in [0, 127] (a valid signed int8), so
//     X'X = sum_{s,t} 2^(7(s+t)) X_s' X_t
// and every X_s' X_t is an int8 GEMM with int32 accumulation, exact while
// K * 127^2 < 2^31 (K < 133 000 bins).  The ns^2 partial products of a tile are
// combined in int64 and converted to double once: S is the correctly rounded
// exact product -- as close to R's dsyrk as the fp64 MFMA product is (both
// differ from it only by rounding), and bit-identical for any tiling or rank
// count.  ns = 2 (counts < 16384) costs 4 int8 products at ~32x the fp64
// MFMA rate each.  Inputs that are not integer counts (balanced / normalised
// matrices) take the fp64 MFMA path (tp_gemm.hip).
//
// Layout: slices are column-major int8 with K padded to a multiple of 64 and
// columns to a multiple of 64 (zero padding), so a fragment load is one
// aligned 16-byte load.  The MFMA operand k order is irrelevant here: A and B
// fragments are loaded with the same k pattern and the product sums over k.
// C/D: col = lane & 15, row = 4 (lane >> 4) + reg (cdna_hip_programming.md §3).
#include "tp_common.cuh"
#include "tp_internal.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace tp {

typedef int i32x4 __attribute__((ext_vector_type(4)));

// max over X and a flag for entries that are not non-negative integers: one
// workgroup per CU-sized chunk, reduced in LDS, ONE atomic per workgroup (a
// per-wave atomic on one address from thousands of waves serialised at L2).
__global__ void __launch_bounds__(256) k_int_scan(const double *X, size_t cnt, unsigned long long *maxbits,
                                                  int *notint) {
    __shared__ double wm[4];
    __shared__ int wb[4];
    double m = 0.0;
    int bad = 0;
    const size_t n2 = cnt / 2;
    const double2 *X2 = (const double2 *)X;
    const size_t G = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * G < n2; i += 4 * G) {   // four 16-byte loads in flight per thread
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = X2[i + u * G];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            bad |= !(v[u].x >= 0.0) || v[u].x != floor(v[u].x) || !(v[u].y >= 0.0) || v[u].y != floor(v[u].y);
            m = fmax(m, fmax(v[u].x, v[u].y));
        }
    }
    for (; i < n2; i += G) {
        const double2 v = X2[i];
        bad |= !(v.x >= 0.0) || v.x != floor(v.x) || !(v.y >= 0.0) || v.y != floor(v.y);
        m = fmax(m, fmax(v.x, v.y));
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && (cnt & 1)) {
        const double x = X[cnt - 1];
        bad |= !(x >= 0.0) || x != floor(x);
        m = fmax(m, x);
    }
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    const int anyb = __ballot(bad) != 0ULL;
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        wm[w] = m;
        wb[w] = anyb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double mm = fmax(fmax(wm[0], wm[1]), fmax(wm[2], wm[3]));
        // non-negative doubles order like their bit patterns
        atomicMax(maxbits, (unsigned long long)__double_as_longlong(mm));
        if (wb[0] | wb[1] | wb[2] | wb[3]) atomicOr(notint, 1);
    }
}

// slice s of column c, rows k..k+3: one thread, four contiguous doubles in,
// one 4-byte word per slice out
__global__ void __launch_bounds__(256) k_slice_i8(const double *X, int n, int Kp, int Np, int ns, int8_t *S) {
    const int c = blockIdx.y;
    const int k = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (k >= Kp) return;
    unsigned v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (c < n && k + u < n) ? (unsigned)X[(size_t)c * n + k + u] : 0u;
    for (int s = 0; s < ns; ++s) {
        unsigned w = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) w |= ((v[u] >> (7 * s)) & 127u) << (8 * u);
        *(unsigned *)(S + (size_t)s * Np * Kp + (size_t)c * Kp + k) = w;
    }
}

// Upper 64 x 64 tiles (tile column tcol0 onward, column by column, as the fp64
// symmetric kernel), 4 waves of 32 x 32 (2 x 2 MFMA tiles), NS^2 products per
// tile; fragments straight from global memory (L2 / MALL resident slices).
template <int NS>
__global__ void __launch_bounds__(256) k_xtx_i8(const int8_t *__restrict__ S, int n, int Kp, int Np,
                                                double *__restrict__ C, int tcol0) {
    int id = blockIdx.x, bn = tcol0;
    while (id > bn) {
        id -= bn + 1;
        ++bn;
    }
    const int bm = id;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i0 = bm * 64 + (w & 1) * 32, j0 = bn * 64 + (w >> 1) * 32;
    const int fr = lane & 15, fk = (lane >> 4) * 16;
    i32x4 acc[NS][NS][2][2];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int t = 0; t < NS; ++t)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[s][t][a][b] = i32x4{0, 0, 0, 0};
    const size_t slice = (size_t)Np * Kp;
    const int8_t *pa = S + (size_t)(i0 + fr) * Kp + fk;
    const int8_t *pb = S + (size_t)(j0 + fr) * Kp + fk;
    // slice rows read: i0 + 31, j0 + 31 (< Np); k bytes kb + fk .. + 15 (< Kp)
    TP_DASSERT(i0 + 31 < Np && j0 + 31 < Np && Kp % 64 == 0);
    for (int kb = 0; kb < Kp; kb += 64) {
        i32x4 fa[NS][2], fb[NS][2];
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                fa[s][a] = *(const i32x4 *)(pa + s * slice + (size_t)a * 16 * Kp + kb);
                fb[s][a] = *(const i32x4 *)(pb + s * slice + (size_t)a * 16 * Kp + kb);
            }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int t = 0; t < NS; ++t)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc[s][t][a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s][a], fb[t][b], acc[s][t][a][b],
                                                                                0, 0, 0);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + 16 * a + (lane >> 4) * 4 + r;
                const int j = j0 + 16 * b + fr;
                if (i >= n || j >= n || i > j) continue;
                long long v = 0;
#pragma unroll
                for (int s = 0; s < NS; ++s)
#pragma unroll
                    for (int t = 0; t < NS; ++t) v += (long long)acc[s][t][a][b][r] << (7 * (s + t));
                const double d = (double)v;
                C[(size_t)i + (size_t)j * n] = d;
                C[(size_t)j + (size_t)i * n] = d;
            }
}

// Large problems: 128 x 128 upper tiles per 8-wave workgroup (waves 2 x 4 of
// 64 x 32, 4 x 2 MFMA tiles each), k-blocks of 128 staged through LDS
// (double-buffered, one barrier per two MFMA k-steps) so each slice fragment
// is read from L2 once per workgroup instead of once per wave.  LDS rows are
// 160 B per column (128 B of k + 32 B pad: the b128 fragment reads of a
// 16-lane group and the staging stores hit distinct banks); the two buffers
// fill the 160 KiB.  Same exact arithmetic as k_xtx_i8.
//
// Tile order (whole triangle, tcol0 = 0 and tn tile columns): workgroups are
// dealt round-robin over the 8 XCDs (blockIdx % 8); each XCD takes a contiguous
// run of an order that walks 8 x 8 supertiles of the triangle (column by
// column inside each), so the ~32-64 tiles one XCD holds at a time share 16
// slice panels instead of one B panel and ~40 A panels (same tiles, same bits).
// Sharded calls (tcol0 > 0) keep the column order.
constexpr int XB = 128, XST = 8;
__device__ __forceinline__ void xtx_supertile(int L, int tn, int &bm, int &bn) {
    const int U = (tn + XST - 1) / XST;
    for (int Q = 0; Q < U; ++Q) {
        const int w = min(XST, tn - XST * Q);
        for (int P = 0; P <= Q; ++P) {
            const int h = min(XST, tn - XST * P);
            const int cnt = P < Q ? h * w : w * (w + 1) / 2;
            if (L < cnt) {
                if (P < Q) {
                    bn = XST * Q + L / h;
                    bm = XST * P + L % h;
                } else {
                    int c = 0;
                    while (L > c) {
                        L -= c + 1;
                        ++c;
                    }
                    bn = XST * Q + c;
                    bm = XST * P + L;
                }
                return;
            }
            L -= cnt;
        }
    }
    bm = bn = 0;   // not reached for L < tn (tn + 1) / 2
}
// COR: the sparse_cor epilogue (R/TADpole.R:96-98,449) applied to each exact
// S_ij before the store -- C holds cor, with k_cor_epilogue's arithmetic (same
// bits), and S is never written or re-read.  m: column means, sd: sqrt(cov_jj).
// Column slab (tiles != nullptr, C5 row-sharded C): workgroup b computes the
// upper tile tiles[b] and stores only the elements whose column lies in
// [c0, c1), at C[row + (col - c0) n] -- the same tiles and arithmetic as the
// whole matrix, so a slab holds exactly those columns' bits.
// k_xtx_i8_glds: 128 x 128 upper tiles, the supertile order above, 8 waves and
// exact arithmetic (the register-staged k_xtx_i8_big before it, removed in
// round 6), with the slices staged by LDS-DMA (global_load_lds_dwordx4)
// into a ring of 64-deep k-blocks (5 stages of 32 KiB for 2 slices): no VGPR round trip and no
// ds_write pass (k_xtx_i8_big's 64 KiB of b128 stores per k-block ran
// between its MFMA blocks), all but two stages in flight across each raw barrier
// (counted vmcnt, never 0 in the loop).  A stage holds, per (operand,
// slice), 8 chunks of 1 KiB = 16 columns x 64 k-bytes -- one MFMA operand
// fragment each.  A DMA writes its chunk lane-linearly, so the bank swizzle
// goes on the source address: lane p of the chunk loads column p >> 2, k
// bytes 16 ((p & 3) ^ sw) .. +16 with sw = ((p >> 4) & 2); the fragment read of
// (row fr, k quarter kc) is then at slot 4 fr + (kc ^ ((fr >> 2) & 2)), which
// puts every ds_read_b128 lane group on 16 distinct 16-byte bank slots.
#ifndef TP_XG_STAGES2
#define TP_XG_STAGES2 5   // ring stages for 2 slices (32 KiB each: 160 KiB)
#endif
#ifndef TP_XG_STAGES1
#define TP_XG_STAGES1 8   // ring stages for 1 slice (16 KiB each)
#endif
__device__ __forceinline__ void glds16(const void *g, void *l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most n (0..16) of this wave's vector-memory operations are outstanding
__device__ __forceinline__ void wait_vm_dyn(int n) {
    switch (n) {
        case 0: wait_vm<0>(); break;
        case 1: wait_vm<1>(); break;
        case 2: wait_vm<2>(); break;
        case 3: wait_vm<3>(); break;
        case 4: wait_vm<4>(); break;
        case 5: wait_vm<5>(); break;
        case 6: wait_vm<6>(); break;
        case 7: wait_vm<7>(); break;
        case 8: wait_vm<8>(); break;
        case 9: wait_vm<9>(); break;
        case 10: wait_vm<10>(); break;
        case 11: wait_vm<11>(); break;
        case 12: wait_vm<12>(); break;
        case 13: wait_vm<13>(); break;
        case 14: wait_vm<14>(); break;
        case 15: wait_vm<15>(); break;
        default: wait_vm<16>(); break;
    }
}
// lgkmcnt(0) as an instruction the compiler's wait insertion sees (an asm
// wait is opaque to it: it then re-waits, lgkmcnt(0) after the next step's
// fragment reads are issued, before the MFMAs on the current ones)
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
// wait until at most `later` (<= MAXL) stages of CPW DMAs each are outstanding
template <int CPW, int MAXL>
__device__ __forceinline__ void wait_stages(int later) {
    if constexpr (MAXL <= 0) {
        wait_vm<0>();
    } else {
        if (later >= MAXL) wait_vm<MAXL * CPW>();
        else wait_stages<CPW, MAXL - 1>(later);
    }
}
template <int NS, bool COR = false>
__global__ void __launch_bounds__(512) k_xtx_i8_glds(const int8_t *__restrict__ S, int n, int Kp, int Np,
                                                     double *__restrict__ C, int tcol0, int tn_all,
                                                     const double *__restrict__ cm = nullptr,
                                                     const double *__restrict__ csd = nullptr,
                                                     const int2 *__restrict__ tiles = nullptr, int c0 = 0,
                                                     int c1 = 0x7fffffff, const unsigned *__restrict__ nzw = nullptr,
                                                     int NW = 0) {
    constexpr int CH = 2 * NS * 8;         // 1 KiB chunks per stage
    constexpr int CPW = CH / 8;            // chunks per wave per stage
    constexpr int STAGE = CH * 1024;
    constexpr int XG_STAGES = NS == 2 ? TP_XG_STAGES2 : TP_XG_STAGES1;
    __shared__ __attribute__((aligned(16))) int8_t L[XG_STAGES * STAGE];   // the only LDS object (DMA waits)
    int bm, bn;
    if (tiles) {
        const int2 tl = tiles[blockIdx.x];
        bm = tl.x;
        bn = tl.y;
    } else if (tn_all > 0) {
        const int total = tn_all * (tn_all + 1) / 2;
        const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
        xtx_supertile(xcd * (total >> 3) + min(xcd, total & 7) + slot, tn_all, bm, bn);
    } else {
        int id = blockIdx.x;
        bn = tcol0;
        while (id > bn) {
            id -= bn + 1;
            ++bn;
        }
        bm = id;
    }
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = (w & 1) * 64, wn = (w >> 1) * 32;
    const size_t slice = (size_t)Np * Kp;
    const int ia = bm * XB, jb = bn * XB;
    // this lane's DMA sources: chunk c = w + 8 i -> operand o = c / (8 NS),
    // slice (c / 8) % NS, column group c % 8 = w; one per-lane base (operand A,
    // slice 0) plus a wave-uniform offset per chunk
    const int8_t *vsrc;
    {
        const int pc = lane >> 2, pk = (lane & 3) ^ ((lane >> 4) & 2);
        TP_DASSERT(ia + 16 * w + pc < Np && jb + 16 * w + pc < Np);
        vsrc = S + (size_t)(ia + 16 * w + pc) * Kp + 16 * pk;
    }
    auto chunk_off = [&](int i) -> size_t {
        const int c = w + 8 * i, o = c / (8 * NS), s = (c >> 3) % NS;
        return (size_t)s * slice + (o ? (size_t)(jb - ia) * Kp : 0);
    };
    const int nk = Kp / 64;
    // Two slices: the high slice X1 of raw Hi-C counts is zero outside a band
    // around the diagonal (C3: 3 % of the 128-column x 64-k blocks hold a count
    // >= 128), so a stage loads and multiplies X1's chunks only where its
    // block-nonzero map (k_slice_nz) has the bit: a1 / b1 for the A / B
    // operand.  Skipped products are exactly zero: same sums, same bits.
    // Lane j holds word j of the tile row's and tile column's maps.
    unsigned za = ~0u, zb = ~0u;
    if (NS == 2 && nzw != nullptr) {
        za = lane < NW ? nzw[(size_t)bm * NW + lane] : 0u;
        zb = lane < NW ? nzw[(size_t)bn * NW + lane] : 0u;
    }
    auto hi_a = [&](int k) -> bool {
        return NS == 2 && ((__builtin_amdgcn_readlane((int)za, k >> 5) >> (k & 31)) & 1);
    };
    auto hi_b = [&](int k) -> bool {
        return NS == 2 && ((__builtin_amdgcn_readlane((int)zb, k >> 5) >> (k & 31)) & 1);
    };
    auto dmas = [&](int k) -> int {   // DMAs per wave of stage k
        return NS == 2 ? 2 + (int)hi_a(k) + (int)hi_b(k) : CPW;
    };
    auto issue = [&](int k) {   // stage k into ring slot k % XG_STAGES
        int8_t *dst = L + (k % XG_STAGES) * STAGE;
        const bool ha = hi_a(k), hb = hi_b(k);
#pragma unroll
        for (int i = 0; i < CPW; ++i) {
            // NS = 2: i = 0 A0, 1 A1, 2 B0, 3 B1
            if (NS == 2 && ((i == 1 && !ha) || (i == 3 && !hb))) continue;
#ifdef TP_XG_DIAG_NODMA   // diagnostic builds only (timing of the MFMA side alone; wrong results)
            if (k < XG_STAGES)
#endif
            glds16(vsrc + chunk_off(i) + (size_t)64 * k, dst + (w + 8 * i) * 1024);
        }
    };
    i32x4 acc[NS][NS][4][2];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int u = 0; u < NS; ++u)
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[s][u][a][b] = i32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < XG_STAGES - 1; ++k)
        if (k < nk) issue(k);
    const int fr = lane & 15, kc = lane >> 4;
    const int roff = (4 * fr + (kc ^ ((fr >> 2) & 2))) * 16;
    // Fragments of stage k + 1 are read while the MFMAs of stage k run, so the
    // LDS read burst after each barrier is off the MFMA chain.  One slice:
    // two register sets.  Two slices (128 accumulator registers): one set,
    // each fragment re-read right after its last MFMA of the step, in the
    // product order (0,0) (1,0) | b0 | (0,1) | a0 | (1,1) | a1 b1.
    struct Frag {
        i32x4 a[NS][4], b[NS][2];
    };
    auto rd_a = [&](Frag &f, int k, int s) {
        const int8_t *Lb = L + (k % XG_STAGES) * STAGE + roff;
#pragma unroll
        for (int a = 0; a < 4; ++a) f.a[s][a] = *(const i32x4 *)(Lb + (s * 8 + (wm >> 4) + a) * 1024);
    };
    auto rd_b = [&](Frag &f, int k, int s) {
        const int8_t *Lb = L + (k % XG_STAGES) * STAGE + roff;
#pragma unroll
        for (int b = 0; b < 2; ++b) f.b[s][b] = *(const i32x4 *)(Lb + ((NS + s) * 8 + (wn >> 4) + b) * 1024);
    };
    auto read_frags = [&](Frag &f, int k) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            rd_a(f, k, s);
            rd_b(f, k, s);
        }
    };
    auto prod = [&](const Frag &f, int s, int u) {
#ifdef TP_XG_DIAG_NOMFMA   // diagnostic builds only (timing of the load side alone; wrong results)
        return;
#endif
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
                acc[s][u][a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[s][a], f.b[u][b], acc[s][u][a][b], 0, 0, 0);
    };
    // step k: stage k + 1 has landed everywhere (this wave's DMAs by the
    // counted wait, the others' by the barrier) and stage k - 1's slot, read
    // at step k - 2, is refilled with stage k + XG_STAGES - 1
    // this wave's DMAs of the stages after `upto` that are issued by step k
    auto later_dmas = [&](int upto, int last) {
        int c = 0;
        for (int j = upto + 1; j <= min(last, nk - 1); ++j) c += dmas(j);
        return c;
    };
    auto sync_issue = [&](int k) {
        if constexpr (NS == 2) wait_vm_dyn(later_dmas(k + 1, k + XG_STAGES - 2));
        else wait_stages<CPW, XG_STAGES - 3>(nk - 2 - k);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (k + XG_STAGES - 1 < nk) issue(k + XG_STAGES - 1);
    };
    if constexpr (NS == 2) wait_vm_dyn(later_dmas(0, XG_STAGES - 2));
    else wait_stages<CPW, XG_STAGES - 2>(nk - 1);
    __builtin_amdgcn_s_barrier();
    if constexpr (NS == 1) {
        Frag f0, f1;
        read_frags(f0, 0);
        auto step = [&](int k, Frag &cur, Frag &nxt) {
            sync_issue(k);
            if (k + 1 < nk) read_frags(nxt, k + 1);
            prod(cur, 0, 0);
        };
        int k = 0;
        for (; k + 1 < nk; k += 2) {
            step(k, f0, f1);
            step(k + 1, f1, f0);
        }
        if (k < nk) step(k, f0, f1);
    } else {
        static_assert(NS == 2, "1 or 2 slices");
        Frag f;
        rd_a(f, 0, 0);
        rd_b(f, 0, 0);
        if (hi_a(0)) rd_a(f, 0, 1);
        if (hi_b(0)) rd_b(f, 0, 1);
        for (int k = 0; k < nk; ++k) {
            sync_issue(k);
            const bool more = k + 1 < nk;
            const bool ha = hi_a(k), hb = hi_b(k);
            prod(f, 0, 0);
            if (ha) prod(f, 1, 0);
            if (more) rd_b(f, k + 1, 0);
            if (hb) prod(f, 0, 1);
            if (more) rd_a(f, k + 1, 0);
            if (ha && hb) prod(f, 1, 1);
            if (more) {
                if (hi_a(k + 1)) rd_a(f, k + 1, 1);
                if (hi_b(k + 1)) rd_b(f, k + 1, 1);
            }
        }
    }
    __syncthreads();   // the ring is free: the epilogue's column statistics reuse it
    double *pm = (double *)L;   // [0,128) m rows, [128,256) m cols, [256,384) sd rows, [384,512) sd cols
    if constexpr (COR) {
        if (t < 128) {
            const int i = min(ia + t, n - 1), j = min(jb + t, n - 1);
            pm[t] = cm[i];
            pm[128 + t] = cm[j];
            pm[256 + t] = csd[i];
            pm[384 + t] = csd[j];
        }
        __syncthreads();
    }
    const double fn = (double)n, fn1 = (double)(n - 1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int il = wm + 16 * a + (lane >> 4) * 4 + r, jl = wn + 16 * b + fr;
                const int i = ia + il;
                const int j = jb + jl;
                if (i >= n || j >= n || i > j) continue;
                long long v = 0;
#pragma unroll
                for (int s = 0; s < NS; ++s)
#pragma unroll
                    for (int u = 0; u < NS; ++u) v += (long long)acc[s][u][a][b][r] << (7 * (s + u));
                double d = (double)v;
                if constexpr (COR) {
                    const double cij = (d - fn * (pm[il] * pm[128 + jl])) / fn1;
                    d = cij / (pm[256 + il] * pm[384 + jl]);
                    if (isnan(d)) d = 0.0;
                }
                if (j >= c0 && j < c1) C[(size_t)i + (size_t)(j - c0) * n] = d;
                if (i >= c0 && i < c1) C[(size_t)j + (size_t)(i - c0) * n] = d;
            }
}

// k_xtx_i8_w: the whole upper triangle in 256 x 128 tiles -- rows 256 P ..,
// columns 128 Q .., every (P, Q) with 2 P <= Q -- by 8 waves of 64 x 64 (4 x 4
// MFMA tiles each; waves 4 x 2).  Why: the 128-tiles are bound by the per-CU
// LDS-DMA fill rate (~25 GB/s a CU: k_xtx_i8_glds's DMA-only build takes 17.8 of
// its 23.6 ms at 24 300 bins, a one-slice ring of twice the depth no less), and
// a 256 x 128 tile stages 24 KiB a 64-deep k step for twice the MACs (12 KiB
// per 128 x 128 instead of 16).  Its compute side is also leaner: the main
// loop stages slice 0 only (a 6-stage ring, 4 stages in flight, one constant
// counted wait a step where the 128-tiles chose among 17 by the high slice's
// map), and reads step k + 1's fragments while step k's 16 MFMAs run.
//
// The high slice (counts >= 128: a band around the diagonal for raw Hi-C) goes
// in a second phase over the k-blocks where either panel's X1 is nonzero
// (k_slice_nz's map; every block when the map is off): A0 A1 B0 B1 of each such
// block are staged (3-slot ring of 48 KiB) and t01 += A1'B0 + A0'B1,
// t11 += A1'B1 in int32 -- the products k_xtx_i8_glds takes inline, exact in
// separate accumulators (|t01| <= 2 * 64 * 127^2 a block: nk <= 1040), so
// S = acc + 2^7 t01 + 2^14 t11 is the same integer and the same double.
// The epilogue is k_xtx_i8_glds's (COR: the sparse_cor epilogue in the store).
constexpr int XW_ST = 6;                 // main-loop ring stages
constexpr int XW_STAGE = 24 * 1024;      // A0 (256 columns) + B0 (128 columns) x 64 k bytes
constexpr int XW_HSTAGE = 48 * 1024;     // phase 2: A0 A1 B0 B1
constexpr int XW_LIST = XW_ST * XW_STAGE;   // hi-block list (u16) + its count, after the ring
constexpr int XW_LDS = XW_LIST + 4096;
static_assert(3 * XW_HSTAGE <= XW_LIST && XW_LDS <= 160 * 1024, "k_xtx_i8_w LDS");
constexpr int XW_MAXNK = 1040;           // k blocks: t01 stays below 2^31

// tile L of the order below -> (P, Q).  Column panels in chunks of 8, row
// panels in chunks of 4 inside: a chunk pair is 32 tiles sharing 12 panels --
// one XCD's 32 CUs at a time (workgroups are dealt to XCDs round-robin and
// each XCD takes a contiguous run of L).  A full column chunk qc holds
// 32 qc + 20 tiles: qc full row chunks of 4 x 8, then the diagonal one.
__device__ __forceinline__ void xtx_w_tile(int L, int tnc, int &P, int &Q) {
    int qc = 0;
    while (true) {
        const int q0 = 8 * qc, wq = min(8, tnc - q0);
        int cnt = 0;
        if (wq == 8) cnt = 32 * qc + 20;
        else
            for (int q = q0; q < q0 + wq; ++q) cnt += q / 2 + 1;
        if (L < cnt) {
            if (L < 4 * wq * qc) {   // a full row chunk: Q-major inside
                const int pc = L / (4 * wq), r = L % (4 * wq);
                Q = q0 + r / 4;
                P = 4 * pc + (r & 3);
                return;
            }
            L -= 4 * wq * qc;
            for (int q = q0; q < q0 + wq; ++q)
                for (int p = 4 * qc; p <= q / 2; ++p)
                    if (L-- == 0) {
                        P = p;
                        Q = q;
                        return;
                    }
        }
        L -= cnt;
        ++qc;
        if (q0 + 8 >= tnc) break;   // not reached for L < the tile count
    }
    P = Q = 0;
}
static long xtx_w_tiles(int tnc) {
    long t = 0;
    for (int q = 0; q < tnc; ++q) t += q / 2 + 1;
    return t;
}

template <int NS, bool COR>
__global__ void __launch_bounds__(512) k_xtx_i8_w(const int8_t *__restrict__ S, int n, int Kp, int Np,
                                                  double *__restrict__ C, int ntiles,
                                                  const double *__restrict__ cm, const double *__restrict__ csd,
                                                  const unsigned *__restrict__ nzw, int NW,
                                                  const int2 *__restrict__ tiles = nullptr, int c0 = 0,
                                                  int c1 = 0x7fffffff) {
    static_assert(NS == 1 || NS == 2, "1 or 2 slices");
    __shared__ __attribute__((aligned(16))) int8_t L[XW_LDS];
    const int tnc = Np / 128;
    int P, Q;
    if (tiles) {   // column slab (C5 row-sharded C): the listed tiles, stores filtered to [c0, c1)
        const int2 tl = tiles[blockIdx.x];
        P = tl.x;
        Q = tl.y;
    } else {
        const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
        xtx_w_tile(xcd * (ntiles >> 3) + min(xcd, ntiles & 7) + slot, tnc, P, Q);
    }
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w & 3, wc = w >> 2;
    const size_t slice = (size_t)Np * Kp;
    const int ia = 256 * P, jb = 128 * Q;
    // DMA sources (k_xtx_i8_glds's swizzle): lane p of a 1 KiB chunk loads
    // column p >> 2, k bytes 16 ((p & 3) ^ ((p >> 4) & 2)) .. + 15.  Chunks of
    // wave w: A columns 16 w .. (slot w), A 128 + 16 w .. (slot 8 + w), B 16 w ..
    // (slot 16 + w).  A's second half may lie past the padded columns (last row
    // panel): it then reads the first half (its rows are >= n, never stored).
    const int pc = lane >> 2, pk = (lane & 3) ^ ((lane >> 4) & 2);
    const int8_t *vA0 = S + (size_t)(ia + 16 * w + pc) * Kp + 16 * pk;
    const int8_t *vA1 = ia + 128 < Np ? vA0 + (size_t)128 * Kp : vA0;
    const int8_t *vB = S + (size_t)(jb + 16 * w + pc) * Kp + 16 * pk;
    TP_DASSERT(ia + 16 * w + pc < Np && jb + 16 * w + pc < Np);
    const int nk = Kp / 64;
    auto issue = [&](int k) {
        int8_t *dst = L + (k % XW_ST) * XW_STAGE + w * 1024;
        const size_t o = (size_t)64 * k;
        glds16(vA0 + o, dst);
        glds16(vA1 + o, dst + 8 * 1024);
        glds16(vB + o, dst + 16 * 1024);
    };
    i32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = i32x4{0, 0, 0, 0};
    const int fr = lane & 15, kc = lane >> 4;
    const int roff = (4 * fr + (kc ^ ((fr >> 2) & 2))) * 16;
    struct Frag {
        i32x4 a[4], b[4];
    };
    auto read_frags = [&](Frag &f, int k) {
        const int8_t *Lb = L + (k % XW_ST) * XW_STAGE + roff;
#pragma unroll
        for (int i = 0; i < 4; ++i) f.a[i] = *(const i32x4 *)(Lb + (4 * wr + i) * 1024);
#pragma unroll
        for (int i = 0; i < 4; ++i) f.b[i] = *(const i32x4 *)(Lb + (16 + 4 * wc + i) * 1024);
    };
    auto prod = [&](i32x4 (&ac)[4][4], const i32x4 (&fa)[4], const i32x4 (&fb)[4]) {
#ifdef TP_XG_DIAG_NOMFMA   // diagnostic builds only (timing of the load side alone; wrong results)
        return;
#endif
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) ac[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[a], fb[b], ac[a][b], 0, 0, 0);
    };
#pragma unroll
    for (int k = 0; k < XW_ST - 1; ++k)
        if (k < nk) issue(k);
    // step k: stage k + 1 has landed everywhere (this wave's DMAs by the
    // counted wait -- stages k + 2 .. k + XW_ST - 2 may stay in flight -- the
    // others' by the barrier); stage k - 1's slot, read at step k - 2, takes
    // stage k + XW_ST - 1
    auto sync_issue = [&](int k) {
        wait_stages<3, XW_ST - 3>(nk - 2 - k);
        wait_lgkm0();
        __builtin_amdgcn_s_barrier();
#ifdef TP_XG_DIAG_NODMA   // diagnostic builds only (timing of the MFMA side alone; wrong results)
        if (k + XW_ST - 1 < XW_ST)
#endif
        if (k + XW_ST - 1 < nk) issue(k + XW_ST - 1);
    };
    wait_stages<3, XW_ST - 2>(nk - 1);
    __builtin_amdgcn_s_barrier();
    {
        Frag f0, f1;
        read_frags(f0, 0);
        auto step = [&](int k, Frag &cur, Frag &nxt) {
            sync_issue(k);
            if (k + 1 < nk) read_frags(nxt, k + 1);
            prod(acc, cur.a, cur.b);
        };
        int k = 0;
        for (; k + 1 < nk; k += 2) {
            step(k, f0, f1);
            step(k + 1, f1, f0);
        }
        if (k < nk) step(k, f0, f1);
    }
    // every DMA landed (the last steps waited vmcnt(0)); all reads done
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    i32x4 t01[4][4], t11[4][4];
    if constexpr (NS == 2) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) t01[a][b] = t11[a][b] = i32x4{0, 0, 0, 0};
        // the k-blocks where A's (two 128-column panels) or B's X1 is nonzero,
        // ascending, into LDS by wave 0 (lane j: word j of the maps)
        unsigned short *hl = (unsigned short *)(L + XW_LIST);
        int *hcount = (int *)(L + XW_LIST + 4096 - 16);
        int nh = nk;
        if (nzw != nullptr) {
            if (w == 0) {
                unsigned u = 0;
                if (lane < NW) {
                    u = nzw[(size_t)(2 * P) * NW + lane] | nzw[(size_t)Q * NW + lane];
                    if (2 * P + 1 < tnc) u |= nzw[(size_t)(2 * P + 1) * NW + lane];
                }
                const int cnt = __popc(u);
                int incl = cnt;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int y = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += y;
                }
                int pos = incl - cnt;
                while (u) {
                    hl[pos++] = (unsigned short)(32 * lane + __ffs(u) - 1);
                    u &= u - 1;
                }
                if (lane == 63) *hcount = incl;
            }
            wait_lgkm0();
            __builtin_amdgcn_s_barrier();
            nh = __builtin_amdgcn_readfirstlane(*hcount);
        }
        auto blk = [&](int h) -> int {
            return nzw != nullptr ? __builtin_amdgcn_readfirstlane((int)hl[h]) : h;
        };
        // stage h: wave w's chunks A0 (slots w, 8 + w), A1 (16 + w, 24 + w),
        // B0 (32 + w), B1 (40 + w)
        auto issue2 = [&](int h) {
            int8_t *dst = L + (h % 3) * XW_HSTAGE + w * 1024;
            const size_t o = (size_t)64 * blk(h);
            glds16(vA0 + o, dst);
            glds16(vA1 + o, dst + 8 * 1024);
            glds16(vA0 + slice + o, dst + 16 * 1024);
            glds16(vA1 + slice + o, dst + 24 * 1024);
            glds16(vB + o, dst + 32 * 1024);
            glds16(vB + slice + o, dst + 40 * 1024);
        };
        if (nh > 0) issue2(0);
        if (nh > 1) issue2(1);
        for (int h = 0; h < nh; ++h) {
            if (h + 1 < nh) wait_vm<6>();
            else wait_vm<0>();
            wait_lgkm0();
            __builtin_amdgcn_s_barrier();
            if (h + 2 < nh) issue2(h + 2);   // the slot of stage h - 1, read before this barrier
            const int8_t *Lb = L + (h % 3) * XW_HSTAGE + roff;
            i32x4 fa[4], fb[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[i] = *(const i32x4 *)(Lb + (16 + 4 * wr + i) * 1024);   // A1
#pragma unroll
            for (int i = 0; i < 4; ++i) fb[i] = *(const i32x4 *)(Lb + (32 + 4 * wc + i) * 1024);   // B0
            prod(t01, fa, fb);
#pragma unroll
            for (int i = 0; i < 4; ++i) fb[i] = *(const i32x4 *)(Lb + (40 + 4 * wc + i) * 1024);   // B1
            prod(t11, fa, fb);
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[i] = *(const i32x4 *)(Lb + (4 * wr + i) * 1024);   // A0
            prod(t01, fa, fb);
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    double *pm = (double *)L;   // [0,256) m rows, [256,384) m cols, [384,640) sd rows, [640,768) sd cols
    if constexpr (COR) {
        if (t < 256) {
            const int i = min(ia + t, n - 1);
            pm[t] = cm[i];
            pm[384 + t] = csd[i];
        } else if (t < 384) {
            const int j = min(jb + t - 256, n - 1);
            pm[t] = cm[j];
            pm[384 + t] = csd[j];
        }
        __syncthreads();
    }
    const double fn = (double)n, fn1 = (double)(n - 1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int il = 64 * wr + 16 * a + 4 * kc + r, jl = 64 * wc + 16 * b + fr;
                const int i = ia + il, j = jb + jl;
                if (i >= n || j >= n || i > j) continue;
                long long v = (long long)acc[a][b][r];
                if constexpr (NS == 2) v += ((long long)t01[a][b][r] << 7) + ((long long)t11[a][b][r] << 14);
                double d = (double)v;
                if constexpr (COR) {
                    const double cij = (d - fn * (pm[il] * pm[256 + jl])) / fn1;
                    d = cij / (pm[384 + il] * pm[640 + jl]);
                    if (isnan(d)) d = 0.0;
                }
                if (j >= c0 && j < c1) C[(size_t)i + (size_t)(j - c0) * n] = d;
                if (i >= c0 && i < c1) C[(size_t)j + (size_t)(i - c0) * n] = d;
            }
}

// the gather's per-column maxima / flags -> the k_int_scan result format
__global__ void __launch_bounds__(256) k_colflags(const double *cmax, const int *cbad, int n,
                                                  unsigned long long *maxbits, int *notint) {
    __shared__ double wm[4];
    __shared__ int wb[4];
    double m = 0.0;
    int bad = 0;
    for (int j = threadIdx.x; j < n; j += 256) {
        m = fmax(m, cmax[j]);
        bad |= cbad[j];
    }
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    const int anyb = __ballot(bad != 0) != 0ULL;
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        wm[w] = m;
        wb[w] = anyb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double mm = fmax(fmax(wm[0], wm[1]), fmax(wm[2], wm[3]));
        *maxbits = (unsigned long long)__double_as_longlong(mm);
        *notint = wb[0] | wb[1] | wb[2] | wb[3];
    }
}

static int slices_for(Ctx &c, unsigned long long *mb) {
    unsigned long long h[2] = {0, 0};
    unsigned long long *ph = (unsigned long long *)c.pinned(16);   // pinned: no staged copy
    TP_HIP(hipMemcpyAsync(ph, mb, 16, hipMemcpyDeviceToHost, c.cur));
    stream_sync(c, c.cur);
    memcpy(h, ph, 16);
    if ((int)h[1]) return 0;
    double mx;
    memcpy(&mx, &h[0], 8);
    if (mx < 128.0) return 1;
    if (mx < 16384.0) return 2;
    if (mx < 2097152.0) return 3;
    return 0;
}

// Decide the path for X (n x n, col-major, device): 0 = fp64, else the slice count.
int xtx_int_slices(Ctx &c, const double *d_X, int n) {
    if (t_knob.xtx_int8 == 0 || n > 130000) return 0;
    unsigned long long *mb = (unsigned long long *)c.buf[S_SHARD2].as<char>(64);
    int *flag = (int *)(mb + 1);
    TP_HIP(hipMemsetAsync(mb, 0, 16, c.cur));
    const size_t cnt = (size_t)n * n;
    const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>(2048, (cnt / 2 + 255) / 256));
    hipLaunchKernelGGL(k_int_scan, dim3(g), dim3(256), 0, c.cur, d_X, cnt, mb, flag);
    TP_HIP(hipGetLastError());
    return slices_for(c, mb);
}

int xtx_kp(int n);
// The same decision from the gather's per-column statistics (k_gather_prep)
int xtx_int_slices_cols(Ctx &c, const double *d_cmax, const int *d_cbad, int n) {
    if (t_knob.xtx_int8 == 0 || n > 130000) return 0;
    unsigned long long *mb = (unsigned long long *)c.buf[S_SMALL2].as<char>(64);
    int *flag = (int *)(mb + 1);
    hipLaunchKernelGGL(k_colflags, dim3(1), dim3(256), 0, c.cur, d_cmax, d_cbad, n, mb, flag);
    TP_HIP(hipGetLastError());
    return slices_for(c, mb);
}

// Slice column stride: whole 64-byte k-blocks, an ODD number of them, so
// consecutive columns do not all start on the same HBM channel / L2 set (a
// power-of-two stride such as 2048 B at n = 2000 ran 3x slower).
int xtx_kp(int n) {
    const int blocks = (n + 63) / 64;
    return 64 * (blocks | 1);
}

// the slice buffer (device scratch, valid until the next call); its first 64
// bytes hold k_int_scan's result
int8_t *xtx_slice_buf(Ctx &c, int n, int ns) {
    const int Kp = xtx_kp(n), Np = (n + 127) / 128 * 128;
    return c.buf[S_SHARD2].as<int8_t>((size_t)ns * Np * Kp + 64) + 64;
}
// int8 slices of X (device scratch, valid until the next call)
const int8_t *xtx_slices(Ctx &c, const double *d_X, int n, int ns) {
    const int Kp = xtx_kp(n), Np = (n + 127) / 128 * 128;
    int8_t *sl = xtx_slice_buf(c, n, ns);
    dim3 g((unsigned)((Kp / 4 + 255) / 256), (unsigned)Np);
    hipLaunchKernelGGL(k_slice_i8, g, dim3(256), 0, c.cur, d_X, n, Kp, Np, ns, sl);
    TP_HIP(hipGetLastError());
    return sl;
}


// Block-nonzero map of the high slice (slice 1): bit kb & 31 of word
// nzw[cb * NW + kb / 32] is set when any byte of columns 128 cb .. + 127, k
// bytes 64 kb .. + 63 is nonzero.  Workgroup (cb, word): thread t reads
// column t / 2, 32-byte half t % 2 of each of the word's 32 k-blocks.
__global__ void __launch_bounds__(256) k_slice_nz(const int8_t *__restrict__ S1, int Kp, int NW,
                                                  unsigned *__restrict__ nzw) {
    __shared__ unsigned red[4];
    const int cb = blockIdx.x, wd = blockIdx.y, t = threadIdx.x;
    const int nk = Kp / 64;
    const int8_t *col = S1 + (size_t)(cb * 128 + (t >> 1)) * Kp + 32 * (t & 1);
    unsigned m = 0;
#pragma unroll 4
    for (int b = 0; b < 32; ++b) {
        const int kb = wd * 32 + b;
        if (kb >= nk) break;
        const int4 *p = (const int4 *)(col + (size_t)64 * kb);
        const int4 x = p[0], y = p[1];
        const bool nz = (x.x | x.y | x.z | x.w | y.x | y.y | y.z | y.w) != 0;
        m |= nz ? (1u << b) : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) m |= (unsigned)__shfl_xor((int)m, o, 64);
    if ((t & 63) == 0) red[t >> 6] = m;
    __syncthreads();
    if (t == 0) nzw[(size_t)cb * NW + wd] = red[0] | red[1] | red[2] | red[3];
}

template <int NS, bool COR>
static void launch_xtx128_t(Ctx &c, unsigned nb, const int8_t *sl, int n, int Kp, int Np, double *d_S, int tc0,
                            int tn_all, const double *cm, const double *csd, const int2 *d_tl, int c0, int c1) {
    unsigned *nzw = nullptr;
    const int NW = (Kp / 64 + 31) / 32;
    if (NS == 2 && cfg_xtx_nz) {
        if (NW > 64) fail(TP_ERR_INTERNAL, "xtx_int8: k blocks past the 64-word nonzero map");
        nzw = c.buf[S_XNZ].as<unsigned>((size_t)(Np / 128) * NW);
        hipLaunchKernelGGL(k_slice_nz, dim3((unsigned)(Np / 128), (unsigned)NW), dim3(256), 0, c.cur,
                           sl + (size_t)Np * Kp, Kp, NW, nzw);
    }
    hipLaunchKernelGGL((k_xtx_i8_glds<NS, COR>), dim3(nb), dim3(512), 0, c.cur, sl, n, Kp, Np, d_S, tc0, tn_all,
                       cm, csd, d_tl, c0, c1, nzw, NW);
}
static void launch_xtx128(Ctx &c, int ns, unsigned nb, const int8_t *sl, int n, int Kp, int Np, double *d_S, int tc0,
                          int tn_all, const double *cm, const double *csd, const int2 *d_tl, int c0, int c1) {
    const bool cor = cm != nullptr;
    if (ns == 1 && !cor) launch_xtx128_t<1, false>(c, nb, sl, n, Kp, Np, d_S, tc0, tn_all, cm, csd, d_tl, c0, c1);
    else if (ns == 2 && !cor) launch_xtx128_t<2, false>(c, nb, sl, n, Kp, Np, d_S, tc0, tn_all, cm, csd, d_tl, c0, c1);
    else if (ns == 1) launch_xtx128_t<1, true>(c, nb, sl, n, Kp, Np, d_S, tc0, tn_all, cm, csd, d_tl, c0, c1);
    else if (ns == 2) launch_xtx128_t<2, true>(c, nb, sl, n, Kp, Np, d_S, tc0, tn_all, cm, csd, d_tl, c0, c1);
    else fail(TP_ERR_ARG, "xtx_int8 (128-tiles): 1..2 slices");
}


template <int NS, bool COR>
static void launch_xtx_w_t(Ctx &c, const int8_t *sl, int n, int Kp, int Np, double *d_S, const double *cm,
                           const double *csd, const int2 *d_tl, long ntl, int c0, int c1) {
    const long nt = d_tl ? ntl : xtx_w_tiles(Np / 128);
    unsigned *nzw = nullptr;
    const int NW = (Kp / 64 + 31) / 32;
    if (NS == 2 && cfg_xtx_nz) {
        nzw = c.buf[S_XNZ].as<unsigned>((size_t)(Np / 128) * NW);
        hipLaunchKernelGGL(k_slice_nz, dim3((unsigned)(Np / 128), (unsigned)NW), dim3(256), 0, c.cur,
                           sl + (size_t)Np * Kp, Kp, NW, nzw);
    }
    if (nt > 0)
        hipLaunchKernelGGL((k_xtx_i8_w<NS, COR>), dim3((unsigned)nt), dim3(512), 0, c.cur, sl, n, Kp, Np, d_S,
                           (int)nt, cm, csd, nzw, NW, d_tl, c0, c1);
    if (!d_tl) {
        c.xtx_w_n = n;
        c.xtx_w_kp = Kp;
        c.xtx_w_np = Np;
        c.xtx_w_ns = NS;
        c.xtx_w_map = nzw != nullptr;
    }
}

// The MACs k_xtx_i8_w executed (host, after the fact): every tile (P, Q), 2P <=
// Q, runs slice 0 over all nk k-blocks (256 x 128 x 64 MACs a block) and, with
// two slices, three products (A1'B0, A0'B1, A1'B1) over the k-blocks where its
// panels' map words have a bit -- the same union the kernel lists.
bool xtx_w_exec(Ctx &c, double *out) {
    if (!c.xtx_w_n) return false;
    const int Kp = c.xtx_w_kp, Np = c.xtx_w_np, tnc = Np / 128, nk = Kp / 64, NW = (nk + 31) / 32;
    std::vector<unsigned> map;
    if (c.xtx_w_ns == 2 && c.xtx_w_map) {
        map.resize((size_t)tnc * NW);
        TP_HIP(hipStreamSynchronize(c.cur));
        TP_HIP(hipMemcpy(map.data(), c.buf[S_XNZ].p, map.size() * 4, hipMemcpyDeviceToHost));
    }
    double tiles = 0, hi = 0;
    for (int Q = 0; Q < tnc; ++Q)
        for (int P = 0; 2 * P <= Q; ++P) {
            tiles += 1;
            if (c.xtx_w_ns != 2) continue;
            if (map.empty()) {
                hi += nk;
                continue;
            }
            for (int w = 0; w < NW; ++w) {
                unsigned u = map[(size_t)(2 * P) * NW + w] | map[(size_t)Q * NW + w];
                if (2 * P + 1 < tnc) u |= map[(size_t)(2 * P + 1) * NW + w];
                hi += __builtin_popcount(u);
            }
        }
    const double blk = 256.0 * 128.0 * 64.0;
    out[1] = tiles * nk * blk;
    out[0] = out[1] + 3.0 * hi * blk;
    out[2] = hi;
    out[3] = tiles;
    out[4] = nk;
    return true;
}
static bool xtx_w_applies(int ns, int Kp) {
    if (!t_knob.xtx_w || (ns != 1 && ns != 2)) return false;
    return ns == 1 || Kp / 64 <= XW_MAXNK;   // t01's int32 bound
}
// the whole upper triangle (d_tl null) or a column slab's tiles by k_xtx_i8_w
static void launch_xtx_w(Ctx &c, int ns, const int8_t *sl, int n, int Kp, int Np, double *d_S, const double *cm,
                         const double *csd, const int2 *d_tl = nullptr, long ntl = 0, int c0 = 0,
                         int c1 = 0x7fffffff) {
    const bool cor = cm != nullptr;
    if (ns == 1 && !cor) launch_xtx_w_t<1, false>(c, sl, n, Kp, Np, d_S, cm, csd, d_tl, ntl, c0, c1);
    else if (ns == 2 && !cor) launch_xtx_w_t<2, false>(c, sl, n, Kp, Np, d_S, cm, csd, d_tl, ntl, c0, c1);
    else if (ns == 1) launch_xtx_w_t<1, true>(c, sl, n, Kp, Np, d_S, cm, csd, d_tl, ntl, c0, c1);
    else launch_xtx_w_t<2, true>(c, sl, n, Kp, Np, d_S, cm, csd, d_tl, ntl, c0, c1);
    TP_HIP(hipGetLastError());
}

// S (n x n) = X'X exactly on the upper tiles of tile columns [tc0, tc1) and
// their mirrors, from ns slices.
// 128-column tiles [tc0, tc1) (tile units of 128) by the LDS-staged kernel
// (the whole triangle by k_xtx_i8_w's 256 x 128 tiles: same products, same bits)
void xtx_int8_tiles128(Ctx &c, const int8_t *sl, int n, int ns, double *d_S, int tc0, int tc1, const double *cm,
                       const double *csd) {
    const int Kp = xtx_kp(n), Np = (n + 127) / 128 * 128;
    const int tn = Np / 128;
    tc0 = std::max(0, tc0);
    tc1 = tc1 < 0 ? tn : std::min(tn, tc1);
    if (tc1 <= tc0) return;
    if (tc0 == 0 && tc1 == tn && cfg_xtx_supertile && xtx_w_applies(ns, Kp)) {
        launch_xtx_w(c, ns, sl, n, Kp, Np, d_S, cm, csd);
        return;
    }
    const unsigned nb = (unsigned)((long)tc1 * (tc1 + 1) / 2 - (long)tc0 * (tc0 + 1) / 2);
    const int tn_all = (tc0 == 0 && tc1 == tn && cfg_xtx_supertile) ? tn : 0;
    launch_xtx128(c, ns, nb, sl, n, Kp, Np, d_S, tc0, tn_all, cm, csd, nullptr, 0, 0x7fffffff);
    TP_HIP(hipGetLastError());
}

// Columns [c0, c1) of S (or of cor with cm / csd) into d_slab (ld n, column c0
// first): every upper 128-tile that holds an element of those columns or of
// their mirror rows -- (P, Q) with Q in the slab's tile columns, or P in them
// and Q past them.
void xtx_int8_slab128(Ctx &c, const int8_t *sl, int n, int ns, double *d_slab, int c0, int c1, const double *cm,
                      const double *csd) {
    if (c1 <= c0) return;
    const int Kp = xtx_kp(n), Np = (n + 127) / 128 * 128;
    const int tn = Np / 128, T0 = c0 / 128, T1 = (c1 + 127) / 128;
    const bool wide = xtx_w_applies(ns, Kp);
    std::vector<int2> tl;
    if (wide) {   // k_xtx_i8_w tiles (256-row panel P, 128-column panel Q, 2P <= Q)
        for (int q = T0; q < T1; ++q)   // the slab's columns, upper part
            for (int p = 0; 2 * p <= q; ++p) tl.push_back(make_int2(p, q));
        for (int p = c0 / 256; p <= (c1 - 1) / 256; ++p)   // its rows' mirrors past the slab
            for (int q = std::max(T1, 2 * p); q < tn; ++q) tl.push_back(make_int2(p, q));
    } else {
        for (int q = T0; q < T1; ++q)
            for (int p = 0; p <= q; ++p) tl.push_back(make_int2(p, q));
        for (int p = T0; p < T1; ++p)
            for (int q = T1; q < tn; ++q) tl.push_back(make_int2(p, q));
    }
    int2 *d_tl = c.buf[S_XTXT].as<int2>(tl.size());
    TP_HIP(hipMemcpyAsync(d_tl, tl.data(), tl.size() * sizeof(int2), hipMemcpyHostToDevice, c.cur));
    if (wide) launch_xtx_w(c, ns, sl, n, Kp, Np, d_slab, cm, csd, d_tl, (long)tl.size(), c0, c1);
    else launch_xtx128(c, ns, (unsigned)tl.size(), sl, n, Kp, Np, d_slab, 0, 0, cm, csd, d_tl, c0, c1);
    TP_HIP(hipGetLastError());
    // the host tile list must outlive the asynchronous copy
    stream_sync(c, c.cur);
}

void xtx_int8_tiles(Ctx &c, const int8_t *sl, int n, int ns, double *d_S, int tc0, int tc1) {
    const int Kp = xtx_kp(n), Np = (n + 127) / 128 * 128;
    const int tn = (n + 63) / 64;   // output column tiles (rows of the slices: < Np)
    tc0 = std::max(0, tc0);
    tc1 = tc1 < 0 ? tn : std::min(tn, tc1);
    if (tc1 <= tc0) return;
    const long nblk = (long)tc1 * (tc1 + 1) / 2 - (long)tc0 * (tc0 + 1) / 2;
    switch (ns) {
        case 1: hipLaunchKernelGGL(k_xtx_i8<1>, dim3((unsigned)nblk), dim3(256), 0, c.cur, sl, n, Kp, Np, d_S, tc0); break;
        case 2: hipLaunchKernelGGL(k_xtx_i8<2>, dim3((unsigned)nblk), dim3(256), 0, c.cur, sl, n, Kp, Np, d_S, tc0); break;
        case 3: hipLaunchKernelGGL(k_xtx_i8<3>, dim3((unsigned)nblk), dim3(256), 0, c.cur, sl, n, Kp, Np, d_S, tc0); break;
        default: fail(TP_ERR_ARG, "xtx_int8: 1..3 slices");
    }
    TP_HIP(hipGetLastError());
}


}  // namespace tp
