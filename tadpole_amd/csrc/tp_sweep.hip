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

#include <algorithm>
#include <cstring>

namespace tp {

// KS: 64-column slots per lane of the kernels that hold all k PCs (4: k <= 256,
// 8: k <= 512, 16: k <= 1024, chosen per launch).  A column past k contributes nothing (its
// slot is skipped or adds fma(0, 0, acc) = acc), so the bits for k <= 256 are
// the same with either instance.
constexpr int KS_MAX = 16;
inline int ks_for(int k) { return k <= 256 ? 4 : (k <= 512 ? 8 : 16); }
constexpr int ROW_PT = 1 << 30;   // CONISS row code flag: the row is in Pt (a singleton)

// pairwise tree over 64 leaves = the xor butterfly's summation tree
template <int W> struct PTree {
    template <class F> __device__ static __forceinline__ double run(const F &f, int m0) {
        return PTree<W / 2>::run(f, m0) + PTree<W / 2>::run(f, m0 + W / 2);
    }
};
template <> struct PTree<1> {
    template <class F> __device__ static __forceinline__ double run(const F &f, int m0) { return f(m0); }
};

// Tree i (1-based) keeps an n x ld(i) slab, ld(i) = 64 * ceil(i / 64): rows
// are padded with zeros to whole 64-column slots, so a lane's loads, stores and
// Ward terms never need a column guard (a zero pad contributes fma(0, 0, acc)
// = acc exactly: the canonical sums are unchanged).  Trees tree0+1..tree0+ntrees
// are packed.  pad_prefix(m) = sum_{t=1..m} ld(t).
static __host__ __device__ inline size_t pad_prefix(long m) {
    const long g = m / 64, r = m % 64;
    return (size_t)64 * (size_t)(64 * g * (g + 1) / 2 + r * (g + 1));
}
static __host__ __device__ inline size_t sums_off(int n, int tree0, int i) {
    return (size_t)n * (pad_prefix(i - 1) - pad_prefix(tree0));
}
size_t sweep_sums_doubles(int n, int tree0, int ntrees) { return sums_off(n, tree0, tree0 + ntrees + 1); }

// keeps a load unconditional (the compiler would otherwise sink a load whose
// value is only selected under a condition into an exec-masked branch)
__device__ __forceinline__ int pin(int x) {
    asm volatile("" : "+v"(x));
    return x;
}
// three loads pinned together: one wait for all of them (pinning each load
// separately waits for it before the next is issued -- serial LDS round trips)
__device__ __forceinline__ void pin3(int &a, int &b, int &c) { asm volatile("" : "+v"(a), "+v"(b), "+v"(c)); }
__device__ __forceinline__ double pin_d(double x) {
    asm volatile("" : "+v"(x));
    return x;
}

__device__ __forceinline__ double nan2inf(double x) { return isnan(x) ? __longlong_as_double(0x7FF0000000000000LL) : x; }

// STAMPS: diagnostic build accumulating s_memtime cycles per merge phase into
// sd.stamps[tree * 16 + phase]: wave A 0..7, wave B 8..15 (phase names in
// tools/diag_kernels.py).  The product launches STAMPS=false.
//
// Argmin without index keys: candidate costs are never NaN (NaN -> +inf) and a
// non-candidate position holds NaN, which v_min ignores.  The smallest value is
// found with a DPP min-reduction; the leftmost position holding it is the
// lowest set bit of a ballot (positions ascend with lane and block), which is
// exactly the oracle's (value, position) lexicographic rule.  Block minima are
// values only (NaN = block has no candidate).
//
// Synchronisation: the workgroup is one wave.  Every lane writes the same value
// to each shared LDS word it updates, so no barrier is needed in the loop.

// four wave minima interleaved, broadcast (lane 63).  The operands are merge
// costs: non-negative doubles, +inf, or the quiet NaN of a non-candidate, whose
// 64-bit patterns order exactly like the values with that NaN largest -- the
// order v_min_f64 gives (NaN ignored unless every lane holds it).  So the
// minimum is taken on the bit patterns, high words first and then the low words
// of the lanes that hold the smallest high word: one DPP-fused v_min_u32 per
// step (a 64-bit step is two DPP moves and a v_min_f64).  Same result bits.
template <int CTRL> __device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ unsigned umin_(unsigned a, unsigned b) { return a < b ? a : b; }
__device__ __forceinline__ void wave_min4(double &a, double &b, double &c, double &d) {
    unsigned h[4], l[4];
    {
        const unsigned long long ua = (unsigned long long)__double_as_longlong(a),
                                 ub = (unsigned long long)__double_as_longlong(b),
                                 uc = (unsigned long long)__double_as_longlong(c),
                                 ud = (unsigned long long)__double_as_longlong(d);
        h[0] = (unsigned)(ua >> 32); l[0] = (unsigned)ua;
        h[1] = (unsigned)(ub >> 32); l[1] = (unsigned)ub;
        h[2] = (unsigned)(uc >> 32); l[2] = (unsigned)uc;
        h[3] = (unsigned)(ud >> 32); l[3] = (unsigned)ud;
    }
    unsigned m[4] = {h[0], h[1], h[2], h[3]};
#define TP_UMIN4(x, ctl)                                                             \
    x[0] = umin_(x[0], dpp_u<ctl>(x[0]));                                            \
    x[1] = umin_(x[1], dpp_u<ctl>(x[1]));                                            \
    x[2] = umin_(x[2], dpp_u<ctl>(x[2]));                                            \
    x[3] = umin_(x[3], dpp_u<ctl>(x[3]));
    TP_UMIN4(m, 0xB1) TP_UMIN4(m, 0x4E) TP_UMIN4(m, 0x141) TP_UMIN4(m, 0x140) TP_UMIN4(m, 0x142)
    TP_UMIN4(m, 0x143)
    unsigned hm[4], lm[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        hm[q] = (unsigned)__builtin_amdgcn_readlane((int)m[q], 63);
        lm[q] = h[q] == hm[q] ? l[q] : 0xFFFFFFFFu;
    }
    TP_UMIN4(lm, 0xB1) TP_UMIN4(lm, 0x4E) TP_UMIN4(lm, 0x141) TP_UMIN4(lm, 0x140) TP_UMIN4(lm, 0x142)
    TP_UMIN4(lm, 0x143)
#undef TP_UMIN4
    double r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)lm[q], 63);
        r[q] = __longlong_as_double((long long)(((unsigned long long)hm[q] << 32) | lo));
    }
    a = r[0];
    b = r[1];
    c = r[2];
    d = r[3];
}

// two wave minima interleaved, broadcast (lane 63)
__device__ __forceinline__ void wave_min2(double &a, double &b) {
#define TP_MIN2(ctl)                    \
    a = vmin(a, dpp_d<ctl>(a));         \
    b = vmin(b, dpp_d<ctl>(b));
    TP_MIN2(0xB1) TP_MIN2(0x4E) TP_MIN2(0x141) TP_MIN2(0x140) TP_MIN2(0x142) TP_MIN2(0x143)
#undef TP_MIN2
    a = readlane_d(a, 63);
    b = readlane_d(b, 63);
}

// two canonical wave sums interleaved (independent chains, same bits as wave_sum)
__device__ __forceinline__ void wave_sum2(double &u, double &v) {
    u = u + dpp_d<0xB1>(u);
    v = v + dpp_d<0xB1>(v);
    u = u + dpp_d<0x4E>(u);
    v = v + dpp_d<0x4E>(v);
    u = u + dpp_d<0x141>(u);
    v = v + dpp_d<0x141>(v);
    u = u + dpp_d<0x140>(u);
    v = v + dpp_d<0x140>(v);
    u = u + dpp_d<0x142>(u);
    v = v + dpp_d<0x142>(v);
    u = u + dpp_d<0x143>(u);
    v = v + dpp_d<0x143>(v);
    u = readlane_d(u, 63);
    v = readlane_d(v, 63);
}


// ---- scores for CONISS with column slots 0 and 1 paired: row p of W (256 or
// 512) doubles, columns l and l + 64 at 2 l and 2 l + 1, columns 128..W-1 plain
// after them (zero past k).  A lane then fetches its first two columns with
// one 16-byte load; the columns a lane holds and their order are those of the
// plain layout (same bits).  Slab rows of merged clusters use the same layout.
// full: slots 2 and 3 paired as well (W = 256, the copy the 4-slot trees read:
// two 16-byte loads a lane per row).  An odd slot count keeps its last slot
// plain (a paired last slot would be read at a 16-byte stride).
__global__ void __launch_bounds__(256) k_pt_pairs(const double *Pt, int n, int ldp, int k, double *Pt2, int W,
                                                  int full) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)n * W) return;
    const int p = (int)(idx / W), q = (int)(idx % W);
    const int c = (q < 128 || (full && q < 256)) ? (q & ~127) + 64 * (q & 1) + ((q & 127) >> 1) : q;
    Pt2[idx] = c < k ? Pt[(size_t)p * ldp + c] : 0.0;
}
static size_t coniss_pt2_offset(int n, int ntrees) {
    return ((size_t)ntrees * (coniss_cost_stride(n) + coniss_link_stride(n)) + 1) & ~(size_t)1;
}

// ---- initial adjacent (singleton) costs of every tree: e_j = x_j - y_j over
// the first i score columns, cost = tot / 2 (canonical order).  One wave per
// (tree, 64 positions).  The trees' cluster-sum slabs are not seeded: a
// singleton's sums are its row of the shared scores Pt (read there by
// k_coniss); a slab row is written only when a merge forms that cluster.
template <int KS>
__global__ void __launch_bounds__(64) k_seed(SweepDev sd, double *cost0) {
    const int n = sd.n, ldp = sd.ldp;
    const int ti = blockIdx.x, i = sd.tree0 + ti + 1;
    const int lane = threadIdx.x;
    double *c0 = cost0 + (size_t)ti * coniss_cost_stride(n);
    const int p0 = blockIdx.y * 64;
    const double QNAN = __longlong_as_double(0x7FF8000000000000LL);
    // rows are fetched RB at a time (all their loads in flight before the first
    // reduction; C3: RB 4 / 8 / 16 = 145 / 150 / 175 us, registers vs latency);
    // the walk over 64 positions is otherwise one load latency a step
    constexpr int RB = 4;
    double x[KS];
#pragma unroll
    for (int t = 0; t < KS; ++t) {
        const int j = lane + 64 * t;
        x[t] = (p0 < n && j < i) ? sd.Pt[(size_t)p0 * ldp + j] : 0.0;
    }
    double mycost = QNAN;
    for (int q0 = 0; q0 < 64 && p0 + q0 + 1 < n; q0 += RB) {
        double z[RB][KS];
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            const int r = p0 + q0 + u + 1;
#pragma unroll
            for (int t = 0; t < KS; ++t) {
                const int j = lane + 64 * t;
                z[u][t] = (r < n && j < i) ? sd.Pt[(size_t)r * ldp + j] : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            const int q = q0 + u;
            if (p0 + q + 1 < n) {                      // uniform over the wave
                double acc = 0.0;
#pragma unroll
                for (int t = 0; t < KS; ++t)
                    if (lane + 64 * t < i) {
                        double e = x[t] - z[u][t];
                        acc = fma(e, e, acc);
                    }
                double tot = wave_sum(acc);
                if (lane == q) mycost = nan2inf(tot / 2.0);
            }
#pragma unroll
            for (int t = 0; t < KS; ++t) x[t] = z[u][t];
        }
    }
    c0[p0 + lane] = mycost;
}

// CONISS link arrays: int (LDS variant, or global memory), or 16-bit indices in
// LDS for the costs-in-global variant (-1 <-> 0xFFFF; n <= ~40k)
template <bool U16> struct LinkArr {
    int *p;
    __device__ __forceinline__ int get(int i) const { return p[i]; }
    __device__ __forceinline__ void set(int i, int v) const { p[i] = v; }
};
template <> struct LinkArr<true> {
    unsigned short *p;
    __device__ __forceinline__ int get(int i) const {
        const int x = p[i];
        return x == 0xFFFF ? -1 : x;
    }
    __device__ __forceinline__ void set(int i, int v) const { p[i] = (unsigned short)v; }
};
// LU = 2 (link-only): rn is not stored.  rn is only read at a cluster start a
// (or the dummy slot DL, whose link is -1), where it is the end of the next
// cluster, link[link[a] + 1] (link[n] = -1 ends the chain), and every rn store
// restates exactly that value -- half the LDS a tree for one dependent LDS
// read more on some merge-chain steps
struct RnDerived {
    LinkArr<true> link;
    __device__ __forceinline__ int get(int i) const {
        const int e = link.get(i);
        return e < 0 ? -1 : link.get(e + 1);
    }
    __device__ __forceinline__ void set(int, int) const {}
};
template <int LU> struct RnOf { using T = LinkArr<LU != 0>; };
template <> struct RnOf<2> { using T = RnDerived; };

// Columns i..ld-1 of a row hold whatever the row was read from (later PCs of
// Pt, or their sums): the last slot's term is selected to 0 there, which adds
// fma(0, 0, acc) = acc -- the canonical sum over the first i columns.
template <int NS>
__device__ __forceinline__ double ward_part(const double (&sa)[NS], double fa, const double (&sb)[NS], double fb,
                                            bool last_in) {
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
        const double t1 = sa[t] * fb;
        const double t2 = sb[t] * fa;
        const double e = (t < NS - 1 || last_in) ? t1 - t2 : 0.0;
        acc = fma(e, e, acc);
    }
    return acc;
}

// One tree's CONISS with NS = ld(i) / 64 column slots per lane and BS block-
// minimum slots per lane (n <= 4096 BS), on two waves of one workgroup (two
// SIMDs) that run the two independent halves of every merge concurrently:
//   wave A (structure): LDS costs/links, masking, block-minimum refresh, the
//     speculative argmin a2 and the descriptions of the three possible next
//     merges; after barrier X only the choice among them;
//   wave B (sums): the rows in registers, merged sums, Ward costs cl/cr, merge
//     records and heights; after X the prefetch of a2's rows.
// Same merges and arithmetic as the oracle (bit-identical).
//
// Speculative prefetch.  After merge s (pair a|b -> m at a) the next merge is
// one of exactly three: the smallest cost among positions merge s does not
// touch (a2, found with ls/a/b masked out), ls|m (new cost cl) or m|r (new cost
// cr).  Their rows are loaded during merge s -- rows a2, b2, ls2, r2 (one that is
// m comes from registers) for a2; sl, sm, row(ll), sr for ls|m; sm, sr, sl,
// row(rr) for m|r -- and the choice is applied at the next merge.
//
// Two barriers per merge.  Before X, A publishes a2's row starts and B cl and
// cr; after X, B prefetches a2's rows while A chooses the next merge among the
// three candidates it holds and publishes its record and cost before Y.  (One
// barrier with both waves choosing was slower: B's prefetch of a2's rows then
// has only B's own choice to hide behind, and HBM latency shows.)  Mailbox
// words are written before one barrier and read after it.
// Variants built and measured slower (in git history): block
// argmin positions in registers, LDS-only barriers, the global variant's next
// cost blocks prefetched after the choice, a2's rows prefetched before X.
// Build switch:
// TP_CONISS_RECB   global variant: the sums wave keeps the merge records (a, b,
//                  cost, height) of 64 merges in registers (lane s % 64) and
//                  stores them once per 64 merges, instead of four stores a merge
#ifndef TP_CONISS_RECB
#define TP_CONISS_RECB 1
#endif
template <bool STAMPS, int NS, int BS, bool GLB, int LU = 0>
__device__ __forceinline__ void coniss_tree2(const SweepDev &sd, double *cost0, double *lds, double *mb_d,
                                             int4 *mb_i) {
    long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long st_t0 = STAMPS ? (long long)__builtin_amdgcn_s_memtime() : 0;
#define TP_STAMP(ph)                                                      \
    if (STAMPS) {                                                         \
        long long _t = (long long)__builtin_amdgcn_s_memtime();           \
        st_acc[ph] += _t - st_t0;                                         \
        st_t0 = _t;                                                       \
    }
    const int n = sd.n;
    const int ti = blockIdx.x;
    const int i = sd.tree0 + ti + 1;
    constexpr int ld = NS * 64;
    const int lane = threadIdx.x & 63;
    const bool waveA = __builtin_amdgcn_readfirstlane((int)threadIdx.x) < 64;   // wave-uniform: a scalar branch
    // measured: 24.3k bins (global variant) 46.8 -> 46.1 ms, C3 (LDS) 9.90 -> 10.09 ms
    constexpr bool kRecb = GLB && TP_CONISS_RECB != 0;
    const int nbk = (n + 63) / 64;
    const double QNAN = __longlong_as_double(0x7FF8000000000000LL);
    // GLB (n above the LDS capacity): costs stay in this tree's slice of cost0
    // (L2 / MALL resident) and links either in LDS as 16-bit indices (LU, n up
    // to ~38k: the link chains of merge_at stay LDS round trips) or in global
    // scratch behind cost0.  Same code path otherwise.
    const size_t cst = coniss_cost_stride(n), lst = coniss_link_stride(n);
    // LU (with GLB): the links are 16-bit indices in LDS, the costs stay global
    double *cost = GLB ? cost0 + (size_t)ti * cst : lds;
    LinkArr<LU != 0> link;
    typename RnOf<LU>::T rn;
    if constexpr (LU != 0) {   // global variant: LDS holds only links; LDS variant: after the costs
        link.p = (unsigned short *)(GLB ? lds : lds + cst);
    } else {
        link.p = GLB ? (int *)(cost0 + (size_t)sd.ntrees * cst) + (size_t)ti * 2 * lst : (int *)(cost + cst);
    }
    if constexpr (LU == 2)
        rn.link = link;
    else
        rn.p = link.p + lst;
    // dummy slots: branch-free code writes absent positions there (an exec-
    // masked `if` costs ~55 cycles on the merge chain, a select ~14)
    const int DC = nbk * 64, DL = n;
    // mailbox (static LDS, so every access is a ds_ op that waits on lgkmcnt
    // only: a generic pointer here made each access a flat_ op whose wait also
    // drained the prefetched row loads): mb_d[0..1] = cl, cr (B -> A before
    // X), mb_d[2] = the next merge's cost (A -> B before Y); mb_i[0..2] = the
    // next merge's record (A -> B before Y), mb_i[3] = a2's row starts
    // (a2s, b2s, ls2, r2) (A -> B before X).
    // Row codes: a cluster's start position, | ROW_PT when the cluster is a
    // singleton (its sums are its row of the shared scores Pt, which no tree
    // writes: slabs hold only merged clusters).  A knows the ends of every
    // cluster it names, so it flags singletons in what it sends B.
    // rows with NS >= 2: slots 0 and 1 paired (lane l: doubles 2l, 2l + 1),
    // slots 2 and 3 plain -- in the tree's slab (stride ld) and in the shared
    // paired copy of the scores (stride sd.pt2_ld); NS = 1: plain rows, the scores
    // read from Pt itself
    // NS = 4: slots (2, 3) paired too, slab rows and the shared copy sd.pt4
    constexpr bool P4 = NS == 4;
    double *S = sd.sums + sums_off(n, sd.tree0, i);
    const double *PP = P4 ? sd.pt4 : (NS >= 2 ? sd.pt2 : sd.Pt);
    const size_t ldpp = P4 ? (size_t)256 : (NS >= 2 ? (size_t)sd.pt2_ld : (size_t)sd.ldp);
    const bool last_in = lane + 64 * (NS - 1) < i;
    int *mrg_a = sd.mrg_a + (size_t)ti * (n - 1);
    int *mrg_b = sd.mrg_b + (size_t)ti * (n - 1);
    double *mcost = sd.cost + (size_t)ti * (n - 1);
    double *height = sd.height + (size_t)ti * (n - 1);
    const double *c0 = cost0 + (size_t)ti * cst;

    double bmr[BS];
    auto argmin_pos = [&](double vmin) -> int {
        if (isnan(vmin)) return -1;
        int blk = 0;
#pragma unroll
        for (int q = BS - 1; q >= 0; --q) {
            const unsigned long long m = __ballot(bmr[q] == vmin);
            if (m) blk = 64 * q + (int)__builtin_ctzll(m);
        }
        const unsigned long long mp = __ballot(cost[blk * 64 + lane] == vmin);
        return blk * 64 + (int)__builtin_ctzll(mp);
    };
    auto gmin = [&]() {
        double g = bmr[0];
#pragma unroll
        for (int q = 1; q < BS; ++q) g = vmin(g, bmr[q]);
        return wave_min(g);
    };
    auto load_row = [&](double (&dst)[NS], int code) {
        code = __builtin_amdgcn_readfirstlane(code);
        const int p = code & (ROW_PT - 1);
        const double *pr = (code & ROW_PT) ? PP + (size_t)p * ldpp : S + (size_t)p * ld;
        if (NS >= 2) {
            const double2 v = *(const double2 *)(pr + 2 * lane);
            dst[0] = v.x;
            dst[1] = v.y;
        } else {
            dst[0] = pr[lane];
        }
        if (P4) {
            const double2 v = *(const double2 *)(pr + 128 + 2 * lane);
            dst[2] = v.x;
            dst[3] = v.y;
        } else {
#pragma unroll
            for (int t = 2; t < NS; ++t) dst[t] = pr[64 * t + lane];
        }
    };
    auto rowc = [](int start, bool single) { return start | (single ? ROW_PT : 0); };
    // A: a merge described by (a, ea, eb, ls, r, er); b = ea + 1; ll = start of
    // the cluster left of ls (its ls|m successor's left row); rre = end of the
    // cluster right of r (rr, its m|r successor's right row)
    struct Mg {
        int a, ea, eb, ls, r, er, ll, rre;
    };
    auto merge_at1 = [&](int p) {   // current links -> the pair starting at p, first level (no branches)
        Mg m;
        m.a = p;
        m.ea = link.get(p);
        m.eb = rn.get(p);
        const int lsv = pin(link.get(p > 0 ? p - 1 : DL));
        m.ls = p > 0 ? lsv : -1;
        m.r = m.eb >= 0 && m.eb + 1 < n ? m.eb + 1 : -1;
        return m;
    };
    auto merge_at2 = [&](Mg &m) {   // second level: the right ends of r and rr, the cluster left of ls
        int erv = rn.get(m.ea + 1 < n ? m.ea + 1 : DL);
        int llv = link.get(m.ls > 0 ? m.ls - 1 : DL);
        int rrev = rn.get(m.r >= 0 ? m.r : DL);
        pin3(erv, llv, rrev);
        m.er = m.r >= 0 ? erv : -1;
        m.ll = m.ls > 0 ? llv : -1;
        m.rre = rrev;
    };
    auto merge_at = [&](int p) {
        Mg m = merge_at1(p);
        merge_at2(m);
        return m;
    };
    struct Rec {
        int4 x, y, z;
    };
    auto make_rec = [&](const Mg &m, int which) {   // A -> B: the record of a next merge
        const int rr = (m.r >= 0 && m.er + 1 < n) ? m.er + 1 : -1;
        const int ac = rowc(m.a, m.ea == m.a);
        Rec rc;
        rc.x = make_int4(m.a, m.ea + 1 < n ? m.ea + 1 : m.a, m.ls, m.r);
        rc.y = make_int4(m.eb - m.a + 1, m.ls >= 0 ? m.a - m.ls : 0, m.r >= 0 ? m.er - m.r + 1 : 0,
                         m.ll >= 0 ? rowc(m.ll, m.ll == m.ls - 1) : ac);
        rc.z = make_int4(rr >= 0 ? rowc(rr, m.rre == rr) : ac, which, 0, 0);
        return rc;
    };
    // the choice after merge (a, ls, r): the lexicographic (cost, position)
    // minimum of (v2, a2), (cl, ls), (cr, a) -- both waves evaluate it
    auto choose = [](int a, int ls, int r, double v2, int a2, double cl, double cr, bool &c1, bool &c2,
                     double &nv) {
        c1 = (ls >= 0) & ((a2 < 0) | (cl < v2) | ((cl == v2) & (ls < a2)));
        nv = c1 ? cl : v2;
        const int np = c1 ? ls : a2;
        c2 = (r >= 0) & ((np < 0) | (cr < nv) | ((cr == nv) & (a < np)));
        nv = c2 ? cr : nv;
    };
    Mg cur = {0, 0, 0, -1, -1, -1, -1, -1};
    double c = 0.0, pcl = QNAN, pcr = QNAN;
    int pls = DC, pa_ = DC;   // A: where the previous merge's new costs go (applied at the next merge's start)
    if (waveA) {
#pragma unroll
        for (int q = 0; q < BS; ++q) bmr[q] = QNAN;
        for (int bk = 0; bk < nbk; ++bk) {
            const int p = bk * 64 + lane;
            const double cp = c0[p];
            if (!GLB) cost[p] = cp;
            if (p < n) {
                link.set(p, p);
                rn.set(p, p + 1 < n ? p + 1 : -1);
            }
            if (bk == 0) {
                link.set(DL + lane, -1);
                rn.set(DL + lane, -1);
            }
            const double m = wave_min(cp);
            if (lane == (bk & 63)) {
#pragma unroll
                for (int q = 0; q < BS; ++q)
                    if (q == (bk >> 6)) bmr[q] = m;
            }
        }
        c = gmin();
        cur = merge_at(argmin_pos(c));
        const Rec rc = make_rec(cur, 0);
        mb_i[0] = rc.x;
        mb_i[1] = rc.y;
        mb_i[2] = rc.z;
        mb_d[2] = c;
    }
    __syncthreads();
    // B's registers
    double pa[NS], pb[NS], pl[NS], pr[NS], pll[NS], prr[NS], sl[NS], sr[NS], sm[NS];
    int ls2p = -1, r2p = -1, aprev = -1;
    double h = 0.0;
    int rec_a = 0, rec_b = 0;          // kRecb: merge s % 64's record in lane s % 64
    double rec_c = 0.0, rec_h = 0.0;
    if (!waveA) {
        const int4 q0 = mb_i[0];
        // the first merge's clusters are all singletons
        load_row(pa, rowc(q0.x, true));
        load_row(pb, rowc(q0.y, true));
        load_row(pl, rowc(q0.z >= 0 ? q0.z : q0.x, true));
        load_row(pr, rowc(q0.w >= 0 ? q0.w : q0.x, true));
        ls2p = q0.z;
        r2p = q0.w;
#pragma unroll
        for (int t = 0; t < NS; ++t) pll[t] = prr[t] = sl[t] = sr[t] = sm[t] = 0.0;
    }
    TP_STAMP(4);

    for (int s = 0; s < n - 1; ++s) {
        if (waveA) {
            // ---- the previous merge's new costs, then this merge's structure
            //      update with ls, a, b masked, refresh, speculative argmin
            const int a = cur.a, eb = cur.eb, ls = cur.ls, b = cur.ea + 1, r = cur.r, er = cur.er;
            // branch-free: absent positions write the dummy slots
            cost[pls] = pcl;
            cost[pa_] = pcr;
            link.set(a, eb);
            link.set(eb, a);
            rn.set(a, er);
            cost[b] = QNAN;
            cost[a] = QNAN;
            cost[ls >= 0 ? ls : DC] = QNAN;
            rn.set(ls >= 0 ? ls : DL, eb);
            // links the two candidate merges next to m need (independent of a2:
            // issued before the argmin's reductions so their latency overlaps)
            int m1llv = link.get(cur.ll > 0 ? cur.ll - 1 : DL);
            int m2erv = rn.get(r >= 0 ? r : DL);
            int m2rrev = rn.get((r >= 0 && er + 1 < n) ? er + 1 : DL);
            // refresh the three touched blocks and, concurrently, the minimum of
            // the untouched ones: four interleaved wave reductions
            const int ba = a >> 6, bb = b >> 6, bl = ls >= 0 ? (ls >> 6) : ba;
            const double va = cost[ba * 64 + lane];
            const double vb = cost[bb * 64 + lane];
            const double vl = cost[bl * 64 + lane];
            double rest = QNAN;
#pragma unroll
            for (int q = 0; q < BS; ++q) {
                const int blk = 64 * q + lane;
                rest = vmin(rest, (blk == ba || blk == bb || blk == bl) ? QNAN : bmr[q]);
            }
            TP_STAMP(6);
            double ma = va, mb = vb, ml = vl, mr = rest;
            wave_min4(ma, mb, ml, mr);
#pragma unroll
            for (int q = 0; q < BS; ++q) {
                bmr[q] = (lane == (ba & 63) && q == (ba >> 6)) ? ma : bmr[q];
                bmr[q] = (lane == (bb & 63) && q == (bb >> 6)) ? mb : bmr[q];
                bmr[q] = (lane == (bl & 63) && q == (bl >> 6)) ? ml : bmr[q];
            }
            const double v2 = vmin(vmin(mr, ma), vmin(mb, ml));
            // leftmost position holding v2: its block from the block minima, then
            // the block's words (v2 NaN: no ballot matches, a2 = -1)
            int blk = 0;
#pragma unroll
            for (int q = BS - 1; q >= 0; --q) {
                const unsigned long long m = __ballot(bmr[q] == v2);
                blk = m ? 64 * q + (int)__builtin_ctzll(m) : blk;
            }
            const unsigned long long mv = __ballot(cost[blk * 64 + lane] == v2);
            const int a2 = mv ? blk * 64 + (int)__builtin_ctzll(mv) : -1;
            TP_STAMP(7);
            // ---- the three possible next merges (post-update links); a2's
            //      clusters go to B at once (its row prefetch starts before X)
            Mg m0 = merge_at1(a2 >= 0 ? a2 : a);
            merge_at2(m0);
            pin3(m1llv, m2erv, m2rrev);   // issued before the reductions; waited for only here
            const int m1ll = cur.ll > 0 ? m1llv : -1;
            const int m2er = (r >= 0 && er + 1 < n) ? m2erv : -1;
            {   // a2's four rows (absent ls / r: -1), singletons flagged
                const int bs2 = m0.ea + 1 < n ? m0.ea + 1 : m0.a;
                mb_i[3] = make_int4(rowc(m0.a, m0.ea == m0.a), rowc(bs2, m0.eb == bs2),
                                    m0.ls >= 0 ? rowc(m0.ls, m0.ls == m0.a - 1) : -1,
                                    m0.r >= 0 ? rowc(m0.r, m0.er == m0.r) : -1);
            }
            Mg m1;   // ls | m
            m1.a = ls; m1.ea = a - 1; m1.eb = eb; m1.ls = cur.ll; m1.r = r; m1.er = er;
            m1.ll = m1ll;
            m1.rre = m2erv;
            Mg m2;   // m | r
            m2.a = a; m2.ea = eb; m2.eb = er; m2.ls = ls;
            m2.r = (r >= 0 && er + 1 < n) ? er + 1 : -1;
            m2.er = m2er;
            m2.ll = cur.ll;
            m2.rre = m2rrev;
            TP_STAMP(0);
            __syncthreads();   // X
            TP_STAMP(1);
            // ---- the choice
            const double cl = mb_d[0], cr = mb_d[1];
            bool c1, c2;
            double nv;
            choose(a, ls, r, v2, a2, cl, cr, c1, c2, nv);
            // field by field (a select of whole structs goes through scratch)
            auto sel = [&](int x0, int x1, int x2) { return c2 ? x2 : (c1 ? x1 : x0); };
            cur.a = sel(m0.a, m1.a, m2.a);
            cur.ea = sel(m0.ea, m1.ea, m2.ea);
            cur.eb = sel(m0.eb, m1.eb, m2.eb);
            cur.ls = sel(m0.ls, m1.ls, m2.ls);
            cur.r = sel(m0.r, m1.r, m2.r);
            cur.er = sel(m0.er, m1.er, m2.er);
            cur.ll = sel(m0.ll, m1.ll, m2.ll);
            cur.rre = sel(m0.rre, m1.rre, m2.rre);
            c = nv;
            {
                const Rec rc = make_rec(cur, c2 ? 2 : (c1 ? 1 : 0));
                mb_i[0] = rc.x;
                mb_i[1] = rc.y;
                mb_i[2] = rc.z;
                mb_d[2] = nv;
            }
            // block minima absorb the new costs now (the LDS words follow at the
            // next merge's start, before its refresh reads them)
#pragma unroll
            for (int q = 0; q < BS; ++q) {
                const double tr = vmin(bmr[q], cr);
                bmr[q] = (lane == (ba & 63) && q == (ba >> 6)) ? tr : bmr[q];
                const double tl = vmin(bmr[q], cl);
                bmr[q] = (ls >= 0 && lane == (bl & 63) && q == (bl >> 6)) ? tl : bmr[q];
            }
            pcl = cl;
            pcr = cr;
            pls = ls >= 0 ? ls : DC;
            pa_ = a;
            TP_STAMP(2);
            __syncthreads();   // Y
            TP_STAMP(3);
        } else {
            // ---- this merge's rows from the previous merge's prefetch
            const int4 q0 = mb_i[0], q1 = mb_i[1], q2 = mb_i[2];
            const double cc = mb_d[2];
            const int a_ = q0.x, b_ = q0.y, ls_ = q0.z, r_ = q0.w;
            const int nm = q1.x, nl = q1.y, nr = q1.z, lls = q1.w;
            const int rrs = q2.x, which = q2.y;
            TP_STAMP(0);
            double sa[NS], sb[NS];
            if (which == 0) {
#pragma unroll
                for (int t = 0; t < NS; ++t) {
                    sa[t] = pa[t];
                    sb[t] = pb[t];
                    sl[t] = ls2p == aprev ? sm[t] : pl[t];
                    sr[t] = r2p == aprev ? sm[t] : pr[t];
                }
            } else if (which == 1) {   // ls | m
#pragma unroll
                for (int t = 0; t < NS; ++t) {
                    sa[t] = sl[t];
                    sb[t] = sm[t];
                    sl[t] = pll[t];
                }
            } else {                   // m | r
#pragma unroll
                for (int t = 0; t < NS; ++t) {
                    sa[t] = sm[t];
                    sb[t] = sr[t];
                    sr[t] = prr[t];
                }
            }
            // rows the ls|m and m|r candidates of the next merge need
            load_row(pll, lls);
            load_row(prr, rrs);
#pragma unroll
            for (int t = 0; t < NS; ++t) sm[t] = sa[t] + sb[t];
            if (NS >= 2)
                *(double2 *)(S + (size_t)a_ * ld + 2 * lane) = make_double2(sm[0], sm[1]);
            else
                S[(size_t)a_ * ld + lane] = sm[0];
            if (P4) {
                *(double2 *)(S + (size_t)a_ * ld + 128 + 2 * lane) = make_double2(sm[2], sm[3]);
            } else {
#pragma unroll
                for (int t = 2; t < NS; ++t) S[(size_t)a_ * ld + 64 * t + lane] = sm[t];
            }
            if (STAMPS) {   // waits for the rows (the stamp below then counts the HBM wait)
                double z = 0.0;
#pragma unroll
                for (int t = 0; t < NS; ++t) z += sm[t];
                asm volatile("" ::"v"(z));
            }
            TP_STAMP(1);
            const double fm = (double)nm, fl = (double)nl, fr = (double)nr;
            double ul = ward_part<NS>(sl, fl, sm, fm, last_in);
            double ur = ward_part<NS>(sm, fm, sr, fr, last_in);
            wave_sum2(ul, ur);
            // both divisions unconditionally (interleaved, no branch), then select
            const double ql = pin_d(ul / (fl * fm * (fl + fm)));
            const double qr = pin_d(ur / (fm * fr * (fm + fr)));
            const double cl = ls_ >= 0 ? nan2inf(ql) : QNAN;
            const double cr = r_ >= 0 ? nan2inf(qr) : QNAN;
            h = h + cc;
            mb_d[0] = cl;
            mb_d[1] = cr;
            // every lane stores the same words (one request each; no exec mask)
            if constexpr (kRecb) {
                const bool mine = lane == (s & 63);
                rec_a = mine ? a_ : rec_a;
                rec_b = mine ? b_ : rec_b;
                rec_c = mine ? cc : rec_c;
                rec_h = mine ? h : rec_h;
                if ((s & 63) == 63 || s == n - 2) {   // uniform: 64 records (or the last ones) at once
                    const int s0 = s & ~63;
                    if (lane <= (s & 63)) {
                        mrg_a[s0 + lane] = rec_a;
                        mrg_b[s0 + lane] = rec_b;
                        mcost[s0 + lane] = rec_c;
                        height[s0 + lane] = rec_h;
                    }
                }
            } else {
                mrg_a[s] = a_;
                mrg_b[s] = b_;
                mcost[s] = cc;
                height[s] = h;
            }
            TP_STAMP(2);
            __syncthreads();   // X
            TP_STAMP(3);
            // ---- prefetch a2's rows for the next merge
            const int4 p0 = mb_i[3];
            load_row(pa, p0.x);
            load_row(pb, p0.y);
            load_row(pl, p0.z >= 0 ? p0.z : p0.x);
            load_row(pr, p0.w >= 0 ? p0.w : p0.x);
            ls2p = p0.z;
            r2p = p0.w;
            aprev = a_;
            TP_STAMP(6);
            __syncthreads();   // Y
            TP_STAMP(7);
        }
    }
    __syncthreads();
    // ---- broken stick (rioja bstick.chclust, vegan bstick.default) on heights
    if (threadIdx.x == 0) {
        const int nobj = n - 1;
        int ncl = -1;
        if (nobj >= 2) {
            const double tot = height[nobj - 1];
            double *cs = cost;
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
    TP_STAMP(5);
    if (STAMPS && lane == 0)   // wave A: slots 0..7, wave B: 8..15
        for (int q = 0; q < 8; ++q) sd.stamps[(size_t)ti * 16 + (waveA ? 0 : 8) + q] = st_acc[q];
#undef TP_STAMP
}

// STAMPS: diagnostic build (see coniss_tree2).  BS: block-minimum slots (n <= 4096 BS).
// LU: the global variant with its links as 16-bit indices in LDS.
// KS: the most column slots a tree of this launch has (4: k <= 256; 8: k <= 512)
template <bool STAMPS, int BS, bool GLB, int LU = 0, int KS = 4>
__global__ void __launch_bounds__(128) k_coniss_t(SweepDev sd, double *cost0) {
    extern __shared__ double lds[];
    __shared__ double mb_d[4];
    __shared__ int4 mb_i[4];
    const int i = sd.tree0 + blockIdx.x + 1;
    switch ((i + 63) / 64) {
        case 1: coniss_tree2<STAMPS, 1, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
        case 2: coniss_tree2<STAMPS, 2, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
        case 3: coniss_tree2<STAMPS, 3, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
        case 4: coniss_tree2<STAMPS, 4, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
        default:
            if constexpr (KS > 4) {
                switch ((i + 63) / 64) {
                    case 5: coniss_tree2<STAMPS, 5, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                    case 6: coniss_tree2<STAMPS, 6, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                    case 7: coniss_tree2<STAMPS, 7, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                    case 8: coniss_tree2<STAMPS, 8, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                    default:
                        if constexpr (KS > 8) {
                            switch ((i + 63) / 64) {
                                case 9: coniss_tree2<STAMPS, 9, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                                case 10: coniss_tree2<STAMPS, 10, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                                case 11: coniss_tree2<STAMPS, 11, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                                case 12: coniss_tree2<STAMPS, 12, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                                case 13: coniss_tree2<STAMPS, 13, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                                case 14: coniss_tree2<STAMPS, 14, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                                case 15: coniss_tree2<STAMPS, 15, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                                default: coniss_tree2<STAMPS, 16, BS, GLB, LU>(sd, cost0, lds, mb_d, mb_i); break;
                            }
                        }
                        break;
                }
            }
            break;
    }
}
template __global__ void k_coniss_t<false, 1, false>(SweepDev, double *);
template __global__ void k_coniss_t<false, 2, false>(SweepDev, double *);
template __global__ void k_coniss_t<false, 3, false>(SweepDev, double *);
template __global__ void k_coniss_t<false, 6, true, true>(SweepDev, double *);
template __global__ void k_coniss_t<false, 8, true, true>(SweepDev, double *);
template __global__ void k_coniss_t<false, 11, true, true>(SweepDev, double *);
template __global__ void k_coniss_t<false, 11, true>(SweepDev, double *);
template __global__ void k_coniss_t<false, 16, true>(SweepDev, double *);
template __global__ void k_coniss_t<false, 32, true>(SweepDev, double *);
#ifdef TP_STAMPS_BUILD   // stamped (diagnostic) kernels: make STAMPS=1
template __global__ void k_coniss_t<true, 1, false>(SweepDev, double *);
template __global__ void k_coniss_t<true, 2, false>(SweepDev, double *);
template __global__ void k_coniss_t<true, 3, false>(SweepDev, double *);
template __global__ void k_coniss_t<true, 6, true, true>(SweepDev, double *);
template __global__ void k_coniss_t<true, 16, true>(SweepDev, double *);
#endif
// k in 257..512 (R accepts any max_pcs, R/TADpole.R:344,452): trees of up to 8 slots
template __global__ void k_coniss_t<false, 1, false, false, 8>(SweepDev, double *);
template __global__ void k_coniss_t<false, 2, false, false, 8>(SweepDev, double *);
template __global__ void k_coniss_t<false, 3, false, false, 8>(SweepDev, double *);
template __global__ void k_coniss_t<false, 6, true, true, 8>(SweepDev, double *);
template __global__ void k_coniss_t<false, 8, true, true, 8>(SweepDev, double *);
template __global__ void k_coniss_t<false, 11, true, true, 8>(SweepDev, double *);
template __global__ void k_coniss_t<false, 11, true, false, 8>(SweepDev, double *);
template __global__ void k_coniss_t<false, 16, true, false, 8>(SweepDev, double *);
template __global__ void k_coniss_t<false, 32, true, false, 8>(SweepDev, double *);
// k in 513..1024: trees of up to 16 slots
template __global__ void k_coniss_t<false, 1, false, false, 16>(SweepDev, double *);
template __global__ void k_coniss_t<false, 2, false, false, 16>(SweepDev, double *);
template __global__ void k_coniss_t<false, 3, false, false, 16>(SweepDev, double *);
template __global__ void k_coniss_t<false, 6, true, true, 16>(SweepDev, double *);
template __global__ void k_coniss_t<false, 8, true, true, 16>(SweepDev, double *);
template __global__ void k_coniss_t<false, 11, true, true, 16>(SweepDev, double *);
template __global__ void k_coniss_t<false, 11, true, false, 16>(SweepDev, double *);
template __global__ void k_coniss_t<false, 16, true, false, 16>(SweepDev, double *);
template __global__ void k_coniss_t<false, 32, true, false, 16>(SweepDev, double *);

// ------------------------------------------------ batched CONISS (round 6)
// The same merges, costs, heights and records as coniss_tree2, produced in
// batches by one workgroup of CB_W waves per tree.  Greedy adjacency-
// constrained Ward merging is sequential, but a run of merges can be taken at
// once when it provably equals the next merges of the sequential order
// (tools/coniss_batch_model.py checks the rule against the oracle):
//   1. candidates: every position whose cost is <= T = g r (g the smallest
//      cost, r an adaptive ratio >= 1), taken from the blocks whose minimum is
//      <= T -- a COMPLETE prefix of the (cost, position) order -- sorted, the
//      first CB_W kept;
//   2. windows: each candidate's clusters LS, A, B, R (starts ls, a, b, r); the
//      candidates are kept up to the first whose window overlaps an earlier
//      one's, so every kept merge reads clusters no other kept merge changes;
//   3. new costs: wave j merges candidate j's A and B from the pre-batch rows
//      (the rows the sequential order would read: nothing earlier in the batch
//      touched them) and forms cl = Ward(LS, M), cr = Ward(M, R) in the
//      canonical arithmetic of coniss_tree2;
//   4. the leading run: candidate i is the next sequential merge unless a new
//      cost of a kept candidate before it, (cl_j, ls_j) or (cr_j, a_j), is
//      lexicographically smaller than (cost_i, a_i) -- the batch stops there;
//   5. the run is applied (costs, links, records, heights summed in merge
//      order, the merged clusters' sums rows), the touched blocks' minima are
//      refreshed, and the next batch starts.
// Typical runs: ~3 merges for trees of 1-3 PCs, 5-7 for wider trees, against
// one merge per ~2 800-cycle step of coniss_tree2.  The overflow case (more
// than CB_CAP positions <= T, or ties at g) takes one merge, the exact argmin.
// Storage modes M: 0 costs and int links / right ends in LDS (16 bytes a bin,
// to ~9.8k bins); 1 costs in LDS, 16-bit links only (10 bytes a bin, rn
// derived as in coniss_tree2's LU = 2, to 12.3k bins); 2 costs in the tree's
// slice of cost0 (global, L2/MALL), 16-bit links only in LDS (2 bytes a bin,
// the C5 arms).  In mode 2 the run's waves read the cost blocks they refresh
// in A2 (with the rows, before the run is known) and apply the run's changes
// in registers, so no global read follows A3's cost stores.
constexpr int CB_W = 8;      // waves a tree = most candidates a batch
constexpr int CB_CAP = 16;   // positions <= T ranked a batch (16 x 16 lane pairs)
constexpr int CB_FMAX = 16;  // flagged blocks a batch (two a wave)
constexpr int CB_SEG = 8;    // positions <= T a wave may contribute
#ifndef TP_CB_NMIN
#define TP_CB_NMIN 2   // (3: C3 6.30 ms, 24.3k 27.5; 2: 6.22, 26.8; 5: 6.53, 28.5)
#endif
constexpr int CB_NMIN = TP_CB_NMIN;   // rescan when the maintained candidate set holds fewer
#ifndef TP_CB_LO             // the gap adapts so a scan finds about LO..HI positions <= T
#define TP_CB_LO 12          // (6..10: C3 7.0 ms; 8..12: 6.8; 10..14: 6.67; 12..15: 6.66; with a
                             // rescan below 2 kept: 8..12 6.38, 10..14 6.33, 12..15 6.26)
#endif
#ifndef TP_CB_HI
#define TP_CB_HI 15
#endif
static_assert(CB_W * CB_SEG == 64, "one segment entry a lane");
struct CbShared {
    double sgc[CB_W * CB_SEG];   // the waves' segments: positions <= T and their costs
    int sgp[CB_W * CB_SEG];
    int segn[CB_W];
    double ccost[CB_CAP];   // the candidate set: every position with cost <= sT (sN of them; -1: rescan)
    int cpos[CB_CAP];
    double sT;
    int sN;
    double key[CB_W], cl[CB_W], cr[CB_W], hgt[CB_W];
    int spos[CB_W], ka[CB_W];
    int4 win[CB_W];   // (lo, hi, ls, r): positions covered by LS..R, the neighbours (-1: none)
    int4 w2[CB_W];    // (b, eb, er, -)
    int kc, cnt;
};
__device__ __forceinline__ int mbcnt64(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
// lexicographic (cost, position) order of the merge choice
__device__ __forceinline__ bool key_lt(double c1, int p1, double c2, int p2) {
    return c1 < c2 || (c1 == c2 && p1 < p2);
}

template <int NS, int BS, int M, bool STAMPS>
__device__ __forceinline__ void coniss_tree_b(const SweepDev &sd, double *cost0, double *lds, CbShared &sh) {
    constexpr bool GL = M == 2, L16 = M >= 1;
    const int n = sd.n;
    const int ti = blockIdx.x;
    const int i = sd.tree0 + ti + 1;
    constexpr int ld = NS * 64;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nbk = (n + 63) / 64;
    const double QNAN = __longlong_as_double(0x7FF8000000000000LL);
    // STAMPS (diagnostic builds): wave 0's cycles per phase, summed over the
    // batches, into sd.stamps[tree * 16 + 0..9]; 13: merges, 14: batches,
    // 15: retries of the candidate pass (too many positions <= T)
    long long st_acc[16] = {};
    long long st_t0 = STAMPS ? (long long)__builtin_amdgcn_s_memtime() : 0;
#define TP_BSTAMP(ph)                                                     \
    if (STAMPS && w == 0) {                                               \
        long long _t = (long long)__builtin_amdgcn_s_memtime();           \
        st_acc[ph] += _t - st_t0;                                         \
        st_t0 = _t;                                                       \
    }
    const size_t cst = coniss_cost_stride(n), lst = coniss_link_stride(n);
    double *cost = GL ? cost0 + (size_t)ti * cst : lds;
    LinkArr<L16> link;
    typename RnOf<L16 ? 2 : 0>::T rn;
    double *bmin;
    if constexpr (L16) {
        link.p = (unsigned short *)(GL ? lds : lds + cst);
        rn.link = link;
        bmin = (double *)((char *)link.p + ((lst * 2 + 7) & ~(size_t)7));
    } else {
        link.p = (int *)(cost + cst);
        rn.p = link.p + lst;
        bmin = (double *)(rn.p + lst);   // 8-byte aligned: 8 cst + 8 lst bytes before it
    }
    const int DC = nbk * 64, DL = n;
    constexpr bool P4 = NS == 4;
    double *S = sd.sums + sums_off(n, sd.tree0, i);
    const double *PP = P4 ? sd.pt4 : (NS >= 2 ? sd.pt2 : sd.Pt);
    const size_t ldpp = P4 ? (size_t)256 : (NS >= 2 ? (size_t)sd.pt2_ld : (size_t)sd.ldp);
    const bool last_in = lane + 64 * (NS - 1) < i;
    int *mrg_a = sd.mrg_a + (size_t)ti * (n - 1);
    int *mrg_b = sd.mrg_b + (size_t)ti * (n - 1);
    double *mcost = sd.cost + (size_t)ti * (n - 1);
    double *height = sd.height + (size_t)ti * (n - 1);
    const double *c0 = cost0 + (size_t)ti * cst;

    auto load_row = [&](double (&dst)[NS], int code) {
        code = __builtin_amdgcn_readfirstlane(code);
        const int p = code & (ROW_PT - 1);
        const double *pr = (code & ROW_PT) ? PP + (size_t)p * ldpp : S + (size_t)p * ld;
        if (NS >= 2) {
            const double2 v = *(const double2 *)(pr + 2 * lane);
            dst[0] = v.x;
            dst[1] = v.y;
        } else {
            dst[0] = pr[lane];
        }
        if (P4) {
            const double2 v = *(const double2 *)(pr + 128 + 2 * lane);
            dst[2] = v.x;
            dst[3] = v.y;
        } else {
#pragma unroll
            for (int t = 2; t < NS; ++t) dst[t] = pr[64 * t + lane];
        }
    };
    auto rowc = [](int start, bool single) { return start | (single ? ROW_PT : 0); };

    // ---- initial costs, links, block minima (all waves)
    for (int bk = w; bk < nbk; bk += CB_W) {
        const int p = bk * 64 + lane;
        const double cp = c0[p];
        if (!GL) cost[p] = cp;   // (mode 2: the costs stay where k_seed wrote them)
        if (p < n) {
            link.set(p, p);
            rn.set(p, p + 1 < n ? p + 1 : -1);
        }
        const double m = wave_min(cp);
        if (lane == 0) bmin[bk] = m;
    }
    if (w == 0) {
        cost[DC + lane] = QNAN;
        link.set(DL + lane, -1);
        rn.set(DL + lane, -1);
        if (GL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();

    if (threadIdx.x == 0) sh.sN = -1;   // (read after the barrier below the initial costs' one)
    __syncthreads();
    double h = 0.0;      // wave 0: the height so far
    double gap = -1.0;   // T = g + gap (every wave the same), adapted to about 6..10 positions <= T
    // waves j < kc: candidate j's window, merged sums, key and new costs
    int a = 0, ea = 0, b = 0, eb = 0, ls = -1, r = -1, er = -1;
    double sm[NS];
    double key = 0.0, cl = 0.0, cr = 0.0;
    double pba = 0.0, pbb = 0.0, pbl = 0.0;   // mode 2: the cost blocks of a, b and ls before the batch
    // rank the candidate set (C entries) by (cost, position) and write the
    // first CB_W to the slots: lane l compares candidate i = 4 p + (l >> 4)
    // with j = l & 15 (in-order LDS: reads the set after this wave's writes)
    auto rank_set = [&](int C) {
        const int j = lane & 15;
        const double kj = sh.ccost[j];
        const int pj = sh.cpos[j];
        double ki[4];
        int pi[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            ki[p] = sh.ccost[4 * p + (lane >> 4)];
            pi[p] = sh.cpos[4 * p + (lane >> 4)];
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int ii = 4 * p + (lane >> 4);
            const unsigned long long mm = __ballot((j < C) & key_lt(kj, pj, ki[p], pi[p]));
            const int rank = __popc((unsigned)(mm >> (16 * (lane >> 4))) & 0xFFFFu);
            if ((j == 0) & (ii < C) & (rank < CB_W)) {
                sh.key[rank] = ki[p];
                sh.spos[rank] = pi[p];
            }
        }
    };
    // the candidate set after a run of cnt merges: drop the changed positions
    // (a, b and ls of every merge), add the new costs <= T -- still every
    // position with cost <= T (costs change only there).  Lane pairs (entry
    // e = 8 h + (l >> 3), merge q = l & 7): does merge q change entry e's
    // position?  Run by the ranking wave during wave 0's A3 (the slots'
    // windows and new costs stay in LDS until the next A2).
    auto update_set = [&](int C, int cnt, bool single) {
        if (single) {
            if (lane == 0) sh.sN = -1;
            return;
        }
        const int sj = lane & 7;
        const int4 wj = sh.win[sj], x2 = sh.w2[sj];
        const int aj = sh.ka[sj];
        const double clj = sh.cl[sj], crj = sh.cr[sj];
        const double sT = sh.sT;
        const double ce = sh.ccost[lane & (CB_CAP - 1)];
        const int pe = sh.cpos[lane & (CB_CAP - 1)];
        const int pe0 = sh.cpos[lane >> 3], pe1 = sh.cpos[8 + (lane >> 3)];
        const bool onq = sj < cnt;
        const unsigned long long r0 = __ballot(onq && (pe0 == aj || pe0 == x2.x || pe0 == wj.z));
        const unsigned long long r1 = __ballot(onq && (pe1 == aj || pe1 == x2.x || pe1 == wj.z));
        const int le = lane & (CB_CAP - 1);
        const bool rm = ((le < 8 ? r0 : r1) >> (8 * (le & 7))) & 0xFFull;
        const bool keep = lane < C && !rm;
        const bool addl = lane < cnt && wj.z >= 0 && clj <= sT;
        const bool addr = lane < cnt && wj.w >= 0 && crj <= sT;
        const unsigned long long mk = __ballot(keep), ml = __ballot(addl), mr = __ballot(addr);
        const int nk = __popcll(mk), nl = __popcll(ml), nr = __popcll(mr);
        if (nk + nl + nr <= CB_CAP) {
            // (every lane read the old set above: in-order LDS, the writes come after)
            if (keep) {
                sh.ccost[mbcnt64(mk)] = ce;
                sh.cpos[mbcnt64(mk)] = pe;
            }
            if (addl) {
                sh.ccost[nk + mbcnt64(ml)] = clj;
                sh.cpos[nk + mbcnt64(ml)] = wj.z;
            }
            if (addr) {
                sh.ccost[nk + nl + mbcnt64(mr)] = crj;
                sh.cpos[nk + nl + mbcnt64(mr)] = aj;
            }
        }
        if (lane == 0) sh.sN = nk + nl + nr <= CB_CAP ? nk + nl + nr : -1;
    };
    int s = 0;
    while (s < n - 1) {
        // ---- A1 (every wave): g and T = g + gap from the block minima (every
        // wave computes the same); wave w scans the flagged blocks (minimum <=
        // T) of flagged index w and w + CB_W and writes its positions with cost
        // <= T to its segment; after B0 every wave reads the segment counts and
        // retries with a smaller gap if they overflow (the same decision in
        // every wave; try 6 takes only the ties at g, try 7 the exact argmin)
        double gq = 0.0;
        bool single = false;
        int C = __builtin_amdgcn_readfirstlane(sh.sN);
        double Tu = 0.0;   // the T of a successful scan
        const bool rescan = C < CB_NMIN;
        if (rescan) {
            double bm[BS];
#pragma unroll
            for (int q = 0; q < BS; ++q) bm[q] = 64 * q + lane < nbk ? bmin[64 * q + lane] : QNAN;
            double x = bm[0];
#pragma unroll
            for (int q = 1; q < BS; ++q) x = vmin(x, bm[q]);
            gq = wave_min(x);
            if (!(gap > 0.0)) gap = gq > 0.0 && gq < 1e300 ? 0.5 * gq : 1e-300;
            for (int tries = 0;; ++tries) {
                double T = gq + gap;
                if (!(T >= gq) || tries >= 6) T = gq;
                int F = 0, mb0 = -1, mb1 = -1;   // this wave's flagged blocks (at most 2)
#pragma unroll
                for (int q = 0; q < BS; ++q) {
                    const bool f = bm[q] <= T;
                    const unsigned long long m = __ballot(f);
                    const int idx = F + mbcnt64(m);
                    const unsigned long long mine = __ballot(f && (idx & (CB_W - 1)) == w);
                    const int i0 = mine ? 64 * q + (int)__builtin_ctzll(mine) : -1;
                    const unsigned long long rest = mine & (mine - 1);
                    const int i1 = rest ? 64 * q + (int)__builtin_ctzll(rest) : -1;
                    if (i0 >= 0) {
                        if (mb0 < 0) mb0 = i0;
                        else if (mb1 < 0) mb1 = i0;
                    }
                    if (i1 >= 0 && mb1 < 0) mb1 = i1;
                    F += __popcll(m);
                }
                int cw = CB_CAP + 1;
                if (F <= CB_FMAX) {
                    const double v0 = cost[(mb0 >= 0 ? mb0 : 0) * 64 + lane];
                    const double v1 = cost[(mb1 >= 0 ? mb1 : 0) * 64 + lane];
                    const bool s0 = (mb0 >= 0) & (v0 <= T), s1 = (mb1 >= 0) & (v1 <= T);
                    const unsigned long long m0 = __ballot(s0), m1 = __ballot(s1);
                    const int i0 = mbcnt64(m0), i1 = __popcll(m0) + mbcnt64(m1);
                    if (s0 && i0 < CB_SEG) {
                        sh.sgc[w * CB_SEG + i0] = v0;
                        sh.sgp[w * CB_SEG + i0] = mb0 * 64 + lane;
                    }
                    if (s1 && i1 < CB_SEG) {
                        sh.sgc[w * CB_SEG + i1] = v1;
                        sh.sgp[w * CB_SEG + i1] = mb1 * 64 + lane;
                    }
                    cw = __popcll(m0) + __popcll(m1);
                }
                if (lane == 0) sh.segn[w] = cw;
                lds_barrier();   // B0
                // the eight counts (two broadcast reads): every wave takes the same decision
                const int4 n0 = *(const int4 *)&sh.segn[0], n1 = *(const int4 *)&sh.segn[4];
                const int c0_ = __builtin_amdgcn_readfirstlane(n0.x), c1_ = __builtin_amdgcn_readfirstlane(n0.y),
                          c2_ = __builtin_amdgcn_readfirstlane(n0.z), c3_ = __builtin_amdgcn_readfirstlane(n0.w),
                          c4_ = __builtin_amdgcn_readfirstlane(n1.x), c5_ = __builtin_amdgcn_readfirstlane(n1.y),
                          c6_ = __builtin_amdgcn_readfirstlane(n1.z), c7_ = __builtin_amdgcn_readfirstlane(n1.w);
                const int tot = c0_ + c1_ + c2_ + c3_ + c4_ + c5_ + c6_ + c7_;
                const int mx = max(max(max(c0_, c1_), max(c2_, c3_)), max(max(c4_, c5_), max(c6_, c7_)));
                if (tot <= CB_CAP && mx <= CB_SEG && tot >= 1) {
                    C = tot;
                    Tu = T;
                    if (tries <= 5) gap *= C < TP_CB_LO ? 1.3 : (C > TP_CB_HI ? 0.8 : 1.0);   // next scan: ~LO..HI positions <= T
                    break;
                }
                if (tries >= 6) {
                    single = true;
                    break;
                }
                lds_barrier();   // every wave has read the counts before a retry rewrites them
                gap *= 0.5;
                if (STAMPS) st_acc[15] += 1;
            }
        }
        TP_BSTAMP(10);
        // ---- A1b (wave 0, after a rescan): gather the segments, rank, the
        // first CB_W into the slots.  Without a rescan the slots were filled
        // during the previous batch's A4 by wave CB_W - 1 (rank_set below), so
        // the batch goes straight to A2
        if (rescan && w == 0) {
            int Kc;
            if (!single) {
                // the segments compacted into the set: lane l holds entry l & 7 of wave l >> 3
                const bool valid = (lane & (CB_SEG - 1)) < sh.segn[lane >> 3];
                const double cv = sh.sgc[lane];
                const int cp = sh.sgp[lane];
                const unsigned long long mv = __ballot(valid);
                const int idx = mbcnt64(mv);
                if (valid) {
                    sh.ccost[idx] = cv;
                    sh.cpos[idx] = cp;
                }
                if (lane == 0) sh.sT = Tu;
                rank_set(C);
                Kc = C < CB_W ? C : CB_W;
            } else {
                // too many positions tie at g: the exact argmin, one merge
                double bm[BS];
#pragma unroll
                for (int q = 0; q < BS; ++q) bm[q] = 64 * q + lane < nbk ? bmin[64 * q + lane] : QNAN;
                int bk = 0;
#pragma unroll
                for (int q = BS - 1; q >= 0; --q) {
                    const unsigned long long m = __ballot(bm[q] == gq);
                    bk = m ? 64 * q + (int)__builtin_ctzll(m) : bk;
                }
                const unsigned long long mv = __ballot(cost[bk * 64 + lane] == gq);
                TP_DASSERT(mv != 0ull);
                if (lane == 0) {
                    sh.key[0] = gq;
                    sh.spos[0] = bk * 64 + (int)__builtin_ctzll(mv);
                }
                Kc = 1;
            }
            if (lane == 0) sh.kc = Kc;
        }
        TP_BSTAMP(0);
        if (rescan) lds_barrier();   // B1
        TP_BSTAMP(1);
        // ---- A2 (wave j < kc): candidate j's window, rows, merged sums, new costs
        const int kc = __builtin_amdgcn_readfirstlane(sh.kc);
        if (w < kc) {
            a = __builtin_amdgcn_readfirstlane(sh.spos[w]);
            key = sh.key[w];
            TP_DASSERT(a >= 0 && a < n - 1);
            int lsv = link.get(a > 0 ? a - 1 : DL);
            ea = link.get(a);
            eb = rn.get(a);
            pin3(lsv, ea, eb);
            ea = __builtin_amdgcn_readfirstlane(ea);
            eb = __builtin_amdgcn_readfirstlane(eb);
            b = ea + 1;
            ls = a > 0 ? __builtin_amdgcn_readfirstlane(lsv) : -1;
            r = eb + 1 < n ? eb + 1 : -1;
            er = r >= 0 ? __builtin_amdgcn_readfirstlane(rn.get(b)) : -1;
            const int ac = rowc(a, ea == a);
            double sa[NS], sb[NS], sl[NS], sr[NS];
            load_row(sa, ac);
            load_row(sb, rowc(b, eb == b));
            load_row(sl, ls >= 0 ? rowc(ls, ls == a - 1) : ac);
            load_row(sr, r >= 0 ? rowc(r, er == r) : ac);
            if (GL) {
                // the blocks A4 refreshes, issued after the rows so the rows'
                // waits leave them in flight (used only after A3)
                pba = cost[(a >> 6) * 64 + lane];
                pbb = cost[(b >> 6) * 64 + lane];
                pbl = cost[((ls >= 0 ? ls : a) >> 6) * 64 + lane];
            }
            if (lane == 0) {
                sh.win[w] = make_int4(ls >= 0 ? ls : a, r >= 0 ? er : eb, ls, r);
                sh.w2[w] = make_int4(b, eb, er, 0);
                sh.ka[w] = a;
            }
#pragma unroll
            for (int t = 0; t < NS; ++t) sm[t] = sa[t] + sb[t];
            const double fm = (double)(eb - a + 1), fl = (double)(a - ls), fr = (double)(er - r + 1);
            double ul = ward_part<NS>(sl, fl, sm, fm, last_in);
            double ur = ward_part<NS>(sm, fm, sr, fr, last_in);
            TP_BSTAMP(7);   // (stamps build: window + rows landed)
            wave_sum2(ul, ur);
            const double ql = pin_d(ul / (fl * fm * (fl + fm)));
            const double qr = pin_d(ur / (fm * fr * (fm + fr)));
            cl = ls >= 0 ? nan2inf(ql) : QNAN;
            cr = r >= 0 ? nan2inf(qr) : QNAN;
            if (lane == 0) {
                sh.cl[w] = cl;
                sh.cr[w] = cr;
            }
        }
        TP_BSTAMP(2);
        lds_barrier();   // B2
        TP_BSTAMP(3);
        if (w == CB_W - 1) {
            // the ranking wave: the run's length as wave 0 finds it below (the
            // same slots, the same ballots), then the candidate set after the
            // run, beside wave 0's A3 (which reads neither the set nor sN)
            const int si = lane >> 3, sj = lane & 7;
            const int4 wi = sh.win[si], wj = sh.win[sj];
            const double ki = sh.key[si];
            const int ai = sh.ka[si], aj = sh.ka[sj];
            const double clj = sh.cl[sj], crj = sh.cr[sj];
            const bool pair = sj < si && si < kc;
            const unsigned long long cm = __ballot(pair && !(wi.y < wj.x || wj.y < wi.x));
            const int kacc = cm ? (int)(__builtin_ctzll(cm) >> 3) : kc;
            const bool und = (wj.z >= 0 && key_lt(clj, wj.z, ki, ai)) || (wj.w >= 0 && key_lt(crj, aj, ki, ai));
            const unsigned long long pm = __ballot(pair && si < kacc && und);
            update_set(C, pm ? (int)(__builtin_ctzll(pm) >> 3) : kacc, single);
        }
        // ---- A3 (wave 0): the conflict-free prefix and the leading run, lane
        // l comparing slot i = l >> 3 with an earlier slot j = l & 7; the
        // run's heights, costs and links
        if (w == 0) {
            const int si = lane >> 3, sj = lane & 7;
            const int4 wi = sh.win[si], wj = sh.win[sj];
            const double ki = sh.key[si];
            const int ai = sh.ka[si], aj = sh.ka[sj];
            const double clj = sh.cl[sj], crj = sh.cr[sj];
            const int4 x2 = sh.w2[sj];
            const bool pair = sj < si && si < kc;
            const unsigned long long cm = __ballot(pair && !(wi.y < wj.x || wj.y < wi.x));
            const int kacc = cm ? (int)(__builtin_ctzll(cm) >> 3) : kc;
            const bool und = (wj.z >= 0 && key_lt(clj, wj.z, ki, ai)) || (wj.w >= 0 && key_lt(crj, aj, ki, ai));
            const unsigned long long pm = __ballot(pair && si < kacc && und);
            const int cnt = pm ? (int)(__builtin_ctzll(pm) >> 3) : kacc;
            // heights in merge order (lane j < 8 holds slot j's key)
            const double kl = sh.key[sj];
            double hh = h, myh = 0.0;
            for (int q = 0; q < cnt; ++q) {
                hh = hh + readlane_d(kl, q);
                myh = lane == q ? hh : myh;
            }
            h = hh;
            // the run's costs and links, lane q < cnt for merge s + q (the
            // windows are disjoint: no two lanes write one word)
            if (lane < cnt) {
                sh.hgt[lane] = myh;
                cost[x2.x] = QNAN;
                cost[aj] = crj;   // QNAN without a right neighbour
                link.set(aj, x2.y);
                link.set(x2.y, aj);
                rn.set(aj, x2.z);
                if (wj.z >= 0) {
                    cost[wj.z] = clj;
                    rn.set(wj.z, x2.y);
                }
            }
            if (lane == 0) sh.cnt = cnt;
            if (STAMPS) st_acc[13] += cnt;
        }
        TP_BSTAMP(4);
        lds_barrier();   // B3
        TP_BSTAMP(5);
        // ---- A4 (wave j < cnt): merge s + j's sums row and record, the touched
        // blocks' minima (every cost of the run is in place); the stores
        // complete before B4 (the next batch's rows may be these)
        const int cnt = __builtin_amdgcn_readfirstlane(sh.cnt);
        if (w < cnt) {
            if (NS >= 2)
                *(double2 *)(S + (size_t)a * ld + 2 * lane) = make_double2(sm[0], sm[1]);
            else
                S[(size_t)a * ld + lane] = sm[0];
            if (P4) {
                *(double2 *)(S + (size_t)a * ld + 128 + 2 * lane) = make_double2(sm[2], sm[3]);
            } else {
#pragma unroll
                for (int t = 2; t < NS; ++t) S[(size_t)a * ld + 64 * t + lane] = sm[t];
            }
            if (lane == 0) {
                mrg_a[s + w] = a;
                mrg_b[s + w] = b;
                mcost[s + w] = key;
                height[s + w] = sh.hgt[w];
            }
            TP_BSTAMP(6);
            const int ba = a >> 6, bb = b >> 6, bl = ls >= 0 ? (ls >> 6) : ba;
            double ma, mb, ml, mx = QNAN;
            if constexpr (GL) {
                // the blocks read in A2 with the run's changes (A3's stores):
                // merge q sets b_q's cost to NaN, a_q's to cr_q, ls_q's to cl_q
                int qb = -1, qa = -1, ql = -1;
                double qcl = 0.0, qcr = 0.0;
                if (lane < cnt) {
                    qb = sh.w2[lane].x;
                    qa = sh.ka[lane];
                    ql = sh.win[lane].z;
                    qcl = sh.cl[lane];
                    qcr = sh.cr[lane];
                }
                ma = pba;
                mb = pbb;
                ml = pbl;
                const int Pa = ba * 64 + lane, Pb = bb * 64 + lane, Pl = bl * 64 + lane;
                for (int q = 0; q < cnt; ++q) {
                    const int xb = __builtin_amdgcn_readlane(qb, q), xa = __builtin_amdgcn_readlane(qa, q),
                              xl = __builtin_amdgcn_readlane(ql, q);
                    const int kb = xb >> 6, ka_ = xa >> 6, kl = xl >> 6;   // xl = -1: no block
                    const bool hit = kb == ba || kb == bb || kb == bl || ka_ == ba || ka_ == bb || ka_ == bl ||
                                     kl == ba || kl == bb || kl == bl;
                    if (!hit) continue;
                    const double vl = readlane_d(qcl, q), vr = readlane_d(qcr, q);
                    ma = Pa == xb ? QNAN : (Pa == xa ? vr : (Pa == xl ? vl : ma));
                    mb = Pb == xb ? QNAN : (Pb == xa ? vr : (Pb == xl ? vl : mb));
                    ml = Pl == xb ? QNAN : (Pl == xa ? vr : (Pl == xl ? vl : ml));
                }
            } else {
                ma = cost[ba * 64 + lane];
                mb = cost[bb * 64 + lane];
                ml = cost[bl * 64 + lane];
            }
            wave_min4(ma, mb, ml, mx);
            if (lane == 0) {
                bmin[ba] = ma;
                bmin[bb] = mb;
                bmin[bl] = ml;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (w == CB_W - 1) {
            // the next batch's slots from the set after the run (updated by
            // this wave during A3); a set that ran low is rescanned and ranked
            // in the next A1 / A1b instead
            const int Cn = __builtin_amdgcn_readfirstlane(sh.sN);   // (in-order LDS: this wave's write)
            if (Cn >= CB_NMIN) {
                rank_set(Cn);
                const int K8 = Cn < CB_W ? Cn : CB_W;
                if (lane == 0) sh.kc = K8;
            }
        }
        s += cnt;
        TP_BSTAMP(8);
        lds_barrier();   // B4
        TP_BSTAMP(9);
        if (STAMPS) st_acc[14] += 1;
    }
    __syncthreads();
    // ---- broken stick (rioja bstick.chclust, vegan bstick.default) on heights
    if (threadIdx.x == 0) {
        const int nobj = n - 1;
        int ncl = -1;
        if (nobj >= 2) {
            const double tot = height[nobj - 1];
            double *cs = cost;
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
    if (STAMPS && threadIdx.x == 0)
        for (int q = 0; q < 16; ++q) sd.stamps[(size_t)ti * 16 + q] = st_acc[q];
#undef TP_BSTAMP
}

// trees of up to 4 column slots (k <= 256); M: the storage mode above
template <int BS, int M, bool STAMPS = false>
__global__ void __launch_bounds__(64 * CB_W) k_coniss_b(SweepDev sd, double *cost0) {
    extern __shared__ double lds[];
    __shared__ CbShared sh;
    const int i = sd.tree0 + blockIdx.x + 1;
    switch ((i + 63) / 64) {
        case 1: coniss_tree_b<1, BS, M, STAMPS>(sd, cost0, lds, sh); break;
        case 2: coniss_tree_b<2, BS, M, STAMPS>(sd, cost0, lds, sh); break;
        case 3: coniss_tree_b<3, BS, M, STAMPS>(sd, cost0, lds, sh); break;
        default: coniss_tree_b<4, BS, M, STAMPS>(sd, cost0, lds, sh); break;
    }
}
template __global__ void k_coniss_b<1, 0>(SweepDev, double *);
template __global__ void k_coniss_b<2, 0>(SweepDev, double *);
template __global__ void k_coniss_b<3, 0>(SweepDev, double *);
template __global__ void k_coniss_b<3, 1>(SweepDev, double *);
template __global__ void k_coniss_b<6, 2>(SweepDev, double *);
template __global__ void k_coniss_b<11, 2>(SweepDev, double *);
#ifdef TP_STAMPS_BUILD
template __global__ void k_coniss_b<1, 0, true>(SweepDev, double *);
template __global__ void k_coniss_b<2, 0, true>(SweepDev, double *);
template __global__ void k_coniss_b<3, 0, true>(SweepDev, double *);
template __global__ void k_coniss_b<3, 1, true>(SweepDev, double *);
template __global__ void k_coniss_b<6, 2, true>(SweepDev, double *);
#endif

// ------------------------------------------------------------ CH over cuts
// canonical segment statistics of rows s..e, by one wave (see tpo_seg_ss)
// RB rows per batch (RB x KS loads in flight); the order of the sums is
// the same for any RB
template <int KS, int RB = 4>
__device__ double seg_ss_wave(const double *Pt, int ldp, int k, int s, int e, double *sumout, int lane) {
    const double fn = (double)(e - s + 1);
    bool ok[KS];
    int jj[KS];
#pragma unroll
    for (int t = 0; t < KS; ++t) {
        jj[t] = lane + 64 * t;
        ok[t] = jj[t] < k;
        if (!ok[t]) jj[t] = 0;   // safe address, value unused
    }
    // pass 1: column sums, sequential over rows per column; RB rows per step
    // so RB x KS independent loads are in flight
    double sj[KS];
#pragma unroll
    for (int t = 0; t < KS; ++t) sj[t] = 0.0;
    int a = s;
    for (; a + RB - 1 <= e; a += RB) {
        double x[RB][KS];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int t = 0; t < KS; ++t) x[r][t] = Pt[(size_t)(a + r) * ldp + jj[t]];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int t = 0; t < KS; ++t) sj[t] = sj[t] + x[r][t];
    }
    for (; a <= e; ++a)
#pragma unroll
        for (int t = 0; t < KS; ++t) sj[t] = sj[t] + Pt[(size_t)a * ldp + jj[t]];
    double mj[KS], ss[KS];
#pragma unroll
    for (int t = 0; t < KS; ++t) ss[t] = 0.0;
#pragma unroll
    for (int t = 0; t < KS; ++t) {
        mj[t] = sj[t] / fn;
        if (sumout && ok[t]) sumout[jj[t]] = sj[t];
    }
    a = s;
    for (; a + RB - 1 <= e; a += RB) {
        double x[RB][KS];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int t = 0; t < KS; ++t) x[r][t] = Pt[(size_t)(a + r) * ldp + jj[t]];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int t = 0; t < KS; ++t) {
                double d = x[r][t] - mj[t];
                ss[t] = fma(d, d, ss[t]);
            }
    }
    for (; a <= e; ++a)
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            double d = Pt[(size_t)a * ldp + jj[t]] - mj[t];
            ss[t] = fma(d, d, ss[t]);
        }
    double part = 0.0;
#pragma unroll
    for (int t = 0; t < KS; ++t)
        if (ok[t]) part = part + ss[t];
    return wave_sum(part);
}

// tr(S) over all rows: thread j owns column j (the canonical sequential sums
// of seg_ss_wave, combined in slot order through LDS exactly as its `part`:
// same bits).  Rows stream in batches of 32 with the next batch's loads
// issued before the current batch is summed (the pass is latency-bound).
template <int KS>
__global__ void __launch_bounds__(64 * KS) k_trS(const double *Pt, int n, int ldp, int k, double *out) {
    __shared__ double ssl[KS][64];
    constexpr int RB = 32;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane + 64 * w;
    const int jj = j < k ? j : 0;
    const double fn = (double)n;
    double x[2][RB];
    auto fetch = [&](double (&d)[RB], int a) {
#pragma unroll
        for (int r = 0; r < RB; ++r) d[r] = a + r < n ? Pt[(size_t)(a + r) * ldp + jj] : 0.0;
    };
    double sj = 0.0;
    fetch(x[0], 0);
    for (int a = 0; a < n; a += 2 * RB) {
        fetch(x[1], a + RB);
#pragma unroll
        for (int r = 0; r < RB; ++r)
            if (a + r < n) sj = sj + x[0][r];
        fetch(x[0], a + 2 * RB);
#pragma unroll
        for (int r = 0; r < RB; ++r)
            if (a + RB + r < n) sj = sj + x[1][r];
    }
    const double mj = sj / fn;
    double ss = 0.0;
    fetch(x[0], 0);
    for (int a = 0; a < n; a += 2 * RB) {
        fetch(x[1], a + RB);
#pragma unroll
        for (int r = 0; r < RB; ++r)
            if (a + r < n) {
                const double d = x[0][r] - mj;
                ss = fma(d, d, ss);
            }
        fetch(x[0], a + 2 * RB);
#pragma unroll
        for (int r = 0; r < RB; ++r)
            if (a + RB + r < n) {
                const double d = x[1][r] - mj;
                ss = fma(d, d, ss);
            }
    }
    ssl[w][lane] = ss;
    __syncthreads();
    if (w == 0) {
        double part = 0.0;
#pragma unroll
        for (int t = 0; t < KS; ++t)
            if (lane + 64 * t < k) part = part + ssl[t][lane];
        const double v = wave_sum(part);
        if (lane == 0) *out = v;
    }
}

// 16 waves per tree: the finest cut's segment statistics spread over them;
// cut boundaries, alive flags and segment SS live in LDS (the coarser levels'
// neighbour scans were chains of dependent global loads).
constexpr int CH_THREADS = 1024, CH_SEGMAX = 1024;

// ---- segment statistics shared across trees.  Consecutive PC prefixes give
// nearly the same finest cuts (at C2 3.7 % of the 15k segments of the 200
// trees are distinct), and a segment's statistics -- column sums over all k
// PCs and the within-segment SS -- do not depend on the tree.  k_ch_cut writes
// each tree's finest cut and inserts its segments [s, e) into an
// open-addressing set; k_ch_segstat computes every distinct one once
// (seg_ss_wave: the same arithmetic, so the same bits); k_ch reads them back.
constexpr unsigned long long kSegEmpty = ~0ULL;
__device__ __forceinline__ unsigned seg_slot(unsigned long long key, unsigned mask) {
    key ^= key >> 31;
    key *= 0x9E3779B97F4A7C15ULL;
    key ^= key >> 29;
    return (unsigned)key & mask;
}
__device__ __forceinline__ unsigned long long seg_key(int s, int e) {
    return ((unsigned long long)(unsigned)s << 32) | (unsigned)e;
}
// finest cut of tree ti: the boundaries removed by the last nc-1 merges,
// ascending, segs[0] = 0, segs[nc] = n (all threads; synchronised on return)
__device__ void finest_cut(const SweepDev &sd, int ti, int nc, int *mbl, int *segs) {
    const int n = sd.n;
    const int *mb = sd.mrg_b + (size_t)ti * (n - 1);
    for (int t = threadIdx.x; t < nc - 1; t += blockDim.x) mbl[t] = mb[n - 2 - t];
    __syncthreads();
    for (int t = threadIdx.x; t < nc - 1; t += blockDim.x) {
        const int bt = mbl[t];
        int rank = 0;
        for (int u = 0; u < nc - 1; ++u) rank += mbl[u] < bt;
        segs[rank + 1] = bt;
    }
    if (threadIdx.x == 0) {
        segs[0] = 0;
        segs[nc] = n;
    }
    __syncthreads();
}
// trees whose cuts k_ch scores (the others it reports or marks NaN itself)
__device__ __forceinline__ bool ch_tree_ok(const SweepDev &sd, int nc) {
    return nc >= 2 && nc <= sd.w_cap && nc <= sd.seg_cap && nc <= CH_SEGMAX;
}

__global__ void __launch_bounds__(256) k_ch_cut(SweepDev sd) {
    __shared__ int segs[CH_SEGMAX + 1], mbl[CH_SEGMAX];
    const int ti = blockIdx.x;
    const int nc = sd.n_cluster[ti];
    if (!ch_tree_ok(sd, nc)) return;
    finest_cut(sd, ti, nc, mbl, segs);
    int *tseg = sd.iseg + (size_t)ti * (2 * sd.seg_cap + 2);
    for (int g = threadIdx.x; g <= nc; g += blockDim.x) tseg[g] = segs[g];
    const unsigned mask = (unsigned)sd.hcap - 1;
    for (int g = threadIdx.x; g < nc; g += blockDim.x) {
        const unsigned long long key = seg_key(segs[g], segs[g + 1]);
        unsigned slot = seg_slot(key, mask);
        for (;;) {   // hcap >= 2 x the insertions: an empty slot is always reached
            const unsigned long long prev = atomicCAS(sd.hkeys + slot, kSegEmpty, key);
            if (prev == kSegEmpty) {
                const int idx = atomicAdd(sd.ucount, 1);
                sd.hidx[slot] = idx < sd.ucap ? idx : -1;
                if (idx < sd.ucap) sd.ukey[idx] = key;
                break;
            }
            if (prev == key) break;
            slot = (slot + 1) & mask;
        }
    }
}

// one wave per distinct segment (grid-stride): k column sums + SS
template <int KS>
__global__ void __launch_bounds__(256) k_ch_segstat(SweepDev sd) {
    const int lane = threadIdx.x & 63;
    const int wv = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nwv = (int)((gridDim.x * blockDim.x) >> 6);
    const int cnt = min(*sd.ucount, sd.ucap);
    const int k = sd.k;
    for (int idx = wv; idx < cnt; idx += nwv) {
        const unsigned long long key = sd.ukey[idx];
        const int s = (int)(key >> 32), e = (int)(unsigned)(key & 0xFFFFFFFFULL);
        double *dst = sd.ustore + (size_t)idx * (k + 1);
        const double ss = seg_ss_wave<KS>(sd.Pt, sd.ldp, k, s, e - 1, dst, lane);
        if (lane == 0) dst[k] = ss;
    }
}

static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }
size_t sweep_dedup_bytes(int n, int k, int ntrees, int seg_cap, int *hcap, int *ucap) {
    const long ins = (long)ntrees * (long)std::max(1, std::min(seg_cap, n));
    long h = 1024;
    while (h < 2 * ins) h <<= 1;
    long u = std::min<long>(ins, std::max<long>(4096, 2L * n));
    if (t_knob.ch_dedup_ucap > 0) u = std::min<long>(u, t_knob.ch_dedup_ucap);
    *hcap = (int)h;
    *ucap = (int)u;
    return al256((size_t)h * 8) + al256((size_t)h * 4) + al256((size_t)u * 8) + al256((size_t)u * (k + 1) * 8) + 256;
}
void sweep_dedup_bind(SweepDev &sd, void *base, int hcap, int ucap) {
    char *q = (char *)base;
    sd.hkeys = (unsigned long long *)q;
    q += al256((size_t)hcap * 8);
    sd.hidx = (int *)q;
    q += al256((size_t)hcap * 4);
    sd.ukey = (unsigned long long *)q;
    q += al256((size_t)ucap * 8);
    sd.ustore = (double *)q;
    q += al256((size_t)ucap * (sd.k + 1) * 8);
    sd.ucount = (int *)q;
    sd.hcap = hcap;
    sd.ucap = ucap;
}
template <int KS>
__global__ void __launch_bounds__(CH_THREADS) k_ch(SweepDev sd) {
    __shared__ int segs[CH_SEGMAX + 1], mbl[CH_SEGMAX];
    __shared__ int src[CH_SEGMAX];   // segment's statistics: ustore index, or -1 = this tree's scratch
    __shared__ int gbl[CH_SEGMAX], lnk_l[CH_SEGMAX], lnk_r[CH_SEGMAX];   // level -> segment, alive list
    __shared__ double ssg[CH_SEGMAX];
    const int n = sd.n, k = sd.k, ldp = sd.ldp;
    const int ti = blockIdx.x;
    const int nc = sd.n_cluster[ti];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (nc < 1) return;
    if (nc > sd.w_cap || nc > sd.seg_cap || nc > CH_SEGMAX) {
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
    // per-tree scratch (global; this workgroup only): column sums of the
    // segments this tree merged (or could not find in the shared store)
    double *seg = sd.seg + (size_t)ti * sd.seg_cap * (k + 1);   // seg_cap x k sums
    if (sd.hkeys) {
        // the finest cut from k_ch_cut, the statistics from the shared store
        const int *tseg = sd.iseg + (size_t)ti * (2 * sd.seg_cap + 2);
        for (int g = threadIdx.x; g <= nc; g += blockDim.x) segs[g] = tseg[g];
        __syncthreads();
        const unsigned mask = (unsigned)sd.hcap - 1;
        for (int g = threadIdx.x; g < nc; g += blockDim.x) {
            const unsigned long long key = seg_key(segs[g], segs[g + 1]);
            unsigned slot = seg_slot(key, mask);
            while (sd.hkeys[slot] != key) slot = (slot + 1) & mask;   // k_ch_cut inserted it
            const int idx = sd.hidx[slot];
            src[g] = idx;
            if (idx >= 0) ssg[g] = sd.ustore[(size_t)idx * (k + 1) + k];
        }
        __syncthreads();
        for (int g = w; g < nc; g += nw)   // the store was full: the tree's own
            if (src[g] < 0) {
                const double ss = seg_ss_wave<KS>(sd.Pt, ldp, k, segs[g], segs[g + 1] - 1, seg + (size_t)g * k, lane);
                if (lane == 0) ssg[g] = ss;
            }
    } else {
        finest_cut(sd, ti, nc, mbl, segs);
        for (int g = w; g < nc; g += nw) {
            double ss = seg_ss_wave<KS>(sd.Pt, ldp, k, segs[g], segs[g + 1] - 1, seg + (size_t)g * k, lane);
            if (lane == 0) { ssg[g] = ss; src[g] = -1; }
        }
    }
    // level structure, in parallel: the segment whose start each level's
    // boundary is (binary search of the sorted cut) and the alive list links
    for (int t = threadIdx.x; t < nc - 1; t += blockDim.x) {
        const int bt = mb[n - 2 - t];   // level lev = t + 1 removes boundary bt
        int lo = 1, hi = nc - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (segs[mid] < bt) lo = mid + 1;
            else hi = mid;
        }
        gbl[t] = lo;
    }
    for (int g = threadIdx.x; g < nc; g += blockDim.x) {
        lnk_l[g] = g - 1;
        lnk_r[g] = g + 1;
    }
    __syncthreads();
    if (w != 0) return;
    // wave 0 only from here.  Level lev merges segment gb (starting at the
    // removed boundary) into its alive left neighbour ga.  The merged sums stay
    // in registers for the next level, whose other operands are loaded while
    // this level's increment is computed.  LDS state is written by every lane
    // with the same value.
    const double trS = *sd.trS;
    double trW = 0.0;
    for (int g = 0; g < nc; ++g) trW = trW + ssg[g];
    if (lane == 0)
        score_row[(size_t)(nc - 1) * ldsc] = ((double)(n - nc) * (trS - trW)) / ((double)(nc - 1) * trW);
    auto sums_of = [&](int g) -> const double * {
        const int ix = src[g];
        return ix >= 0 ? sd.ustore + (size_t)ix * (k + 1) : seg + (size_t)g * k;
    };
    auto load4 = [&](double (&d)[KS], const double *p) {
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            const int j = lane + 64 * t;
            d[t] = j < k ? p[j] : 0.0;
        }
    };
    int lev = nc - 1;
    double A[KS], B[KS], M[KS], A2[KS], B2[KS];
    int ga = 0, gb = 0, nx = 0;
    if (lev >= m && lev >= 1) {
        gb = gbl[lev - 1];
        ga = lnk_l[gb];
        nx = lnk_r[gb];
        load4(A, sums_of(ga));
        load4(B, sums_of(gb));
    }
    for (; lev >= m && lev >= 1; --lev) {
        const int b = segs[gb];
        const int na = b - segs[ga];
        const int nbb = (nx < nc ? segs[nx] : n) - b;
        // unlink gb; ga's sums move to this tree's scratch (stored below)
        lnk_r[ga] = nx;
        if (nx < nc) lnk_l[nx] = ga;
        src[ga] = -1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the next level's operands other than the merged segment: loads in flight now
        const bool more = lev - 1 >= m && lev - 1 >= 1;
        int ga2 = ga, gb2 = gb, nx2 = nx;
        if (more) {
            gb2 = gbl[lev - 2];
            ga2 = lnk_l[gb2];
            nx2 = lnk_r[gb2];
            if (ga2 != ga) load4(A2, sums_of(ga2));
            if (gb2 != ga) load4(B2, sums_of(gb2));
        }
        const double fa = (double)na, fb = (double)nbb;
        double acc = 0.0;
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            const int j = lane + 64 * t;
            if (j < k) {
                const double t1 = A[t] * fb;
                const double t2 = B[t] * fa;
                const double e = t1 - t2;
                acc = fma(e, e, acc);
            }
        }
        const double tot = wave_sum(acc);
        trW = trW + tot / (fa * fb * (fa + fb));
        double *DA = seg + (size_t)ga * k;   // the merged segment's sums
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            const int j = lane + 64 * t;
            M[t] = A[t] + B[t];
            if (j < k) DA[j] = M[t];
        }
        if (lane == 0)
            score_row[(size_t)(lev - 1) * ldsc] =
                lev == 1 ? r_nan() : ((double)(n - lev) * (trS - trW)) / ((double)(lev - 1) * trW);
        if (more) {
#pragma unroll
            for (int t = 0; t < KS; ++t) {
                A[t] = ga2 == ga ? M[t] : A2[t];
                B[t] = gb2 == ga ? M[t] : B2[t];
            }
            ga = ga2;
            gb = gb2;
            nx = nx2;
        }
    }
}

// ---- CH for trees whose finest cut exceeds k_ch's LDS capacity (more than
// CH_SEGMAX = 1024 significant broken-stick levels; R's loop at
// R/TADpole.R:117-120 has no limit): the same arithmetic as k_ch without the
// shared segment store, with the cut, the level structure and the segment sums
// in global scratch.  slot_of[ti]: the tree's scratch slot (-1: k_ch scored it).
template <int KS>
__global__ void __launch_bounds__(256) k_ch_glb(SweepDev sd, const int *slot_of, double *scratch,
                                                size_t slot_doubles) {
    const int ti = blockIdx.x;
    const int sl = slot_of[ti];
    if (sl < 0) return;
    const int n = sd.n, k = sd.k, ldp = sd.ldp;
    const int nc = sd.n_cluster[ti];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    double *base = scratch + (size_t)sl * slot_doubles;
    double *seg = base;                                 // nc x k segment sums
    double *ssg = seg + (size_t)nc * k;                 // nc segment SS
    int *segs = (int *)(ssg + nc);                      // nc + 1 cut positions
    int *mbl = segs + nc + 1, *gbl = mbl + nc, *lnk_l = gbl + nc, *lnk_r = lnk_l + nc;
    const int ldsc = sd.ntrees;
    double *score_row = sd.scores + ti;
    const int m = sd.min_clusters < nc ? sd.min_clusters : nc;
    const int *mb = sd.mrg_b + (size_t)ti * (n - 1);
    // finest cut (as finest_cut, in global memory)
    for (int t = threadIdx.x; t < nc - 1; t += blockDim.x) mbl[t] = mb[n - 2 - t];
    __syncthreads();
    for (int t = threadIdx.x; t < nc - 1; t += blockDim.x) {
        const int bt = mbl[t];
        int rank = 0;
        for (int u = 0; u < nc - 1; ++u) rank += mbl[u] < bt;
        segs[rank + 1] = bt;
    }
    if (threadIdx.x == 0) {
        segs[0] = 0;
        segs[nc] = n;
    }
    __syncthreads();
    for (int g = w; g < nc; g += nw) {
        const double ss = seg_ss_wave<KS>(sd.Pt, ldp, k, segs[g], segs[g + 1] - 1, seg + (size_t)g * k, lane);
        if (lane == 0) ssg[g] = ss;
    }
    for (int t = threadIdx.x; t < nc - 1; t += blockDim.x) {
        const int bt = mb[n - 2 - t];
        int lo = 1, hi = nc - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (segs[mid] < bt) lo = mid + 1;
            else hi = mid;
        }
        gbl[t] = lo;
    }
    for (int g = threadIdx.x; g < nc; g += blockDim.x) {
        lnk_l[g] = g - 1;
        lnk_r[g] = g + 1;
    }
    __syncthreads();
    if (w != 0) return;
    const double trS = *sd.trS;
    double trW = 0.0;
    for (int g = 0; g < nc; ++g) trW = trW + ssg[g];
    if (lane == 0)
        score_row[(size_t)(nc - 1) * ldsc] = ((double)(n - nc) * (trS - trW)) / ((double)(nc - 1) * trW);
    for (int lev = nc - 1; lev >= m && lev >= 1; --lev) {
        const int gb = gbl[lev - 1];
        const int ga = lnk_l[gb];
        const int nx = lnk_r[gb];
        const int b = segs[gb];
        const int na = b - segs[ga];
        const int nbb = (nx < nc ? segs[nx] : n) - b;
        const double fa = (double)na, fb = (double)nbb;
        double *DA = seg + (size_t)ga * k;
        const double *DB = seg + (size_t)gb * k;
        double acc = 0.0, Mv[KS];
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            const int j = lane + 64 * t;
            const double a = j < k ? DA[j] : 0.0, bv = j < k ? DB[j] : 0.0;
            if (j < k) {
                const double t1 = a * fb;
                const double t2 = bv * fa;
                const double e = t1 - t2;
                acc = fma(e, e, acc);
            }
            Mv[t] = a + bv;
        }
        const double tot = wave_sum(acc);
        trW = trW + tot / (fa * fb * (fa + fb));
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            const int j = lane + 64 * t;
            if (j < k) DA[j] = Mv[t];
        }
        lnk_r[ga] = nx;
        if (nx < nc) lnk_l[nx] = ga;
        if (lane == 0)
            score_row[(size_t)(lev - 1) * ldsc] =
                lev == 1 ? r_nan() : ((double)(n - lev) * (trS - trW)) / ((double)(lev - 1) * trW);
    }
}

size_t ch_glb_slot_doubles(int nc, int k) { return (size_t)nc * (k + 1) + (size_t)(5 * nc + 2) / 2 + 8; }
void launch_ch_glb(const SweepDev &sd, const int *d_slot_of, double *scratch, size_t slot_doubles, hipStream_t s) {
    if (ks_for(sd.k) == 4)
        hipLaunchKernelGGL(k_ch_glb<4>, dim3(sd.ntrees), dim3(256), 0, s, sd, d_slot_of, scratch, slot_doubles);
    else if (ks_for(sd.k) == 8)
        hipLaunchKernelGGL(k_ch_glb<8>, dim3(sd.ntrees), dim3(256), 0, s, sd, d_slot_of, scratch, slot_doubles);
    else
        hipLaunchKernelGGL(k_ch_glb<16>, dim3(sd.ntrees), dim3(256), 0, s, sd, d_slot_of, scratch, slot_doubles);
    TP_HIP(hipGetLastError());
}

__global__ void k_fill(double *p, size_t cnt, double v) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < cnt) p[t] = v;
}

static size_t coniss_lds_bytes(int n) {   // costs, links, right ends (the mailbox is static LDS)
    return coniss_cost_stride(n) * 8 + coniss_link_stride(n) * 8;
}
constexpr size_t kConissGlbLds = 16;   // nothing: the mailbox is static LDS
constexpr int kConissMaxN = 64 * 64 * 32;             // global variant: up to 32 block-minimum slots
static bool coniss_in_lds(int n) { return coniss_lds_bytes(n) <= 160 * 1024 - 256 && n <= 64 * 64 * 3; }   // 256: static mailbox
// the LDS variant with one 16-bit link array (LU = 2): 10 bytes a bin instead of 16
static size_t coniss_lds2_bytes(int n) { return coniss_cost_stride(n) * 8 + coniss_link_stride(n) * 2; }
static bool coniss_in_lds2(int n) { return coniss_lds2_bytes(n) <= 160 * 1024 - 256 && n <= 64 * 64 * 3; }
// knob 49: the LDS variant link-only -- 3 (default): where the 16-byte variant
// does not fit (~10.2k-12.3k bins; 11 000 bins: sweep 21.5 -> 18.8 ms against the
// global variant), 2: every sweep, 1: lean sweeps, 0: never.  Not below: at C3
// the extra dependent LDS read on the merge chain costs 10.9 -> 12.8 ms

// seed kernel + CONISS (cost0 = initial adjacent costs, ntrees x nbk*64, then
// the global-variant link scratch: see sweep_cost0_doubles)
template <bool STAMPS, int BS, bool GLB, int LU = 0>
static void launch_coniss_bs(const SweepDev &sd, double *cost0, size_t lds, hipStream_t s) {
    if (sd.tree0 + sd.ntrees > 512) {   // trees of 9..16 column slots
        if constexpr (!STAMPS) {
            TP_HIP(hipFuncSetAttribute((const void *)k_coniss_t<false, BS, GLB, LU, 16>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL((k_coniss_t<false, BS, GLB, LU, 16>), dim3(sd.ntrees), dim3(128), lds, s, sd, cost0);
            return;
        }
        fail(TP_ERR_UNSUPPORTED, "stamped CONISS: at most 256 columns");
    }
    if (sd.tree0 + sd.ntrees > 256) {   // trees of 5..8 column slots
        if constexpr (!STAMPS) {
            TP_HIP(hipFuncSetAttribute((const void *)k_coniss_t<false, BS, GLB, LU, 8>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL((k_coniss_t<false, BS, GLB, LU, 8>), dim3(sd.ntrees), dim3(128), lds, s, sd, cost0);
            return;
        }
        fail(TP_ERR_UNSUPPORTED, "stamped CONISS: at most 256 columns");
    }
    TP_HIP(hipFuncSetAttribute((const void *)k_coniss_t<STAMPS, BS, GLB, LU>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_coniss_t<STAMPS, BS, GLB, LU>), dim3(sd.ntrees), dim3(128), lds, s, sd, cost0);
}
// knob 52: the batched CONISS kernel (k_coniss_b) where it applies (k <= 256,
// up to ~38k bins) -- 3 (default): also for lean sweeps, which take storage
// mode 1 where mode 0 would fit (10 bytes a bin: two trees share a CU; C4, 8
// streams: 0.224 -> 0.214 s), 2: lean sweeps in mode 0 (C4 0.265 -> 0.229 s
// against the two-wave kernel), 1: not for lean sweeps, 0: never (k_coniss_t)
// lean sweeps (another pipeline in flight on the device) of matrices that fit
// LDS, from this many bins (knob 48; 0: never): costs global and only the
// links in LDS (2 bytes a bin) so several trees share a CU -- the LDS
// variant's 16 bytes a bin hold a whole CU from ~5k bins while the tree's two
// waves use two of its SIMDs.  Measured on C4 (8 streams): 0.27-0.29 s at
// 4096 or 2048 vs 0.26 s off -- the global costs slow each tree more than
// the sharing gains -- so off

static void run_coniss(const SweepDev &sd_in, hipStream_t s, bool stamped, Ctx *prof) {
    SweepDev sd = sd_in;
    const int nbk = (sd.n + 63) / 64;
    double *cost0 = sd.cost0;
    const int ks = ks_for(sd.tree0 + sd.ntrees);   // slots of the widest tree of this launch
    if (sd.tree0 + sd.ntrees > 64) {   // trees with two or more slots read the paired copy
        double *pt2 = cost0 + coniss_pt2_offset(sd.n, sd.ntrees);
        sd.pt2_ld = 64 * ks;
        const size_t cnt = (size_t)sd.n * sd.pt2_ld;
        hipLaunchKernelGGL(k_pt_pairs, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, sd.Pt, sd.n, sd.ldp, sd.k,
                           pt2, sd.pt2_ld, 0);
        TP_HIP(hipGetLastError());
        sd.pt2 = pt2;
        if (sd.tree0 + sd.ntrees > 192 && sd.tree0 < 256) {   // 4-slot trees: the fully paired copy
            double *pt4 = pt2 + cnt;
            const size_t c4 = (size_t)sd.n * 256;
            hipLaunchKernelGGL(k_pt_pairs, dim3((unsigned)((c4 + 255) / 256)), dim3(256), 0, s, sd.Pt, sd.n, sd.ldp,
                               sd.k, pt4, 256, 1);
            TP_HIP(hipGetLastError());
            sd.pt4 = pt4;
        }
    }
    if (ks == 4)
        hipLaunchKernelGGL(k_seed<4>, dim3(sd.ntrees, nbk), dim3(64), 0, s, sd, cost0);
    else if (ks == 8)
        hipLaunchKernelGGL(k_seed<8>, dim3(sd.ntrees, nbk), dim3(64), 0, s, sd, cost0);
    else
        hipLaunchKernelGGL(k_seed<16>, dim3(sd.ntrees, nbk), dim3(64), 0, s, sd, cost0);
    TP_HIP(hipGetLastError());
    const bool lean_small = sd.lds_lean && t_knob.coniss_lean_min > 0 && sd.n >= t_knob.coniss_lean_min;
    const bool in_lds2 = !lean_small && coniss_in_lds2(sd.n) &&
                         (t_knob.coniss_lds2 == 2 || (t_knob.coniss_lds2 == 1 && sd.lds_lean) ||
                          (t_knob.coniss_lds2 == 3 && !coniss_in_lds(sd.n)));
    const bool in_lds = (coniss_in_lds(sd.n) || in_lds2) && !lean_small;
    // global variant: 16-bit links in LDS when they fit (costs stay global)
    const size_t lu_bytes = coniss_link_stride(sd.n) * 4;
    const int bs = (nbk + 63) / 64;   // block-minimum slots per lane
    // lds_lean (TP_FLAG_LDS_LEAN: another pipeline runs beside this one): only
    // the link array in LDS, rn derived from it (LU = 2, half the bytes), so
    // these trees fit on CUs whose LDS the other pipeline's trees hold
    const bool lu_ok = !in_lds && cfg_coniss_lu && sd.n + 64 < 0xFFFF && bs <= 11;
    const bool lu2 = lu_ok && sd.lds_lean;
    const bool lu = lu_ok && !lu2 && lu_bytes <= 150 * 1024;
    const size_t lds = in_lds2 ? coniss_lds2_bytes(sd.n)
                               : (in_lds ? coniss_lds_bytes(sd.n) : (lu ? lu_bytes : (lu2 ? lu_bytes / 2 : kConissGlbLds)));
    if (!stamped && prof) kprof_begin(*prof, K_CONISS);
    // the batched kernel (round 6), trees of up to 4 column slots: mode 0
    // (costs, int links and the block minima in LDS) where it fits, else mode 1
    // (16-bit links only) up to 3 block-minimum slots, else mode 2 (costs global)
    const size_t l16 = (coniss_link_stride(sd.n) * 2 + 7) & ~(size_t)7;
    const size_t cap_b = 160 * 1024 - 64 - sizeof(CbShared);
    const size_t lds_b0 = coniss_lds_bytes(sd.n) + (size_t)nbk * 8;
    const size_t lds_b1 = coniss_cost_stride(sd.n) * 8 + l16 + (size_t)nbk * 8;
    const size_t lds_b2 = l16 + (size_t)nbk * 8;
    // knob 52 = 3: lean sweeps (another pipeline in flight) take mode 1 where
    // mode 0 would fit, so two trees share a CU's LDS
    const bool lean1 = sd.lds_lean && t_knob.coniss_batch == 3;
    const int mode = (bs <= 3 && lds_b0 <= cap_b && !lean1) ? 0 : (bs <= 3 && lds_b1 <= cap_b) ? 1
                     : (bs <= 11 && sd.n + 64 < 0xFFFF && lds_b2 <= cap_b) ? 2 : -1;
    if (t_knob.coniss_batch && sd.tree0 + sd.ntrees <= 256 && mode >= 0 && !lean_small &&
        !(sd.lds_lean && t_knob.coniss_batch < 2)) {
        const size_t lds_b = mode == 0 ? lds_b0 : (mode == 1 ? lds_b1 : lds_b2);
        auto go = [&](auto kern) {
            TP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_b));
            hipLaunchKernelGGL(kern, dim3(sd.ntrees), dim3(64 * CB_W), lds_b, s, sd, cost0);
        };
        if (stamped) {
#ifdef TP_STAMPS_BUILD
            if (mode == 2 && bs <= 6) go(k_coniss_b<6, 2, true>);
            else if (mode == 2) fail(TP_ERR_UNSUPPORTED, "stamped batched CONISS: at most 24 576 bins in mode 2");
            else if (mode == 1) go(k_coniss_b<3, 1, true>);
            else if (bs == 1) go(k_coniss_b<1, 0, true>);
            else if (bs == 2) go(k_coniss_b<2, 0, true>);
            else go(k_coniss_b<3, 0, true>);
#else
            fail(TP_ERR_UNSUPPORTED, "stamped CONISS kernels are in the diagnostic build only (make STAMPS=1)");
#endif
        } else if (mode == 2 && bs <= 6) go(k_coniss_b<6, 2>);
        else if (mode == 2) go(k_coniss_b<11, 2>);
        else if (mode == 1) go(k_coniss_b<3, 1>);
        else if (bs == 1) go(k_coniss_b<1, 0>);
        else if (bs == 2) go(k_coniss_b<2, 0>);
        else go(k_coniss_b<3, 0>);
        if (!stamped && prof) kprof_end(*prof, K_CONISS);
        TP_HIP(hipGetLastError());
        return;
    }
    // global variant: as few block-minimum slots as the size needs (every
    // per-slot loop of the merge chain -- the untouched minimum, the argmin
    // ballots, the block-minimum updates -- runs over all of them)
    if (stamped) {
#ifdef TP_STAMPS_BUILD
        if (lu && bs <= 6) launch_coniss_bs<true, 6, true, true>(sd, cost0, lds, s);
        else if (!in_lds && bs <= 16) launch_coniss_bs<true, 16, true>(sd, cost0, lds, s);
        else if (!in_lds) fail(TP_ERR_UNSUPPORTED, "stamped CONISS: at most 65 536 bins");
        else if (bs == 1) launch_coniss_bs<true, 1, false>(sd, cost0, lds, s);
        else if (bs == 2) launch_coniss_bs<true, 2, false>(sd, cost0, lds, s);
        else launch_coniss_bs<true, 3, false>(sd, cost0, lds, s);
#else
        fail(TP_ERR_UNSUPPORTED, "stamped CONISS kernels are in the diagnostic build only (make STAMPS=1)");
#endif
    } else {
        if (in_lds2 && bs == 1) launch_coniss_bs<false, 1, false, 2>(sd, cost0, lds, s);
        else if (in_lds2 && bs == 2) launch_coniss_bs<false, 2, false, 2>(sd, cost0, lds, s);
        else if (in_lds2) launch_coniss_bs<false, 3, false, 2>(sd, cost0, lds, s);
        else if (lu2 && bs <= 2) launch_coniss_bs<false, 2, true, 2>(sd, cost0, lds, s);
        else if (lu2 && bs <= 3) launch_coniss_bs<false, 3, true, 2>(sd, cost0, lds, s);
        else if (lu2 && bs <= 6) launch_coniss_bs<false, 6, true, 2>(sd, cost0, lds, s);
        else if (lu2 && bs <= 8) launch_coniss_bs<false, 8, true, 2>(sd, cost0, lds, s);
        else if (lu2) launch_coniss_bs<false, 11, true, 2>(sd, cost0, lds, s);
        else if (lu && bs <= 6) launch_coniss_bs<false, 6, true, true>(sd, cost0, lds, s);
        else if (lu && bs <= 8) launch_coniss_bs<false, 8, true, true>(sd, cost0, lds, s);
        else if (lu) launch_coniss_bs<false, 11, true, true>(sd, cost0, lds, s);
        else if (!in_lds && bs <= 11) launch_coniss_bs<false, 11, true>(sd, cost0, lds, s);
        else if (!in_lds && bs <= 16) launch_coniss_bs<false, 16, true>(sd, cost0, lds, s);
        else if (!in_lds) launch_coniss_bs<false, 32, true>(sd, cost0, lds, s);   // > 65 536 bins
        else if (bs == 1) launch_coniss_bs<false, 1, false>(sd, cost0, lds, s);
        else if (bs == 2) launch_coniss_bs<false, 2, false>(sd, cost0, lds, s);
        else launch_coniss_bs<false, 3, false>(sd, cost0, lds, s);
    }
    if (!stamped && prof) kprof_end(*prof, K_CONISS);
    TP_HIP(hipGetLastError());
}

void launch_sweep(const SweepDev &sd, hipStream_t s, Ctx *prof) {
    if (sd.k > 64 * KS_MAX)
        fail(TP_ERR_UNSUPPORTED, "min(max_pcs, n_good) > 1024: this build's sweep kernels hold at most 1024 PC "
                                 "columns per lane group (R accepts any max_pcs, R/TADpole.R:344,452)");
    const int ks = ks_for(sd.k);
    if (sd.n < 3) fail(TP_ERR_NO_BSTICK, "fewer than 3 good bins: no broken-stick level");
    if (sd.n > kConissMaxN) fail(TP_ERR_UNSUPPORTED, "more than 131072 bins per matrix");
    if (sd.ntrees < 1 || sd.tree0 < 0 || sd.tree0 + sd.ntrees > sd.k) fail(TP_ERR_ARG, "bad tree range");
    size_t cnt = (size_t)sd.ntrees * sd.w_cap;
    double na;
    {
        uint64_t u = kRNaBits;
        memcpy(&na, &u, 8);
    }
    hipLaunchKernelGGL(k_fill, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, sd.scores, cnt, na);
    TP_HIP(hipGetLastError());
    hipStream_t ts = prof ? side_fork(*prof) : s;
    if (ks == 4) hipLaunchKernelGGL(k_trS<4>, dim3(1), dim3(256), 0, ts, sd.Pt, sd.n, sd.ldp, sd.k, sd.trS);
    else if (ks == 8) hipLaunchKernelGGL(k_trS<8>, dim3(1), dim3(512), 0, ts, sd.Pt, sd.n, sd.ldp, sd.k, sd.trS);
    else hipLaunchKernelGGL(k_trS<16>, dim3(1), dim3(1024), 0, ts, sd.Pt, sd.n, sd.ldp, sd.k, sd.trS);
    TP_HIP(hipGetLastError());
    run_coniss(sd, s, false, prof);
    if (prof) side_join(*prof);
    trace_mark(s, "coniss + trS");
    if (prof) kprof_begin(*prof, K_CH);
    if (sd.hkeys) {
        TP_HIP(hipMemsetAsync(sd.hkeys, 0xFF, (size_t)sd.hcap * sizeof(unsigned long long), s));
        TP_HIP(hipMemsetAsync(sd.ucount, 0, sizeof(int), s));
        hipLaunchKernelGGL(k_ch_cut, dim3(sd.ntrees), dim3(256), 0, s, sd);
        TP_HIP(hipGetLastError());
        trace_mark(s, "ch_cut");
        const int g = std::max(1, std::min(256, (sd.ucap + 3) / 4));
        if (ks == 4) hipLaunchKernelGGL(k_ch_segstat<4>, dim3(g), dim3(256), 0, s, sd);
        else if (ks == 8) hipLaunchKernelGGL(k_ch_segstat<8>, dim3(g), dim3(256), 0, s, sd);
        else hipLaunchKernelGGL(k_ch_segstat<16>, dim3(g), dim3(256), 0, s, sd);
        TP_HIP(hipGetLastError());
        trace_mark(s, "ch_segstat");
        if (ks == 4) hipLaunchKernelGGL(k_ch<4>, dim3(sd.ntrees), dim3(256), 0, s, sd);
        else if (ks == 8) hipLaunchKernelGGL(k_ch<8>, dim3(sd.ntrees), dim3(256), 0, s, sd);
        else hipLaunchKernelGGL(k_ch<16>, dim3(sd.ntrees), dim3(256), 0, s, sd);
    } else {
        if (ks == 4) hipLaunchKernelGGL(k_ch<4>, dim3(sd.ntrees), dim3(CH_THREADS), 0, s, sd);
        else if (ks == 8) hipLaunchKernelGGL(k_ch<8>, dim3(sd.ntrees), dim3(CH_THREADS), 0, s, sd);
        else hipLaunchKernelGGL(k_ch<16>, dim3(sd.ntrees), dim3(CH_THREADS), 0, s, sd);
    }
    TP_HIP(hipGetLastError());
    trace_mark(s, "ch");
    if (prof) kprof_end(*prof, K_CH);
}

void launch_coniss_stamped(const SweepDev &sd, hipStream_t s) { run_coniss(sd, s, true, nullptr); }

void launch_coniss_only(const SweepDev &sd, hipStream_t s) {
    if (sd.tree0 + sd.ntrees > 64 * KS_MAX) fail(TP_ERR_UNSUPPORTED, "more than 1024 columns");
    if (sd.n > kConissMaxN) fail(TP_ERR_UNSUPPORTED, "more than 131072 bins per matrix");
    run_coniss(sd, s, false, nullptr);
}

// ------------------------------------------- single calinhara (tp_ch entry)
template <int KS>
__global__ void __launch_bounds__(256) k_ch_single(const double *Pt, int n, int ldp, int k, const int *bnd, int cn,
                                                   double *ssg, double *trS_out, double *out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int g = w; g < cn + 1; g += 4) {
        // g == cn: the whole matrix (tr S)
        int s0 = g == cn ? 0 : bnd[g], e0 = g == cn ? n - 1 : bnd[g + 1] - 1;
        double ss = seg_ss_wave<KS>(Pt, ldp, k, s0, e0, nullptr, lane);
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
    if (k > 64 * KS_MAX) fail(TP_ERR_UNSUPPORTED, "calinhara: more than 1024 columns");
    if (k <= 256)
        hipLaunchKernelGGL(k_ch_single<4>, dim3(1), dim3(256), 0, s, d_Pt, n, ldp, k, d_bnd, cn, d_seg,
                           d_seg + cn + 1, d_out);
    else if (k <= 512)
        hipLaunchKernelGGL(k_ch_single<8>, dim3(1), dim3(256), 0, s, d_Pt, n, ldp, k, d_bnd, cn, d_seg,
                           d_seg + cn + 1, d_out);
    else
        hipLaunchKernelGGL(k_ch_single<16>, dim3(1), dim3(256), 0, s, d_Pt, n, ldp, k, d_bnd, cn, d_seg,
                           d_seg + cn + 1, d_out);
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
