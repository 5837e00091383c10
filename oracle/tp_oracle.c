/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of TADpole's per-matrix sweep (R/TADpole.R:102-140) and of the
 * third-party arithmetic it calls: stats::dist (R distance.c R_euclidean),
 * rioja::chclust(method="coniss") (rioja >= 0.9-21, Grimm 1987 CONISS),
 * rioja::bstick.chclust + vegan::bstick.default, stats::cutree and
 * fpc::calinhara (fpc >= 2.1-11.1).  None of rioja / fpc / R is present in
 * this container, so the [ext] semantics are restated from their published
 * algorithms (see DESIGN.md "Oracle").  PARITY UNPINNED: the reference ships no
 * tests or fixtures for this path and cannot be run here.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product path (libtadpole_hip.so) never links it.
 *
 * Two flavours live here:
 *   - "canonical" functions (tpo_coniss, tpo_ch_levels, tpo_bstick_dd, ...) fix
 *     one floating-point evaluation order.  The HIP kernels follow the same
 *     order, so GPU and oracle agree BIT FOR BIT given identical PC scores.
 *     The order is: 64-lane strided partial sums, then an xor butterfly
 *     (masks 1,2,4,8,16,32), explicit fma() where noted, no contraction.
 *   - "R-faithful" functions (tpo_bstick_ld, tpo_rowmeans_ld, tpo_dist_r,
 *     tpo_coniss_bruteforce) follow R's own arithmetic (long double
 *     accumulators, R_euclidean's loop, a distance-matrix CONISS) and are used
 *     to show the canonical versions make the same decisions.
 *
 * Compile with -ffp-contract=off (see oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define LANES 64

/* R's NA_real_ is a NaN with payload 1954 (R arithmetic.c R_ValueOfNA). */
static double r_na_real(void) {
    union { uint64_t u; double d; } v;
    v.u = 0x7FF00000000007A2ULL;
    return v.d;
}
static double r_nan(void) {
    union { uint64_t u; double d; } v;
    v.u = 0x7FF8000000000000ULL;
    return v.d;
}

/* xor butterfly over 64 lane partials; every lane ends with the same bits. */
static double butterfly64(double *part) {
    double tmp[LANES];
    for (int m = 1; m < LANES; m <<= 1) {
        for (int l = 0; l < LANES; ++l) tmp[l] = part[l] + part[l ^ m];
        memcpy(part, tmp, sizeof(tmp));
    }
    return part[0];
}

/*
 * Ward increment of merging adjacent clusters A (na rows, column sums SA) and
 * B: |A||B|/(|A|+|B|) * ||SA/na - SB/nb||^2 over the first ncols columns,
 * evaluated division-free as sum_j (SA_j nb - SB_j na)^2 / (na nb (na+nb)).
 * This is CONISS's "increase in total dispersion" (Grimm 1987; rioja chclust
 * called at R/TADpole.R:108,374,460).  Canonical order: e_j = SA_j*nb - SB_j*na
 * (two rounded products, one subtraction); lane l accumulates j = l, l+64, ...
 * with fma(e, e, acc); xor butterfly; one division by na*nb*(na+nb).
 */
double tpo_ward(const double *SA, int na, const double *SB, int nb, int ncols) {
    double part[LANES];
    const double fa = (double)na, fb = (double)nb;
    for (int l = 0; l < LANES; ++l) {
        double acc = 0.0;
        for (int j = l; j < ncols; j += LANES) {
            double t1 = SA[j] * fb;
            double t2 = SB[j] * fa;
            double e = t1 - t2;
            acc = fma(e, e, acc);
        }
        part[l] = acc;
    }
    double tot = butterfly64(part);
    return tot / (fa * fb * (fa + fb));
}

static inline double nan2inf(double x) { return isnan(x) ? INFINITY : x; }

/*
 * Canonical CONISS on rows 0..n-1 of Pt (row-major, leading dim ldp), first
 * ncols columns.  Greedy: at each of the n-1 steps merge the adjacent pair with
 * the smallest Ward increment; ties go to the leftmost pair.  Outputs per step
 * s: mrg_a[s] = start of the left cluster, mrg_b[s] = start of the right
 * cluster (the boundary the merge removes), cost[s] = increment,
 * height[s] = running total dispersion (cumulative sum of increments).
 * Returns 0, or -1 on allocation failure.
 */
int tpo_coniss(const double *Pt, int n, int ldp, int ncols,
               int *mrg_a, int *mrg_b, double *cost_out, double *height) {
    if (n < 2) return 0;
    double *S = (double *)malloc((size_t)n * ncols * sizeof(double));
    double *cost = (double *)malloc((size_t)n * sizeof(double));
    int *link = (int *)malloc((size_t)n * sizeof(int));
    if (!S || !cost || !link) { free(S); free(cost); free(link); return -1; }
    for (int a = 0; a < n; ++a) {
        memcpy(S + (size_t)a * ncols, Pt + (size_t)a * ldp, ncols * sizeof(double));
        link[a] = a;
    }
    for (int a = 0; a < n - 1; ++a)
        cost[a] = nan2inf(tpo_ward(S + (size_t)a * ncols, 1, S + (size_t)(a + 1) * ncols, 1, ncols));
    cost[n - 1] = INFINITY;
    /* cand[p]: p starts a cluster that has a right neighbour.  Argmin key is
     * (cost with NaN -> +inf, p) for candidates and (+inf, p + n) otherwise,
     * compared lexicographically: the leftmost smallest candidate wins. */
    unsigned char *cand = (unsigned char *)malloc((size_t)n);
    if (!cand) { free(S); free(cost); free(link); return -1; }
    for (int p = 0; p < n; ++p) cand[p] = (unsigned char)(p < n - 1);
    double h = 0.0;
    for (int s = 0; s < n - 1; ++s) {
        int a = -1;
        double best = INFINITY;
        long bidx = 2L * n;
        for (int p = 0; p < n - 1; ++p) {
            double v = cand[p] ? cost[p] : INFINITY;
            long idx = cand[p] ? p : (long)p + n;
            if (v < best || (v == best && idx < bidx)) { best = v; bidx = idx; a = p; }
        }
        int ea = link[a];
        int b = ea + 1;
        int eb = link[b];
        double c = cost[a];
        mrg_a[s] = a;
        mrg_b[s] = b;
        cost_out[s] = c;
        h = h + c;
        height[s] = h;
        link[a] = eb;
        link[eb] = a;
        double *SA = S + (size_t)a * ncols, *SB = S + (size_t)b * ncols;
        for (int j = 0; j < ncols; ++j) SA[j] = SA[j] + SB[j];
        int nm = eb - a + 1;
        cost[b] = INFINITY;
        cand[b] = 0;
        if (a > 0) {
            int ls = link[a - 1];
            cost[ls] = nan2inf(tpo_ward(S + (size_t)ls * ncols, a - ls, SA, nm, ncols));
        }
        if (eb + 1 < n) {
            int r = eb + 1, er = link[r];
            cost[a] = nan2inf(tpo_ward(SA, nm, S + (size_t)r * ncols, er - r + 1, ncols));
        } else {
            cost[a] = INFINITY;
            cand[a] = 0;
        }
    }
    free(S); free(cost); free(link); free(cand);
    return 0;
}

/*
 * Definitional CONISS on a dissimilarity matrix, the way rioja's C code works
 * on x = as.matrix(dist)^2/2: a cluster's dispersion is sum_{a,b in C} x_ab/|C|
 * (full square, so = within-cluster sum of squares), the cost of a merge is
 * disp(A u B) - disp(A) - disp(B).  O(n^3); for cross-checking the Ward form's
 * merge order on small fixtures only.  P is column-major n x ncols (ld ldp).
 */
int tpo_coniss_bruteforce(const double *P, int n, int ldp, int ncols,
                          int *mrg_b, double *height) {
    double *x = (double *)malloc((size_t)n * n * sizeof(double));
    int *start = (int *)malloc((size_t)n * sizeof(int));
    int *len = (int *)malloc((size_t)n * sizeof(int));
    double *disp = (double *)malloc((size_t)n * sizeof(double));
    if (!x || !start || !len || !disp) { free(x); free(start); free(len); free(disp); return -1; }
    for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) {
            double s = 0.0;
            for (int j = 0; j < ncols; ++j) {
                double dv = P[a + (size_t)j * ldp] - P[b + (size_t)j * ldp];
                s += dv * dv;
            }
            double d = sqrt(s);
            x[a + (size_t)b * n] = d * d / 2.0;
        }
    int nc = n;
    for (int c = 0; c < n; ++c) { start[c] = c; len[c] = 1; disp[c] = 0.0; }
    double tot = 0.0;
    for (int s = 0; s < n - 1; ++s) {
        int best = -1;
        double bestinc = INFINITY, bestdisp = 0.0;
        for (int c = 0; c < nc - 1; ++c) {
            int s0 = start[c], e0 = start[c + 1] + len[c + 1];
            double sum = 0.0;
            for (int a = s0; a < e0; ++a)
                for (int b = s0; b < e0; ++b) sum += x[a + (size_t)b * n];
            double du = sum / (double)(e0 - s0);
            double inc = du - disp[c] - disp[c + 1];
            if (inc < bestinc) { bestinc = inc; best = c; bestdisp = du; }
        }
        mrg_b[s] = start[best + 1];
        tot += bestinc;
        height[s] = tot;
        len[best] += len[best + 1];
        disp[best] = bestdisp;
        for (int c = best + 1; c < nc - 1; ++c) {
            start[c] = start[c + 1]; len[c] = len[c + 1]; disp[c] = disp[c + 1];
        }
        --nc;
    }
    free(x); free(start); free(len); free(disp);
    return 0;
}

/* ---- broken stick (rioja bstick.chclust + vegan bstick.default) ---------- */

/* R-faithful: R's cumsum accumulates in LDOUBLE (R cum.c). */
int tpo_bstick_ld(const double *height, int n, int *n_cluster) {
    int nobj = n - 1;               /* length(height) */
    if (nobj < 2) { *n_cluster = -1; return -1; }
    double tot = height[nobj - 1];
    double *cs = (double *)malloc((size_t)(nobj + 1) * sizeof(double));
    if (!cs) return -1;
    long double acc = 0.0L;
    for (int t = 1; t <= nobj; ++t) {
        acc += (long double)(tot / (double)(nobj - t + 1));
        cs[t] = (double)acc;
    }
    int run = 0, started = 0;
    for (int j = 1; j <= nobj - 1; ++j) {
        double disp = fabs(height[nobj - 1 - j] - height[nobj - j]);
        double bs = cs[nobj - j + 1] / (double)nobj;
        int gt = disp > bs;
        if (gt) { started = 1; ++run; }
        else if (started) break;
    }
    free(cs);
    *n_cluster = started ? run : -1;
    return started ? 0 : -1;
}

/* double-double helpers (canonical; the HIP kernels use the same steps). */
static inline void two_sum(double a, double b, double *s, double *e) {
    double x = a + b;
    double bv = x - a;
    double av = x - bv;
    *s = x;
    *e = (a - av) + (b - bv);
}
static inline void dd_add_d(double *hi, double *lo, double x) {
    double s, e;
    two_sum(*hi, x, &s, &e);
    e = e + *lo;
    double h2 = s + e;
    *lo = e - (h2 - s);
    *hi = h2;
}
/* (hi+lo)/d rounded to double; d > 0 exact integer-valued. */
static inline double dd_div_d(double hi, double lo, double d) {
    double q1 = hi / d;
    double r = fma(-q1, d, hi);
    r = r + lo;
    return q1 + r / d;
}

/* Canonical: the long double cumsum replaced by a double-double cumsum. */
int tpo_bstick_dd(const double *height, int n, int *n_cluster) {
    int nobj = n - 1;
    if (nobj < 2) { *n_cluster = -1; return -1; }
    double tot = height[nobj - 1];
    double *cs = (double *)malloc((size_t)(nobj + 1) * sizeof(double));
    if (!cs) return -1;
    double hi = 0.0, lo = 0.0;
    for (int t = 1; t <= nobj; ++t) {
        dd_add_d(&hi, &lo, tot / (double)(nobj - t + 1));
        cs[t] = hi + lo;
    }
    int run = 0, started = 0;
    for (int j = 1; j <= nobj - 1; ++j) {
        double disp = fabs(height[nobj - 1 - j] - height[nobj - j]);
        double bs = cs[nobj - j + 1] / (double)nobj;
        int gt = disp > bs;
        if (gt) { started = 1; ++run; }
        else if (started) break;
    }
    free(cs);
    *n_cluster = started ? run : -1;
    return started ? 0 : -1;
}

/* ---- Calinski-Harabasz over nested cutree levels ------------------------ */

/*
 * Canonical segment statistics of rows s..e (inclusive) over k columns:
 * sum_j sequential over rows, mean_j = sum_j / n, ss_j = sum fma(d,d,.) over
 * rows, total = 64-lane strided partials of ss_j (plain adds) + butterfly.
 */
double tpo_seg_ss(const double *Pt, int ldp, int k, int s, int e, double *sum) {
    double part[LANES];
    const double fn = (double)(e - s + 1);
    for (int l = 0; l < LANES; ++l) part[l] = 0.0;
    for (int j = 0; j < k; ++j) {
        double sj = 0.0;
        for (int a = s; a <= e; ++a) sj = sj + Pt[(size_t)a * ldp + j];
        sum[j] = sj;
        double mj = sj / fn;
        double ss = 0.0;
        for (int a = s; a <= e; ++a) {
            double d = Pt[(size_t)a * ldp + j] - mj;
            ss = fma(d, d, ss);
        }
        part[j % LANES] = part[j % LANES] + ss;
    }
    return butterfly64(part);
}

double tpo_trS(const double *Pt, int n, int ldp, int k) {
    double *sum = (double *)malloc((size_t)k * sizeof(double));
    double r = tpo_seg_ss(Pt, ldp, k, 0, n - 1, sum);
    free(sum);
    return r;
}

static int cmp_int(const void *a, const void *b) {
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

/*
 * Scores of one tree (R/TADpole.R:115-120): score[n-1] = calinhara(P, cutree(k=n))
 * for n = min(min_clusters, nc)..nc; other entries NA.  cutree(k=n) is the set
 * of boundaries removed by the last n-1 merges.  tr(W) at the finest level is
 * the sum of canonical segment SS; each coarser level adds the Ward increment
 * (all k columns) of the two segments that merge.  CH = (N-n) tr(B) /
 * ((n-1) tr(W)) with tr(B) = trS - tr(W) (fpc calinhara); n = 1 gives NaN as in R.
 */
int tpo_ch_levels(const double *Pt, int n, int ldp, int k, const int *mrg_b,
                  int nc, int min_clusters, double trS, double *score) {
    const double NA = r_na_real();
    for (int t = 0; t < nc; ++t) score[t] = NA;
    int m = min_clusters < nc ? min_clusters : nc;
    if (nc == 1) { score[0] = r_nan(); return 0; }
    int *bnd = (int *)malloc((size_t)nc * sizeof(int));
    int *segs = (int *)malloc((size_t)(nc + 1) * sizeof(int));
    double *S = (double *)malloc((size_t)nc * k * sizeof(double));
    int *alive = (int *)malloc((size_t)nc * sizeof(int));
    if (!bnd || !segs || !S || !alive) { free(bnd); free(segs); free(S); free(alive); return -1; }
    for (int t = 1; t <= nc - 1; ++t) bnd[t - 1] = mrg_b[n - 1 - t];
    qsort(bnd, nc - 1, sizeof(int), cmp_int);
    segs[0] = 0;
    for (int t = 0; t < nc - 1; ++t) segs[t + 1] = bnd[t];
    segs[nc] = n;
    double trW = 0.0;
    for (int g = 0; g < nc; ++g) {
        double ss = tpo_seg_ss(Pt, ldp, k, segs[g], segs[g + 1] - 1, S + (size_t)g * k);
        trW = trW + ss;
        alive[g] = 1;
    }
    if (nc >= m && nc >= 2)
        score[nc - 1] = ((double)(n - nc) * (trS - trW)) / ((double)(nc - 1) * trW);
    for (int lev = nc - 1; lev >= m && lev >= 1; --lev) {
        int b = mrg_b[n - lev - 1];
        int gb = -1;
        for (int g = 0; g < nc; ++g) if (alive[g] && segs[g] == b) { gb = g; break; }
        int ga = gb - 1;
        while (ga >= 0 && !alive[ga]) --ga;
        if (gb < 0 || ga < 0) { free(bnd); free(segs); free(S); free(alive); return -2; }
        int na = 0, nb = 0;
        int ea = gb;  /* segment ga spans segs[ga] .. start of next alive */
        na = segs[ea] - segs[ga];
        int nx = gb + 1;
        while (nx < nc && !alive[nx]) ++nx;
        nb = (nx < nc ? segs[nx] : n) - segs[gb];
        double dw = tpo_ward(S + (size_t)ga * k, na, S + (size_t)gb * k, nb, k);
        trW = trW + dw;
        for (int j = 0; j < k; ++j) S[(size_t)ga * k + j] = S[(size_t)ga * k + j] + S[(size_t)gb * k + j];
        alive[gb] = 0;
        if (lev == 1) score[0] = r_nan();
        else score[lev - 1] = ((double)(n - lev) * (trS - trW)) / ((double)(lev - 1) * trW);
    }
    free(bnd); free(segs); free(S); free(alive);
    return 0;
}

/*
 * Whole find_params sweep (R/TADpole.R:102-123), trees i = 1..k in parallel
 * (OpenMP stands in for doParallel's fork workers, R/TADpole.R:103-104).
 * Pt: n x k row-major (ld ldp).  Outputs: n_cluster[k] (-1 where R would
 * error), scores k x wcap column-major (R matrix layout), and per tree the
 * merge record (k x (n-1) each) when the arrays are non-NULL.
 * bstick_mode: 0 canonical (double-double), 1 R-faithful (long double).
 * Returns 0 ok, 1 if some tree has no broken-stick level (R errors there),
 * 2 if wcap is too small, <0 on allocation failure.
 */
int tpo_sweep(const double *Pt, int n, int ldp, int k, int min_clusters,
              int bstick_mode, int nthreads, int *n_cluster, double *scores,
              int wcap, int *mrg_a_all, int *mrg_b_all, double *cost_all,
              double *height_all) {
    const double NA = r_na_real();
    for (size_t t = 0; t < (size_t)k * wcap; ++t) scores[t] = NA;
    double trS = tpo_trS(Pt, n, ldp, k);
    int err = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int i = 1; i <= k; ++i) {
        int *ma = (int *)malloc((size_t)n * sizeof(int));
        int *mb = (int *)malloc((size_t)n * sizeof(int));
        double *co = (double *)malloc((size_t)n * sizeof(double));
        double *he = (double *)malloc((size_t)n * sizeof(double));
        double *sc = (double *)malloc((size_t)n * sizeof(double));
        if (!ma || !mb || !co || !he || !sc) { err |= 4; goto done; }
        if (tpo_coniss(Pt, n, ldp, i, ma, mb, co, he)) { err |= 4; goto done; }
        int nc = -1;
        if (bstick_mode == 1) tpo_bstick_ld(he, n, &nc);
        else tpo_bstick_dd(he, n, &nc);
        n_cluster[i - 1] = nc;
        if (nc < 1) { err |= 1; }
        else if (nc > wcap) { err |= 2; }
        else {
            tpo_ch_levels(Pt, n, ldp, k, mb, nc, min_clusters, trS, sc);
            for (int t = 0; t < nc; ++t) scores[(size_t)(i - 1) + (size_t)t * k] = sc[t];
        }
        if (mrg_a_all) memcpy(mrg_a_all + (size_t)(i - 1) * (n - 1), ma, (size_t)(n - 1) * sizeof(int));
        if (mrg_b_all) memcpy(mrg_b_all + (size_t)(i - 1) * (n - 1), mb, (size_t)(n - 1) * sizeof(int));
        if (cost_all) memcpy(cost_all + (size_t)(i - 1) * (n - 1), co, (size_t)(n - 1) * sizeof(double));
        if (height_all) memcpy(height_all + (size_t)(i - 1) * (n - 1), he, (size_t)(n - 1) * sizeof(double));
    done:
        free(ma); free(mb); free(co); free(he); free(sc);
    }
    if (err & 4) return -1;
    if (err & 2) return 2;
    if (err & 1) return 1;
    return 0;
}

/* ---- stats::dist, euclidean (R distance.c R_euclidean) ------------------ */
/* P column-major n x ncols (ld ldp); d = lower triangle by columns, R order. */
void tpo_dist_r(const double *P, int n, int ldp, int ncols, double *d) {
    size_t ij = 0;
    for (int j = 0; j < n; ++j)
        for (int i = j + 1; i < n; ++i) {
            double dist = 0.0;
            for (int c = 0; c < ncols; ++c) {
                double dev = P[i + (size_t)c * ldp] - P[j + (size_t)c * ldp];
                dist += dev * dev;
            }
            d[ij++] = sqrt(dist);
        }
}

/* ---- rowMeans with R's long double accumulator (R array.c do_colsum) ---- */
void tpo_rowmeans_ld(const double *M, int n, int ld, int col_major, double *r) {
    for (int i = 0; i < n; ++i) {
        long double s = 0.0L;
        for (int j = 0; j < n; ++j)
            s += col_major ? M[i + (size_t)j * ld] : M[(size_t)i * ld + j];
        s /= n;
        r[i] = (double)s;
    }
}

/* Canonical device rule: double-double row sum, then dd / n. */
void tpo_rowmeans_dd(const double *M, int n, int ld, int col_major, double *r) {
    for (int i = 0; i < n; ++i) {
        double hi = 0.0, lo = 0.0;
        for (int j = 0; j < n; ++j)
            dd_add_d(&hi, &lo, col_major ? M[i + (size_t)j * ld] : M[(size_t)i * ld + j]);
        r[i] = dd_div_d(hi, lo, (double)n);
    }
}
