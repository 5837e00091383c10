/* ORACLE — TEST INFRASTRUCTURE ONLY.  AddressSanitizer / UBSan driver for the C
 * half of the oracle (tp_oracle.c, compiled into this binary by `make -C
 * oracle asan`): runs every entry point on seeded random inputs at ragged
 * sizes (n = 2, 3, 65, 257, k up to 70, min_clusters 1..n) and cross-checks
 * the Ward-form CONISS against the distance-matrix definition, so an
 * out-of-bounds access or undefined behaviour in the restatement fails the CPU
 * test suite (tests/test_oracle.py::test_oracle_under_asan). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

int tpo_coniss(const double *Pt, int n, int ldp, int ncols, int *mrg_a, int *mrg_b, double *cost_out,
               double *height);
int tpo_coniss_bruteforce(const double *P, int n, int ldp, int ncols, int *mrg_b, double *height);
int tpo_bstick_ld(const double *height, int n, int *n_cluster);
int tpo_bstick_dd(const double *height, int n, int *n_cluster);
int tpo_sweep(const double *Pt, int n, int ldp, int k, int min_clusters, int bstick_mode, int nthreads,
              int *n_cluster, double *scores, int wcap, int *mrg_a_all, int *mrg_b_all, double *cost_all,
              double *height_all);
void tpo_dist_r(const double *P, int n, int ldp, int ncols, double *d);
void tpo_rowmeans_ld(const double *M, int n, int ld, int col_major, double *r);
void tpo_rowmeans_dd(const double *M, int n, int ld, int col_major, double *r);

static unsigned long long st = 0x9E3779B97F4A7C15ULL;
static double urand(void) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) * (1.0 / 9007199254740992.0);
}

static int run(int n, int k, int mc) {
    double *Pt = malloc(sizeof(double) * n * k), *P = malloc(sizeof(double) * n * k);
    for (int a = 0; a < n; ++a)
        for (int j = 0; j < k; ++j) {
            double v = (urand() - 0.5) * 10.0 / (1.0 + j) + (double)((a / 7) % 3);
            Pt[(size_t)a * k + j] = v;
            P[a + (size_t)j * n] = v;
        }
    int *ma = malloc(sizeof(int) * (n > 1 ? n - 1 : 1)), *mb = malloc(sizeof(int) * (n > 1 ? n - 1 : 1));
    int *mb2 = malloc(sizeof(int) * (n > 1 ? n - 1 : 1));
    double *co = malloc(sizeof(double) * (n > 1 ? n - 1 : 1)), *he = malloc(sizeof(double) * (n > 1 ? n - 1 : 1));
    double *he2 = malloc(sizeof(double) * (n > 1 ? n - 1 : 1));
    int bad = 0;
    tpo_coniss(Pt, n, k, k, ma, mb, co, he);
    if (n <= 300) {
        tpo_coniss_bruteforce(P, n, n, k, mb2, he2);
        for (int s = 0; s < n - 1; ++s)
            if (mb[s] != mb2[s]) { bad = 1; break; }
    }
    int nc = 0;
    if (n > 2) { tpo_bstick_ld(he, n - 1, &nc); tpo_bstick_dd(he, n - 1, &nc); }
    double *d = malloc(sizeof(double) * ((size_t)n * (n - 1) / 2 + 1));
    tpo_dist_r(P, n, n, k, d);
    double *r = malloc(sizeof(double) * n), *M = malloc(sizeof(double) * n * n);
    for (size_t t = 0; t < (size_t)n * n; ++t) M[t] = floor(urand() * 100);
    tpo_rowmeans_ld(M, n, n, 0, r);
    tpo_rowmeans_dd(M, n, n, 1, r);
    if (n >= 3) {
        int *ncl = malloc(sizeof(int) * k);
        double *sc = malloc(sizeof(double) * k * n);
        int *A = malloc(sizeof(int) * k * (n - 1)), *B = malloc(sizeof(int) * k * (n - 1));
        double *C = malloc(sizeof(double) * k * (n - 1)), *H = malloc(sizeof(double) * k * (n - 1));
        tpo_sweep(Pt, n, k, k, mc, 0, 1, ncl, sc, n, A, B, C, H);
        tpo_sweep(Pt, n, k, k, mc, 1, 2, ncl, sc, n, A, B, C, H);
        free(ncl); free(sc); free(A); free(B); free(C); free(H);
    }
    free(Pt); free(P); free(ma); free(mb); free(mb2); free(co); free(he); free(he2); free(d); free(r); free(M);
    return bad;
}

int main(void) {
    const int cases[][3] = {{2, 1, 2}, {3, 1, 1}, {3, 2, 2}, {65, 7, 2}, {65, 64, 5}, {257, 70, 2}, {120, 3, 50}};
    int fails = 0;
    for (unsigned c = 0; c < sizeof cases / sizeof cases[0]; ++c) {
        int b = run(cases[c][0], cases[c][1], cases[c][2]);
        printf("n=%d k=%d min_clusters=%d: %s\n", cases[c][0], cases[c][1], cases[c][2], b ? "MISMATCH" : "ok");
        fails += b;
    }
    return fails ? 1 : 0;
}
