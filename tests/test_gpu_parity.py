"""GPU parity: every stage through the C ABI of libtadpole_hip.so against the
CPU oracle (oracle/), at sizes the oracle finishes in seconds.

Bars: bit-exact for indices (mask, merge order, boundaries, n_cluster,
n_pcs/n_clusters, TAD coordinates) and for the canonical-order sweep floats
(heights, CH scores given identical PC scores); R's dist order bit-exact;
correlation / PCA (different algorithm from LAPACK) within the tolerances
written in each test; end-to-end CH within 1e-6 relative (north_star).
"""
import numpy as np
import pytest

import gpu_helpers as G
import tadpole_oracle as O
from tadpole_amd.synth import synth_hic

pytestmark = pytest.mark.gpu


def _pcs(n0, seed, k=200):
    m = synth_hic(n0, seed)
    r = O.tadpole(m, max_pcs=k)
    return r.pcs


# ------------------------------------------------------------------ mask

@pytest.mark.parametrize("n0,seed", [(200, 1), (333, 2), (1000, 3)])
def test_mask_integer_counts(gpu, n0, seed):
    m = synth_hic(n0, seed)
    bad, rm, good = G.mask(m)
    obad, orm, _ = O.bad_mask(O.clean_symmetrize(m), 0.01)
    assert np.array_equal(bad, obad)
    assert np.array_equal(rm, orm)            # integer sums: exact
    assert np.array_equal(good, np.flatnonzero(~obad))


@pytest.mark.parametrize("frac", [0.0, 0.01, 0.05, 0.3, 1.0])
def test_mask_real_values_nan_and_asymmetric(gpu, frac):
    rng = np.random.default_rng(7)
    n0 = 257
    m = rng.gamma(2.0, 3.0, (n0, n0))          # asymmetric on purpose: upper must win
    m[rng.random((n0, n0)) < 0.01] = np.nan
    m[5, 5] = 0.0
    bad, rm, good = G.mask(m, frac)
    cm = O.clean_symmetrize(m)
    obad, orm, _ = O.bad_mask(cm, frac)
    assert np.array_equal(bad, obad)
    np.testing.assert_allclose(rm, orm, rtol=2e-16, atol=0)
    # column-major buffer of the same matrix gives the same answer
    bad2, _, _ = G.mask(np.asfortranarray(m), frac, flags=0)
    assert np.array_equal(bad2, obad)


@pytest.mark.parametrize("n0", [64, 257, 1000])
def test_clean_symmetrize_in_place(gpu, n0):
    """tp_mask_dev's in-place NA -> 0 and forceSymmetric(uplo='U')
    (R/TADpole.R:19-20) leave exactly the oracle's matrix in the buffer: NaNs on
    both sides of the diagonal and on it, the lower triangle overwritten."""
    import torch
    from tadpole_amd.api import mask_dev
    rng = np.random.default_rng(n0)
    m = rng.gamma(2.0, 3.0, (n0, n0))
    m[rng.random((n0, n0)) < 0.02] = np.nan
    m[3, 3] = np.nan
    dm = torch.from_numpy(m).cuda()
    mask_dev(dm, 0.01)
    assert np.array_equal(dm.cpu().numpy(), O.clean_symmetrize(m))


def test_mask_ties_and_all_equal(gpu):
    m = np.ones((64, 64))
    bad, _, _ = G.mask(m, 0.01)
    assert not bad.any()                       # r < q is false for ties
    m[:, 3] = m[3, :] = 0.5
    bad, _, _ = G.mask(m, 0.01)
    obad, _, _ = O.bad_mask(O.clean_symmetrize(m), 0.01)
    assert np.array_equal(bad, obad)


# ------------------------------------------------------------------- cor

@pytest.mark.parametrize("n", [64, 198, 515])
def test_cor(gpu, n):
    m = synth_hic(n + 3, 11 + n)
    obad, _, _ = O.bad_mask(O.clean_symmetrize(m), 0.01)
    g = np.flatnonzero(~obad)
    x = O.clean_symmetrize(m)[np.ix_(g, g)]
    c = G.cor(x)
    oc = O.sparse_cor(x)
    assert np.array_equal(c, c.T)              # exactly symmetric, as dsyrk + copy
    np.testing.assert_allclose(c, oc, rtol=0, atol=5e-12)


def test_cor_constant_column_nan_to_zero(gpu):
    rng = np.random.default_rng(3)
    x = rng.random((40, 40))
    x = x + x.T
    x[:, 7] = 2.0
    x[7, :] = 2.0
    c = G.cor(x)
    oc = O.sparse_cor(x)
    assert np.all(c[7, :] == 0) or np.allclose(c[7, :], oc[7, :], atol=1e-12)
    np.testing.assert_allclose(c, oc, atol=1e-10)


# ------------------------------------------------------------------- pca

def _proj(p, i):
    q, _ = np.linalg.qr(p[:, :i])
    return q @ q.T


@pytest.mark.parametrize("n0,k", [(120, 120), (200, 200), (700, 200)])
def test_pca_scores(gpu, n0, k):
    m = synth_hic(n0, 40 + n0)
    cm = O.clean_symmetrize(m)
    obad, _, _ = O.bad_mask(cm, 0.01)
    g = np.flatnonzero(~obad)
    c = O.sparse_cor(cm[np.ix_(g, g)])
    kk = min(k, len(g))
    p, sd = G.pca(c, kk)
    op = O.prcomp_x(c, kk)
    # column signs are arbitrary (irrelevant downstream); compare |columns|
    s = np.sign(np.sum(p * op, axis=0))
    s[s == 0] = 1
    scale = np.abs(op).max()
    # well separated leading components: elementwise
    np.testing.assert_allclose(p[:, :20] * s[:20], op[:, :20], atol=1e-9 * scale)
    # every prefix subspace the sweep uses (distances only see span(P[:, :i]))
    sv = np.linalg.svd(op, compute_uv=False)
    for i in (1, 5, 20, kk // 2, kk):
        if i < kk and sv[i - 1] / max(sv[i], 1e-300) < 1.0 + 1e-6:
            continue                           # degenerate prefix: not defined by the reference either
        assert np.abs(_proj(p, i) - _proj(op, i)).max() < 1e-7, i


# ------------------------------------------------- Rayleigh-Ritz eigensolver

def _spectrum(kind, b, rng):
    if kind == "graded":          # like a filtered PCA block: lambda_1 / lambda_b ~ 400
        return np.sort(np.exp(rng.uniform(np.log(2.5e-3), 0, b)))[::-1] * 1e5
    if kind == "clustered":       # near-degenerate groups and exact repeats
        base = np.repeat(rng.uniform(1, 100, (b + 3) // 4), 4)[:b]
        return np.sort(base + rng.standard_normal(b) * 1e-9 * (rng.random(b) < 0.5))[::-1]
    if kind == "rankdef":         # centred-Gram style: several exact zeros
        ev = rng.gamma(1.0, 1.0, b) ** 2
        ev[rng.choice(b, size=max(1, b // 8), replace=False)] = 0.0
        return np.sort(ev)[::-1]
    return rng.standard_normal(b)  # indefinite


@pytest.mark.parametrize("b,kind", [(1, "graded"), (2, "indefinite"), (3, "graded"), (5, "clustered"),
                                    (64, "graded"), (200, "rankdef"), (256, "graded"), (256, "clustered"),
                                    (16, "graded"), (240, "clustered"), (208, "rankdef"),
                                    (300, "graded"), (512, "graded"), (640, "clustered"),
                                    (768, "graded"), (1000, "rankdef"), (1280, "clustered")])
def test_eigsym(gpu, b, kind):
    rng = np.random.default_rng(b * 7 + len(kind))
    ev = _spectrum(kind, b, rng)
    q, _ = np.linalg.qr(rng.standard_normal((b, b)))
    h = (q * ev) @ q.T
    h = (h + h.T) / 2
    theta, v = G.eigsym(h)
    ref = np.linalg.eigvalsh(h)
    scale = max(np.abs(ref).max(), 1e-300)
    assert np.all(np.diff(theta) >= -1e-13 * scale)
    np.testing.assert_allclose(theta, ref, atol=1e-12 * scale, rtol=0)
    # residual and orthogonality (bars: LAPACK-level backward error)
    assert np.abs(h @ v - v * theta).max() <= 1e-12 * scale
    assert np.abs(v.T @ v - np.eye(b)).max() <= 1e-9


@pytest.mark.parametrize("b,cond,rel", [(16, 1e2, 0.0), (48, 1e4, 0.0), (128, 1e6, 0.0), (256, 1e6, 0.0),
                                         (256, 1e12, 1e-14), (96, 1.0, 0.0), (64, 1e8, 1e-14), (32, 1e3, 0.0)])
def test_chol_inv_register_kernel(gpu, b, cond, rel):
    """PCA CholQR kernels (k_chol_inv + k_trsm_frag) on Z = I: Y = U^{-1} for
    U'U = W + rel diag(W) (Jacobi-scaled shift).  Checks Y upper triangular,
    Y'(W + rel diag W)Y = I (bar ~ eps kappa(S W S)) and diag(U) = diag of
    the Cholesky factor (bar ~ b eps kappa)."""
    import ctypes
    rng = np.random.default_rng(b + int(np.log10(cond)))
    q, _ = np.linalg.qr(rng.standard_normal((b, b)))
    ev = np.logspace(0, -np.log10(cond), b)
    dsc = 10.0 ** rng.uniform(-3, 3, b)          # column norms spread (Jacobi scaling)
    W = ((q * ev) @ q.T) * dsc[:, None] * dsc[None, :]
    W = np.asfortranarray((W + W.T) / 2)
    dg = np.zeros(b)
    Y = np.zeros((b, b), order="F")
    ms = np.zeros(8)
    st = ctypes.c_int(0)
    D = ctypes.POINTER(ctypes.c_double)
    gpu.tp_debug_chol_inv(W.ctypes.data_as(D), ctypes.byref(ctypes.c_int(b)), ctypes.byref(ctypes.c_double(rel)),
                          ctypes.byref(ctypes.c_int(3)), dg.ctypes.data_as(D), Y.ctypes.data_as(D),
                          ms.ctypes.data_as(D), ctypes.byref(st))
    assert st.value == 0
    assert ms[1] == 0, "not positive definite"
    assert np.all(np.tril(Y, -1) == 0.0)
    s = np.sqrt(np.diag(W))
    Wr = W + rel * np.diag(np.diag(W))
    kap = np.linalg.cond(Wr / s[:, None] / s[None, :])
    assert np.abs(Y.T @ Wr @ Y - np.eye(b)).max() <= 100 * b * 2.2e-16 * kap
    Uref = np.linalg.cholesky(Wr).T
    np.testing.assert_allclose(dg, np.diag(Uref), rtol=100 * b * 2.2e-16 * np.sqrt(kap))
    print(f"chol_inv b={b}: chol {ms[0] * 1e3:.1f} us (product, 4 waves for b <= 64), {ms[2] * 1e3:.1f} us (16 waves), "
          f"trsm {ms[6] * 1e3:.1f} us; cycles prologue {ms[3]:.0f} factor {ms[4]:.0f} diag {ms[5]:.0f}")


def _q_from_reflectors(A, tau, b):
    """Q = H_0 H_1 ... H_{b-3} (LAPACK dsytrd 'L' storage: u[j+1] = 1,
    u[r] = A[r, j] for r >= j+2)."""
    Q = np.eye(b)
    for j in range(b - 3, -1, -1):
        u = np.zeros(b)
        u[j + 1] = 1.0
        u[j + 2:] = A[j + 2:, j]
        Q = Q - tau[j] * np.outer(u, u @ Q)
    return Q


@pytest.mark.parametrize("b,which", [(256, 0), (96, 0), (256, 2), (240, 2), (208, 2), (200, 2), (96, 2), (48, 2),
                                     (33, 2), (16, 2), (5, 2), (3, 2)])
def test_sytrd_kernels(gpu, b, which):
    """Tridiagonalisation kernels of the Rayleigh-Ritz eigensolver: Q'HQ = T
    with Q from the stored reflectors (bar ~ b eps |H|) and Q orthogonal;
    which = 2: the 32 x 32-tile register kernel (the product path for b <=
    256), 0: the L2-resident one (b > 256)."""
    import ctypes
    rng = np.random.default_rng(b)
    h = rng.standard_normal((b, b))
    h = np.asfortranarray(h + h.T)
    hl = np.asfortranarray(np.tril(h))   # only the lower triangle is read
    d = np.zeros(b); e = np.zeros(b); tau = np.zeros(b)
    A = np.zeros((b, b), order="F")
    ms = np.zeros(8)
    st = ctypes.c_int(0)
    D = ctypes.POINTER(ctypes.c_double)
    gpu.tp_debug_sytrd2(hl.ctypes.data_as(D), ctypes.byref(ctypes.c_int(b)), ctypes.byref(ctypes.c_int(which)),
                        ms.ctypes.data_as(D), d.ctypes.data_as(D), e.ctypes.data_as(D), tau.ctypes.data_as(D),
                        A.ctypes.data_as(D), ctypes.byref(st))
    assert st.value == 0
    Q = _q_from_reflectors(A, tau, b)
    Tm = np.diag(d) + np.diag(e[:b - 1], 1) + np.diag(e[:b - 1], -1)
    scale = np.abs(h).max()
    print(f"sytrd b={b} kernel={['l2', '-', 'reg32'][which]}: {ms[0] * 1e3:.1f} us")
    # run-to-run determinism (three more calls, identical bits)
    for _ in range(3):
        d2 = np.zeros(b); e2 = np.zeros(b); t2 = np.zeros(b); A2 = np.zeros((b, b), order="F")
        gpu.tp_debug_sytrd2(hl.ctypes.data_as(D), ctypes.byref(ctypes.c_int(b)), ctypes.byref(ctypes.c_int(which)),
                            ms.ctypes.data_as(D), d2.ctypes.data_as(D), e2.ctypes.data_as(D),
                            t2.ctypes.data_as(D), A2.ctypes.data_as(D), ctypes.byref(st))
        assert st.value == 0
        assert np.array_equal(d2, d) and np.array_equal(e2, e) and np.array_equal(t2, tau) and np.array_equal(A2, A)
    assert np.abs(Q.T @ h @ Q - Tm).max() <= 200 * b * 2.2e-16 * scale
    assert np.abs(Q.T @ Q - np.eye(b)).max() <= 100 * b * 2.2e-16


# ---------------------------------------------------------- coniss / dist

@pytest.mark.parametrize("n,c,seed", [(2, 1, 0), (3, 1, 1), (50, 1, 2), (97, 7, 3), (300, 64, 4), (300, 65, 5),
                                      (400, 200, 6), (513, 256, 7)])
def test_coniss_bit_exact(gpu, n, c, seed):
    rng = np.random.default_rng(seed)
    p = rng.standard_normal((n, c)) * rng.random(c)[None, :] * 10
    merge, h, bnd = G.coniss(p)
    ma, mb, co, he = O.coniss(p)
    assert np.array_equal(bnd, mb)
    assert np.array_equal(h, he)               # canonical order: bit-identical
    # hclust merge matrix (R/TADpole.R:465; cutree / ggdendro consume it)
    assert np.array_equal(merge, O.hclust_merge(ma, mb, n))
    # cutree from merge + height alone reproduces every cut's segments
    for kk in sorted({1, 2, min(n, 3), min(n, 7), n // 2 or 1, n}):
        assert np.array_equal(O.hclust_cutree(merge, n, kk), O.cutree_labels(mb, n, kk)), kk


def test_coniss_ties_leftmost(gpu):
    p = np.repeat(np.arange(6.0), 2)[:, None]  # equal adjacent pairs everywhere
    _, h, bnd = G.coniss(p)
    _, mb, _, he = O.coniss(p)
    assert np.array_equal(bnd, mb)
    assert np.array_equal(h, he)


def test_coniss_matches_distance_matrix_definition(gpu):
    rng = np.random.default_rng(9)
    p = rng.standard_normal((80, 5))
    _, h, bnd = G.coniss(p)
    mb, he = O.coniss_bruteforce(p)
    assert np.array_equal(bnd, mb)
    np.testing.assert_allclose(h, he, rtol=1e-10)


@pytest.mark.parametrize("n,c", [(2, 1), (33, 3), (300, 20)])
def test_dist_r_order_bit_exact(gpu, n, c):
    from scipy.spatial.distance import pdist
    rng = np.random.default_rng(n)
    p = rng.standard_normal((n, c))
    d = G.dist(p)
    assert np.array_equal(d, O.dist_r(p))
    np.testing.assert_allclose(d, pdist(p), rtol=1e-13)


# -------------------------------------------------------------------- ch

def test_ch_single(gpu):
    from sklearn.metrics import calinski_harabasz_score
    rng = np.random.default_rng(5)
    p = rng.standard_normal((150, 30))
    lab = np.repeat(np.arange(1, 7), 25)
    v = G.ch(p, lab)
    np.testing.assert_allclose(v, calinski_harabasz_score(p, lab), rtol=1e-12)
    assert np.isnan(G.ch(p, np.ones(150, np.int32)))   # cn = 1: 0/0 as in fpc


# ----------------------------------------------------------------- sweep

@pytest.mark.parametrize("n0,k,seed", [(200, 200, 20261016), (420, 60, 12), (700, 200, 13)])
def test_sweep_bit_exact(gpu, n0, k, seed):
    p = _pcs(n0, seed, k)
    got = G.sweep_dev(p)
    ref = O.sweep(p)
    assert np.array_equal(got["n_cluster"], ref.n_cluster)
    assert np.array_equal(got["mrg_b"], ref.mrg_b)
    assert np.array_equal(got["mrg_a"], ref.mrg_a)
    assert np.array_equal(got["height"], ref.height)
    a, b = got["scores"], ref.scores
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))   # incl. NA bit patterns


def _structured_pcs(n, k, seed):
    """Piecewise-constant PC scores + noise (TAD-like segments of 10-60 bins)."""
    rng = np.random.default_rng(seed)
    cuts = np.cumsum(rng.integers(10, 60, size=n))
    seg = np.searchsorted(cuts, np.arange(n), side="right")
    means = rng.standard_normal((seg.max() + 1, k)) * (1.0 / (1 + np.arange(k)))
    return means[seg] + 0.05 * rng.standard_normal((n, k))


@pytest.mark.parametrize("n,k,seed", [(10600, 6, 3), (20000, 3, 4), (38000, 2, 5), (40000, 2, 6)])
def test_sweep_bit_exact_global_variant(gpu, n, k, seed):
    # 10.6k / 20k: 6 block-minimum slots; 38k: 11 slots with 16-bit LDS links
    # (the largest size they fit); 40k: links in global memory whatever lu says
    # n beyond the LDS capacity (10 200): the CONISS keeps its costs in global
    # memory, its links as 16-bit indices in LDS (40k: in global memory too)
    # -- the C5 arm sizes
    p = _structured_pcs(n, k, seed)
    got = G.sweep_dev(p)
    ref = O.sweep(p)
    assert np.array_equal(got["n_cluster"], ref.n_cluster)
    assert np.array_equal(got["mrg_b"], ref.mrg_b)
    assert np.array_equal(got["height"], ref.height)
    assert np.array_equal(got["scores"].view(np.uint64), ref.scores.view(np.uint64))


def test_sweep_selection_and_bstick_r_faithful(gpu):
    p = _pcs(300, 21)
    got = G.sweep(p)
    ref = O.sweep(p)
    ld = O.sweep(p, bstick="ld")                # R's long double cumsum decides the same
    assert np.array_equal(ref.n_cluster, ld.n_cluster)
    assert (got["n_pcs"], got["n_clusters"]) == O.select_params(ref.scores)


@pytest.mark.parametrize("ucap", [0, 7])
def test_sweep_shared_segment_stats(gpu, ucap):
    """CH segment statistics shared across trees (k_ch_cut / k_ch_segstat) give
    the oracle's bits -- also when the shared store overflows (ucap 7, knob 1:
    most segments take the per-tree fallback)."""
    p = _pcs(700, 13, 200)
    old = G.knob(1, ucap)
    try:
        got = G.sweep_dev(p)
    finally:
        G.knob(1, old)
    ref = O.sweep(p)
    assert np.array_equal(got["n_cluster"], ref.n_cluster)
    assert np.array_equal(got["scores"].view(np.uint64), ref.scores.view(np.uint64))


@pytest.mark.parametrize("mc", [1, 2, 5, 50])
def test_sweep_min_clusters(gpu, mc):
    p = _pcs(250, 22, 40)
    got = G.sweep_dev(p, min_clusters=mc)
    ref = O.sweep(p, min_clusters=mc)
    assert np.array_equal(got["scores"].view(np.uint64), ref.scores.view(np.uint64))


# -------------------------------------------------------------- pipeline

@pytest.mark.parametrize("n0,seed,max_pcs", [(200, 20261016, 200), (150, 5, 200), (600, 6, 200),
                                              (900, 7, 50), (64, 8, 10)])
def test_pipeline_end_to_end(gpu, n0, seed, max_pcs):
    import tadpole_amd as tp
    m = synth_hic(n0, seed)
    got = tp.TADpole(m, max_pcs=max_pcs)
    ref = O.tadpole(m, max_pcs=max_pcs)
    assert got.n_pcs == ref.n_pcs
    assert got.optimal_n_clusters == ref.optimal_n_clusters
    assert set(got.clusters) == {str(q) for q in ref.clusters}
    for q, v in ref.clusters.items():
        assert np.array_equal(got.clusters[str(q)], v), q
    assert np.array_equal(got.bad_columns, np.flatnonzero(ref.bad) + 1)
    a, b = got.scores, ref.scores
    assert a.shape == b.shape
    fin = ~np.isnan(b)
    assert np.array_equal(np.isnan(a), ~fin)
    assert np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin])) < 1e-6
    np.testing.assert_allclose(got.dendro.height, ref.height, rtol=1e-8)


def test_pipeline_file_input_and_nan(gpu, tmp_path):
    import tadpole_amd as tp
    m = synth_hic(180, 31).astype(float)
    m[3, 100] = np.nan
    f = tmp_path / "m.tsv"
    np.savetxt(f, m, delimiter="\t", fmt="%.17g")
    got = tp.TADpole(str(f))
    ref = O.tadpole(m)
    assert (got.n_pcs, got.optimal_n_clusters) == (ref.n_pcs, ref.optimal_n_clusters)


def test_read_tsv_dev_blocks_equal_host_parse(gpu, tmp_path):
    # tp_read_tsv_dev (parse in 8 row blocks on 4 threads, each block's upload
    # overlapping the next block's parse) gives the host parser's bits: reals,
    # NA, a short line padded with NaN, CRLF line ends
    import ctypes
    import torch
    from tadpole_amd import _lib, read_matrix
    rng = np.random.default_rng(7)
    n = 400
    m = rng.standard_normal((n, n)) * 1e3
    lines = ["\t".join(f"{v:.17g}" for v in row) for row in m]
    lines[5] = lines[5].replace(lines[5].split("\t")[7], "NA", 1)
    lines[9] = "\t".join(lines[9].split("\t")[:n - 3])
    f = tmp_path / "blocks.tsv"
    f.write_bytes(("\r\n".join(lines) + "\r\n").encode())
    host = read_matrix(str(f))
    assert np.isnan(host[5, 7]) and np.all(np.isnan(host[9, n - 3:]))
    d = torch.full((n, n), -1.0, dtype=torch.float64, device="cuda:0")
    st = ctypes.c_int(0)
    path = ctypes.c_char_p(str(f).encode())
    s = torch.cuda.current_stream(0)
    gpu.tp_read_tsv_dev(ctypes.byref(path), ctypes.byref(ctypes.c_int(n)), ctypes.byref(ctypes.c_int(n)),
                        ctypes.byref(ctypes.c_int(4)), ctypes.byref(ctypes.c_int(0)), ctypes.c_void_p(s.cuda_stream),
                        ctypes.c_void_p(d.data_ptr()), ctypes.byref(st))
    _lib.check(st)
    got = d.cpu().numpy()
    assert np.array_equal(got.view(np.uint64)[~np.isnan(host)], host.view(np.uint64)[~np.isnan(host)])
    assert np.array_equal(np.isnan(got), np.isnan(host))
    # wrong row count: an argument error, not a partial matrix
    gpu.tp_read_tsv_dev(ctypes.byref(path), ctypes.byref(ctypes.c_int(n + 1)), ctypes.byref(ctypes.c_int(n)),
                        ctypes.byref(ctypes.c_int(4)), ctypes.byref(ctypes.c_int(0)), ctypes.c_void_p(s.cuda_stream),
                        ctypes.c_void_p(d.data_ptr()), ctypes.byref(st))
    assert st.value == _lib.TP_ERR_ARG


def test_pipeline_errors(gpu):
    import tadpole_amd as tp
    with pytest.raises(tp.TadpoleError):
        tp.TADpole(np.zeros((10, 10)))         # everything bad


# ------------------------------------------------------ X'X int8-exact path

def _xtx(gpu, x, mode):
    import ctypes
    n = x.shape[0]
    xf = np.asfortranarray(x, np.float64)
    S = np.zeros((n, n), order="F")
    ns = ctypes.c_int(-1); ms = ctypes.c_double(0); st = ctypes.c_int(0)
    D = ctypes.POINTER(ctypes.c_double)
    gpu.tp_debug_xtx(xf.ctypes.data_as(D), ctypes.byref(ctypes.c_int(n)), ctypes.byref(ctypes.c_int(mode)),
                     S.ctypes.data_as(D), ctypes.byref(ns), ctypes.byref(ms), ctypes.byref(st))
    return S, ns.value, ms.value, st.value


def _exact_xtx(x):
    """X'X of a non-negative integer matrix, exactly: in float64 (BLAS) every
    partial sum is an integer below 2^53 when n * max^2 < 2^53, so any summation
    order is exact; numpy's int64 product (no BLAS) otherwise."""
    n, mx = x.shape[0], float(x.max())
    if n * mx * mx < 2.0 ** 53:
        return x.T @ x
    xi = x.astype(np.int64)
    return (xi.T @ xi).astype(np.float64)


@pytest.mark.parametrize("n,maxv,slices", [(64, 100, 1), (200, 5000, 2), (515, 16383, 2), (1000, 3000, 2),
                                           (333, 2_000_000, 3), (2000, 4000, 2), (1100, 120, 1),
                                           (1500, 16000, 2), (4100, 9000, 2)])
def test_xtx_int8_exact(gpu, n, maxv, slices):
    """sparse_cor's crossprod (R/TADpole.R:96) on the int8 matrix cores: for
    integer counts the product is EXACT -- equal to numpy's int64 X'X rounded
    once to double -- and symmetric; ragged n (not a multiple of 64)."""
    rng = np.random.default_rng(n + maxv)
    x = rng.integers(0, maxv, size=(n, n)).astype(np.float64)
    x[0, 0] = maxv - 1
    S, ns, ms, st = _xtx(gpu, x, 1)
    assert st == 0 and ns == slices
    ref = _exact_xtx(x)
    assert np.array_equal(S, ref)
    S64, _, ms64, st64 = _xtx(gpu, x, 0)
    assert st64 == 0
    assert np.max(np.abs(S64 - ref) / np.maximum(ref, 1)) < 1e-13
    print(f"xtx n={n} slices={ns}: int8 {ms * 1e3:.1f} us, fp64 {ms64 * 1e3:.1f} us")


@pytest.mark.parametrize("wide", [1, 0])
@pytest.mark.parametrize("n,maxv,slices", [(1100, 120, 1), (1500, 16000, 2), (2000, 127, 1), (4100, 9000, 2),
                                           (1025, 300, 2), (300, 9000, 2), (130, 50, 1)])
def test_xtx_int8_tiles128_exact(gpu, n, maxv, slices, wide):
    """The pipeline's whole-triangle int8 X'X kernels -- k_xtx_i8_w's 256 x 128
    tiles (knob 44 = 1) and the 128-tile LDS-DMA ring: exact X'X at ragged n (odd tile-column counts:
    the last 256-row panel past the padded columns), both slice counts."""
    rng = np.random.default_rng(n * 3 + maxv)
    x = rng.integers(0, maxv, size=(n, n)).astype(np.float64)
    x[0, 0] = maxv - 1
    oldw = G.knob(44, wide)
    try:
        S, ns, ms, st = _xtx(gpu, x, 2)
    finally:
        G.knob(44, oldw)
    assert st == 0 and ns == slices
    assert np.array_equal(S, _exact_xtx(x))
    print(f"xtx128 n={n} slices={ns} wide={wide}: {ms * 1e3:.1f} us")


@pytest.mark.parametrize("wide", [1, 0])
@pytest.mark.parametrize("n", [1100, 3000, 4100])
def test_xtx_int8_tiles128_sparse_high_slice(gpu, n, wide):
    """Counts >= 128 only in a band around the diagonal and at a few scattered
    entries (raw Hi-C): the LDS-DMA kernels skip the high slice's all-zero
    128 x 64 blocks (k_xtx_i8_w, knob 44, takes the nonzero ones in
    its second phase) and the product stays exact."""
    rng = np.random.default_rng(n)
    x = rng.integers(0, 128, size=(n, n)).astype(np.float64)
    i = np.arange(n)
    for d in range(-5, 6):
        j = i + d
        ok = (j >= 0) & (j < n)
        x[i[ok], j[ok]] = rng.integers(128, 16000, size=int(ok.sum()))
    r, c = rng.integers(0, n, 40), rng.integers(0, n, 40)
    x[r, c] = 15000
    old44 = G.knob(44, wide)
    try:
        S, ns, ms, st = _xtx(gpu, x, 2)
    finally:
        G.knob(44, old44)
    assert st == 0 and ns == 2
    assert np.array_equal(S, _exact_xtx(x))
    print(f"xtx128 sparse-high n={n} wide={wide}: {ms * 1e3:.1f} us")


@pytest.mark.parametrize("n,maxv", [(515, 16000), (1100, 9000), (1100, 120)])
def test_xtx_int8_exact_fresh_context(gpu, n, maxv):
    """Regression for the out-of-bounds slice reads fixed in 5295f4f (64-tile
    int8 X'X kernel: slice tiles counted from the padded k stride; it faulted
    only when the scratch was exactly sized).  tp_shutdown() frees every
    context, so this call runs with freshly allocated, exactly sized scratch
    at ragged n (not a multiple of 64)."""
    gpu.tp_shutdown()
    rng = np.random.default_rng(n * 7 + maxv)
    x = rng.integers(0, maxv, size=(n, n)).astype(np.float64)
    S, ns, _, st = _xtx(gpu, x, 1)
    assert st == 0 and ns >= 1
    assert np.array_equal(S, _exact_xtx(x))


def test_xtx_int8_rejects_non_counts(gpu):
    x = np.random.default_rng(0).random((100, 100))
    _, _, _, st = _xtx(gpu, x, 1)
    assert st == 1
    x = -np.ones((80, 80))
    _, _, _, st = _xtx(gpu, x, 1)
    assert st == 1


# ------------------------------------------------ fp64 GEMM kernels agree

def _gemm(gpu, A, B, M, N, K, ta, sym, kernel):
    import ctypes
    C = np.zeros((M, N), order="F")
    ms = ctypes.c_double(0); st = ctypes.c_int(0)
    D = ctypes.POINTER(ctypes.c_double)
    I = lambda v: ctypes.byref(ctypes.c_int(v))  # noqa: E731
    gpu.tp_debug_gemm(A.ctypes.data_as(D), B.ctypes.data_as(D), I(M), I(N), I(K), I(ta), I(sym), I(kernel),
                      C.ctypes.data_as(D), ctypes.byref(ms), ctypes.byref(st))
    assert st.value == 0
    return C, ms.value


@pytest.mark.parametrize("M,N,K,ta,sym", [(1500, 1500, 700, 1, 1), (16500, 256, 600, 1, 0), (16500, 200, 300, 0, 0),
                                          (3000, 3000, 1000, 1, 1)])
def test_gemm_big_tiles_same_bits(gpu, M, N, K, ta, sym):
    """The 128 x 128 fp64 MFMA kernel keeps the k order of the 64 x 64 one: the
    products agree bit for bit (so shard layouts / tile choices never change
    results), and both match numpy to ~K eps."""
    rng = np.random.default_rng(M + N + K)
    A = np.asfortranarray(rng.standard_normal((K, M) if ta else (M, K)))
    B = np.asfortranarray(A if sym else rng.standard_normal((K, N)))
    c0, t0 = _gemm(gpu, A, B, M, N, K, ta, sym, 0)
    c1, t1 = _gemm(gpu, A, B, M, N, K, ta, sym, 1)
    assert np.array_equal(c0.view(np.uint64), c1.view(np.uint64))
    ref = (A.T if ta else A) @ B
    assert np.abs(c1 - ref).max() <= 1e-13 * np.abs(ref).max() * np.sqrt(K)
    print(f"gemm {M}x{N}x{K} sym={sym}: 64-tile {t0 * 1e3:.0f} us, 128-tile {t1 * 1e3:.0f} us")


@pytest.mark.parametrize("M,N,K,ta", [(1980, 256, 1980, 1), (1980, 200, 1980, 1), (1980, 256, 256, 0),
                                      (4100, 130, 1001, 1), (8000, 64, 333, 0)])
def test_gemm_panel_same_bits(gpu, M, N, K, ta):
    """The 32 x 64 tall-skinny kernel (Z = G Q, scores, Ritz rotation) keeps the
    k order of the 64 x 64 kernel without split-K: identical bits; timings of
    the panel kernel vs the split-K policy it replaces are printed."""
    rng = np.random.default_rng(M * 3 + N + K)
    A = np.asfortranarray(rng.standard_normal((K, M) if ta else (M, K)))
    B = np.asfortranarray(rng.standard_normal((K, N)))
    c0, t0 = _gemm(gpu, A, B, M, N, K, ta, 0, 0)
    c2, t2 = _gemm(gpu, A, B, M, N, K, ta, 0, 2)
    c3, t3 = _gemm(gpu, A, B, M, N, K, ta, 0, 3)
    t2 = min(t2, _gemm(gpu, A, B, M, N, K, ta, 0, 2)[1])
    t3 = min(t3, _gemm(gpu, A, B, M, N, K, ta, 0, 3)[1])
    if K < 512:   # the panel kernel's range (longer K keeps the split-K policy)
        assert np.array_equal(c0.view(np.uint64), c2.view(np.uint64))
    ref = (A.T if ta else A) @ B
    assert np.abs(c2 - ref).max() <= 1e-13 * np.abs(ref).max() * np.sqrt(K)
    assert np.abs(c3 - ref).max() <= 1e-13 * np.abs(ref).max() * np.sqrt(K)
    tf = 2.0 * M * N * K / 1e9
    print(f"gemm {M}x{N}x{K}: 64-tile {t0 * 1e3:.1f} us, panel {t2 * 1e3:.1f} us ({tf / t2:.1f} TF/s), "
          f"split-K policy {t3 * 1e3:.1f} us ({tf / t3:.1f} TF/s)")


def test_gemm_splitk_sweep(gpu):
    """Z = G Q at the C2 shape with every split-K factor: all agree with numpy
    to ~K eps (timings printed; the policy in gemm_f64 picks from them)."""
    M, N, K = 1980, 256, 1980
    rng = np.random.default_rng(7)
    A = np.asfortranarray(rng.standard_normal((K, M)))
    B = np.asfortranarray(rng.standard_normal((K, N)))
    ref = A.T @ B
    for S in (1, 2, 3, 4, 6, 8, 12, 16):
        for kb, base in ((32, 10), (16, 110)):
            c, t = _gemm(gpu, A, B, M, N, K, 1, 0, base + S)
            t = min(t, _gemm(gpu, A, B, M, N, K, 1, 0, base + S)[1], _gemm(gpu, A, B, M, N, K, 1, 0, base + S)[1])
            assert np.abs(c - ref).max() <= 1e-13 * np.abs(ref).max() * np.sqrt(K)
            if kb == 32:
                c32 = c
            else:   # the stage depth never changes the k order
                assert np.array_equal(c.view(np.uint64), c32.view(np.uint64))
            print(f"splitk {S} stage {kb}: {t * 1e3:.1f} us, {2.0 * M * N * K / t / 1e9:.1f} TF/s")


@pytest.mark.parametrize("M,N,K", [(3000, 64, 4100), (1300, 200, 5000), (7729, 64, 7729), (24300, 200, 4096)])
def test_gemm_rows_kernel_row_independent(gpu, M, N, K):
    """The 128 x 64 long-K kernel of the PCA's Xc products (k chunks fixed by K):
    any row slice of the product -- a row shard on another GPU -- has the bits of
    the same rows of the full product; repeat runs are identical; numpy to ~K eps."""
    rng = np.random.default_rng(M + 7 * N + K)
    A = np.asfortranarray(rng.standard_normal((K, M)))
    B = np.asfortranarray(rng.standard_normal((K, N)))
    c, t = _gemm(gpu, A, B, M, N, K, 1, 0, 4)
    c2, _ = _gemm(gpu, A, B, M, N, K, 1, 0, 4)
    assert np.array_equal(c.view(np.uint64), c2.view(np.uint64))
    for r0, r1 in ((0, 64), (640, 1280), (M - 193, M)):
        cs, _ = _gemm(gpu, np.asfortranarray(A[:, r0:r1]), B, r1 - r0, N, K, 1, 0, 4)
        assert np.array_equal(cs.view(np.uint64), c[r0:r1].view(np.uint64)), (r0, r1)
    ref = A.T @ B
    assert np.abs(c - ref).max() <= 1e-13 * np.abs(ref).max() * np.sqrt(K)
    print(f"rows gemm {M}x{N}x{K}: {t * 1e3:.1f} us, {2.0 * M * N * K / t / 1e9:.1f} TF/s")


@pytest.mark.parametrize("K,M,N", [(4100, 302, 64), (7808, 130, 64), (4160, 9, 64), (9000, 200, 64),
                                   (4100, 302, 32), (9000, 330, 32), (4160, 9, 32)])
def test_prod_i8_digit_product(gpu, K, M, N):
    """The Krylov products on the int8 MFMA (digit images, knob 36) against
    an 80-bit reference of the same A'B with the rank-1 epilogue: within
    1e-14 of sum |A||B| elementwise (measured 5e-16..9e-16 with six digits of
    A; the fp64 k_gemm_ts path ~5e-17).
    Columns with a non-unit scale, a zero column and a column of ones (the
    [C | m | 1] layout) ride along."""
    import ctypes
    rng = np.random.default_rng(K + M + N)
    A = rng.uniform(-1, 1, size=(K, M))
    A[:, 3] *= 1e-5
    A[:, 5] = 0.0
    A[:, 7] *= 37.5
    A[:, M - 1] = 1.0
    B = rng.standard_normal((K, N)) / np.sqrt(K)
    B[:, 1] *= 1e6
    Af, Bf = np.asfortranarray(A), np.asfortranarray(B)
    O8 = np.zeros((M - 1, N), order="F")
    O64 = np.zeros((M - 1, N), order="F")
    ms = np.zeros(2)
    st = ctypes.c_int(0)
    D = ctypes.POINTER(ctypes.c_double)
    I = lambda v: ctypes.byref(ctypes.c_int(v))  # noqa: E731
    gpu.tp_debug_prod_i8(Af.ctypes.data_as(D), I(K), I(M), Bf.ctypes.data_as(D), I(N), O8.ctypes.data_as(D),
                         O64.ctypes.data_as(D), ms.ctypes.data_as(D), ctypes.byref(st))
    assert st.value == 0
    P = A.astype(np.longdouble).T @ B.astype(np.longdouble)
    ref = (P[:M - 1] - P[M - 1]).astype(np.float64)
    absP = np.abs(A).T @ np.abs(B)
    bound = absP[:M - 1] + absP[M - 1]
    e8 = float(np.max(np.abs(O8 - ref) / bound))
    e64 = float(np.max(np.abs(O64 - ref) / bound))
    print(f"prod_i8 K={K} M={M} N={N}: int8 {ms[0] * 1e3:.1f} us err {e8:.2e} | fp64 {ms[1] * 1e3:.1f} us err {e64:.2e}")
    assert e8 < 1e-14


def _digits_ref(x, nd):
    """The digit image's restatement for one column: e from the largest |x|
    (frexp, clamped at -968), q = rint(x 2^(54 - e)), balanced base-256 digits
    least significant first (d = the signed low byte of r, r = (r - d) / 256),
    the top digit last; the first nd digits, most significant first."""
    mx = np.max(np.abs(x)) if x.size else 0.0
    e = max(int(np.frexp(mx)[1]) if mx > 0 else 0, -968)
    q = np.rint(x * np.ldexp(1.0, 54 - e)).astype(np.int64)
    r = q.copy()
    dig = [None] * 7
    for s in range(6, 0, -1):
        d = ((r & 0xFF) ^ 0x80) - 0x80
        dig[s] = d
        r = (r - d) >> 8
    dig[0] = r
    return np.stack(dig[:nd]).astype(np.int8), np.ldexp(1.0, e - 54)


@pytest.mark.parametrize("K,M", [(7729, 260), (1000, 67), (4160, 130), (9000, 70), (20000, 66)])
@pytest.mark.parametrize("fused", [1, 0])
def test_pd_image_digits_and_fused_means(gpu, K, M, fused):
    """A's int8 digit image against the restated digitisation (every byte, the
    pd_off layout: ((c / 64) Kp / 64 + k / 64) ND 4096 + s 4096 + (c % 64) 64 +
    k % 64), the per-column scales, zero digits past K and past M; with fused
    = 1 (k_pd_digits_cm, the PCA's default) the column means of the first
    M - 2 columns carry k_colmean's bits -- a zero column, tiny and huge
    columns and a column of integers ride along.  K > 8192: the 1024-thread
    register digitiser (the C-space path's long columns; no fused means there)."""
    import ctypes
    if fused and K > 8192:
        pytest.skip("the fused means are for K <= 8192")
    rng = np.random.default_rng(K + M)
    A = rng.uniform(-1, 1, size=(K, M))
    A[:, 1] = 0.0
    A[:, 4] *= 1e-9
    A[:, 6] *= 3.7e12
    A[:, 9] = np.rint(A[:, 9] * 1000)
    A[:, M - 2] = A[:, :M - 2].mean(axis=0)[:K] if K <= M - 2 else rng.uniform(-1, 1, K)
    A[:, M - 1] = 1.0
    A = np.asfortranarray(A)
    cp = (M + 63) // 64 * 64
    Kp = (K + 63) // 64 * 64
    img = np.zeros(7 * cp * Kp, dtype=np.int8)
    scale = np.zeros(cp)
    cm = np.zeros(M - 2)
    cm_ref = np.zeros(M - 2)
    nd = ctypes.c_int(0)
    st = ctypes.c_int(0)
    D = ctypes.POINTER(ctypes.c_double)
    I = lambda v: ctypes.byref(ctypes.c_int(v))  # noqa: E731
    gpu.tp_debug_pd_image(A.ctypes.data_as(D), I(K), I(M), I(fused), img.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)),
                          scale.ctypes.data_as(D), cm.ctypes.data_as(D), cm_ref.ctypes.data_as(D), ctypes.byref(nd),
                          ctypes.byref(st))
    assert st.value == 0
    ND = nd.value
    nsteps = Kp // 64
    # image[tile, kstep, s, col % 64, k % 64]
    im = img[:ND * cp * Kp].reshape(cp // 64, nsteps, ND, 64, 64)
    for c in range(cp):
        got = im[c // 64, :, :, c % 64, :].transpose(1, 0, 2).reshape(ND, Kp)
        if c >= M:
            assert not got.any() and scale[c] == 0.0, c
            continue
        ref, sc = _digits_ref(A[:, c], ND)
        assert scale[c] == sc, c
        assert np.array_equal(got[:, :K], ref), c
        assert not got[:, K:].any(), c
    if fused:
        assert np.array_equal(cm.view(np.uint64), cm_ref.view(np.uint64))
    import math
    exact = np.array([math.fsum(A[:, j]) / K for j in range(M - 2)])   # double-double: within an ulp or two
    np.testing.assert_allclose(cm_ref, exact, rtol=5e-16, atol=0)


@pytest.mark.parametrize("K", [64, 1000, 4100, 7729, 8192])
def test_prod_i8_block_digitizers(gpu, K):
    """The block's digit image by (column, 1024-row slice) workgroups
    (k_pd_digits_blk): the products against fp64 within 1e-14 of sum |A||B|,
    a NaN column (NaN products), a zero column and a huge column included."""
    import ctypes
    M = 200
    rng = np.random.default_rng(K)
    A = np.asfortranarray(rng.uniform(-1, 1, size=(K, M)))
    B = rng.standard_normal((K, 64)) / np.sqrt(K)
    B[:, 2] = 0.0
    B[:, 9] *= 1e200
    B[K // 2, 11] = np.nan
    B = np.asfortranarray(B)
    D = ctypes.POINTER(ctypes.c_double)
    I = lambda v: ctypes.byref(ctypes.c_int(v))  # noqa: E731
    O = np.zeros((M, 64), order="F")
    st = ctypes.c_int(0)
    gpu.tp_debug_prod_i8_rows(A.ctypes.data_as(D), I(K), I(M), B.ctypes.data_as(D), I(64), I(0), I(0),
                              I(M), O.ctypes.data_as(D), ctypes.byref(st))
    assert st.value == 0
    outs = [O]
    assert np.all(np.isnan(outs[0][:, 11])) and np.all(outs[0][:, 2] == 0.0)
    ok = [j for j in range(64) if j != 11]
    ref = A.T @ B[:, ok]
    assert np.abs(outs[0][:, ok] - ref).max() <= 1e-14 * (np.abs(A).T @ np.abs(B[:, ok])).max(axis=0).max()


@pytest.mark.parametrize("K,M,col0,r0", [(4100, 330, 64, 64), (9000, 300, 128, 192), (7729, 400, 0, 128)])
@pytest.mark.parametrize("kernel", [1, 5])
def test_prod_i8_rows_slab_same_bits(gpu, K, M, col0, r0, kernel):
    """A rank's row shard of an int8-digit product, from the digit image of
    its own column slab [col0, M) (the C5 schedule: tp_shard.hip), carries
    the bits of the same rows of the whole product; K > 8192 takes the
    two-pass digitizers of the block (k_pd_colmax + k_pd_digits_sl) and of
    A (k_pd_digits).  kernel: the product kernel (knob 36: 1 = k_pd_prod,
    5 = k_pd_prodA), which must agree bit for bit with each other."""
    import ctypes
    rng = np.random.default_rng(K + M + col0)
    A = np.asfortranarray(rng.uniform(-1, 1, size=(K, M)))
    A[:, 70] *= 1e-7
    B = np.asfortranarray(rng.standard_normal((K, 64)) / np.sqrt(K))
    D = ctypes.POINTER(ctypes.c_double)
    I = lambda v: ctypes.byref(ctypes.c_int(v))  # noqa: E731

    def rows(c0, q0, nr):
        O = np.zeros((nr, 64), order="F")
        st = ctypes.c_int(0)
        gpu.tp_debug_prod_i8_rows(A.ctypes.data_as(D), I(K), I(M), B.ctypes.data_as(D), I(64), I(c0), I(q0),
                                  I(nr), O.ctypes.data_as(D), ctypes.byref(st))
        assert st.value == 0
        return O

    old = G.knob(36, 1)
    try:
        base = rows(0, 0, M)
        G.knob(36, kernel)
        full = rows(0, 0, M)
        part = rows(col0, r0, M - r0)
    finally:
        G.knob(36, old)
    assert np.array_equal(full.view(np.uint64), base.view(np.uint64))
    assert np.array_equal(part.view(np.uint64), full[r0:].view(np.uint64))
    ref = A.T @ B
    assert np.abs(full - ref).max() <= 1e-14 * (np.abs(A).T @ np.abs(B)).max()


# ------------------------------------------------------------------- upload

def test_upload_counts_bit_exact(gpu):
    """tp_upload_counts_dev (tp_pipeline's host path, and the stream path of
    TADpole() on a host matrix): 16 MB blocks of exact 16-bit counts travel
    packed and are widened on the device; every other block (a fraction, NaN
    with a payload, -0.0, 65536, a negative count) travels as float64 -- the
    device copy equals the host matrix bit for bit either way; tp_upload_dev
    copies raw bytes."""
    import ctypes
    import torch
    blk = (16 << 20) // 8                       # values a block
    n = 5 * blk + 12345                         # ragged last block
    rng = np.random.default_rng(3)
    h = rng.integers(0, 65536, n).astype(np.float64)
    specials = {1: 0.5, 2: np.frombuffer(np.uint64(0x7FF8000000000123).tobytes(), np.float64)[0],
                3: -0.0, 4: 65536.0}
    for b, v in specials.items():
        h[b * blk + 777] = v
    h[5 * blk + 5] = -1.0                       # the ragged block
    d = torch.empty(n, dtype=torch.float64, device="cuda:0")
    packed = ctypes.c_longlong(0)
    st = ctypes.c_int(0)
    s = torch.cuda.Stream()
    old = G.knob(43, 3)   # packed count blocks, uploads in turn (both paths of the switch)
    try:
        _upload_checks(gpu, h, d, n, blk, packed, st, s, rng)
    finally:
        G.knob(43, old)


def _upload_checks(gpu, h, d, n, blk, packed, st, s, rng):
    import ctypes
    import torch
    gpu.tp_upload_counts_dev(ctypes.c_void_p(h.ctypes.data), ctypes.byref(ctypes.c_longlong(n)),
                             ctypes.c_void_p(d.data_ptr()), ctypes.byref(ctypes.c_int(4)), ctypes.byref(ctypes.c_int(0)),
                             ctypes.c_void_p(s.cuda_stream), ctypes.byref(packed), ctypes.byref(st))
    assert st.value == 0
    out = d.cpu().numpy()
    assert np.array_equal(out.view(np.uint64), h.view(np.uint64))
    assert packed.value == 16 << 20             # only block 0 is all counts
    # all counts: everything packed; raw copy of arbitrary bytes
    h2 = rng.integers(0, 1000, 3 * blk).astype(np.float64)
    d2 = torch.empty(3 * blk, dtype=torch.float64, device="cuda:0")
    gpu.tp_upload_counts_dev(ctypes.c_void_p(h2.ctypes.data), ctypes.byref(ctypes.c_longlong(h2.size)),
                             ctypes.c_void_p(d2.data_ptr()), ctypes.byref(ctypes.c_int(1)), ctypes.byref(ctypes.c_int(0)),
                             ctypes.c_void_p(s.cuda_stream), ctypes.byref(packed), ctypes.byref(st))
    assert st.value == 0 and packed.value == h2.nbytes
    assert np.array_equal(d2.cpu().numpy(), h2)
    raw = rng.standard_normal(blk + 3)
    d3 = torch.empty(blk + 3, dtype=torch.float64, device="cuda:0")
    gpu.tp_upload_dev(ctypes.c_void_p(raw.ctypes.data), ctypes.byref(ctypes.c_longlong(raw.nbytes)),
                      ctypes.c_void_p(d3.data_ptr()), ctypes.byref(ctypes.c_int(2)), ctypes.byref(ctypes.c_int(0)),
                      ctypes.c_void_p(s.cuda_stream), ctypes.byref(st))
    assert st.value == 0
    assert np.array_equal(d3.cpu().numpy().view(np.uint64), raw.view(np.uint64))


@pytest.mark.parametrize("n,k,seed", [(150, 5, 31), (1999, 70, 32), (4100, 200, 33), (7729, 200, 34),
                                      (9500, 24, 35), (3000, 256, 36), (11000, 12, 37), (24300, 66, 38),
                                      (40000, 3, 39)])
def test_coniss_batched_same_bits(gpu, n, k, seed):
    """The batched CONISS (k_coniss_b, knob 52: candidate runs taken several
    merges at a time by 8 waves a tree) gives every tree's merge order, costs,
    heights, broken-stick count and CH scores of the two-wave kernel bit for
    bit (the run rule of tools/coniss_batch_model.py), on TAD-like scores with
    1..256 PCs (1..4 column slots, 1..3 block-minimum slots) -- storage mode 0
    (everything in LDS), 11 000 bins mode 1 (16-bit links), 24 300 and 40 000
    bins mode 2 (costs in global memory, 6 and 11 block-minimum slots)."""
    p = _structured_pcs(n, k, seed)
    old = G.knob(52, 0)
    try:
        ref = G.sweep_dev(p)
        G.knob(52, 1)
        got = G.sweep_dev(p)
    finally:
        G.knob(52, old)
    for f in ("n_cluster", "mrg_a", "mrg_b"):
        assert np.array_equal(got[f], ref[f]), f
    for f in ("cost", "height", "scores"):
        assert np.array_equal(got[f].view(np.uint64), ref[f].view(np.uint64)), f
