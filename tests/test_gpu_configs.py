"""GPU parity at the BASELINE configs (BASELINE.json configs[1..4]) and on the
paths around them, against committed oracle fixtures (tests/golden/, made by
make_golden.py from oracle/tadpole_oracle.py) or, at full C5 size, through
size-independent properties.

Bars (north_star): TAD start/end indices, n_pcs, optimal_n_clusters, bad
columns, n_cluster per tree, the final tree's boundary order and hclust merge
matrix bit-exact; CH scores within 1e-6 relative (NA pattern exact); heights
within 1e-8 relative (different PCA algorithm from LAPACK: the PC scores agree
to ~1e-12, not bit for bit).

The hclust ``merge`` comparison is oracle self-consistency: the row order of
rioja's merge matrix is restated (hclust's hcass2 convention) in both the
library and the oracle, and no reference-held fixture pins it (parity with R
unpinned).
"""
import os

import numpy as np
import pytest

import gpu_helpers as G
import tadpole_oracle as O
from tadpole_amd.synth import (SEED_BASE, early_centromere_matrix, genome_bins, genome_matrix, matrix_checksum,
                               synth_hic, synth_hic_par)

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _coords_dict(z, prefix=""):
    lev = z[prefix + "levels"]
    co = z[prefix + "coords"]
    return {int(q): co[co[:, 0] == q][:, 1:] for q in lev}


def _check(got, z, prefix="", bad=True):
    assert got.n_pcs == int(z[prefix + "n_pcs"])
    assert got.optimal_n_clusters == int(z[prefix + "optimal_n_clusters"])
    ref = _coords_dict(z, prefix)
    assert set(got.clusters) == {str(q) for q in ref}
    for q, v in ref.items():
        assert np.array_equal(got.clusters[str(q)], v), q
    if bad and (prefix + "bad_idx1") in z:
        assert np.array_equal(got.bad_columns, z[prefix + "bad_idx1"])
    a, b = got.scores, z[prefix + "scores"]
    assert a.shape == b.shape
    fin = ~np.isnan(b)
    assert np.array_equal(np.isnan(a), ~fin)
    assert np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin])) < 1e-6
    assert np.array_equal(got.dendro.boundary - 1, z[prefix + "merge_b"])
    assert np.array_equal(got.dendro.merge, z[prefix + "merge"])
    np.testing.assert_allclose(got.dendro.height, z[prefix + "height"], rtol=1e-8)


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_config_golden(gpu, name):
    """C2 (synthetic 2000 x 2000) and C3 (chr18 @10kb shape, 7808 bins), full
    size, max_pcs = 200, end to end through TADpole() vs the oracle's outputs."""
    import tadpole_amd as tp
    z = np.load(os.path.join(GOLD, f"{name}.npz"))
    m = synth_hic(int(z["n0"]), int(z["seed"]))
    got = tp.TADpole(m, max_pcs=int(z["max_pcs"]))
    _check(got, z)
    # the PCA residual the pipeline accepted (||G v - theta v|| / theta_1)
    assert got.timings_ms[13] <= 1e-11


@pytest.mark.parametrize("prod", [0, 1])
def test_config_c3_golden_product_paths(gpu, prod):
    """C3 with the Krylov products on the paths the default does not take
    (knob 36: 0 the fp64 k_gemm_ts, 1 the 64-row-tile int8-digit kernel
    k_pd_prod; the default, k_pd_prodA, is test_config_golden): the
    golden's n_pcs, clusters, merge order and every level, CH within 1e-6."""
    import tadpole_amd as tp
    z = np.load(os.path.join(GOLD, "c3.npz"))
    m = synth_hic(int(z["n0"]), int(z["seed"]))
    old = G.knob(36, prod)
    try:
        got = tp.TADpole(m, max_pcs=200)
    finally:
        G.knob(36, old)
    _check(got, z)


def test_config_c3_from_hbm(gpu):
    """C3 with the matrix already resident in HBM (a torch tensor: the bench's
    input form) gives the same result as from host memory."""
    import torch
    import tadpole_amd as tp
    z = np.load(os.path.join(GOLD, "c3.npz"))
    m = synth_hic(int(z["n0"]), int(z["seed"]))
    got = tp.TADpole(torch.from_numpy(m).cuda(), max_pcs=200)
    _check(got, z)


@pytest.mark.parametrize("forced,space", [(True, "C"), (True, "G"), (True, "G-int8"), (False, "G")])
def test_pca_krylov_path_vs_lapack(gpu, forced, space):
    """The block Krylov PCA (G never formed; Krylov space of G, the default,
    or of C: knob 20; G with the products on the int8
    MFMA from digit images -- six digits of C, seven of each block: knob 36) against LAPACK's SVD on a matrix below its default
    size threshold (forced) and the G-formed path on the same matrix: every
    prefix subspace the sweep uses agrees."""
    n0 = 2600
    m = synth_hic(n0, SEED_BASE + 77)
    cm = O.clean_symmetrize(m)
    obad, _, _ = O.bad_mask(cm, 0.01)
    g = np.flatnonzero(~obad)
    c = O.sparse_cor(cm[np.ix_(g, g)])
    old = G.knob(8, 0 if forced else 1 << 30)
    old20 = G.knob(20, 1 if space.startswith("C") else 0)
    old36 = G.knob(36, 1 if space == "G-int8" else 0)   # the other spaces on the fp64 products
    try:
        p, _ = G.pca(c, 200)
    finally:
        G.knob(8, old)
        G.knob(20, old20)
        G.knob(36, old36)
    op = O.prcomp_x(c, 200)
    s = np.sign(np.sum(p * op, axis=0))
    s[s == 0] = 1
    scale = np.abs(op).max()
    np.testing.assert_allclose(p[:, :20] * s[:20], op[:, :20], atol=1e-9 * scale)
    sv = np.linalg.svd(op, compute_uv=False)

    def proj(x, i):
        q, _ = np.linalg.qr(x[:, :i])
        return q @ q.T
    for i in (1, 5, 20, 100, 199, 200):
        if i < 200 and sv[i - 1] / max(sv[i], 1e-300) < 1.0 + 1e-6:
            continue
        assert np.abs(proj(p, i) - proj(op, i)).max() < 1e-7, i


@pytest.mark.parametrize("space", ["C", "G"])
def test_pipeline_krylov_forced_end_to_end(gpu, space):
    """A whole TADpole() through the Krylov PCA (in C or in G) at a size the
    oracle runs live."""
    import tadpole_amd as tp
    m = synth_hic(2400, SEED_BASE + 78)
    old = G.knob(8, 0)
    old20 = G.knob(20, 1 if space == "C" else 0)
    try:
        got = tp.TADpole(m, max_pcs=200)
    finally:
        G.knob(8, old)
        G.knob(20, old20)
    assert got.timings_ms[16] > 0          # the Krylov path ran
    ref = O.tadpole(m, max_pcs=200)
    assert (got.n_pcs, got.optimal_n_clusters) == (ref.n_pcs, ref.optimal_n_clusters)
    for q, v in ref.clusters.items():
        assert np.array_equal(got.clusters[str(q)], v), q
    a, b = got.scores, ref.scores
    fin = ~np.isnan(b)
    assert np.array_equal(np.isnan(a), ~fin)
    assert np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin])) < 1e-6


@pytest.mark.parametrize("case", ["counts", "large_counts", "real"])
def test_cor_in_xtx_store_same_bits(gpu, case):
    """The correlation epilogue applied in the int8 X'X store with the gather's
    column statistics (knob 18, default) gives the bits of X'X into S plus the
    separate epilogue -- on counts (the fused path), on counts >= 2^14 (3
    slices: the fallback) and on non-integer data (the fp64 product)."""
    import tadpole_amd as tp
    m = synth_hic(2100, SEED_BASE + 80)
    if case == "large_counts":
        m = m * 7.0                        # maxima past 2^14
    elif case == "real":
        m = m * 0.37                       # not integers
    runs = []
    for fused in (1, 0):
        old = G.knob(18, fused)
        try:
            runs.append(tp.TADpole(m, max_pcs=150))
        finally:
            G.knob(18, old)
    a, b = runs
    assert (a.n_pcs, a.optimal_n_clusters) == (b.n_pcs, b.optimal_n_clusters)
    assert np.array_equal(np.asarray(a.scores).view(np.uint64), np.asarray(b.scores).view(np.uint64))
    assert a.clusters.keys() == b.clusters.keys()
    for q in a.clusters:
        assert np.array_equal(a.clusters[q], b.clusters[q]), q
    assert np.array_equal(a.dendro.height.view(np.uint64), b.dendro.height.view(np.uint64))


@pytest.mark.parametrize("n", [2100, 4500])
def test_cor_wide_tiles_same_bits(gpu, n):
    """The correlation in k_xtx_i8_w's 256 x 128 tile store (knob 44, default)
    against the 128-tile kernel: the same exact X'X and epilogue, so the same
    pipeline bits (ragged n with an odd tile-column count; 4500 bins: the
    block Krylov path)."""
    import tadpole_amd as tp
    m = synth_hic(n, SEED_BASE + 82)
    runs = []
    for wide in (1, 0):
        old = G.knob(44, wide)
        try:
            runs.append(tp.TADpole(m, max_pcs=150))
        finally:
            G.knob(44, old)
    a, b = runs
    assert (a.n_pcs, a.optimal_n_clusters) == (b.n_pcs, b.optimal_n_clusters)
    assert np.array_equal(np.asarray(a.scores).view(np.uint64), np.asarray(b.scores).view(np.uint64))
    for q in a.clusters:
        assert np.array_equal(a.clusters[q], b.clusters[q]), q


@pytest.mark.parametrize("n", [4500, 10500])
def test_cspace_int8_products(gpu, n):
    """The C-space Krylov path (knob 20 = 1 forces it at 4500 bins; the default
    from 10 000) with its 32-column products on the int8 digits of C (knob 45,
    k_pd_prodA<1, 2>) against the fp64 products: the same PC count, cluster
    count and clusters at every level, dendrogram heights within 1e-9 (the
    digit products are within ~1e-15 of sum |A||B|, not bit-equal)."""
    import tadpole_amd as tp
    m = synth_hic(n, SEED_BASE + 83)
    runs = []
    old20 = G.knob(20, 1)
    try:
        for i8 in (1, 0):
            old = G.knob(45, i8)
            try:
                runs.append(tp.TADpole(m, max_pcs=150))
            finally:
                G.knob(45, old)
    finally:
        G.knob(20, old20)
    a, b = runs
    assert a.timings_ms[16] > 0                       # the Krylov path ran
    assert (a.n_pcs, a.optimal_n_clusters) == (b.n_pcs, b.optimal_n_clusters)
    assert a.clusters.keys() == b.clusters.keys()
    for q in a.clusters:
        assert np.array_equal(a.clusters[q], b.clusters[q]), q
    np.testing.assert_allclose(a.dendro.height, b.dendro.height, rtol=1e-9, atol=0)


# ------------------------------------------------------------ arm path (C5)

@pytest.mark.parametrize("name", ["arm_c5layout", "arm_early"])
@pytest.mark.parametrize("mode", ["bug", "fixed"])
def test_arms_golden(gpu, name, mode):
    """centromere_search=TRUE (R/TADpole.R:58-85,351-442) against the oracle:
    merging_arms, and per arm n_pcs, optimal_n_clusters, scores, dendro and
    every `cluster` level; bug-compatible (q-arm bad bins removed by original
    index) and fixed modes."""
    import tadpole_amd as tp
    z = np.load(os.path.join(GOLD, f"{name}.npz"))
    n0, seed = int(z["n0"]), int(z["seed"])
    early = tuple(int(x) for x in z["early"])
    m = early_centromere_matrix(n0, seed, *early) if early[0] >= 0 else synth_hic(n0, seed, centromere=True)
    got = tp.TADpole(m, max_pcs=200, centromere_search=True, fixed_centromere=(mode == "fixed"))
    assert np.array_equal(got.merging_arms, z[f"{mode}_merging_arms"])
    for arm in ("p", "q"):
        sub = getattr(got, arm)
        assert np.array_equal(sub.dendro.labels, z[f"{mode}_{arm}_names"].astype(str).tolist())
        _check(sub, z, f"{mode}_{arm}_", bad=False)
        assert sub.cluster is sub.clusters        # R's `$cluster` slot on the arm branch


@pytest.mark.parametrize("mode", ["bug", "fixed"])
def test_arms_golden_device_input(gpu, mode):
    """The same golden arms from a GPU-resident matrix: each arm's pipeline
    reads its rows and columns from the cleaned whole matrix (TP_FLAG_SUBSET)
    instead of a copied submatrix."""
    import torch
    import tadpole_amd as tp
    z = np.load(os.path.join(GOLD, "arm_c5layout.npz"))
    m = synth_hic(int(z["n0"]), int(z["seed"]), centromere=True)
    got = tp.TADpole(torch.from_numpy(m).cuda(), max_pcs=200, centromere_search=True,
                     fixed_centromere=(mode == "fixed"))
    assert np.array_equal(got.merging_arms, z[f"{mode}_merging_arms"])
    for arm in ("p", "q"):
        sub = getattr(got, arm)
        assert np.array_equal(sub.dendro.labels, z[f"{mode}_{arm}_names"].astype(str).tolist())
        _check(sub, z, f"{mode}_{arm}_", bad=False)


@pytest.mark.parametrize("n0,take", [(400, 300), (2600, 2100)])
def test_subset_pipeline_same_bits(gpu, n0, take):
    """TP_FLAG_SUBSET on a ragged index list (gaps, both ends dropped) gives
    the bits of the pipeline on the copied principal submatrix; bad lists
    (descending, repeated, out of range) are TP_ERR_ARG."""
    import torch
    from tadpole_amd import _lib
    from tadpole_amd.api import _pipeline
    rng = np.random.default_rng(7)
    m = synth_hic(n0, SEED_BASE + 91)
    names = np.sort(rng.choice(np.arange(2, n0), take, replace=False)) + 1     # 1-based, ragged
    dm = torch.from_numpy(m).cuda()
    a = _pipeline(dm, 200, 2, 0.0, _lib.TP_FLAG_CLEAN, 0, subset=names)
    sel = torch.as_tensor(names - 1, device=dm.device)
    sub = dm.index_select(0, sel).index_select(1, sel).contiguous()
    b = _pipeline(sub, 200, 2, 0.0, _lib.TP_FLAG_NO_MASK | _lib.TP_FLAG_CLEAN, 0)
    assert np.array_equal(a["good"], names)
    assert not a["bad"].any() and a["bad"].size == take
    for key in ("k", "w", "n_pcs", "n_clusters"):
        assert a[key] == b[key], key
    for key in ("n_cluster", "scores", "merge", "height", "boundary"):
        assert np.array_equal(a[key], b[key], equal_nan=key in ("scores", "height")), key
    for bad in (names[::-1].copy(), np.r_[names[:5], names[4:10]], np.r_[0, names[1:]], np.r_[names[:-1], n0 + 1]):
        with pytest.raises(RuntimeError, match="TP_FLAG_SUBSET"):
            _pipeline(dm, 200, 2, 0.0, _lib.TP_FLAG_CLEAN, 0, subset=bad)


@pytest.mark.parametrize("n", [2100, 5000, 10500, 16000])
def test_lds_lean_coniss_same_bits(gpu, n):
    """TP_FLAG_LDS_LEAN (pipelines sharing a GPU: the C5 arms, run_genome's
    streams): CONISS keeps only its link array in LDS and derives each next
    cluster's end from it (from 4096 bins also for matrices whose costs would
    fit LDS); every merge, height and score is the default sweep's."""
    from tadpole_amd import _lib
    from tadpole_amd.api import _pipeline
    m = synth_hic(n, SEED_BASE + 97)
    a = _pipeline(m, 60, 2, 0.01, 0, 0)
    old = G.knob(48, 4096)          # the in-LDS sizes' lean variant is opt-in
    try:
        b = _pipeline(m, 60, 2, 0.01, _lib.TP_FLAG_LDS_LEAN, 0)
    finally:
        G.knob(48, old)
    for key in ("k", "w", "n_pcs", "n_clusters"):
        assert a[key] == b[key], key
    for key in ("good", "n_cluster", "scores", "merge", "height", "boundary"):
        assert np.array_equal(a[key], b[key], equal_nan=key in ("scores", "height")), key


@pytest.mark.parametrize("n", [2100, 7808, 16000])
def test_lds_lean_batched_coniss_same_bits(gpu, n):
    """The default lean sweep (TP_FLAG_LDS_LEAN, knob 52 = 3): the batched CONISS
    in storage mode 1 (costs in LDS, 16-bit links: two trees a CU) where the
    default sweep takes mode 0, mode 2 at 16 000 bins -- every merge, height and
    score is the default sweep's."""
    from tadpole_amd import _lib
    from tadpole_amd.api import _pipeline
    m = synth_hic(n, SEED_BASE + 96)
    a = _pipeline(m, 60, 2, 0.01, 0, 0)
    b = _pipeline(m, 60, 2, 0.01, _lib.TP_FLAG_LDS_LEAN, 0)
    for key in ("k", "w", "n_pcs", "n_clusters"):
        assert a[key] == b[key], key
    for key in ("good", "n_cluster", "scores", "merge", "height", "boundary"):
        assert np.array_equal(a[key], b[key], equal_nan=key in ("scores", "height")), key


@pytest.mark.parametrize("n", [700, 2100, 7808, 11000])
def test_lds_link_only_coniss_same_bits(gpu, n):
    """Knob 49: the LDS variant keeps one 16-bit link array after the costs (10
    bytes a bin instead of 16; by default only where the 16-byte variant does not
    fit, so 11 000 bins fit LDS instead of taking the global variant).  Every
    size on it (2) against the 16-byte and global variants (0): same merges,
    heights and scores."""
    from tadpole_amd.api import _pipeline
    m = synth_hic(n, SEED_BASE + 98)
    old = G.knob(49, 0)
    try:
        a = _pipeline(m, 60, 2, 0.01, 0, 0)
    finally:
        G.knob(49, old)
    old = G.knob(49, 2)
    try:
        b = _pipeline(m, 60, 2, 0.01, 0, 0)
    finally:
        G.knob(49, old)
    for key in ("k", "w", "n_pcs", "n_clusters"):
        assert a[key] == b[key], key
    for key in ("good", "n_cluster", "scores", "merge", "height", "boundary"):
        assert np.array_equal(a[key], b[key], equal_nan=key in ("scores", "height")), key


def test_arms_bug_mode_errors_like_r(gpu):
    import tadpole_amd as tp
    m = synth_hic(300, 5)
    m[:20, :] = 0
    m[:, :20] = 0                                 # longest bad run touches the start
    with pytest.raises(TypeError):
        tp.TADpole(m, centromere_search=True)
    got = tp.TADpole(m, centromere_search=True, fixed_centromere=True)
    ref = tp.TADpole(m)
    assert got.n_pcs == ref.n_pcs and got.clusters.keys() == ref.clusters.keys()


# ----------------------------------------------------------- genome (C4)

def test_genome_c4_one_gpu(gpu):
    """C4: the 23 hg19 chromosomes @25 kb through run_genome on one GPU
    (concurrent streams): every result equals its own single-stream run, and
    the three smallest equal the oracle fixtures."""
    import tadpole_amd as tp
    from tadpole_amd.genome import run_genome
    sizes = genome_bins()
    mats = {c: genome_matrix(c) for c in sizes}
    res, secs = run_genome(mats, sizes=sizes, streams=4, max_pcs=200)
    assert set(res) == set(sizes)
    for c in sizes:
        one = tp.TADpole(mats[c], max_pcs=200)
        r = res[c]
        assert (r.n_pcs, r.optimal_n_clusters) == (one.n_pcs, one.optimal_n_clusters), c
        assert r.clusters.keys() == one.clusters.keys(), c
        for q in one.clusters:
            assert np.array_equal(r.clusters[q], one.clusters[q]), (c, q)
        assert np.array_equal(r.scores.view(np.uint64), one.scores.view(np.uint64)), c
    for c in ("chr21", "chr22", "chr19"):
        _check(res[c], np.load(os.path.join(GOLD, f"genome_{c}.npz")))
    print("C4 seconds per chromosome:", {c: round(s, 3) for c, s in sorted(secs.items())})


# ------------------------------------ the largest single matrices (oracle)

LARGE = {"genome_chr1": lambda: genome_matrix("chr1"),           # C4's largest chromosome, 9 971 bins
         "c5arm": lambda: synth_hic_par(24300, SEED_BASE + 5)}   # C5's p-arm shape, 24 300 bins


@pytest.mark.parametrize("name", sorted(LARGE))
def test_large_golden(gpu, name):
    """The largest single matrices of the BASELINE configs end to end against
    the oracle (tests/golden/make_golden.py large: LAPACK dsyevr PCA, the C
    sweep): identical n_pcs, optimal_n_clusters, bad columns, merge order and
    every level's coordinates, CH within 1e-6 relative.  These are the sizes
    where the dense PC tail makes CONISS near-ties likeliest
    (R/TADpole.R:351-442,444-497)."""
    import tadpole_amd as tp
    z = np.load(os.path.join(GOLD, f"{name}.npz"))
    m = LARGE[name]()
    assert np.array_equal(matrix_checksum(m), z["matrix_checksum"])   # same input as the fixture
    got = tp.TADpole(m, max_pcs=int(z["max_pcs"]))
    del m
    sv = z["pc_norms"]
    print(f"{name}: n={int(got.timings_ms[14])} n_pcs={got.n_pcs} k*={got.optimal_n_clusters} "
          f"pca resid {got.timings_ms[13]:.1e} krylov steps {int(got.timings_ms[16])} "
          f"sigma_k-1/sigma_k {sv[-2] / sv[-1]:.6f}")
    assert got.timings_ms[13] <= 1e-11
    _check(got, z)


# ------------------------------------------------- C5 at full size (properties)

def _nested(clusters):
    """Boundaries of level k are a subset of those of level k+1 (cuts of one
    tree) and every level tiles its bins in order."""
    levels = sorted(int(q) for q in clusters)
    prev = None
    for q in levels:
        c = clusters[str(q)]
        assert np.all(c[:, 0] <= c[:, 1]) and np.all(c[1:, 0] > c[:-1, 1])
        starts = set(c[:, 0].tolist())
        if prev is not None:
            assert prev <= starts
        prev = starts


def test_c5_full_golden_and_sharded_bit_identical(gpu):
    # (also: the arm-group schedule -- p and q each sharded over its own rank
    # group, tadpole_amd.multi.init_arm_comms -- gives the same bits)
    """BASELINE config 5 at full size (chr1 @5kb shape: synth_hic_par(49 851,
    SEED_BASE + 5, centromere=True), the CPU-generated matrix of
    tests/golden/c5full.npz): TADpole(centromere_search=TRUE), bug-compatible
    (the q arm keeps its ~100 zeroed bins: constant columns, NaN -> 0 in cor,
    identical PC rows, exact CONISS ties), against the CPU oracle --
    merging_arms, and per arm n_pcs, optimal_n_clusters, bit-exact merge
    order and every level's coordinates, CH within 1e-6 relative
    (R/TADpole.R:58-85,351-442).  The same matrix split over 8 virtual shards
    (the C5 schedule: column slabs of C, row-split Krylov products, tree-split
    sweep) gives the unsharded bits; the levels nest."""
    import torch
    import tadpole_amd as tp
    from tadpole_amd import multi
    z = np.load(os.path.join(GOLD, "c5full.npz"))
    m = synth_hic_par(int(z["n0"]), int(z["seed"]), centromere=True)
    assert np.array_equal(matrix_checksum(m), z["matrix_checksum"])   # same input as the fixture
    dm = torch.from_numpy(m).cuda()
    del m
    got = tp.TADpole(dm, max_pcs=200, centromere_search=True, inplace=True)
    assert np.array_equal(got.merging_arms, z["bug_merging_arms"])
    for arm in ("p", "q"):
        sub = getattr(got, arm)
        sv = z[f"bug_{arm}_pc_norms"]
        print(f"C5 arm {arm}: n={int(sub.timings_ms[14])} n_pcs={sub.n_pcs} k*={sub.optimal_n_clusters} "
              f"pca resid {sub.timings_ms[13]:.1e} sigma_k-1/sigma_k {sv[-2] / sv[-1]:.6f}")
        assert sub.timings_ms[13] <= 1e-11
        assert np.array_equal(sub.dendro.label_ids, z[f"bug_{arm}_names"])
        _check(sub, z, f"bug_{arm}_", bad=False)
        _nested(sub.clusters)
    multi.set_virtual_shards(8)
    try:
        g8 = tp.TADpole(dm, max_pcs=200, centromere_search=True, sharded=True, inplace=True)
    finally:
        multi.set_virtual_shards(1)
    # the arm-group schedule of N = 5 ranks (bench.py --gpus 5: p over 3, q
    # over 2): each arm sharded over its own group, merged after
    from tadpole_amd import api
    p_r, q_r = multi.arm_group_ranks(5)
    bad, _, _ = api.mask_dev(dm, 0.01)
    plan = api._arm_plan(bad)
    subs = {}
    for arm, nv in (("p", len(p_r)), ("q", len(q_r))):
        multi.set_virtual_shards(nv)
        try:
            subs[arm] = api._run_arm(dm, plan, arm, 200, 2, 0, api._lib.TP_FLAG_SHARDED)
        finally:
            multi.set_virtual_shards(1)
    g5 = api._merge_arms(plan, subs)
    del dm
    torch.cuda.empty_cache()
    for g in (g8, g5):
        assert np.array_equal(g.merging_arms, got.merging_arms)
        for arm in ("p", "q"):
            x, y = getattr(got, arm), getattr(g, arm)
            assert (x.n_pcs, x.optimal_n_clusters) == (y.n_pcs, y.optimal_n_clusters)
            assert np.array_equal(x.scores.view(np.uint64), y.scores.view(np.uint64))
            assert np.array_equal(x.dendro.boundary, y.dendro.boundary)
            assert np.array_equal(x.dendro.height.view(np.uint64), y.dendro.height.view(np.uint64))


def test_non_integer_counts_gather_x_on_demand(gpu):
    """The fused gather writes X only for the fp64 correlation product: a
    balanced (non-integer) matrix above the int8 size threshold takes the fp64
    path through the on-demand gather and gives the bits of the plain gather
    (knob 5 = 0: no int8 prep at all), and the oracle's TADs."""
    import tadpole_amd as tp
    m = synth_hic(1500, SEED_BASE + 83).astype(np.float64)
    rng = np.random.default_rng(5)
    w = rng.uniform(0.5, 1.5, m.shape[0])
    m = m * w[:, None] * w[None, :]                     # balanced-style weights: not integers
    a = tp.TADpole(m, max_pcs=100)
    old = G.knob(5, 0)
    try:
        b = tp.TADpole(m, max_pcs=100)
    finally:
        G.knob(5, old)
    assert np.array_equal(a.scores.view(np.uint64), b.scores.view(np.uint64))
    ref = O.tadpole(m, max_pcs=100)
    assert (a.n_pcs, a.optimal_n_clusters) == (ref.n_pcs, ref.optimal_n_clusters)
    for q, v in ref.clusters.items():
        assert np.array_equal(a.clusters[str(q)], v), q
