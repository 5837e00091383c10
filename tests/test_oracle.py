"""CPU: the oracle against independent implementations and the committed
golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

PARITY UNPINNED against R itself (no R / rioja / fpc in the image, no reference
tests); what pins the oracle here: numpy's type-7 quantile and LAPACK SVD,
scipy's pdist, sklearn's Calinski-Harabasz, a brute-force distance-matrix
CONISS, the reference's own diffT data + published curve, and self-consistency
of the canonical (GPU) vs R-faithful (long double) arithmetic.
"""
import json
import os

import numpy as np
import pytest

import tadpole_oracle as O
from tadpole_amd.synth import synth_hic

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_quantile7_matches_numpy_linear():
    rng = np.random.default_rng(0)
    for n in (1, 2, 7, 200, 1999):
        x = rng.random(n)
        for p in (0.0, 0.01, 0.013, 0.05, 0.5, 1.0):
            assert O.quantile7(x, p) == pytest.approx(np.quantile(x, p, method="linear"), abs=1e-15)
    x = np.array([3.0, 3.0, 3.0, 5.0])
    assert O.quantile7(x, 0.2) == 3.0      # x[hi] == x[lo]: no interpolation rounding


def test_mask_rules():
    m = np.ones((10, 10)) * 5
    m[2, 2] = 0                            # diag == 0
    m[7, :] = m[:, 7] = 0.1                # low coverage
    m[7, 7] = 1
    bad, r, q = O.bad_mask(m, 0.1)
    assert bad[2] and bad[7] and bad.sum() == 2
    bad0, _, _ = O.bad_mask(m, 0.0)        # `if (bad_frac)` is FALSE
    assert bad0.sum() == 1 and bad0[2]


def test_rowmeans_canonical_equals_r_faithful():
    rng = np.random.default_rng(1)
    m = rng.gamma(2, 3, (300, 300))
    a = np.empty(300); b = np.empty(300)
    mm = np.ascontiguousarray(m)
    O.lib().tpo_rowmeans_ld(O._dp(mm), 300, 300, 0, O._dp(a))
    O.lib().tpo_rowmeans_dd(O._dp(mm), 300, 300, 0, O._dp(b))
    assert np.array_equal(a, b)


def test_clean_symmetrize_upper_wins():
    m = np.arange(16.0).reshape(4, 4)
    m[0, 3] = np.nan
    s = O.clean_symmetrize(m)
    assert np.array_equal(s, s.T)
    assert s[3, 0] == 0.0 and s[2, 1] == m[1, 2]


def test_sparse_cor_matches_corrcoef():
    m = synth_hic(150, 3)
    bad, _, _ = O.bad_mask(O.clean_symmetrize(m), 0.01)
    g = np.flatnonzero(~bad)
    x = O.clean_symmetrize(m)[np.ix_(g, g)]
    np.testing.assert_allclose(O.sparse_cor(x), np.corrcoef(x, rowvar=False), atol=1e-10)


def test_prcomp_scores_are_svd_scores():
    rng = np.random.default_rng(2)
    c = rng.standard_normal((60, 60))
    c = c + c.T
    p = O.prcomp_x(c, 10)
    xc = c - c.mean(0)
    u, s, _ = np.linalg.svd(xc)
    np.testing.assert_allclose(np.abs(p), np.abs(u[:, :10] * s[:10]), atol=1e-10)


@pytest.mark.parametrize("seed", range(12))
def test_ward_coniss_equals_distance_matrix_coniss(seed):
    rng = np.random.default_rng(seed)
    n, c = int(rng.integers(3, 70)), int(rng.integers(1, 20))
    p = rng.standard_normal((n, c))
    _, mb, _, he = O.coniss(p)
    mb2, he2 = O.coniss_bruteforce(p)
    assert np.array_equal(mb, mb2)
    np.testing.assert_allclose(he, he2, rtol=1e-9)


def test_coniss_heights_monotone_and_total():
    rng = np.random.default_rng(4)
    p = rng.standard_normal((90, 6))
    _, _, co, he = O.coniss(p)
    assert np.all(co >= 0) and np.all(np.diff(he) >= 0)
    tot = np.sum((p - p.mean(0)) ** 2)     # final height = total sum of squares
    assert he[-1] == pytest.approx(tot, rel=1e-12)


def test_dist_r_matches_pdist():
    from scipy.spatial.distance import pdist
    rng = np.random.default_rng(5)
    p = rng.standard_normal((40, 9))
    np.testing.assert_allclose(O.dist_r(p), pdist(p), rtol=1e-14)


def test_ch_levels_match_sklearn():
    from sklearn.metrics import calinski_harabasz_score
    p = np.load(os.path.join(GOLD, "sweep_p120.npz"))["p"]
    n, k = p.shape
    ma, mb, _, he = O.coniss(p[:, :5])
    nc = 9
    sc = np.empty(nc)
    trS = O.lib().tpo_trS(O._dp(np.ascontiguousarray(p)), n, k, k)
    O.lib().tpo_ch_levels(O._dp(np.ascontiguousarray(p)), n, k, k, O._ip(mb), nc, 2, trS, O._dp(sc))
    assert O.is_r_na(sc[:1]).all()
    for q in range(2, nc + 1):
        lab = O.cutree_labels(mb, n, q)
        assert sc[q - 1] == pytest.approx(calinski_harabasz_score(p, lab), rel=1e-11)


def test_bstick_canonical_equals_r_faithful():
    for name in ("n200", "n300"):
        g = np.load(os.path.join(GOLD, f"{name}.npz"))
        a = O.sweep(g["pcs"], bstick="dd")
        b = O.sweep(g["pcs"], bstick="ld")
        assert np.array_equal(a.n_cluster, b.n_cluster)


@pytest.mark.parametrize("name", ["n64", "n200", "n300"])
def test_golden_regression(name):
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    m = g["matrix"].astype(np.float64)
    assert np.array_equal(m, synth_hic(m.shape[0], int(g["seed"])))   # generator is stable
    r = O.tadpole(m, max_pcs=int(g["max_pcs"]), pcs=g["pcs"])
    assert np.array_equal(r.bad, g["bad"])
    assert (r.n_pcs, r.optimal_n_clusters) == (int(g["n_pcs"]), int(g["optimal_n_clusters"]))
    assert np.array_equal(r.scores.view(np.uint64), g["scores"].view(np.uint64))
    assert np.array_equal(r.merge_b, g["merge_b"])
    coords = np.concatenate([np.c_[np.full(len(r.clusters[q]), q), r.clusters[q]] for q in sorted(r.clusters)])
    assert np.array_equal(coords, g["coords"])
    # the LAPACK PCA reproduces the committed scores' subspaces
    p2 = O.prcomp_x(O.sparse_cor(O.clean_symmetrize(m)[np.ix_(~r.bad, ~r.bad)]), g["pcs"].shape[1])
    np.testing.assert_allclose(np.abs(p2[:, :3]), np.abs(g["pcs"][:, :3]), atol=1e-8)


def test_golden_sweep_fixture():
    g = np.load(os.path.join(GOLD, "sweep_p120.npz"))
    sw = O.sweep(g["p"], 2)
    assert np.array_equal(sw.n_cluster, g["n_cluster"])
    assert np.array_equal(sw.mrg_b, g["mrg_b"])
    assert np.array_equal(sw.height, g["height"])
    assert np.array_equal(sw.scores.view(np.uint64), g["scores"].view(np.uint64))


def test_sweep_no_bstick_level_is_an_error():
    p = np.zeros((10, 2))                  # all costs 0: dispersion never beats the stick
    sw = O.sweep(p)
    assert sw.status == 1


def _bed(path):
    rows = []
    with open(path) as f:
        for line in f:
            c, s, e = line.split()
            rows.append((c, int(s), int(e)))
    return rows


def test_diffT_reference_example_curve():
    x = _bed(os.path.join(GOLD, "control.bed"))
    y = _bed(os.path.join(GOLD, "case.bed"))
    d = O.diffT(x, y)
    cur = json.load(open(os.path.join(GOLD, "diffT_curve.json")))
    assert len(d) == cur["length"]
    for b, v in cur["breakpoints"].items():
        assert round(float(d[int(b) - 1]), 3) == v, b


def test_cutree_and_fix_values():
    mb = np.array([3, 1, 5, 4, 2])           # n = 6
    assert list(O.cutree_labels(mb, 6, 1)) == [1] * 6
    assert list(O.cutree_labels(mb, 6, 3)) == [1, 1, 2, 2, 3, 3]   # last merges removed 4, 2
    lens, vals = O.fix_values(*O.rle(np.array([0, 1, 1, 0, 1, 2, 0, 0, 3, 0])))
    assert list(vals) == [0, 1, 1, 1, 2, 0, 3, 0]   # interior 0 between equal labels absorbed
    c = O.coords_for(np.array([1, 1, 2, 2]), np.array([1, 2, 4, 6]), np.array([3, 5]))
    assert c.tolist() == [[1, 2], [4, 6]]        # bin 5 absorbed, bin 3 is a gap


def test_oracle_under_asan():
    """The C half of the oracle built with AddressSanitizer + UBSan (make -C
    oracle asan) runs every entry point at ragged sizes without a memory or
    UB error, and its Ward-form CONISS equals the distance-matrix definition."""
    import os
    import subprocess
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    subprocess.run(["make", "-s", "-C", here, "asan"], check=True)
    r = subprocess.run([os.path.join(here, "_asan", "tp_oracle_asan")], capture_output=True, text=True,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"), timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "MISMATCH" not in r.stdout


@pytest.mark.parametrize("name", ["genome_chr21", "genome_chr22", "genome_chr19", "genome_chr1", "c5arm"])
def test_large_fixture_generator_pinned(name):
    """The parallel generator (synth_hic_par) reproduces the inputs of the
    outputs-only fixtures exactly (their matrix_checksum), for any thread count."""
    from tadpole_amd.synth import SEED_BASE, genome_matrix, matrix_checksum, synth_hic_par
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    if name.startswith("genome_"):
        m = genome_matrix(name[len("genome_"):])
    else:
        m = synth_hic_par(int(g["n0"]), int(g["seed"]), threads=3)
    assert m.shape[0] == int(g["n0"])
    assert np.array_equal(matrix_checksum(m), g["matrix_checksum"])


def test_write_tsv_round_trip(tmp_path):
    """The bench's TSV writer (read.big.matrix input) parses back to the matrix."""
    from tadpole_amd.synth import synth_hic_par, write_tsv
    m = synth_hic_par(300, 9)
    m[5, 7] = m[7, 5] = 123456789       # wide field
    p = tmp_path / "m.tsv"
    nb = write_tsv(m, str(p), block_rows=7, threads=3)
    assert nb == p.stat().st_size
    rows = p.read_text().split("\n")
    assert rows[-1] == "" and len(rows) == 301
    back = np.array([[float(x) for x in r.split("\t")] for r in rows[:-1]])
    assert np.array_equal(back, m)
