"""R-legal inputs past the round-2 build's limits (R accepts any max_pcs,
R/TADpole.R:344,452; the CH loop at :117-120 has no level limit):

* k = min(max_pcs, N) up to 1024 in the sweep kernels (column-slot templates
  of 4, 8 and 16 slots), with the PCA's Rayleigh-Ritz block up to 1280 on the
  library's own eigensolver and CholQR (the library links no rocSOLVER);
* more than 1024 significant broken-stick levels (k_ch_glb, the global-memory
  CH kernel for cuts past k_ch's LDS capacity);
* more than 65 536 bins in CONISS (32 block-minimum slots).

Bars as everywhere: the sweep bit-identical to the oracle (merge order,
heights, n_cluster, every CH score with R's NA bits); end to end identical TAD
coordinates, n_pcs, optimal_n_clusters, CH within 1e-6 relative.
"""
import numpy as np
import pytest

import gpu_helpers as G
import tadpole_oracle as O
from tadpole_amd.synth import synth_hic

pytestmark = pytest.mark.gpu


def _same_sweep(got, ref):
    assert np.array_equal(got["n_cluster"], ref.n_cluster)
    assert np.array_equal(got["mrg_b"], ref.mrg_b)
    assert np.array_equal(got["mrg_a"], ref.mrg_a)
    assert np.array_equal(got["height"], ref.height)
    a, b = got["scores"], ref.scores
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))   # incl. NA bit patterns


def _segment_pcs(n, k, seed):
    """TAD-like piecewise-constant scores with a decaying spectrum + noise."""
    rng = np.random.default_rng(seed)
    cuts = np.cumsum(rng.integers(10, 60, size=n))
    seg = np.searchsorted(cuts, np.arange(n), side="right")
    means = rng.standard_normal((seg.max() + 1, k)) * (1.0 / (1 + 0.05 * np.arange(k)))
    return means[seg] + 0.05 * rng.standard_normal((n, k))


def hier_pcs(levels, k, seed=1):
    """Scores of a balanced binary hierarchy of 2**levels bins in which every
    sibling merge costs exactly 1 (children of a node sit at +-u_d / sqrt(2m),
    u_d orthonormal): every level of the tree is significant against the broken
    stick, so a prefix with all `levels` structural columns has ~0.63 n levels
    -- past k_ch's 1024-segment LDS capacity at 2048 bins."""
    n = 2 ** levels
    p = np.zeros((n, k))
    for d in range(levels):
        m = 2 ** (levels - 1 - d)
        p[:, d] = np.where((np.arange(n) // m) % 2 == 0, 1.0, -1.0) / np.sqrt(2 * m)
    p[:, levels:] = np.random.default_rng(seed).standard_normal((n, k - levels)) * 1e-3
    return p


@pytest.mark.parametrize("k", [300, 400, 512, 600, 1024])
def test_sweep_k_above_256_bit_exact(gpu, k):
    """Trees of 5..8 and 9..16 column slots (the KS = 8 / 16 instances of
    CONISS, k_seed, k_trS, the CH kernels) against the oracle, bit for bit."""
    p = _segment_pcs(max(900, k + 100), k, 40 + k)
    got = G.sweep_dev(p)
    ref = O.sweep(p)
    _same_sweep(got, ref)


def test_sweep_k_above_256_global_variant(gpu):
    """k > 256 above the LDS capacity of CONISS (global costs, 16-bit links)."""
    p = _segment_pcs(11000, 270, 7)
    got = G.sweep_dev(p)
    ref = O.sweep(p, nthreads=16)
    assert np.array_equal(got["n_cluster"], ref.n_cluster)
    assert np.array_equal(got["mrg_b"], ref.mrg_b)
    assert np.array_equal(got["height"], ref.height)
    assert np.array_equal(got["scores"].view(np.uint64), ref.scores.view(np.uint64))


@pytest.mark.parametrize("levels,k", [(11, 16), (12, 24), (11, 300)])
def test_more_than_1024_broken_stick_levels(gpu, levels, k):
    """Cuts of 1293 / 2587 segments: k_ch_glb scores them with k_ch's
    arithmetic (the oracle's tpo_ch_levels has no level limit)."""
    p = hier_pcs(levels, k)
    ref = O.sweep(p, nthreads=16)
    assert ref.n_cluster.max() > 1024
    got = G.sweep_dev(p)
    _same_sweep(got, ref)
    # the selection over the full score matrix (R/TADpole.R:134-135)
    sel = G.sweep(p)
    assert (sel["n_pcs"], sel["n_clusters"]) == O.select_params(ref.scores)


def test_coniss_above_65536_bins(gpu):
    """CONISS of one tree at 70 000 bins (32 block-minimum slots, links in
    global memory) against the oracle's merge order and heights."""
    rng = np.random.default_rng(70000)
    n = 70000
    cuts = np.cumsum(rng.integers(10, 60, size=n))
    seg = np.searchsorted(cuts, np.arange(n), side="right")
    p = rng.standard_normal((seg.max() + 1, 3))[seg] + 0.05 * rng.standard_normal((n, 3))
    merge, h, bnd = G.coniss(p)
    ma, mb, _, he = O.coniss(p)
    assert np.array_equal(bnd, mb)
    assert np.array_equal(h.view(np.uint64), he.view(np.uint64))
    assert np.array_equal(merge, O.hclust_merge(ma, mb, n).astype(np.int32))


def _check_pipeline(got, ref):
    assert (got.n_pcs, got.optimal_n_clusters) == (ref.n_pcs, ref.optimal_n_clusters)
    assert set(got.clusters) == {str(q) for q in ref.clusters}
    for q, v in ref.clusters.items():
        assert np.array_equal(got.clusters[str(q)], v), q
    a, b = got.scores, ref.scores
    fin = ~np.isnan(b)
    assert np.array_equal(np.isnan(a), ~fin)
    assert np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin])) < 1e-6


@pytest.mark.parametrize("max_pcs", [300, 480, 600])
def test_pipeline_max_pcs_above_256(gpu, max_pcs):
    """TADpole(max_pcs = 300 / 480 / 600) end to end against the oracle
    (LAPACK SVD): Rayleigh-Ritz blocks of 384 / 608 / 768 on the library's
    eigensolver (768: the b > 640 kernels -- k_sytrd_l<20>, one-vector
    k_invit, the chunked k_trsm_ru_big); R accepts any max_pcs
    (R/TADpole.R:344,452)."""
    import tadpole_amd as tp
    m = synth_hic(1400, 900 + max_pcs)
    got = tp.TADpole(m, max_pcs=max_pcs)
    assert got.timings_ms[12] > 256                 # the Rayleigh-Ritz block
    ref = O.tadpole(m, max_pcs=max_pcs, nthreads=16)
    _check_pipeline(got, ref)


def test_pipeline_krylov_max_pcs_300(gpu):
    """The block Krylov PCA (n >= 4096) with k = 300."""
    import tadpole_amd as tp
    m = synth_hic(4300, 4300)
    got = tp.TADpole(m, max_pcs=300)
    assert got.timings_ms[16] > 0                    # the Krylov path ran
    assert got.timings_ms[13] <= 1e-11
    ref = O.tadpole(m, max_pcs=300, nthreads=16, pca="eigh")
    _check_pipeline(got, ref)


def test_sweep_k_above_1024_unsupported(gpu):
    """k > 1024 is refused with TP_ERR_UNSUPPORTED (a clear error, not a
    silent truncation)."""
    from tadpole_amd._lib import TadpoleError, TP_ERR_UNSUPPORTED
    p = _segment_pcs(1200, 1030, 3)
    with pytest.raises(TadpoleError) as e:
        G.sweep_dev(p)
    assert e.value.status == TP_ERR_UNSUPPORTED
