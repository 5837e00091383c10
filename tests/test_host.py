"""CPU: host-side logic of the R mirror (no GPU calls): cutree on the
boundary order, fix_values / bad-column re-insertion / coordinates (R/TADpole.R
:470-510) against the oracle's independent restatement, the centromere arm
split helpers (R/TADpole.R:58-85), diffT (R/DiffT.R) and random_bed."""
import os

import numpy as np
import pandas as pd
import pytest

import tadpole_oracle as O
from tadpole_amd import _lib, api

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _chclust(mb, n):
    return api.Chclust(merge=np.zeros((n - 1, 2), np.int32), height=np.arange(n - 1, dtype=float),
                       order=np.arange(1, n + 1), label_ids=np.arange(1, n + 1),
                       boundary=np.asarray(mb) + 1)


@pytest.mark.parametrize("seed", range(5))
def test_cutree_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(3, 60))
    mb = rng.permutation(np.arange(1, n))
    ch = _chclust(mb, n)
    for k in range(1, n + 1):
        assert np.array_equal(ch.cutree(k), O.cutree_labels(mb, n, k))


@pytest.mark.parametrize("name", ["n64", "n200", "n300"])
def test_assembly_matches_oracle_on_golden(name):
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    bad = g["bad"]
    good1 = np.flatnonzero(~bad).astype(np.int32) + 1
    n = len(good1)
    res = dict(good=good1, merge=np.zeros((n - 1, 2), np.int32), height=g["height"], boundary=g["merge_b"] + 1,
               n_pcs=int(g["n_pcs"]), n_clusters=int(g["optimal_n_clusters"]), scores=g["scores"],
               timings=np.zeros(32))
    t = api._assemble(res, np.flatnonzero(bad) + 1)
    coords = np.concatenate([np.c_[np.full(len(t.clusters[q]), int(q)), t.clusters[q]]
                             for q in sorted(t.clusters, key=int)])
    assert np.array_equal(coords, g["coords"])
    assert t.dendro.labels == [str(x) for x in good1]


@pytest.mark.parametrize("seed", range(12))
def test_vectorised_assembly_equals_literal_rle(seed):
    # api._level_coords (one slice per level) against the literal cutree + c(good,
    # bad) + order + rle + fix_values + runs of R/TADpole.R:470-488, with bad runs
    # at both ends, adjacent bad runs and arm-style names (not 1..n0)
    rng = np.random.default_rng(100 + seed)
    n0 = int(rng.integers(5, 120))
    bad = rng.random(n0) < rng.choice([0.0, 0.1, 0.4])
    if seed % 3 == 0:
        bad[:2] = True
        bad[-3:] = True
    if bad.sum() > n0 - 3:
        bad[: n0 - 3] = False
    names = np.arange(1, n0 + 1) + (0 if seed % 2 else 500)
    good1, bad1 = names[~bad], names[bad]
    n = len(good1)
    mb = rng.permutation(np.arange(1, n))
    scores = np.full((3, n - 1), np.nan)
    scores[1, rng.choice(n - 1, size=min(n - 1, 7), replace=False)] = 1.0
    res = dict(good=good1, merge=np.zeros((n - 1, 2), np.int32), height=np.arange(n - 1, dtype=float),
               boundary=mb + 1, n_pcs=2, n_clusters=2, scores=scores, timings=np.zeros(32))
    for b in (bad1, None):
        fast = api._assemble(res, b)
        slow = api._assemble_rle(api.Tadpole(), fast.dendro, np.flatnonzero(~np.isnan(scores[1])) + 1, good1, b)
        assert set(fast.clusters) == set(slow.clusters)
        for q in fast.clusters:
            assert np.array_equal(fast.clusters[q], slow.clusters[q]), (q, b is None)


def test_level_coords_rejects_bad_arguments():
    # tp_level_coords (host-only C-ABI): levels outside 1..n and boundaries
    # outside 2..n fail with TP_ERR_ARG instead of reading out of bounds
    n = 6
    pos = np.arange(1, n + 1, dtype=np.int64)
    with pytest.raises(_lib.TadpoleError) as e:
        api._all_level_coords(np.array([2, 3, 4, 5, 6]), n, [n + 1], pos)
    assert e.value.status == _lib.TP_ERR_ARG
    with pytest.raises(_lib.TadpoleError) as e:
        api._all_level_coords(np.array([2, 3, 1, 5, 6]), n, [4], pos)
    assert e.value.status == _lib.TP_ERR_ARG
    assert [c.tolist() for c in api._all_level_coords(np.array([4, 2, 6, 3, 5]), n, [1, 3], pos)] == \
        [[[1, 6]], [[1, 2], [3, 4], [5, 6]]]


def test_assembly_without_bad_columns_branch():
    # R/TADpole.R:490-494 (table(good_clusters)) equals the bad-column branch
    n = 30
    mb = np.random.default_rng(1).permutation(np.arange(1, n))
    lab = O.cutree_labels(mb, n, 5)
    eb = np.cumsum(np.bincount(lab)[1:])
    a = np.stack([np.concatenate([[1], eb[:-1] + 1]), eb], axis=1)
    b = api._coords(api._fixed_clusters(lab, np.arange(1, n + 1), np.zeros(0, np.int64))[0])
    assert np.array_equal(a, b)


def test_fix_values_edges():
    lens, v = api.fix_values(*api.rle(np.array([0, 0, 1, 0, 1, 0, 2, 2, 0])))
    assert list(v) == [0, 1, 1, 1, 0, 2, 0]
    ref = O.fix_values(*O.rle(np.array([0, 0, 1, 0, 1, 0, 2, 2, 0])))
    assert list(ref[1]) == list(v)


def test_arm_split_helpers_bug_compatible():
    # R: mat_q[-bad_q, -bad_q] with ORIGINAL indices; out-of-range ignored
    keep = api._r_negative_keep(10, np.array([3, 12, 40]))
    assert list(keep) == [0, 1, 3, 4, 5, 6, 7, 8, 9]
    runs = api._runs(np.array([2, 3, 4, 9, 10, 20]))
    assert [list(r) for r in runs] == [[2, 3, 4], [9, 10], [20]]


def _bed(name):
    return pd.read_csv(os.path.join(GOLD, name), sep="\t", header=None)


def test_diffT_matches_oracle_and_figure():
    x, y = _bed("control.bed"), _bed("case.bed")
    d = api.diffT(x, y)
    rows = lambda df: [tuple(r) for r in df.itertuples(index=False)]
    assert np.array_equal(d, O.diffT(rows(x), rows(y)))
    assert len(d) == 194 and d[-1] == 1.0


def test_diffT_random_pairs_match_oracle():
    rng = np.random.default_rng(3)
    for _ in range(20):
        nt = int(rng.integers(2, 8))
        def mk(off):
            cuts = np.sort(rng.choice(np.arange(1, 60), nt - 1, replace=False)) + off
            st = np.concatenate([[off], cuts]); en = np.concatenate([cuts - 1, [off + 60 + int(rng.integers(0, 3))]])
            return [("chr1", int(a), int(b)) for a, b in zip(st, en)]
        a, b = mk(int(rng.integers(0, 3))), mk(int(rng.integers(0, 3)))
        assert np.array_equal(api.diffT(a, b), O.diffT(a, b))


def test_diffT_errors():
    with pytest.raises(ValueError):
        api.diffT([("c", 1, 5)], [("c", 1, 2), ("c", 3, 5)])


def test_random_bed_shape():
    x = _bed("control.bed")
    r = api.random_bed(x, rng=0)
    assert len(r) == len(x)
    assert r["start"].iloc[0] == x[1].iloc[0] and r["end"].iloc[-1] == x[2].iloc[-1]
    assert (r["start"].to_numpy()[1:] > r["start"].to_numpy()[:-1]).all()


def test_read_matrix_na(tmp_path):
    f = tmp_path / "m.tsv"
    f.write_text("1\t2\tNA\n2\tNaN\t3\n0\t3\t4\n")
    m = api.read_matrix(str(f))
    assert m.shape == (3, 3) and np.isnan(m[0, 2]) and np.isnan(m[1, 1])
    c = api.clean_symmetrize(m)
    assert c[2, 0] == 0.0 and c[1, 1] == 0.0 and np.array_equal(c, c.T)


@pytest.mark.parametrize("n,k,seed", [(150, 5, 31), (300, 1, 7), (65, 2, 4), (3, 1, 1)])
def test_coniss_batch_emulation(n, k, seed):
    """The batched CONISS kernel's control flow (tools/coniss_batch_emu.py: the
    candidate scan over the waves' segments, slot_of, ranks, windows,
    conflicts, runs), emulated with range checks on every index, makes the
    sequential CONISS's merges on TAD-like scores."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("coniss_batch_emu", os.path.join(root, "tools", "coniss_batch_emu.py"))
    E = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(E)
    p = E.structured(n, k, seed)
    got, _ = E.kernel(p)
    ref = E.seq_coniss(p)
    assert [(a, b) for a, b, _ in got] == [(a, b) for a, b, _ in ref]
