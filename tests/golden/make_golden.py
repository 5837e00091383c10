"""Generate the committed golden fixtures from the CPU oracle (run here, on
CPU; the reference itself is R and cannot run in this image).

  python tests/golden/make_golden.py [small|configs|arms|genome|all]

Fixtures (outputs of oracle/tadpole_oracle.py, a restatement of
R/TADpole.R:15-140,344-510):

* small: synthetic Hi-C inputs (SURVEY.md §8(d) generator) at N0 = 64, 200,
  300 with the matrix and the oracle's TADpole() outputs (mask, n_pcs,
  optimal_n_clusters, NA-padded CH scores, merge boundaries, hclust merge
  matrix and heights of the final tree, TAD coordinates of every significant
  level), plus a PC-score fixture for the sweep alone;
* configs: the BASELINE configs C2 (synth_hic(2000, SEED_BASE+2)) and C3
  (synth_hic(7808, SEED_BASE+3)), outputs only (the generator is pinned by
  test_golden_regression);
* arms: centromere_search=TRUE (R/TADpole.R:58-85,351-442), bug-compatible and
  fixed, on a C5-layout matrix (centromere past the middle: the q-arm index bug
  drops nothing) and on an early-centromere matrix (the bug drops wrong bins);
* genome: the three smallest C4 chromosomes (chr21, chr22, chr19 @25 kb).
* large: the largest single matrices of the BASELINE configs, outputs only:
  C4's chr1 @25 kb (9 971 bins) and a C5-arm-size matrix
  (synth_hic_par(24300, SEED_BASE + 5), the p arm's size; the bench's c5_arm
  line runs the same matrix).  The PCA is LAPACK dsyevr on Xc'Xc (``pca="eigh"``:
  the same top-k subspaces as R's full SVD at a fraction of its cost); peak
  host memory ~35 GB at 24.3k bins.

control.bed / case.bed are the reference's own diffT example data
(inst/extdata) and diffT_curve.json the breakpoints of misc/DiffT_score.png.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import tadpole_oracle as O  # noqa: E402
from tadpole_amd.synth import (SEED_BASE, early_centromere_matrix, genome_bins, genome_matrix,  # noqa: E402
                               genome_seed, synth_hic, synth_hic_par, matrix_checksum)

CASES = [("n64", 64, 20261101, 200), ("n200", 200, 20261016, 200), ("n300", 300, 20261102, 100)]
CONFIGS = [("c2", 2000, SEED_BASE + 2), ("c3", 7808, SEED_BASE + 3)]
ARMS = [("arm_c5layout", 600, 20261104, None), ("arm_early", 500, 20261105, (100, 130))]
GENOME = ["chr21", "chr22", "chr19"]
THREADS = int(os.environ.get("OMP_NUM_THREADS", "8"))


def outputs(r, prefix=""):
    lev = sorted(r.clusters)
    d = {"n_pcs": r.n_pcs, "optimal_n_clusters": r.optimal_n_clusters, "scores": r.scores,
         "merge_b": r.merge_b, "height": r.height, "merge": r.merge.astype(np.int32),
         "n_cluster": r.sweep.n_cluster, "levels": np.array(lev, np.int32),
         "coords": np.concatenate([np.c_[np.full(len(r.clusters[q]), q), r.clusters[q]] for q in lev])}
    if r.bad is not None:
        d["bad_idx1"] = (np.flatnonzero(r.bad) + 1).astype(np.int32)
    return {prefix + k: v for k, v in d.items()}


def small():
    for name, n0, seed, max_pcs in CASES:
        m = synth_hic(n0, seed)
        r = O.tadpole(m, max_pcs=max_pcs, nthreads=THREADS)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), matrix=m.astype(np.int32), max_pcs=max_pcs,
                            seed=seed, bad=r.bad, pcs=r.pcs, **outputs(r))
        print(name, r.n_pcs, r.optimal_n_clusters, r.scores.shape)
    rng = np.random.default_rng(20261103)
    p = rng.standard_normal((120, 24)) * np.linspace(3, 0.2, 24)[None, :]
    sw = O.sweep(p, 2)
    np.savez_compressed(os.path.join(HERE, "sweep_p120.npz"), p=p, n_cluster=sw.n_cluster, scores=sw.scores,
                        mrg_b=sw.mrg_b, height=sw.height)
    # misc/DiffT_score.png breakpoints (1-based bin -> value), SURVEY.md §4
    curve = {"1": 0.003, "23": 0.065, "28": 0.169, "42": 0.208, "53": 0.214, "54": 0.231, "100": 0.288,
             "103": 0.367, "122": 0.400, "134": 0.447, "141": 0.577, "156": 0.687, "162": 0.798,
             "173": 0.872, "179": 0.958, "194": 1.000}
    with open(os.path.join(HERE, "diffT_curve.json"), "w") as f:
        json.dump({"source": "misc/DiffT_score.png (reference), control.bed vs case.bed", "length": 194,
                   "breakpoints": curve}, f, indent=1)


def configs():
    for name, n0, seed in CONFIGS:
        t0 = time.time()
        m = synth_hic(n0, seed)
        r = O.tadpole(m, max_pcs=200, nthreads=THREADS)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), n0=n0, seed=seed, max_pcs=200, **outputs(r))
        print(name, r.n_pcs, r.optimal_n_clusters, r.scores.shape, f"{time.time() - t0:.1f} s")


def arms():
    for name, n0, seed, early in ARMS:
        m = (early_centromere_matrix(n0, seed, *early) if early
             else synth_hic(n0, seed, centromere=True))
        out = {"n0": n0, "seed": seed, "early": np.array(early if early else (-1, -1))}
        for mode, fixed in (("bug", False), ("fixed", True)):
            a = O.tadpole_arms(m, max_pcs=200, fixed=fixed, nthreads=THREADS)
            out[f"{mode}_merging_arms"] = a.merging_arms
            out[f"{mode}_centromere"] = a.centromere
            for arm in ("p", "q"):
                r = getattr(a, arm)
                out.update(outputs(r, f"{mode}_{arm}_"))
                out[f"{mode}_{arm}_names"] = np.asarray(r.good_idx1, np.int32)
            print(name, mode, a.p.n_pcs, a.q.n_pcs, len(a.merging_arms),
                  "q kept", len(a.q.good_idx1))
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)


def genome():
    for name in GENOME:
        m = genome_matrix(name)
        r = O.tadpole(m, max_pcs=200, nthreads=THREADS)
        np.savez_compressed(os.path.join(HERE, f"genome_{name}.npz"), n0=genome_bins()[name],
                            seed=genome_seed(name), max_pcs=200, matrix_checksum=matrix_checksum(m),
                            **outputs(r))
        print(name, m.shape[0], r.n_pcs, r.optimal_n_clusters)


def large():
    for name, make, seed in (("genome_chr1", lambda: genome_matrix("chr1"), genome_seed("chr1")),
                             ("c5arm", lambda: synth_hic_par(C5ARM_BINS, SEED_BASE + 5), SEED_BASE + 5)):
        t0 = time.time()
        m = make()
        n0 = m.shape[0]
        ck = matrix_checksum(m)
        r = O.tadpole(m, max_pcs=200, nthreads=THREADS, pca="eigh")
        del m
        pcs = r.pcs
        # the spectral gap at k (how well the top-k subspace is defined) for the tests' log
        sv = np.linalg.norm(pcs, axis=0)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), n0=n0, seed=seed, max_pcs=200,
                            pc_norms=sv, matrix_checksum=ck, **outputs(r))
        print(name, n0, r.n_pcs, r.optimal_n_clusters, r.scores.shape, f"{time.time() - t0:.1f} s", flush=True)
        del r


C5ARM_BINS = 24300
C5_BINS = 49851


def c5full():
    """BASELINE config 5 at full size: synth_hic_par(49 851, SEED_BASE + 5,
    centromere=True) -- chr1 @5kb -- through TADpole(centromere_search=TRUE)
    (R/TADpole.R:58-85,351-442), bug-compatible (the q arm keeps its bad bins,
    :78-80) and with the PCA by LAPACK dsyevr.  Outputs only (+ the matrix
    checksum).  The 19.9 GB matrix is cleaned in place and freed before the
    arms run (peak ~35 GB)."""
    t0 = time.time()
    m = synth_hic_par(C5_BINS, SEED_BASE + 5, centromere=True)
    ck = matrix_checksum(m)
    print("c5 matrix", f"{time.time() - t0:.1f} s", ck, flush=True)
    loaded = O.load_mat_arms(m, 0.01, fixed=False, inplace=True)
    del m
    out = {"n0": C5_BINS, "seed": SEED_BASE + 5, "max_pcs": 200, "matrix_checksum": ck}

    def log(arm, r):
        print("c5 arm", arm, len(r.good_idx1), r.n_pcs, r.optimal_n_clusters, r.scores.shape,
              f"{time.time() - t0:.1f} s", flush=True)

    a = O.arms_from_loaded(loaded, max_pcs=200, nthreads=THREADS, pca="eigh", log=log)
    out["bug_merging_arms"] = a.merging_arms
    out["bug_centromere"] = a.centromere
    for arm in ("p", "q"):
        r = getattr(a, arm)
        out.update(outputs(r, f"bug_{arm}_"))
        out[f"bug_{arm}_names"] = np.asarray(r.good_idx1, np.int32)
        out[f"bug_{arm}_pc_norms"] = np.linalg.norm(r.pcs, axis=0)
    np.savez_compressed(os.path.join(HERE, "c5full.npz"), **out)
    print("c5full", len(a.merging_arms), f"{time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "large":   # tens of minutes and ~35 GB: never part of "all"
        large()
    if what == "c5full":  # ~1 h and ~35 GB: never part of "all"
        c5full()
    for fn in (small, arms, genome, configs):
        if what in ("all", fn.__name__):
            fn()
