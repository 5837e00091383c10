"""Generate the committed golden fixtures from the CPU oracle (run here, on
CPU; the reference itself is R and cannot run in this image).

  python tests/golden/make_golden.py

Fixtures: synthetic Hi-C inputs (SURVEY.md §8(d) generator) at N0 = 64, 200,
300 with the oracle's TADpole() outputs (mask, n_pcs, optimal_n_clusters,
NA-padded CH scores, merge boundaries and heights of the final tree, TAD
coordinates of every significant level), plus a PC-score fixture for the sweep
alone.  control.bed / case.bed are the reference's own diffT example data
(inst/extdata) and diffT_curve.json the breakpoints of misc/DiffT_score.png.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import tadpole_oracle as O  # noqa: E402
from tadpole_amd.synth import synth_hic  # noqa: E402

CASES = [("n64", 64, 20261101, 200), ("n200", 200, 20261016, 200), ("n300", 300, 20261102, 100)]


def main():
    for name, n0, seed, max_pcs in CASES:
        m = synth_hic(n0, seed)
        r = O.tadpole(m, max_pcs=max_pcs, nthreads=4)
        lev = sorted(r.clusters)
        np.savez_compressed(
            os.path.join(HERE, f"{name}.npz"),
            matrix=m.astype(np.int32), max_pcs=max_pcs, seed=seed,
            bad=r.bad, n_pcs=r.n_pcs, optimal_n_clusters=r.optimal_n_clusters,
            scores=r.scores, merge_b=r.merge_b, height=r.height,
            n_cluster=r.sweep.n_cluster,
            levels=np.array(lev, np.int32),
            coords=np.concatenate([np.c_[np.full(len(r.clusters[q]), q), r.clusters[q]] for q in lev]),
            pcs=r.pcs)
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


if __name__ == "__main__":
    main()
