"""PCA degree margin vs parity: for each margin, TADpole on several synthetic
matrices against the oracle (boundaries, n_pcs, CH error) plus PCA iterations
and residual from the pipeline's timing record.  GPU box only."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "oracle"), os.path.join(HERE, "tests")]
import gpu_helpers as G  # noqa: E402
import tadpole_amd as tp  # noqa: E402
import tadpole_oracle as O  # noqa: E402
from tadpole_amd.synth import synth_hic  # noqa: E402

cases = [(2000, 20261017), (2000, 5), (1500, 6), (1000, 7), (2500, 8)]
refs = {}
for n0, seed in cases:
    m = synth_hic(n0, seed)
    refs[(n0, seed)] = (m, O.tadpole(m, max_pcs=200))
for margin in [int(x) for x in sys.argv[1:]] or [2, 1, 0]:
    old = G.knob(6, margin)
    for (n0, seed), (m, ref) in refs.items():
        got = tp.TADpole(m, max_pcs=200)
        same = (got.n_pcs == ref.n_pcs and got.optimal_n_clusters == ref.optimal_n_clusters
                and set(got.clusters) == {str(q) for q in ref.clusters}
                and all(np.array_equal(got.clusters[str(q)], v) for q, v in ref.clusters.items()))
        a, b = got.scores, ref.scores
        fin = ~np.isnan(b)
        rel = float(np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin]))) if a.shape == b.shape else None
        tm = getattr(got, "timings_ms", None)
        it = int(tm[11]) if tm is not None else -1
        rs = float(tm[13]) if tm is not None else -1
        print(f"margin {margin} n0 {n0} seed {seed}: match {same} ch_rel {rel:.2e} iters {it} resid {rs:.2e}",
              flush=True)
    G.knob(6, old)
