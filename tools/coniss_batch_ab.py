"""CONISS time of the batched kernel (knob 52 = 1) against the two-wave kernel
(knob 52 = 0) on one synthetic matrix, same library: python
tools/coniss_batch_ab.py N0 [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import tadpole_amd as tp  # noqa: E402
import gpu_helpers as G  # noqa: E402
from tadpole_amd.synth import synth_hic, synth_hic_par  # noqa: E402

n0 = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
m = synth_hic(n0, 20261018) if n0 < 8000 else synth_hic_par(n0, 20261018)
dm = torch.from_numpy(m).cuda()
res = {}
for kb in (0, 1, 0, 1):
    G.knob(52, kb)
    r0 = tp.TADpole(dm)
    t = np.array([tp.TADpole(dm).timings_ms[:11] for _ in range(reps)])
    med = np.median(t, axis=0)
    res.setdefault(kb, []).append((med[9], med[3], med[4], r0))
    print(f"knob52={kb} n0={n0}: coniss {med[9]:.3f} ms  sweep {med[3]:.3f}  total {med[4]:.3f}  "
          f"(min coniss {t[:, 9].min():.3f})", flush=True)
a, b = res[0][0][3], res[1][0][3]
same = (a.n_pcs == b.n_pcs and a.optimal_n_clusters == b.optimal_n_clusters
        and np.array_equal(a.scores.view(np.uint64), b.scores.view(np.uint64))
        and all(np.array_equal(a.clusters[q], b.clusters[q]) for q in a.clusters))
print("same results:", same, flush=True)
