"""A/B timing of library switches (tp_debug_knob) on one synthetic matrix:
python tools/ab_knobs.py N0 'which=value,...' ['which=value,...' ...]
Prints per-configuration stage times (median of 3 runs) and PCA iterations."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "tests")]
import gpu_helpers as G  # noqa: E402
import tadpole_amd as tp  # noqa: E402
from tadpole_amd.synth import synth_hic, synth_hic_par  # noqa: E402

n0 = int(sys.argv[1])
m = synth_hic(n0, 20261017) if n0 < 8000 else synth_hic_par(n0, 20261017)
tp.TADpole(m, max_pcs=200)   # warm-up (contexts, code objects)
for cfg in sys.argv[2:]:
    sets = [tuple(int(v) for v in kv.split("=")) for kv in cfg.split(",") if kv]
    olds = [(w, G.knob(w, v)) for w, v in sets]
    runs = []
    for _ in range(3):
        t = tp.TADpole(m, max_pcs=200)
        runs.append(np.array(t.timings_ms))
    for w, v in olds:
        G.knob(w, v)
    tm = np.median(np.array(runs), axis=0)
    print(f"{cfg or 'default'}: total {tm[4]:.2f} ms  cor {tm[1]:.3f}  pca {tm[2]:.2f} sweep {tm[3]:.2f}  G {tm[6]:.2f} "
          f"GQ {tm[7]:.2f} ({int(tm[8])})  iters {int(tm[11])} resid {tm[13]:.1e} krylov {int(tm[16])}x{int(tm[17])}", flush=True)
