"""A/B timing of library switches (tp_debug_knob) on one synthetic matrix:
python tools/ab_knobs.py N0 'which=value,...' ['which=value,...' ...]
Prints per-configuration stage times (median of REPS runs, env, default 3),
the wall time of the TADpole() call on a GPU-resident copy of the matrix, and
PCA iterations.  Configurations are interleaved round-robin (ROUNDS, default
1) so drift on the box hits them alike."""
import time
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
import torch  # noqa: E402

md = torch.from_numpy(np.ascontiguousarray(m, dtype=np.float64)).to("cuda:0")
tp.TADpole(md, max_pcs=200)   # warm-up (contexts, code objects)
REPS = int(os.environ.get("REPS", "3"))
cfgs = sys.argv[2:]
runs = {c: [] for c in cfgs}
walls = {c: [] for c in cfgs}
for _ in range(int(os.environ.get("ROUNDS", "1"))):
    for cfg in cfgs:
        sets = [tuple(int(v) for v in kv.split("=")) for kv in cfg.split(",") if kv]
        olds = [(w, G.knob(w, v)) for w, v in sets]
        for _ in range(REPS):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            t = tp.TADpole(md, max_pcs=200)
            walls[cfg].append(time.perf_counter() - t0)
            runs[cfg].append(np.array(t.timings_ms))
        for w, v in olds:
            G.knob(w, v)
for cfg in cfgs:
    tm = np.median(np.array(runs[cfg]), axis=0)
    print(f"{cfg or 'default'}: wall {1e3 * np.median(walls[cfg]):.2f} ms  total {tm[4]:.2f} ms  mask {tm[0]:.3f} "
          f"cor {tm[1]:.3f}  pca {tm[2]:.2f} sweep {tm[3]:.2f}  G {tm[6]:.2f} GQ {tm[7]:.2f} ({int(tm[8])})  "
          f"iters {int(tm[11])} resid {tm[13]:.1e} krylov {int(tm[16])}x{int(tm[17])}", flush=True)
