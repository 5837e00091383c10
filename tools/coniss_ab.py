"""CONISS / sweep time of one synthetic matrix with the library named by
TADPOLE_LIB (A/B builds): python tools/coniss_ab.py N0 [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tadpole_amd as tp  # noqa: E402
from tadpole_amd.synth import synth_hic, synth_hic_par  # noqa: E402

n0 = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
m = synth_hic(n0, 20261018) if n0 < 8000 else synth_hic_par(n0, 20261018)
dm = torch.from_numpy(m).cuda()
tp.TADpole(dm)
t = np.array([tp.TADpole(dm).timings_ms[:11] for _ in range(reps)])
med = np.median(t, axis=0)
print(f"{os.path.basename(os.environ.get('TADPOLE_LIB', 'default'))} n0={n0}: coniss {med[9]:.3f} ms  "
      f"sweep {med[3]:.3f}  total {med[4]:.3f}  (min coniss {t[:, 9].min():.3f})", flush=True)
