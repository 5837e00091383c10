"""Three TADpole() calls on the 24 300-bin C5-arm-shape matrix resident in
HBM (the bench's c5_arm workload), for rocprofv3 --kernel-trace --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tadpole_amd as tp  # noqa: E402
from tadpole_amd.synth import SEED_BASE, synth_hic_par  # noqa: E402

n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 24300
dm = torch.from_numpy(synth_hic_par(n0, SEED_BASE + 5)).cuda()
for _ in range(3):
    r = tp.TADpole(dm, inplace=True)
    print({k: round(float(v), 2) for k, v in zip(("mask", "cor", "pca", "sweep", "total"), r.timings_ms[:5])},
          flush=True)
