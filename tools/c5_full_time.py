"""c5_full alone (BASELINE config 5: TADpole(centromere_search=TRUE) on the
49 851-bin chr1 @5kb matrix resident in HBM, one GPU), for kernel traces of its
two arms: python tools/c5_full_time.py [reps] [knob=value ...]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "tests")]
import torch  # noqa: E402

import bench  # noqa: E402
import gpu_helpers as G  # noqa: E402
from tadpole_amd.api import TADpole  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for kv in sys.argv[2:]:
    w, v = (int(x) for x in kv.split("="))
    G.knob(w, v)
dm, info = bench._c5_resident(1, 0, 0)
print(info, flush=True)
TADpole(dm, max_pcs=200, centromere_search=True, inplace=True)   # warm-up
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = TADpole(dm, max_pcs=200, centromere_search=True, inplace=True)
    torch.cuda.synchronize()
    print(f"c5_full {time.perf_counter() - t0:.4f} s  p {r.p.n_pcs}/{r.p.optimal_n_clusters}  "
          f"q {r.q.n_pcs}/{r.q.optimal_n_clusters}", flush=True)
