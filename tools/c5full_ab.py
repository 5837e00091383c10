"""c5_full arm schedules: median of 3 TADpole(centromere_search=True) calls on
the bench's 49 851-bin matrix (resident in HBM) per schedule.
python tools/c5full_ab.py [schedule ...]   schedules: conc (both arms at once),
serial (TADPOLE_ARMS_SERIAL=1), qN (q starts at p's progress stage N)"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402
import bench  # noqa: E402
from tadpole_amd.api import TADpole  # noqa: E402

dm, _ = bench._c5_resident(1, 0, 0)
for sch in sys.argv[1:] or ["conc", "serial"]:
    os.environ.pop("TADPOLE_ARMS_SERIAL", None)
    os.environ.pop("TADPOLE_ARMS_Q_AT", None)
    if sch == "serial":
        os.environ["TADPOLE_ARMS_SERIAL"] = "1"
    elif sch.startswith("q"):
        os.environ["TADPOLE_ARMS_Q_AT"] = sch[1:]
    TADpole(dm, max_pcs=200, centromere_search=True, inplace=True)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = TADpole(dm, max_pcs=200, centromere_search=True, inplace=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"{sch}: {np.median(ts):.4f} s  {[round(t, 4) for t in ts]}  p {np.round(r.p.timings_ms[:5], 1)} "
          f"q {np.round(r.q.timings_ms[:5], 1)}", flush=True)
