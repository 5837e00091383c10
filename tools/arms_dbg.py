"""Timeline of the two centromere arms run concurrently (tadpole_amd.api
_tadpole_arms): both arms' progress words polled from a third thread (GPU box).
  python tools/arms_dbg.py [n0]"""
import ctypes
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tadpole_amd as tp  # noqa: E402
from tadpole_amd import _lib, api  # noqa: E402
from tadpole_amd.synth import SEED_BASE, synth_hic_par  # noqa: E402

n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 49851
dm = torch.from_numpy(synth_hic_par(n0, SEED_BASE + 5, centromere=True)).cuda()
tp.TADpole(dm, centromere_search=True, inplace=True)   # warm-up
sp, sq = api._arm_streams(0)
L = _lib.load()
pq = np.zeros(1, np.int32)
st = _lib.cint(0)
for rep in range(2):
    pq[0] = -1
    L.tp_progress_attach(ctypes.byref(_lib.cint(0)), ctypes.c_void_p(sq.cuda_stream), pq.ctypes.data_as(ctypes.c_void_p),
                         ctypes.byref(st))
    seen = []
    done = [False]
    t0 = time.perf_counter()

    def poll():
        last = None
        while not done[0]:
            v = int(pq[0])
            if v != last:
                seen.append((round(1e3 * (time.perf_counter() - t0), 1), "q", v))
                last = v
            time.sleep(1e-4)

    th = threading.Thread(target=poll)
    th.start()
    torch.cuda.synchronize()
    r = tp.TADpole(dm, centromere_search=True, inplace=True)
    torch.cuda.synchronize()
    done[0] = True
    th.join()
    print(f"rep {rep}: {1e3 * (time.perf_counter() - t0):.1f} ms", seen,
          {a: [round(x, 1) for x in getattr(r, a).timings_ms[:5]] for a in ("p", "q")}, flush=True)
L.tp_progress_attach(ctypes.byref(_lib.cint(0)), ctypes.c_void_p(sq.cuda_stream), None, ctypes.byref(st))
