"""Per-phase cycles of the batched CONISS (k_coniss_b, STAMPS build of the same
source) on the PC scores of a synthetic matrix: python tools/coniss_b_stamps.py
[N0].  Needs the diagnostic build (`make -C tadpole_amd/csrc STAMPS=1`: the
product build leaves the stamped kernels out)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import gpu_helpers as G  # noqa: E402
import tadpole_amd as tp  # noqa: E402
from tadpole_amd import _lib  # noqa: E402
from tadpole_amd.synth import synth_hic, synth_hic_par  # noqa: E402

n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 7808
res = tp.TADpole(synth_hic(n0, 20261018) if n0 < 8000 else synth_hic_par(n0, 20261018))
L = _lib.load()
n, k = int(res.timings_ms[14]), int(res.timings_ms[15])
P = np.zeros((n, k), order="F")
st = ctypes.c_int(0)
L.tp_debug_last_scores(ctypes.byref(ctypes.c_int(n)), ctypes.byref(ctypes.c_int(k)),
                       P.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(st))
_lib.check(st)
names = ["A1b rank", "B1", "A2 ward+writes", "B2", "A3 run+costs", "B3", "A4 stores", "A2 window+rows", "A4 blkmin",
         "B4", "A1 scan+B0"]

for kb in (1, 0):
    G.knob(52, kb)
    stamps = np.zeros(k * 16, np.int64)
    ms = ctypes.c_double(0)
    D = ctypes.POINTER(ctypes.c_double)
    L.tp_debug_coniss_stamps(P.ctypes.data_as(D), ctypes.byref(ctypes.c_int(n)), ctypes.byref(ctypes.c_int(k)),
                             stamps.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), ctypes.byref(ms),
                             ctypes.byref(st))
    _lib.check(st)
    print(f"knob52={kb} n={n} k={k}: stamped kernel {ms.value:.3f} ms", flush=True)
    if kb != 1:
        continue
    s = stamps.reshape(k, 16).astype(float)
    for t in (1, 2, 8, 64, 128, 200):
        if t > k:
            continue
        row = s[t - 1]
        nb = max(1.0, row[14])
        ph = ", ".join(f"{nm} {row[q] / nb:.0f}" for q, nm in enumerate(names))
        print(f"  tree {t:3d}: {int(nb)} batches ({row[13] / nb:.2f} merges each, {int(row[15])} retries), "
              f"{row[:11].sum() / nb:.0f} cycles a batch, {row[:11].sum() / (n - 1):.0f} a merge", flush=True)
        print(f"            {ph}", flush=True)
G.knob(52, 1)
