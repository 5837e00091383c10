"""X'X kernel A/B: time of the pipeline's 128-column int8 tile kernels
(tp_debug_xtx mode 2, mean of 3) with knob 32 = 0 (register-staged) and 1
(LDS-DMA ring) on a synthetic count matrix, and bitwise equality of the two.
python tools/xtx_ab.py N [maxv (0: synthetic Hi-C)] [knob=value ...]"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "tests")]
import gpu_helpers as G  # noqa: E402
from tadpole_amd import _lib  # noqa: E402

n = int(sys.argv[1])
maxv = int(sys.argv[2]) if len(sys.argv) > 2 else 9000   # 0: a synthetic Hi-C matrix
knobs = [tuple(int(v) for v in kv.split("=")) for kv in sys.argv[3:]]   # which=value, set for both arms
L = _lib.load()
if maxv == 0:
    from tadpole_amd.synth import synth_hic, synth_hic_par
    x = np.asfortranarray(synth_hic(n, 20261017) if n < 8000 else synth_hic_par(n, 20261017))
else:
    x = np.asfortranarray(np.random.default_rng(n).integers(0, maxv, size=(n, n)).astype(np.float64))
for w, v in knobs:
    G.knob(w, v)
D = ctypes.POINTER(ctypes.c_double)
out = {}
for glds in (0, 1, 0, 1):
    old = G.knob(32, glds)
    S = np.zeros((n, n), order="F")
    ns = ctypes.c_int(-1); ms = ctypes.c_double(0); st = ctypes.c_int(0)
    L.tp_debug_xtx(x.ctypes.data_as(D), ctypes.byref(ctypes.c_int(n)), ctypes.byref(ctypes.c_int(2)),
                   S.ctypes.data_as(D), ctypes.byref(ns), ctypes.byref(ms), ctypes.byref(st))
    G.knob(32, old)
    _lib.check(st)
    out[glds] = S
    macs = ns.value ** 2 * n * n / 2 * n
    print(f"n={n} slices={ns.value} glds={glds}: {ms.value:.3f} ms = {2 * macs / ms.value / 1e9:.0f} TOP/s int8 "
          f"(upper-half MACs)", flush=True)
print("bit-identical" if np.array_equal(out[0], out[1]) else "DIFFERENT", flush=True)
