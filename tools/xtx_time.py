"""Device time of the pipeline's 128-column int8 X'X tile kernel (tp_debug_xtx
mode 2, mean of 3 launches) on a synthetic Hi-C count matrix, for the library
TADPOLE_LIB names (A/B builds from tools/build_variant.sh), and a checksum of S.
python tools/xtx_time.py N [reps] [knob=value ...]   (env CLIP=c: counts clipped to c)"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "tests")]
import gpu_helpers as G  # noqa: E402
from tadpole_amd import _lib  # noqa: E402
from tadpole_amd.synth import synth_hic, synth_hic_par  # noqa: E402

n = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
knobs = [tuple(int(v) for v in kv.split("=")) for kv in sys.argv[3:]]
L = _lib.load()
x = np.asfortranarray(synth_hic(n, 20261017) if n < 8000 else synth_hic_par(n, 20261017))
if os.environ.get("CLIP"):   # counts clipped to CLIP (127: one 7-bit slice)
    np.minimum(x, float(os.environ["CLIP"]), out=x)
for w, v in knobs:
    G.knob(w, v)
D = ctypes.POINTER(ctypes.c_double)
S = np.zeros((n, n), order="F")
for r in range(reps):
    ns = ctypes.c_int(-1); ms = ctypes.c_double(0); st = ctypes.c_int(0)
    L.tp_debug_xtx(x.ctypes.data_as(D), ctypes.byref(ctypes.c_int(n)), ctypes.byref(ctypes.c_int(2)),
                   S.ctypes.data_as(D), ctypes.byref(ns), ctypes.byref(ms), ctypes.byref(st))
    _lib.check(st)
    print(f"{os.path.basename(_lib.LIB_PATH)} n={n} slices={ns.value}: {ms.value:.3f} ms", flush=True)
u = S.view(np.uint64)
print(f"checksum {int(np.bitwise_xor.reduce(u.ravel())):#018x} sum {S.sum():.17g}", flush=True)
