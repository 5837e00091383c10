"""A's int8 digit image at C3 size (K = 7729 rows, M = 7731 columns of
[C | m | 1]) built both ways -- fused = 1: k_pd_digits_cm (digits + the
means, two columns a workgroup), 0: k_pd_digits_reg + k_colmean -- three times
each, for `rocprofv3 --kernel-trace --stats -- python tools/pd_image_time.py`.
Checks the two images, scales and means agree bit for bit."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tadpole_amd import _lib  # noqa: E402

L = _lib.load()
D = ctypes.POINTER(ctypes.c_double)
I = lambda v: ctypes.byref(ctypes.c_int(v))  # noqa: E731
K = int(sys.argv[1]) if len(sys.argv) > 1 else 7729
M = K + 2
rng = np.random.default_rng(5)
A = np.asfortranarray(rng.uniform(-1, 1, size=(K, M)))
cp, Kp = (M + 63) // 64 * 64, (K + 63) // 64 * 64
res = {}
for fused in (0, 1, 0, 1, 0, 1):
    img = np.zeros(7 * cp * Kp, dtype=np.int8)
    sc, cm, cr = np.zeros(cp), np.zeros(M - 2), np.zeros(M - 2)
    nd, st = ctypes.c_int(0), ctypes.c_int(0)
    L.tp_debug_pd_image(A.ctypes.data_as(D), I(K), I(M), I(fused), img.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)),
                        sc.ctypes.data_as(D), cm.ctypes.data_as(D), cr.ctypes.data_as(D), ctypes.byref(nd),
                        ctypes.byref(st))
    _lib.check(st)
    res[fused] = (img, sc, cm if fused else cr)
same = all(np.array_equal(res[0][q].view(np.uint8), res[1][q].view(np.uint8)) for q in range(3))
print(f"K={K} M={M}: fused and separate images, scales and means identical: {same}")
