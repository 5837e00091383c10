"""k_chol_inv cycle stamps (tp_debug_chol_inv): prologue, factorisation +
output, cycles inside the diagonal factors; b = 64 and 256."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tadpole_amd import _lib  # noqa: E402

L = _lib.load()
D = ctypes.POINTER(ctypes.c_double)
rng = np.random.default_rng(0)
for b in (64, 256):
    Z = rng.standard_normal((4 * b, b))
    W = np.asfortranarray(Z.T @ Z)
    dg = np.zeros(b); Y = np.zeros((b, b), order="F"); ms = np.zeros(8); st = ctypes.c_int(0)
    L.tp_debug_chol_inv(W.ctypes.data_as(D), ctypes.byref(ctypes.c_int(b)), ctypes.byref(ctypes.c_double(0.0)),
                        ctypes.byref(ctypes.c_int(5)), dg.ctypes.data_as(D), Y.ctypes.data_as(D),
                        ms.ctypes.data_as(D), ctypes.byref(st))
    _lib.check(st)
    print(f"chol_inv b={b}: {ms[0] * 1e3:.1f} us (trsm of I {ms[6] * 1e3:.1f} us); cycles: prologue {ms[3]:.0f}, "
          f"factor+output {ms[4]:.0f}, inside diagonal factors {ms[5]:.0f}", flush=True)
