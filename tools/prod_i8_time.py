"""Device time of one C3-size int8-digit product (tp_debug_prod_i8 at K = 7808,
M = 7810, N = 64) against the fp64 path; no reference check (diagnostic builds
give wrong results by design)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tadpole_amd import _lib  # noqa: E402

L = _lib.load()
D = ctypes.POINTER(ctypes.c_double)
K, M, N = 7808, 7810, 64
rng = np.random.default_rng(1)
A = np.asfortranarray(rng.uniform(-1, 1, size=(K, M)))
B = np.asfortranarray(rng.standard_normal((K, N)) / np.sqrt(K))
O8 = np.zeros((M - 1, N), order="F"); O64 = np.zeros((M - 1, N), order="F"); ms = np.zeros(2); st = ctypes.c_int(0)
I = lambda v: ctypes.byref(ctypes.c_int(v))  # noqa: E731
L.tp_debug_prod_i8(A.ctypes.data_as(D), I(K), I(M), B.ctypes.data_as(D), I(N), O8.ctypes.data_as(D),
                   O64.ctypes.data_as(D), ms.ctypes.data_as(D), ctypes.byref(st))
_lib.check(st)
print(f"{os.path.basename(os.environ.get('TADPOLE_LIB', 'default'))}: int8 product {ms[0] * 1e3:.1f} us, "
      f"fp64 {ms[1] * 1e3:.1f} us, max |diff| {np.max(np.abs(O8 - O64)):.2e}", flush=True)
