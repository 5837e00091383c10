"""Device time of one C3-size int8-digit product (tp_debug_prod_i8 at K = 7729,
M = 7731, N = 64: B's digits + the product + the split-K reduce) for each
product kernel (knob 36: 1 = k_pd_prod<1>, 5 = k_pd_prodA)
against the fp64 path, and whether the kernels give the same bits.
python tools/prod_i8_time.py [K]   (env N=32: the C-space block width; KNOBS="1 5")"""
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
N = int(os.environ.get("N", "64"))   # 32: the C-space blocks (k_pd_prodA<1, 2> whatever knob 36 says)
M = K + 2
rng = np.random.default_rng(1)
A = np.asfortranarray(rng.uniform(-1, 1, size=(K, M)))
B = np.asfortranarray(rng.standard_normal((K, N)) / np.sqrt(K))
outs = {}
for kn in [int(v) for v in os.environ.get("KNOBS", "1 5 1 5").split()]:
    old = ctypes.c_int(0); st = ctypes.c_int(0)
    L.tp_debug_knob(I(36), I(kn), ctypes.byref(old), ctypes.byref(st))
    _lib.check(st)
    O8 = np.zeros((M - 1, N), order="F"); O64 = np.zeros((M - 1, N), order="F"); ms = np.zeros(2)
    L.tp_debug_prod_i8(A.ctypes.data_as(D), I(K), I(M), B.ctypes.data_as(D), I(N), O8.ctypes.data_as(D),
                       O64.ctypes.data_as(D), ms.ctypes.data_as(D), ctypes.byref(st))
    _lib.check(st)
    outs[kn] = O8
    first = next(iter(outs.values()))
    same = np.array_equal(O8.view(np.uint64), first.view(np.uint64))
    print(f"K={K} N={N} knob36={kn}: int8 product {ms[0] * 1e3:.1f} us, fp64 {ms[1] * 1e3:.1f} us, "
          f"max |int8 - fp64| {np.max(np.abs(O8 - O64)):.2e}, bits == the first: {same}", flush=True)
L.tp_debug_knob(I(36), I(5), ctypes.byref(ctypes.c_int(0)), ctypes.byref(ctypes.c_int(0)))
