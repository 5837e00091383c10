"""Runs one diagnostic kernel entry (for rocprofv3 PMC passes):
python tools/run_kernel.py sytrd B WHICH | chol B"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tadpole_amd import _lib  # noqa: E402

L = _lib.load()
D = ctypes.POINTER(ctypes.c_double)
what = sys.argv[1]
b = int(sys.argv[2])
rng = np.random.default_rng(b)
st = ctypes.c_int(0)
if what == "sytrd":
    which = int(sys.argv[3])
    h = rng.standard_normal((b, b))
    h = np.asfortranarray(np.tril(h + h.T))
    d = np.zeros(b); e = np.zeros(b); tau = np.zeros(b); A = np.zeros((b, b), order="F"); ms = np.zeros(8)
    L.tp_debug_sytrd2(h.ctypes.data_as(D), ctypes.byref(ctypes.c_int(b)), ctypes.byref(ctypes.c_int(which)),
                      ms.ctypes.data_as(D), d.ctypes.data_as(D), e.ctypes.data_as(D), tau.ctypes.data_as(D),
                      A.ctypes.data_as(D), ctypes.byref(st))
    print(f"sytrd b={b} which={which}: {ms[0]*1e3:.1f} us")
elif what == "chol":
    q, _ = np.linalg.qr(rng.standard_normal((b, b)))
    W = np.asfortranarray((q * np.logspace(0, -6, b)) @ q.T)
    dg = np.zeros(b); Y = np.zeros((b, b), order="F"); ms = np.zeros(8)
    L.tp_debug_chol_inv(W.ctypes.data_as(D), ctypes.byref(ctypes.c_int(b)), ctypes.byref(ctypes.c_double(0.0)),
                        ctypes.byref(ctypes.c_int(3)), dg.ctypes.data_as(D), Y.ctypes.data_as(D),
                        ms.ctypes.data_as(D), ctypes.byref(st))
    print(f"chol b={b}: {ms[0]*1e3:.1f} us, trsm {ms[6]*1e3:.1f} us")
_lib.check(st)
if what == "xtx":
    mode = int(sys.argv[3])
    x = rng.integers(0, 4000, size=(b, b)).astype(np.float64)
    xf = np.asfortranarray(x)
    S = np.zeros((b, b), order="F")
    ns = ctypes.c_int(0); ms = ctypes.c_double(0)
    L.tp_debug_xtx(xf.ctypes.data_as(D), ctypes.byref(ctypes.c_int(b)), ctypes.byref(ctypes.c_int(mode)),
                   S.ctypes.data_as(D), ctypes.byref(ns), ctypes.byref(ms), ctypes.byref(st))
    _lib.check(st)
    print(f"xtx b={b} mode={mode} slices={ns.value}: {ms.value*1e3:.1f} us")
if what == "gemm":   # Z = G Q at the C2 shape by the library's policy: gemm M N K [reps]
    M, N, K = b, int(sys.argv[3]), int(sys.argv[4])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    A = np.asfortranarray(rng.standard_normal((K, M)))
    Bm = np.asfortranarray(rng.standard_normal((K, N)))
    C = np.zeros((M, N), order="F")
    ms = ctypes.c_double(0)
    I = lambda v: ctypes.byref(ctypes.c_int(v))  # noqa: E731
    for _ in range(reps):
        L.tp_debug_gemm(A.ctypes.data_as(D), Bm.ctypes.data_as(D), I(M), I(N), I(K), I(1), I(0), I(2),
                        C.ctypes.data_as(D), ctypes.byref(ms), ctypes.byref(st))
        _lib.check(st)
    print(f"gemm {M}x{N}x{K}: {ms.value*1e3:.1f} us")
