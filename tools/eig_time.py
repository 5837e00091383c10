"""Rayleigh-Ritz eigensolver timings on one GPU: the tridiagonalisation
kernels A/B (tp_debug_sytrd2: 1 = k_sytrd_reg, 2 = k_sytrd32, mean of 3
launches), the stamped k_sytrd32 phases, and one whole eig_sym call.
python tools/eig_time.py [b ...]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tadpole_amd import _lib  # noqa: E402

L = _lib.load()
D = ctypes.POINTER(ctypes.c_double)
B = ctypes.byref
for b in [int(x) for x in sys.argv[1:]] or [256]:
    rng = np.random.default_rng(b)
    h = rng.standard_normal((b, b))
    h = np.asfortranarray(h + h.T)
    ev = np.linalg.eigvalsh(h)
    for which in (1, 2):
        if which == 1 and b % 16:
            continue
        ms = np.zeros(1); d = np.zeros(b); e = np.zeros(b); tau = np.zeros(b)
        A = np.zeros((b, b), order="F"); st = ctypes.c_int(0)
        for _ in range(2):
            L.tp_debug_sytrd2(h.ctypes.data_as(D), B(ctypes.c_int(b)), B(ctypes.c_int(which)), ms.ctypes.data_as(D),
                              d.ctypes.data_as(D), e.ctypes.data_as(D), tau.ctypes.data_as(D), A.ctypes.data_as(D), B(st))
            _lib.check(st)
        T = np.diag(d) + np.diag(e[:b - 1], 1) + np.diag(e[:b - 1], -1)
        err = np.abs(np.sort(np.linalg.eigvalsh(T)) - ev).max() / np.abs(ev).max()
        print(f"b={b} which={which}: {ms[0] * 1e3:.1f} us, eigenvalue err {err:.1e}", flush=True)
    ms = ctypes.c_double(0); st = ctypes.c_int(0); stamps = np.zeros(4, np.int64)
    L.tp_debug_sytrd(h.ctypes.data_as(D), B(ctypes.c_int(b)), B(ms), stamps.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), B(st))
    _lib.check(st)
    per = ", ".join(f"{n} {v / max(1, b - 2):.0f}" for n, v in zip(["reflector", "partials+B1", "p+B2", "update+B0"], stamps))
    print(f"b={b} k_sytrd32 stamped: {ms.value * 1e3:.1f} us; cycles a step: {per}", flush=True)
    th = np.zeros(b); V = np.zeros((b, b), order="F")
    for _ in range(3):
        t0 = time.perf_counter()
        L.tp_debug_eigsym(h.ctypes.data_as(D), B(ctypes.c_int(b)), B(ctypes.c_int(1)), th.ctypes.data_as(D),
                          V.ctypes.data_as(D), B(st))
        _lib.check(st)
        wall = (time.perf_counter() - t0) * 1e3
    res = np.abs(h @ V - V * th).max() / np.abs(ev).max()
    print(f"b={b} eig_sym call {wall:.3f} ms (host wall incl. copies), |th-ev| {np.abs(th - ev).max() / np.abs(ev).max():.1e}, "
          f"resid {res:.1e}, |V'V-I| {np.abs(V.T @ V - np.eye(b)).max():.1e}", flush=True)
