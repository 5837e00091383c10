"""k_sytrd_reg A/B: time (mean of 3 launches) and output bits of one b x b
tridiagonalisation with the library named by TADPOLE_LIB; the outputs go to
gpurun_out/sytrd_<tag>_<b>.npz for a bitwise comparison between builds.
python tools/sytrd_ab.py TAG [b ...]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tadpole_amd import _lib  # noqa: E402

tag = sys.argv[1]
L = _lib.load()
D = ctypes.POINTER(ctypes.c_double)
I = ctypes.POINTER(ctypes.c_int)
for b in [int(x) for x in sys.argv[2:]] or [256, 224]:
    rng = np.random.default_rng(b)
    h = rng.standard_normal((b, b))
    h = np.asfortranarray(h + h.T)
    ms = np.zeros(1); d = np.zeros(b); e = np.zeros(b); tau = np.zeros(b)
    A = np.zeros((b, b), order="F"); st = ctypes.c_int(0)
    for _ in range(2):
        L.tp_debug_sytrd2(h.ctypes.data_as(D), ctypes.byref(ctypes.c_int(b)), ctypes.byref(ctypes.c_int(1)),
                          ms.ctypes.data_as(D), d.ctypes.data_as(D), e.ctypes.data_as(D),
                          tau.ctypes.data_as(D), A.ctypes.data_as(D), ctypes.byref(st))
        _lib.check(st)
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez(f"gpurun_out/sytrd_{tag}_{b}.npz", d=d, e=e, tau=tau, A=A)
    ev = np.linalg.eigvalsh(h)
    T = np.diag(d) + np.diag(e[:b - 1], 1) + np.diag(e[:b - 1], -1)
    err = np.abs(np.sort(np.linalg.eigvalsh(T)) - ev).max() / np.abs(ev).max()
    print(f"{tag} b={b}: k_sytrd_reg {ms[0] * 1e3:.1f} us, eigenvalue err {err:.1e}", flush=True)
