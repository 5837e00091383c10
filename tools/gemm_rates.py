"""fp64 MFMA GEMM rates of the library kernels on this GPU (tp_debug_gemm):
the 128 x 128 square kernel, the 64 x 64 kernel and the long-K row kernel
(k_gemm_ts, the Krylov product shape) on random operands."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tadpole_amd import _lib  # noqa: E402

L = _lib.load()
D = ctypes.POINTER(ctypes.c_double)
B = ctypes.byref


def run(m, n, k, ta, sym, kernel, reps=3):
    rng = np.random.default_rng(1)
    A = np.asfortranarray(rng.standard_normal((k, m) if ta else (m, k)))
    Bm = np.asfortranarray(rng.standard_normal((k, n)))
    C = np.zeros((m, n), order="F")
    ms = ctypes.c_double(0)
    st = ctypes.c_int(0)
    best = 1e9
    for _ in range(reps):
        L.tp_debug_gemm(A.ctypes.data_as(D), Bm.ctypes.data_as(D), B(ctypes.c_int(m)), B(ctypes.c_int(n)),
                        B(ctypes.c_int(k)), B(ctypes.c_int(int(ta))), B(ctypes.c_int(int(sym))),
                        B(ctypes.c_int(kernel)), C.ctypes.data_as(D), B(ms), B(st))
        _lib.check(st)
        best = min(best, ms.value)
    flops = (m * n * k if sym else 2.0 * m * n * k)
    print(f"M={m} N={n} K={k} ta={ta} sym={sym} kernel={kernel}: {best * 1e3:.1f} us  {flops / best / 1e9:.1f} TF/s",
          flush=True)


if __name__ == "__main__":
    run(8192, 8192, 8192, True, False, 1)
    run(8192, 8192, 8192, True, False, 0)
    run(7729, 7729, 7729, True, True, 1)
    run(7729, 64, 7729, True, False, 4, reps=5)
    run(7729, 128, 7729, True, False, 4, reps=5)
    run(24057, 64, 24057, True, False, 4, reps=3)
