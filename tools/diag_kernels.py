"""GPU diagnostics: k_chol_inv accuracy + time, and per-phase cycle stamps of
the CONISS merge loop (tp_debug_* entries of libtadpole_hip.so)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from tadpole_amd import _lib  # noqa: E402

L = _lib.load()
B = ctypes.byref
D = ctypes.POINTER(ctypes.c_double)


def chol(b=256, cond=1e6):
    rng = np.random.default_rng(0)
    q, _ = np.linalg.qr(rng.standard_normal((b, b)))
    ev = np.logspace(0, -np.log10(cond), b)
    W = np.asfortranarray((q * ev) @ q.T)
    U = np.zeros((b, b), order="F"); X = np.zeros((b, b), order="F")
    ms = np.zeros(8); st = ctypes.c_int(0)
    L.tp_debug_chol(W.ctypes.data_as(D), B(ctypes.c_int(b)), B(ctypes.c_double(0.0)), B(ctypes.c_int(5)),
                    U.ctypes.data_as(D), X.ctypes.data_as(D), ms.ctypes.data_as(D), B(st))
    _lib.check(st)
    Uu = np.triu(U)
    e1 = np.abs(Uu.T @ Uu - W).max() / np.abs(W).max()
    e2 = np.abs(X @ Uu - np.eye(b)).max()
    print(f"chol b={b} cond={cond:.0e}: chol {ms[0]:.3f} ms, trsm(I) {ms[1]:.3f} ms  "
          f"|U'U-W|/|W|={e1:.2e}  |XU-I|={e2:.2e}\n    cycles: diag {ms[2]:.0f} panel {ms[3]:.0f} "
          f"trailing {ms[4]:.0f} prologue {ms[5]:.0f}", flush=True)


def coniss(n0=2000, k=200):
    """Per-merge cycle budget of both CONISS waves on the scores of a synthetic
    matrix (mask on the host, correlation and PCA through the library)."""
    import tadpole_oracle as O
    from tadpole_amd.synth import synth_hic
    m = synth_hic(n0, 20261017)
    cm = O.clean_symmetrize(m)
    bad, _, _ = O.bad_mask(cm, 0.01)
    g = np.flatnonzero(~bad)
    x = np.asfortranarray(cm[np.ix_(g, g)])
    n = x.shape[0]
    cor = np.zeros((n, n), order="F")
    p = np.zeros((n, k), order="F")
    st = ctypes.c_int(0)
    L.tp_cor(x.ctypes.data_as(D), B(ctypes.c_int(n)), B(ctypes.c_int(0)), cor.ctypes.data_as(D), B(st))
    _lib.check(st)
    L.tp_pca(cor.ctypes.data_as(D), B(ctypes.c_int(n)), B(ctypes.c_int(k)), B(ctypes.c_int(0)), p.ctypes.data_as(D),
             None, B(st))
    _lib.check(st)
    stamps = np.zeros(k * 16, np.int64)
    ms = ctypes.c_double(0)
    for _ in range(2):   # second run: warm code objects
        L.tp_debug_coniss_stamps(p.ctypes.data_as(D), B(ctypes.c_int(n)), B(ctypes.c_int(k)),
                                 stamps.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), B(ms), B(st))
        _lib.check(st)
    s = stamps.reshape(k, 16).astype(float) / (n - 1)
    na = {6: "writes+block loads", 7: "reductions+argmin", 0: "merge_at+records", 1: "wait X", 2: "choice",
          3: "wait Y"}
    nb = {8: "rec read", 9: "row wait+sums", 10: "ward+records", 11: "wait X", 14: "prefetch", 15: "wait Y"}
    print(f"coniss n={n} k={k}: stamped kernel {ms.value:.3f} ms ({ms.value * 1e3 / (n - 1):.2f} us/merge)",
          flush=True)
    for i in (0, 63, 127, 128, 160, 191, 192, k - 1):
        print(f"  tree {i + 1:3d}: A " + ", ".join(f"{v} {s[i, q]:.0f}" for q, v in na.items()) +
              f" (sum {sum(s[i, q] for q in na):.0f})", flush=True)
        print(f"            B " + ", ".join(f"{v} {s[i, q]:.0f}" for q, v in nb.items()) +
              f" (sum {sum(s[i, q] for q in nb):.0f})", flush=True)


def eig(b=256):
    """The library's b x b eigensolver (tp_debug_eigsym) on a graded spectrum:
    wall time of the call, accuracy, orthogonality (rocSOLVER is no longer
    linked, so there is nothing to compare against but LAPACK's values)."""
    import time
    rng = np.random.default_rng(1)
    q, _ = np.linalg.qr(rng.standard_normal((b, b)))
    ev = np.sort(rng.gamma(1.0, 1.0, b))[::-1] ** 4
    H = np.asfortranarray(((q * ev) @ q.T + ((q * ev) @ q.T).T) / 2)
    th = np.zeros(b); V = np.zeros((b, b), order="F"); st = ctypes.c_int(0)
    for _ in range(2):
        t0 = time.perf_counter()
        L.tp_debug_eigsym(H.ctypes.data_as(D), B(ctypes.c_int(b)), B(ctypes.c_int(1)), th.ctypes.data_as(D),
                          V.ctypes.data_as(D), B(st))
        _lib.check(st)
        ms = (time.perf_counter() - t0) * 1e3
    ref = np.sort(ev)
    res = np.abs(H @ V - V * th).max() / ref.max()
    orth = np.abs(V.T @ V - np.eye(b)).max()
    print(f"eig b={b}: {ms:.3f} ms (call)  max|dev|/max={np.abs(th - ref).max() / ref.max():.2e}  "
          f"resid/max {res:.2e}  |V'V-I| {orth:.2e}", flush=True)


def sytrd(b=256):
    rng = np.random.default_rng(2)
    h = rng.standard_normal((b, b))
    h = np.asfortranarray(h + h.T)
    ms = ctypes.c_double(0); st = ctypes.c_int(0); stamps = np.zeros(4, np.int64)
    L.tp_debug_sytrd(h.ctypes.data_as(D), B(ctypes.c_int(b)), B(ms),
                     stamps.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), B(st))
    _lib.check(st)
    names = (["reflector", "partials+B1", "p+B2", "update+B0"] if b <= 256 else
             ["reflector", "pass", "combine", "-"])
    per = ", ".join(f"{n} {v / max(1, b - 2):.0f}" for n, v in zip(names, stamps))
    print(f"sytrd b={b}: {ms.value:.3f} ms (stamped build); cycles a step: {per}; "
          f"total {stamps.sum() / max(1, b - 2):.0f}", flush=True)


if __name__ == "__main__":
    import sys
    what = sys.argv[1:] or ["chol", "coniss"]
    if "eig" in what:
        eig(256)
    if "sytrd" in what:
        sytrd(256)
        sytrd(480)
    if "chol" in what:
        chol(256, 1e3)
        chol(256, 1e10)
        chol(480, 1e6)
    if "coniss" in what:
        coniss()
    if "coniss3" in what:
        coniss(7808, 200)
    if "coniss24" in what:   # above the LDS capacity: the global-memory variant
        coniss(24300, 200)

