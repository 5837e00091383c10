"""Thin ctypes wrappers around the stage entry points (tests only)."""
import ctypes

import numpy as np

from tadpole_amd import _lib
from tadpole_amd._lib import cdbl, cint, dp, ip

B = ctypes.byref


def _st():
    return cint(0)


def mask(m, bad_frac=0.01, flags=None):
    L = _lib.load()
    if flags is None:
        mm = np.ascontiguousarray(m, np.float64)
        flags = _lib.TP_FLAG_ROW_MAJOR
    else:
        mm = m
    n0 = mm.shape[0]
    bad = np.zeros(n0, np.int32); rm = np.zeros(n0); good = np.zeros(n0, np.int32)
    ng, st = cint(0), _st()
    L.tp_mask(dp(mm), B(cint(n0)), B(cdbl(bad_frac)), B(cint(flags)), B(cint(0)), ip(bad), dp(rm), B(ng),
              ip(good), B(st))
    _lib.check(st)
    return bad.astype(bool), rm, good[:ng.value] - 1


def cor(x):
    L = _lib.load()
    xf = np.asfortranarray(x, np.float64)
    n = xf.shape[0]
    out = np.zeros((n, n), order="F")
    st = _st()
    L.tp_cor(dp(xf), B(cint(n)), B(cint(0)), dp(out), B(st))
    _lib.check(st)
    return out


def pca(c, k):
    L = _lib.load()
    cf = np.asfortranarray(c, np.float64)
    n = cf.shape[0]
    p = np.zeros((n, k), order="F")
    sd = np.zeros(k)
    st = _st()
    L.tp_pca(dp(cf), B(cint(n)), B(cint(k)), B(cint(0)), dp(p), dp(sd), B(st))
    _lib.check(st)
    return p, sd


def coniss(p):
    L = _lib.load()
    pf = np.asfortranarray(p, np.float64)
    n, c = pf.shape
    merge = np.zeros(2 * (n - 1), np.int32); h = np.zeros(n - 1); bnd = np.zeros(n - 1, np.int32)
    st = _st()
    L.tp_coniss(dp(pf), B(cint(n)), B(cint(c)), B(cint(0)), ip(merge), dp(h), ip(bnd), B(st))
    _lib.check(st)
    return merge.reshape(2, n - 1).T.copy(), h, bnd - 1


def dist(p):
    L = _lib.load()
    pf = np.asfortranarray(p, np.float64)
    n, c = pf.shape
    d = np.zeros(n * (n - 1) // 2)
    st = _st()
    L.tp_dist(dp(pf), B(cint(n)), B(cint(c)), B(cint(0)), dp(d), B(st))
    _lib.check(st)
    return d


def ch(p, labels):
    L = _lib.load()
    pf = np.asfortranarray(p, np.float64)
    n, k = pf.shape
    lab = np.ascontiguousarray(labels, np.int32)
    out = cdbl(0.0)
    st = _st()
    L.tp_ch(dp(pf), B(cint(n)), B(cint(k)), ip(lab), B(cint(int(lab.max()))), B(cint(0)), B(out), B(st))
    _lib.check(st)
    return out.value


def sweep_dev(p, min_clusters=2):
    """tp_sweep_dev on a device copy of p; returns per-tree records."""
    import torch
    L = _lib.load()
    n, k = p.shape
    dP = torch.from_numpy(np.asfortranarray(p, np.float64).ravel(order="F").copy()).cuda()
    w_cap = n
    nclu = np.zeros(k, np.int32); sc = np.zeros(k * w_cap)
    ma = np.zeros(k * (n - 1), np.int32); mb = np.zeros(k * (n - 1), np.int32)
    co = np.zeros(k * (n - 1)); he = np.zeros(k * (n - 1))
    w, st = cint(0), _st()
    torch.cuda.synchronize()
    L.tp_sweep_dev(ctypes.c_void_p(dP.data_ptr()), B(cint(n)), B(cint(k)), B(cint(min_clusters)), B(cint(0)),
                   None, B(cint(w_cap)), ip(nclu), dp(sc), B(w), ip(ma), ip(mb), dp(co), dp(he), B(st))
    _lib.check(st)
    ww = w.value
    return dict(n_cluster=nclu, scores=sc[:k * ww].reshape(ww, k).T.copy(),
                mrg_a=ma.reshape(k, n - 1), mrg_b=mb.reshape(k, n - 1), cost=co.reshape(k, n - 1),
                height=he.reshape(k, n - 1))


def sweep(p, min_clusters=2):
    L = _lib.load()
    pf = np.asfortranarray(p, np.float64)
    n, k = pf.shape
    w_cap = n
    nclu = np.zeros(k, np.int32); sc = np.zeros(k * w_cap)
    merge = np.zeros(2 * (n - 1), np.int32); h = np.zeros(n - 1)
    w, npcs, ncl, st = cint(0), cint(0), cint(0), _st()
    L.tp_sweep(dp(pf), B(cint(n)), B(cint(k)), B(cint(min_clusters)), B(cint(0)), B(cint(w_cap)), ip(nclu),
               dp(sc), B(w), B(npcs), B(ncl), ip(merge), dp(h), B(st))
    _lib.check(st)
    ww = w.value
    return dict(n_cluster=nclu, scores=sc[:k * ww].reshape(ww, k).T.copy(), n_pcs=npcs.value,
                n_clusters=ncl.value, merge=merge.reshape(2, n - 1).T.copy(), height=h)


def eigsym(h, method=1):
    """PCA Rayleigh-Ritz eigensolver test hook (tp_debug_eigsym)."""
    L = _lib.load()
    hf = np.asfortranarray(h, np.float64)
    b = hf.shape[0]
    theta = np.zeros(b)
    v = np.zeros((b, b), order="F")
    st = _st()
    L.tp_debug_eigsym(dp(hf), B(cint(b)), B(cint(method)), dp(theta), dp(v), B(st))
    _lib.check(st)
    return theta, v


def knob(which, value):
    """tp_debug_knob: set a tuning switch, return its previous value."""
    L = _lib.load()
    old, st = cint(0), _st()
    L.tp_debug_knob(B(cint(which)), B(cint(value)), B(old), B(st))
    _lib.check(st)
    return old.value
