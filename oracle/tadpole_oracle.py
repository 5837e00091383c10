"""ORACLE — TEST INFRASTRUCTURE ONLY.  PARITY UNPINNED.

CPU restatement of the reference's per-matrix path, ``R/TADpole.R:15-140,
344-510`` and ``R/DiffT.R:1-73``, in numpy (+ the C sweep in ``tp_oracle.c``).
The reference is R and calls third-party R packages (rioja, fpc, vegan, stats,
bigmemory, Matrix) that are absent from this container, and it ships no tests
or fixtures for this path; R cannot be installed (no network).  So this oracle
is pinned only by (a) independent implementations available here
(``numpy.quantile(method='linear')`` = R type 7, ``numpy.linalg.svd`` = LAPACK
gesdd as in R's ``La.svd``, ``scipy.spatial.distance.pdist``,
``sklearn.metrics.calinski_harabasz_score``), (b) a brute-force distance-matrix
CONISS, and (c) the reference README facts that need no input file.  See
DESIGN.md "Oracle".

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  The product (``tadpole_amd``) never does.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

NA_BITS = 0x7FF00000000007A2     # R NA_real_
NA_REAL = struct.unpack("<d", struct.pack("<Q", NA_BITS))[0]


def is_r_na(x: np.ndarray) -> np.ndarray:
    """True where x carries R's NA_real_ bit pattern (not a plain NaN)."""
    return np.asarray(x, np.float64).view(np.uint64) == np.uint64(NA_BITS)


def lib():
    """Load (building if needed) the C half of the oracle."""
    global _LIB
    if _LIB is None:
        so = os.path.join(_HERE, "libtp_oracle.so")
        src = os.path.join(_HERE, "tp_oracle.c")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(so)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        c_int, c_double = ctypes.c_int, ctypes.c_double
        L.tpo_ward.restype = c_double
        L.tpo_ward.argtypes = [dp, c_int, dp, c_int, c_int]
        L.tpo_coniss.argtypes = [dp, c_int, c_int, c_int, ip, ip, dp, dp]
        L.tpo_coniss_bruteforce.argtypes = [dp, c_int, c_int, c_int, ip, dp]
        L.tpo_bstick_ld.argtypes = [dp, c_int, ip]
        L.tpo_bstick_dd.argtypes = [dp, c_int, ip]
        L.tpo_seg_ss.restype = c_double
        L.tpo_seg_ss.argtypes = [dp, c_int, c_int, c_int, c_int, dp]
        L.tpo_trS.restype = c_double
        L.tpo_trS.argtypes = [dp, c_int, c_int, c_int]
        L.tpo_ch_levels.argtypes = [dp, c_int, c_int, c_int, ip, c_int, c_int, c_double, dp]
        L.tpo_sweep.argtypes = [dp, c_int, c_int, c_int, c_int, c_int, c_int, ip, dp,
                                c_int, ip, ip, dp, dp]
        L.tpo_dist_r.argtypes = [dp, c_int, c_int, c_int, dp]
        L.tpo_rowmeans_ld.argtypes = [dp, c_int, c_int, c_int, dp]
        L.tpo_rowmeans_dd.argtypes = [dp, c_int, c_int, c_int, dp]
        _LIB = L
    return _LIB


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


# ---------------------------------------------------------------- load_mat ---

def clean_symmetrize(mat: np.ndarray, inplace: bool = False) -> np.ndarray:
    """``R/TADpole.R:19-20``: NA/NaN -> 0, then ``forceSymmetric(uplo='U')``.
    ``inplace`` (a C-contiguous float64 array, the 49 851-bin C5 fixture):
    the same assignments in row blocks, no N^2 index arrays or copy."""
    if not inplace:
        m = np.array(mat, dtype=np.float64, copy=True)
        m[np.isnan(m)] = 0.0
        iu = np.triu_indices(m.shape[0], 1)
        m.T[iu] = m[iu]
        return m
    m = mat
    if m.dtype != np.float64 or not m.flags["C_CONTIGUOUS"]:
        raise ValueError("inplace clean_symmetrize needs a C-contiguous float64 array")
    n = m.shape[0]
    blk = 256
    for r0 in range(0, n, blk):
        r1 = min(n, r0 + blk)
        rows = m[r0:r1]
        rows[np.isnan(rows)] = 0.0
    for r0 in range(0, n, blk):        # lower (row > col) <- upper (col, row)
        r1 = min(n, r0 + blk)
        m[r0:r1, :r0] = m[:r0, r0:r1].T
        sub = m[r0:r1, r0:r1]
        il = np.tril_indices(r1 - r0, -1)
        sub[il] = sub.T[il]
    return m


def quantile7(x: np.ndarray, p: float) -> float:
    """R ``quantile(type=7)`` (stats quantile.default [ext]):
    index = 1 + (n-1) p; lo = floor, hi = ceiling; q = x[lo], replaced by
    (1-h) x[lo] + h x[hi] where index > lo and x[hi] != x[lo]."""
    xs = np.sort(np.asarray(x, np.float64))
    n = xs.size
    index = 1.0 + float(max(n - 1, 0)) * float(p)
    lo = int(np.floor(index))
    hi = int(np.ceil(index))
    q = xs[lo - 1]
    if index > lo and xs[hi - 1] != q:
        h = index - lo
        q = (1.0 - h) * q + h * xs[hi - 1]
    return float(q)


def bad_mask(m: np.ndarray, bad_frac: float, rowmeans: str = "ld"):
    """``R/TADpole.R:35-37``.  Returns (bad bool[N0], r, q)."""
    n0 = m.shape[0]
    r = np.empty(n0)
    mm = np.ascontiguousarray(m)
    fn = lib().tpo_rowmeans_ld if rowmeans == "ld" else lib().tpo_rowmeans_dd
    fn(_dp(mm), n0, n0, 0, _dp(r))
    bad = np.diag(m) == 0
    q = None
    if bad_frac:
        # seq(0, 1, by = bad_frac)[2] == bad_frac
        q = quantile7(r, bad_frac)
        bad = bad | (r < q)
    return bad, r, q


# -------------------------------------------------------------- sparse_cor ---

def sparse_cor(x: np.ndarray) -> np.ndarray:
    """``R/TADpole.R:94-100`` + NaN -> 0 (``:449``)."""
    n = x.shape[0]
    m = np.array([float(np.sum(x[:, j], dtype=np.longdouble) / n) for j in range(n)])
    s = x.T @ x
    cov = (s - n * np.outer(m, m)) / (n - 1)
    sd = np.sqrt(np.diag(cov))
    with np.errstate(invalid="ignore", divide="ignore"):
        cor = cov / np.outer(sd, sd)
    cor[np.isnan(cor)] = 0.0
    return cor


def prcomp_x(c: np.ndarray, k: int, method: str = "svd") -> np.ndarray:
    """``prcomp(cor, rank.=k)$x`` (``R/TADpole.R:453``): centre columns,
    LAPACK gesdd SVD (as R's La.svd), scores = Xc V[:, :k].  ``method="eigh"``:
    the top-k eigenvectors of Xc'Xc by LAPACK dsyevr instead (same subspaces,
    several times cheaper than the full SVD; used only for the bench's CPU
    baseline timing)."""
    mu = np.array([float(np.sum(c[:, j], dtype=np.longdouble) / c.shape[0])
                   for j in range(c.shape[1])])
    xc = c - mu[None, :]
    if method == "eigh" and k < xc.shape[1]:
        import scipy.linalg as sl
        n = xc.shape[1]
        _, v = sl.eigh(xc.T @ xc, subset_by_index=[n - k, n - 1], driver="evr")
        return xc @ v[:, ::-1]
    _, _, vt = np.linalg.svd(xc, full_matrices=False)
    return xc @ vt[:k].T


# ------------------------------------------------------------------- sweep ---

@dataclass
class Sweep:
    n_cluster: np.ndarray          # k ints
    scores: np.ndarray             # k x w (NA = R NA_real_)
    mrg_a: np.ndarray              # k x (N-1)
    mrg_b: np.ndarray
    cost: np.ndarray
    height: np.ndarray
    status: int = 0


def sweep(p: np.ndarray, min_clusters: int = 2, bstick: str = "dd",
          nthreads: int = 0) -> Sweep:
    """``find_params`` loop body for every i (``R/TADpole.R:104-123``)."""
    n, k = p.shape
    pt = np.ascontiguousarray(p, dtype=np.float64)
    wcap = max(1, n)
    nc = np.full(k, -1, np.int32)
    sc = np.empty(k * wcap)
    ma = np.empty((k, n - 1), np.int32)
    mb = np.empty((k, n - 1), np.int32)
    co = np.empty((k, n - 1))
    he = np.empty((k, n - 1))
    st = lib().tpo_sweep(_dp(pt), n, k, k, int(min_clusters), 1 if bstick == "ld" else 0,
                         int(nthreads), _ip(nc), _dp(sc), wcap, _ip(ma), _ip(mb),
                         _dp(co), _dp(he))
    if st < 0:
        raise MemoryError("oracle sweep allocation failed")
    w = int(nc.max()) if (nc > 0).any() else 1
    scores = sc.reshape(wcap, k).T[:, :w].copy()
    return Sweep(nc, scores, ma, mb, co, he, st)


def coniss(p: np.ndarray):
    """Canonical CONISS of one prefix matrix (all columns of ``p``)."""
    n, c = p.shape
    pt = np.ascontiguousarray(p, dtype=np.float64)
    ma = np.empty(n - 1, np.int32); mb = np.empty(n - 1, np.int32)
    co = np.empty(n - 1); he = np.empty(n - 1)
    lib().tpo_coniss(_dp(pt), n, c, c, _ip(ma), _ip(mb), _dp(co), _dp(he))
    return ma, mb, co, he


def coniss_bruteforce(p: np.ndarray):
    n, c = p.shape
    pf = np.asfortranarray(p, dtype=np.float64)
    mb = np.empty(n - 1, np.int32); he = np.empty(n - 1)
    lib().tpo_coniss_bruteforce(_dp(pf), n, n, c, _ip(mb), _dp(he))
    return mb, he


def dist_r(p: np.ndarray) -> np.ndarray:
    n, c = p.shape
    pf = np.asfortranarray(p, dtype=np.float64)
    d = np.empty(n * (n - 1) // 2)
    lib().tpo_dist_r(_dp(pf), n, n, c, _dp(d))
    return d


def select_params(scores: np.ndarray):
    """``R/TADpole.R:134-135``: rowMeans(na.rm=TRUE) in long double, first max."""
    means = np.full(scores.shape[0], np.nan)
    for i in range(scores.shape[0]):
        row = scores[i]
        ok = ~np.isnan(row)
        if ok.any():
            means[i] = float(np.sum(row[ok].astype(np.longdouble)) / np.longdouble(ok.sum()))
    if np.all(np.isnan(means)):
        raise ValueError("no finite CH row mean")
    n_pcs = int(np.nanargmax(means)) + 1
    row = scores[n_pcs - 1]
    n_clusters = int(np.nanargmax(row)) + 1
    return n_pcs, n_clusters


# ----------------------------------------------------------------- cutree ---

def hclust_merge(mrg_a: np.ndarray, mrg_b: np.ndarray, n: int) -> np.ndarray:
    """``chclust(...)$merge`` (rioja, ``R/TADpole.R:108,460,465``) in
    ``stats::hclust`` encoding [ext: hclust's hcass2 conventions; rioja's own
    row order is unverified here]: row s joins the adjacent clusters whose
    first bins are mrg_a[s] (left) and mrg_b[s] (right), 0-based; an
    observation is -(bin+1) and a cluster the 1-based step that formed it (a
    merged cluster keeps the id of its left part, as hclust keeps the smaller
    index); a singleton comes before a cluster, and of two clusters the
    earlier step comes first; two singletons in observation order."""
    ident = -(np.arange(n, dtype=np.int64) + 1)
    out = np.empty((n - 1, 2), np.int64)
    for s in range(n - 1):
        x, y = int(ident[mrg_a[s]]), int(ident[mrg_b[s]])
        if (x > 0 > y) or (x > 0 and y > 0 and x > y):
            x, y = y, x
        out[s] = (x, y)
        ident[mrg_a[s]] = s + 1
    return out


def hclust_cutree(merge: np.ndarray, n: int, kk: int) -> np.ndarray:
    """``stats::cutree(tree, k)`` on an hclust merge matrix, from its
    definition: apply the first n-k merges (union-find), then number the
    groups 1..k in order of their first observation.  Independent of the
    constrained-tree shortcut in ``cutree_labels``."""
    parent = np.arange(n)

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x
    rep = {}
    for s in range(n - kk):
        ends = []
        for v in merge[s]:
            ends.append(-v - 1 if v < 0 else rep[v])
        ra, rb = find(ends[0]), find(ends[1])
        parent[max(ra, rb)] = min(ra, rb)
        rep[s + 1] = min(ra, rb)
    roots = np.array([find(x) for x in range(n)])
    lab = np.zeros(n, np.int64)
    seen = {}
    for x in range(n):
        if roots[x] not in seen:
            seen[roots[x]] = len(seen) + 1
        lab[x] = seen[roots[x]]
    return lab


def cutree_labels(mrg_b: np.ndarray, n: int, kk: int) -> np.ndarray:
    """``stats::cutree(clust, k)`` for a constrained tree: the boundaries of the
    last kk-1 merges, labels 1..kk left to right."""
    lab = np.ones(n, np.int64)
    if kk > 1:
        b = np.sort(np.asarray(mrg_b[n - kk:], np.int64))
        lab[b] += 1
        lab = np.cumsum(lab) - np.arange(n)
    return lab


def rle(x):
    x = np.asarray(x)
    if x.size == 0:
        return np.array([], np.int64), x
    cut = np.flatnonzero(x[1:] != x[:-1]) + 1
    starts = np.concatenate([[0], cut])
    lengths = np.diff(np.concatenate([starts, [x.size]]))
    return lengths, x[starts]


def fix_values(lengths, values):
    """``R/TADpole.R:503-510``."""
    values = np.array(values, copy=True)
    zeros = [i for i in np.flatnonzero(values == 0) if i != 0 and i != len(values) - 1]
    for i in zeros:
        if values[i - 1] == values[i + 1]:
            values[i] = values[i - 1]
    return lengths, values


def coords_for(labels_good: np.ndarray, good_idx1: np.ndarray, bad_idx1: np.ndarray):
    """``R/TADpole.R:471-494``: re-insert bad columns as 0 by original index,
    fix_values, RLE -> (start, end) rows with value != 0."""
    names = np.concatenate([good_idx1, bad_idx1]).astype(np.float64)
    vals = np.concatenate([labels_good.astype(np.float64), np.zeros(len(bad_idx1))])
    order = np.argsort(names, kind="stable")
    clusters = vals[order]
    lens, v = fix_values(*rle(clusters))
    fixed = np.repeat(v, lens)
    lens2, v2 = rle(fixed)
    eb = np.cumsum(lens2)
    start = np.concatenate([[1], eb[:-1] + 1])
    keep = v2 != 0
    return np.stack([start[keep], eb[keep]], axis=1).astype(np.int64)


@dataclass
class OracleResult:
    n_pcs: int
    optimal_n_clusters: int
    scores: np.ndarray
    clusters: dict = field(default_factory=dict)
    bad: np.ndarray = None
    good_idx1: np.ndarray = None
    pcs: np.ndarray = None
    cor: np.ndarray = None
    sweep: Sweep = None
    merge_b: np.ndarray = None
    height: np.ndarray = None
    merge: np.ndarray = None
    fixed_opt: np.ndarray = None      # fixed cluster vector at optimal_n_clusters (arm merge input)


def _core(x: np.ndarray, good_names1: np.ndarray, bad_idx1: np.ndarray, max_pcs: int,
          min_clusters: int, bstick: str, nthreads: int, pcs=None, pca: str = "svd") -> OracleResult:
    """``R/TADpole.R:444-497`` (and the per-arm body ``:359-432``) on a masked
    matrix x whose rows carry the 1-based names ``good_names1``."""
    c = None
    if pcs is None:
        c = sparse_cor(x)
        k = min(max_pcs, x.shape[0])
        pcs = prcomp_x(c, k, pca)
    sw = sweep(pcs, min_clusters, bstick=bstick, nthreads=nthreads)
    if sw.status == 1:
        raise ValueError("invalid 'times' argument (no broken-stick level)")
    n_pcs, n_clusters = select_params(sw.scores)
    n = x.shape[0]
    mb = sw.mrg_b[n_pcs - 1]
    res = OracleResult(n_pcs, n_clusters, sw.scores, good_idx1=good_names1,
                       pcs=pcs, cor=c, sweep=sw, merge_b=mb, height=sw.height[n_pcs - 1],
                       merge=hclust_merge(sw.mrg_a[n_pcs - 1], mb, n))
    row = sw.scores[n_pcs - 1]
    for kk in np.flatnonzero(~np.isnan(row)) + 1:
        lab = cutree_labels(mb, n, int(kk))
        res.clusters[int(kk)] = coords_for(lab, good_names1, bad_idx1)
    lab = cutree_labels(mb, n, n_clusters)
    res.fixed_opt = fixed_vector(lab, good_names1, bad_idx1)
    return res


def tadpole(mat: np.ndarray, max_pcs: int = 200, min_clusters: int = 2,
            bad_frac: float = 0.01, pcs: np.ndarray | None = None,
            bstick: str = "dd", nthreads: int = 0, pca: str = "svd") -> OracleResult:
    """``TADpole(..., centromere_search=FALSE)`` body, ``R/TADpole.R:344-349,
    444-497``, from an in-memory matrix (``load_mat`` minus the plots).
    ``pca``: "svd" (R's full SVD) or "eigh" (see ``prcomp_x``)."""
    m = clean_symmetrize(mat)
    bad, _, _ = bad_mask(m, bad_frac)
    good = np.flatnonzero(~bad)
    x = m[np.ix_(good, good)]
    res = _core(x, good + 1, np.flatnonzero(bad) + 1, max_pcs, min_clusters, bstick, nthreads, pcs, pca)
    res.bad = bad
    return res


def fixed_vector(labels_good, names1, bad_idx1) -> np.ndarray:
    """``R/TADpole.R:413-432``: c(good, bad = 0) ordered by numeric name,
    fix_values, inverse.rle (duplicate names kept, stable order)."""
    names = np.concatenate([np.asarray(names1), np.asarray(bad_idx1)]).astype(np.float64)
    vals = np.concatenate([np.asarray(labels_good, np.float64), np.zeros(len(bad_idx1))])
    order = np.argsort(names, kind="stable")
    lens, v = fix_values(*rle(vals[order]))
    return np.repeat(v, lens)


def _r_drop(n: int, neg) -> np.ndarray:
    """Positions 0..n-1 kept by R's ``x[-neg, ]`` for numeric ``neg`` (R
    negativeSubscript [ext]: in-range values drop that position, out-of-range
    ones are ignored)."""
    neg = np.asarray(neg, np.int64)
    drop = neg[(neg >= 1) & (neg <= n)] - 1
    return np.setdiff1d(np.arange(n), drop)


def load_mat_arms(mat: np.ndarray, bad_frac: float = 0.01, fixed: bool = False, inplace: bool = False):
    """``load_mat(..., centromere_search=TRUE)`` (``R/TADpole.R:15-92``)
    without plots.  Returns ``("matrix", x, names1, bad_idx1)`` when there is no
    bad bin or the longest bad run touches an end (``:66-70``), else
    ``("arms", {"p": (x, names1, bad_idx1), "q": ...}, centromere1)``.

    Bug-compatible by default: the q-arm bad bins are removed with their
    ORIGINAL indices as positions in the arm-local matrix (``:78-80``), so an
    index inside the arm's length drops the wrong bin and one beyond it is
    ignored.  ``fixed=True`` removes them at their arm-local positions.
    ``inplace``: clean ``mat`` itself (see ``clean_symmetrize``)."""
    m = clean_symmetrize(mat, inplace)
    n0 = m.shape[0]
    bad, _, _ = bad_mask(m, bad_frac)
    idx = np.flatnonzero(bad) + 1
    if idx.size == 0:
        return ("matrix", m, np.arange(1, n0 + 1), idx)
    cut = np.flatnonzero(np.diff(idx) > 1) + 1
    runs = np.split(idx, cut)
    longest = runs[int(np.argmax([len(r) for r in runs]))]   # which.max: first max
    cs, ce = int(longest[0]), int(longest[-1])
    if cs == 1 or ce == n0:
        good = np.flatnonzero(~bad)
        return ("matrix", m[np.ix_(good, good)], good + 1, idx)
    arms = {}
    for arm, lo, hi, bad_arm in (("p", 1, cs - 1, idx[idx < cs]), ("q", ce + 1, n0, idx[idx > ce])):
        names = np.arange(lo, hi + 1)
        sub = np.ascontiguousarray(m[lo - 1:hi, lo - 1:hi])
        if bad_arm.size:
            keep = _r_drop(len(names), (bad_arm - lo + 1) if fixed else bad_arm)
            sub = sub[np.ix_(keep, keep)]
            names = names[keep]
        arms[arm] = (sub, names, bad_arm)
    return ("arms", arms, np.arange(cs, ce + 1))


@dataclass
class ArmsResult:
    p: OracleResult
    q: OracleResult
    merging_arms: np.ndarray
    centromere: np.ndarray


def tadpole_arms(mat: np.ndarray, max_pcs: int = 200, min_clusters: int = 2,
                 bad_frac: float = 0.01, fixed: bool = False, nthreads: int = 0, pca: str = "svd"):
    """``TADpole(..., centromere_search=TRUE)`` (``R/TADpole.R:351-442``).
    Returns an ``ArmsResult``; when ``load_mat`` returned a plain matrix R
    fails at ``mat$centromer`` (``:356``): bug-compatible mode raises, fixed
    mode runs the single-matrix path instead."""
    loaded = load_mat_arms(mat, bad_frac, fixed)
    if loaded[0] == "matrix":
        if not fixed:
            raise TypeError("$ operator is invalid for atomic vectors")
        return tadpole(mat, max_pcs, min_clusters, bad_frac, nthreads=nthreads, pca=pca)
    return arms_from_loaded(loaded, max_pcs, min_clusters, nthreads, pca)


def arms_from_loaded(loaded, max_pcs: int = 200, min_clusters: int = 2, nthreads: int = 0,
                     pca: str = "svd", log=None) -> "ArmsResult":
    """The arm loop and arm merge of ``R/TADpole.R:357-442`` on the output of
    ``load_mat_arms`` (split out so a caller can free the full matrix first).
    Each arm's matrix is dropped from ``loaded`` once its result exists."""
    kind, arms, cen = loaded
    if kind != "arms":
        raise ValueError("arms_from_loaded needs load_mat_arms' arm split")
    out = {}
    parts = []
    for arm in ("p", "q"):
        x, names, bad_arm = arms[arm]
        arms[arm] = (None, names, bad_arm)
        r = _core(x, names, bad_arm, max_pcs, min_clusters, "dd", nthreads, pca=pca)
        del x
        r.cor = None
        out[arm] = r
        if log:
            log(arm, r)
        parts += [r.fixed_opt, np.zeros(len(cen))]
    allv = np.concatenate(parts)[:-len(cen)]
    lens, v = rle(allv)
    eb = np.cumsum(lens)
    start = np.concatenate([[1], eb[:-1] + 1])
    keep = v != 0
    coords = np.stack([start[keep], eb[keep]], axis=1).astype(np.int64)
    return ArmsResult(out["p"], out["q"], coords, cen)


# ------------------------------------------------------------------ diffT ---

def bin_index(bed, size):
    """``R/DiffT.R:1-9``."""
    tad_index = np.zeros(size, np.int64)
    first = bed[0][1]
    for t, (_, s, e) in enumerate(bed, start=1):
        for b in range(s, e + 1):
            tad_index[b - first] = t
    return tad_index


def diffT(bed_x, bed_y):
    """``R/DiffT.R:19-50`` (O(L^2) as in R)."""
    if len(bed_x) != len(bed_y):
        raise ValueError("Both calls must have the same number of TADs.")
    sx, sy = bed_x[0][1], bed_y[0][1]
    ex, ey = bed_x[-1][2], bed_y[-1][2]
    tx = bin_index(bed_x, ex - sx + 1)
    ty = bin_index(bed_y, ey - sy + 1)
    tx = np.concatenate([np.ones(max(0, sx - sy), np.int64), tx,
                         np.full(max(0, ey - ex), tx.max(), np.int64)])
    ty = np.concatenate([np.ones(max(0, sy - sx), np.int64), ty,
                         np.full(max(0, ex - ey), ty.max(), np.int64)])
    assert len(tx) == len(ty)
    scores = []
    for b in range(len(tx)):
        x = (tx[b] != tx) | (tx[b] == 0)
        y = (ty[b] != ty) | (ty[b] == 0)
        scores.append(int(np.sum(x ^ y)))
    s = np.cumsum(scores).astype(np.float64)
    return s if max(scores) == 0 else s / s.max()
