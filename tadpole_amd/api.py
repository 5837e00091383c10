"""Host-side mirror of the reference R API (NAMESPACE:3-8): ``TADpole``,
``load_mat``, ``diffT``, ``random_bed`` and the ``tadpole`` result object.

The numeric hot path (mask, correlation, PCA, CONISS sweep, broken stick,
Calinski-Harabasz) runs in ``libtadpole_hip.so`` on the GPU; this module does
what the R host code does around it: file parsing, the NA-padded result
assembly, cutree, bad-column re-insertion and ``fix_values`` (R/TADpole.R:
470-510), the centromere arm split (R/TADpole.R:58-85, 351-442), and diffT.
Plots (``load_mat``'s levelplot/histogram, ``plot_hierarchy``, ``CH_map``) are
out of scope: they draw, they do not compute.
"""
from __future__ import annotations

import ctypes
import time
import logging
import os
import struct
import sys
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import TadpoleError, cdbl, cint, dp, ip

_log = logging.getLogger("tadpole_amd")

NA_BITS = 0x7FF00000000007A2
NA_REAL = struct.unpack("<d", struct.pack("<Q", NA_BITS))[0]


def is_na(x) -> np.ndarray:
    """R ``is.na`` on a score matrix: NA and NaN."""
    return np.isnan(np.asarray(x, np.float64))


def is_r_na(x) -> np.ndarray:
    """True only where the value carries R's NA_real_ bits (not NaN)."""
    return np.asarray(x, np.float64).view(np.uint64) == np.uint64(NA_BITS)


# ------------------------------------------------------------------ objects

@dataclass
class Chclust:
    """``rioja::chclust`` object (class c("chclust", "hclust")): what
    ``plot_hierarchy`` feeds to ``cutree`` / ``ggdendro::dendro_data``."""
    merge: np.ndarray            # (n-1) x 2 int, hclust encoding
    height: np.ndarray           # n-1 cumulative total dispersion
    order: np.ndarray            # 1..n
    label_ids: np.ndarray        # original bin indices (R's labels, as integers)
    boundary: np.ndarray         # 1-based first bin (in 1..n) of the right cluster per merge
    method: str = "coniss"
    dist_method: str = "euclidean"
    call: str = "rioja::chclust(d = dist(pcs))"

    @property
    def labels(self) -> List[str]:
        """R's ``labels`` (character): built on first use, not per pipeline."""
        lab = self.__dict__.get("_labels")
        if lab is None:
            lab = self.__dict__["_labels"] = np.asarray(self.label_ids, np.int64).astype(str).tolist()
        return lab

    @property
    def n(self) -> int:
        return len(self.order)

    def cutree(self, k: int) -> np.ndarray:
        """``stats::cutree(tree, k)``: labels 1..k in observation order."""
        n = self.n
        lab = np.ones(n, np.int64)
        if k > 1:
            b = np.sort(self.boundary[n - k:] - 1)
            lab[b] += 1
            lab = np.cumsum(lab) - np.arange(n)
        return lab

    def __repr__(self):
        return (f"\nCall:\n{self.call}\n\nCluster method   : {self.method}\n"
                f"Distance         : {self.dist_method}\nNumber of objects: {self.n}\n")


@dataclass
class Tadpole:
    """The ``tadpole`` list of R/TADpole.R:463-468 (plus ``merging_arms`` /
    per-arm ``p``, ``q`` entries when ``centromere_search`` is on)."""
    n_pcs: Optional[int] = None
    optimal_n_clusters: Optional[int] = None
    dendro: Optional[Chclust] = None
    clusters: Dict[str, np.ndarray] = field(default_factory=dict)   # "k" -> (m x 2) start, end
    scores: Optional[np.ndarray] = None                             # k x w, NA = R NA bits
    merging_arms: Optional[np.ndarray] = None
    p: Optional["Tadpole"] = None
    q: Optional["Tadpole"] = None
    bad_columns: Optional[np.ndarray] = None                        # 1-based original indices
    timings_ms: Optional[np.ndarray] = None
    # host seconds of this call's phases (upload through the pinned staging,
    # the library call, the Python assembly); not part of R's object
    host_s: Dict[str, float] = field(default_factory=dict)

    def __getitem__(self, key):
        return getattr(self, key)

    # R's cluster slot name on the arm branch is `cluster` (R/TADpole.R:407)
    @property
    def cluster(self):
        return self.clusters


# --------------------------------------------------------------- load_mat

def read_matrix(mat_file, nthreads: int = 0) -> np.ndarray:
    """``bigmemory::read.big.matrix(sep='\\t', type='double')`` (R/TADpole.R:17):
    a headerless tab-separated numeric matrix, parsed natively (memory-mapped,
    multi-threaded: ``tp_read_tsv``); NA/NaN/empty fields become NaN."""
    L = _lib.load()
    path = ctypes.c_char_p(os.fsencode(os.fspath(mat_file)))
    nr, nc, st = cint(0), cint(0), cint(0)
    L.tp_tsv_dims(ctypes.byref(path), ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(st))
    _lib.check(st)
    out = np.empty((nr.value, nc.value), np.float64)
    if out.size:
        th = nthreads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        L.tp_read_tsv(ctypes.byref(path), ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(cint(min(th, 64))),
                      ctypes.byref(cint(_lib.TP_FLAG_ROW_MAJOR)), dp(out), ctypes.byref(st))
        _lib.check(st)
    return out


def _read_to_device(mat_file, device: int, stream=None):
    """A matrix file parsed straight into a new float64 device tensor
    (``tp_read_tsv_dev``: row blocks through the library's pinned staging, each
    block's upload overlapping the parse of the next).  TADpole(path) never
    returns the matrix, so the pipeline may clean this copy in place."""
    L = _lib.load()
    if L.tp_device_count() <= 0:
        raise _lib.TadpoleError(_lib.TP_ERR_HIP, "no HIP device: there is no CPU path")
    import torch
    path = ctypes.c_char_p(os.fsencode(os.fspath(mat_file)))
    nr, nc, st = cint(0), cint(0), cint(0)
    L.tp_tsv_dims(ctypes.byref(path), ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(st))
    _lib.check(st)
    d = torch.empty((nr.value, nc.value), dtype=torch.float64, device=f"cuda:{device}")
    if d.numel():
        s = stream if stream is not None else torch.cuda.current_stream(device)
        th = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        L.tp_read_tsv_dev(ctypes.byref(path), ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(cint(min(th, 64))),
                          ctypes.byref(cint(device)), ctypes.c_void_p(s.cuda_stream), ctypes.c_void_p(d.data_ptr()),
                          ctypes.byref(st))
        _lib.check(st)
    return d


def _is_path(mat) -> bool:
    return isinstance(mat, (str, bytes)) or hasattr(mat, "__fspath__")


def _as_matrix(mat) -> np.ndarray:
    if _is_path(mat):
        return read_matrix(mat)
    m = np.asarray(mat, dtype=np.float64)
    if m.ndim != 2 or m.shape[0] != m.shape[1]:
        raise ValueError("the interaction matrix must be square")
    return m


def _layout(m: np.ndarray):
    if m.flags["F_CONTIGUOUS"] and not m.flags["C_CONTIGUOUS"]:
        return m, 0
    return np.ascontiguousarray(m), _lib.TP_FLAG_ROW_MAJOR


def clean_symmetrize(m: np.ndarray) -> np.ndarray:
    """R/TADpole.R:19-20 on the host (load_mat's return value): NaN -> 0, then
    forceSymmetric(uplo='U').  Row blocks, so no N^2 index arrays (the
    pipeline does the same on the device)."""
    out = np.array(m, dtype=np.float64, copy=True)
    np.nan_to_num(out, copy=False, nan=0.0, posinf=np.inf, neginf=-np.inf)
    n = out.shape[0]
    blk = max(1, min(n, (1 << 22) // max(n, 1)))
    for r0 in range(0, n, blk):
        r1 = min(n, r0 + blk)
        out[r0:r1, :r0] = out[:r0, r0:r1].T
        sub = out[r0:r1, r0:r1]
        il = np.tril_indices(r1 - r0, -1)
        sub[il] = sub.T[il]
    return out


def mask(mat, bad_frac: float = 0.01, device: int = 0):
    """GPU bad-column mask (R/TADpole.R:35-37).  Returns (bad bool[N0],
    rowMeans, good 1-based indices)."""
    L = _lib.load()
    m, flags = _layout(_as_matrix(mat))
    n0 = m.shape[0]
    bad = np.zeros(n0, np.int32)
    rm = np.zeros(n0)
    good = np.zeros(n0, np.int32)
    ng = cint(0)
    st = cint(0)
    L.tp_mask(dp(m), ctypes.byref(cint(n0)), ctypes.byref(cdbl(bad_frac)), ctypes.byref(cint(flags)),
              ctypes.byref(cint(device)), ip(bad), dp(rm), ctypes.byref(ng), ip(good), ctypes.byref(st))
    _lib.check(st)
    return bad.astype(bool), rm, good[:ng.value].copy()


class Mat(np.ndarray):
    """ndarray with R's ``attr(mat, 'bad_columns')`` and its row names (the
    1-based original bin index of every row)."""
    bad_columns: np.ndarray
    names: np.ndarray

    def __new__(cls, arr, bad_columns, names):
        obj = np.asarray(arr).view(cls)
        obj.bad_columns = np.asarray(bad_columns, np.int64)
        obj.names = np.asarray(names, np.int64)
        return obj

    def __array_finalize__(self, obj):
        self.bad_columns = getattr(obj, "bad_columns", np.zeros(0, np.int64))
        self.names = getattr(obj, "names", np.zeros(0, np.int64))


def _runs(idx: np.ndarray) -> List[np.ndarray]:
    """``split(idx, cumsum(seq_along(idx) %in% (which(diff(idx) > 1) + 1)))``."""
    if idx.size == 0:
        return []
    cut = np.flatnonzero(np.diff(idx) > 1) + 1
    return np.split(idx, cut)


def _message(text: str, verbose: bool) -> None:
    """R ``message()`` (R/TADpole.R:55-56,65,67,136-137,358): logged on the
    ``tadpole_amd`` logger, and written to stderr when ``verbose``."""
    _log.info(text)
    if verbose:
        print(text, file=sys.stderr, flush=True)


def _arm_plan(bad: np.ndarray, fixed: bool = False, verbose: bool = False):
    """The centromere split of load_mat (R/TADpole.R:58-85) as index sets.

    Returns None when R returns a plain matrix (no bad bin, R/TADpole.R:87-90,
    or the longest bad run touches an end, :66-70), else
    ``{"p": (names1, bad1), "q": (names1, bad1), "centromere": idx1}`` where
    names1 are the 1-based original bins each arm keeps.  Bug-compatible by
    default: the q-arm bad bins are removed with their ORIGINAL indices used
    as arm-local positions (R/TADpole.R:78-80; R ignores out-of-range negative
    subscripts and drops in-range ones, so the wrong bins go or none do);
    ``fixed=True`` removes them at their arm-local positions."""
    idx = np.flatnonzero(bad) + 1
    n0 = len(bad)
    if idx.size == 0:
        return None
    runs = _runs(idx)
    longest = runs[int(np.argmax([len(r) for r in runs]))]    # which.max: first max
    cs, ce = int(longest[0]), int(longest[-1])
    _message(f"centromere position: {cs} {ce}", verbose)
    if cs == 1 or ce == n0:
        _message("longest stretch of bad rows/columns at the ends, not splitting the matrix.", verbose)
        return None
    names_p, names_q = np.arange(1, cs), np.arange(ce + 1, n0 + 1)
    bad_p, bad_q = idx[idx < cs], idx[idx > ce]
    keep_p = _r_negative_keep(len(names_p), bad_p)
    keep_q = _r_negative_keep(len(names_q), bad_q - ce if fixed else bad_q)
    return {"p": (names_p[keep_p], bad_p), "q": (names_q[keep_q], bad_q), "centromere": np.arange(cs, ce + 1)}


def load_mat(mat_file, chr=None, start=None, end=None, resol=None, bad_frac: float = 0.01,
             centromere_search: bool = False, device: int = 0, fixed_centromere: bool = False,
             verbose: bool = False):
    """``load_mat`` (R/TADpole.R:15-92) without its plots.

    Returns the masked matrix (``Mat`` with ``bad_columns``) or, with
    ``centromere_search``, ``{"p": Mat, "q": Mat, "centromere": ndarray}``,
    bug-compatible with the reference unless ``fixed_centromere`` (see
    ``_arm_plan``); a plain matrix when the longest bad run touches an end
    (R/TADpole.R:66-70)."""
    raw = _as_matrix(mat_file)
    bad, _, good = mask(raw, bad_frac, device)
    bad_idx = np.flatnonzero(bad) + 1
    _message(f"{len(bad_idx)} bad columns found at position(s):", verbose)
    _message(" ".join(str(int(b)) for b in bad_idx), verbose)
    plan = _arm_plan(bad, fixed_centromere, verbose) if (bad.any() and centromere_search) else None
    if plan is None:
        return Mat(clean_symmetrize(raw[np.ix_(good - 1, good - 1)]), bad_idx, good)
    out = {arm: Mat(clean_symmetrize(raw[np.ix_(plan[arm][0] - 1, plan[arm][0] - 1)]), plan[arm][1], plan[arm][0])
           for arm in ("p", "q")}
    out["centromere"] = plan["centromere"]
    return out


def _r_negative_keep(n: int, neg: np.ndarray) -> np.ndarray:
    """Positions kept by R's ``x[-neg]`` on length n: negative subscripts are
    positions (the reference passes original bin indices here, R/TADpole.R:80),
    and out-of-range ones are silently ignored."""
    if neg.size == 0:
        return np.arange(n)
    drop = neg[(neg >= 1) & (neg <= n)] - 1
    return np.setdiff1d(np.arange(n), drop)


# ---------------------------------------------------------------- pipeline

def _is_device(m) -> bool:
    """A torch tensor resident on a GPU (the matrix is already in HBM)."""
    return type(m).__module__.startswith("torch") and getattr(m, "is_cuda", False)


def _pipeline(m, max_pcs: int, min_clusters: int, bad_frac: float, flags: int,
              device: int, stream=None, subset=None):
    """One tp_pipeline call.  ``m``: a host array, or a square float64 torch
    tensor on the GPU (tp_pipeline_dev on it: no host staging; unless
    TP_FLAG_CLEAN it is cleaned in place).  ``stream`` (a torch.cuda.Stream):
    the pipeline is queued on that stream with its own library context, so
    several pipelines can run concurrently on one GPU.  ``subset`` (1-based,
    strictly ascending bin indices): TP_FLAG_SUBSET, the pipeline runs on that
    principal submatrix of ``m``, read in place (no copy of it is made)."""
    L = _lib.load()
    dev_in = _is_device(m)
    if dev_in:
        if m.dim() != 2 or m.shape[0] != m.shape[1]:
            raise ValueError("the interaction matrix must be square")
        import torch
        if m.dtype != torch.float64 or not m.is_contiguous():
            m = m.to(torch.float64).contiguous()
        flags |= _lib.TP_FLAG_ROW_MAJOR
        device = m.device.index if m.device.index is not None else device
    else:
        m, lay = _layout(m)
        flags |= lay
    n0 = m.shape[0]
    t0 = time.perf_counter()
    t_up = 0.0
    good = np.zeros(n0, np.int32)
    nsub = n0
    if subset is not None:
        subset = np.asarray(subset, np.int64)
        nsub = int(subset.size)
        if nsub < 1 or nsub > n0:
            raise ValueError("subset: 1..n0 bin indices")
        good[:nsub] = subset
        flags |= _lib.TP_FLAG_SUBSET
    k_cap = max(1, min(max_pcs, nsub))
    w_cap = max(1, nsub)
    bad = np.zeros(n0, np.int32)
    nclu = np.zeros(k_cap, np.int32)
    scores = np.zeros(k_cap * w_cap)
    merge = np.zeros(2 * max(1, n0 - 1), np.int32)
    height = np.zeros(max(1, n0 - 1))
    boundary = np.zeros(max(1, n0 - 1), np.int32)
    timings = np.zeros(32)
    out = [cint(0) for _ in range(6)]
    n_good, k, w, n_pcs, n_clusters, st = out
    n_good.value = nsub if subset is not None else 0
    if stream is None and not dev_in:
        L.tp_pipeline(dp(m), ctypes.byref(cint(n0)), ctypes.byref(cint(max_pcs)), ctypes.byref(cint(min_clusters)),
                      ctypes.byref(cdbl(bad_frac)), ctypes.byref(cint(flags)), ctypes.byref(cint(device)),
                      ctypes.byref(cint(k_cap)), ctypes.byref(cint(w_cap)), ip(bad), ctypes.byref(n_good),
                      ip(good), ctypes.byref(k), ip(nclu), dp(scores), ctypes.byref(w), ctypes.byref(n_pcs),
                      ctypes.byref(n_clusters), ip(merge), dp(height), ip(boundary), dp(timings),
                      ctypes.byref(st))
    else:
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(device)
        if dev_in:
            dm = m
            # the library's own stream (handle 0 selects it) does not order
            # with torch's default stream: finish the producer of m first
            if stream.cuda_stream == 0:
                torch.cuda.current_stream(device).synchronize()
            else:
                stream.wait_stream(torch.cuda.current_stream(device))
        else:
            host = m if m.flags["C_CONTIGUOUS"] else np.ascontiguousarray(m.T)   # same buffer order as `lay`
            host = np.ascontiguousarray(host, dtype=np.float64)
            with torch.cuda.stream(stream):
                dm = torch.empty(host.shape, dtype=torch.float64, device=f"cuda:{device}")
            # through this stream's context's pinned staging (tp_upload_dev): a
            # pageable .to(device) shares the runtime's one staging path with
            # every other stream of the process
            # (tp_upload_counts_dev): blocks of exact 16-bit counts travel packed
            ust = cint(0)
            L.tp_upload_counts_dev(ctypes.c_void_p(host.ctypes.data), ctypes.byref(ctypes.c_longlong(host.size)),
                                   ctypes.c_void_p(dm.data_ptr()), ctypes.byref(cint(_upload_threads(host.nbytes))),
                                   ctypes.byref(cint(device)), ctypes.c_void_p(stream.cuda_stream), None,
                                   ctypes.byref(ust))
            _lib.check(ust)
            t_up = time.perf_counter() - t0
        L.tp_pipeline_dev(ctypes.c_void_p(dm.data_ptr()), ctypes.byref(cint(n0)), ctypes.byref(cint(max_pcs)),
                          ctypes.byref(cint(min_clusters)), ctypes.byref(cdbl(bad_frac)), ctypes.byref(cint(flags)),
                          ctypes.byref(cint(device)), ctypes.c_void_p(stream.cuda_stream),
                          ctypes.byref(cint(k_cap)), ctypes.byref(cint(w_cap)), ip(bad), ctypes.byref(n_good),
                          ip(good), ctypes.byref(k), ip(nclu), dp(scores), ctypes.byref(w), ctypes.byref(n_pcs),
                          ctypes.byref(n_clusters), ip(merge), dp(height), ip(boundary), dp(timings),
                          ctypes.byref(st))
        del dm
    _lib.check(st)
    t_call = time.perf_counter() - t0 - t_up
    n = n_good.value
    kk, ww = k.value, w.value
    sc = scores[:kk * ww].reshape(ww, kk).T.copy()
    return dict(bad=bad[:n].astype(bool) if subset is not None else bad.astype(bool), good=good[:n].copy(), k=kk, w=ww, n_cluster=nclu[:kk].copy(),
                scores=sc, n_pcs=n_pcs.value, n_clusters=n_clusters.value,
                merge=merge[:2 * (n - 1)].reshape(2, n - 1).T.copy(), height=height[:n - 1].copy(),
                boundary=boundary[:n - 1].copy(), timings=timings,
                host_s={"upload": t_up, "call": t_call})


_UPLOAD_THREADS = int(os.environ.get("TP_UPLOAD_THREADS", "0"))


def _upload_threads(nbytes: int) -> int:
    """Host threads for one tp_upload_dev copy (TP_UPLOAD_THREADS overrides):
    the library runs one upload at a time per device (FIFO), and four threads
    of host copy keep up with the PCIe link (~52 of ~56 GB/s measured)."""
    if _UPLOAD_THREADS > 0:
        return _UPLOAD_THREADS
    return 1 if nbytes < (16 << 20) else 4


def mask_dev(dm, bad_frac: float = 0.01, stream=None):
    """tp_mask_dev on a GPU-resident square float64 tensor (cleaned and
    symmetrised in place, R/TADpole.R:19-20).  Returns (bad bool[N0],
    rowMeans, good 1-based indices)."""
    import torch
    L = _lib.load()
    device = dm.device.index if dm.device.index is not None else 0
    if dm.dtype != torch.float64 or not dm.is_contiguous():
        raise ValueError("mask_dev needs a contiguous float64 tensor")
    stream = stream or torch.cuda.current_stream(device)
    if stream.cuda_stream == 0:       # see _pipeline: order with torch's default stream
        torch.cuda.current_stream(device).synchronize()
    else:
        stream.wait_stream(torch.cuda.current_stream(device))
    n0 = dm.shape[0]
    bad = np.zeros(n0, np.int32)
    rm = np.zeros(n0)
    good = np.zeros(n0, np.int32)
    ng, st = cint(0), cint(0)
    L.tp_mask_dev(ctypes.c_void_p(dm.data_ptr()), ctypes.byref(cint(n0)), ctypes.byref(cdbl(bad_frac)),
                  ctypes.byref(cint(_lib.TP_FLAG_ROW_MAJOR)), ctypes.byref(cint(device)),
                  ctypes.c_void_p(stream.cuda_stream), ip(bad), dp(rm), ctypes.byref(ng), ip(good),
                  ctypes.byref(st))
    _lib.check(st)
    return bad.astype(bool), rm, good[:ng.value].copy()


def rle(x):
    x = np.asarray(x)
    if x.size == 0:
        return np.zeros(0, np.int64), x
    cut = np.flatnonzero(x[1:] != x[:-1]) + 1
    starts = np.concatenate([[0], cut])
    return np.diff(np.concatenate([starts, [x.size]])), x[starts]


def fix_values(lengths, values):
    """``fix_values`` (R/TADpole.R:503-510)."""
    values = np.array(values, copy=True)
    for i in np.flatnonzero(values == 0):
        if i == 0 or i == len(values) - 1:
            continue
        if values[i - 1] == values[i + 1]:
            values[i] = values[i - 1]
    return lengths, values


def _fixed_clusters(labels_good, good_idx1, bad_idx1):
    """R/TADpole.R:474-483: c(good, bad=0), order by numeric name, fix_values,
    inverse.rle.  Returns (vector over all bins in original order, names)."""
    names = np.concatenate([good_idx1, bad_idx1]).astype(np.float64)
    vals = np.concatenate([np.asarray(labels_good, np.float64), np.zeros(len(bad_idx1))])
    order = np.argsort(names, kind="stable")
    lens, v = fix_values(*rle(vals[order]))
    return np.repeat(v, lens), names[order]


def _coords(fixed):
    """R/TADpole.R:485-488: runs of the fixed vector -> (start, end), 0-runs dropped."""
    lens, v = rle(fixed)
    eb = np.cumsum(lens)
    start = np.concatenate([[1], eb[:-1] + 1])
    keep = v != 0
    return np.stack([start[keep], eb[keep]], axis=1).astype(np.int64)


def _level_coords(boundary, n, kk, pos):
    """TAD coordinates of the cut into ``kk`` clusters (R/TADpole.R:470-488).

    The cut's segments are runs of good bins in good order; a run of bad bins
    (value 0 after ``c(good, bad)`` + ``order``) between two bins of the same
    segment is filled by ``fix_values`` and one between two segments stays 0,
    so every TAD spans from its first to its last good bin: (start, end) =
    (pos[first], pos[last]) with ``pos`` the 1-based rank of each good bin in
    the name-sorted union of good and bad bins."""
    out = np.empty((kk, 2), np.int64)
    out[0, 0] = pos[0]
    out[kk - 1, 1] = pos[n - 1]
    if kk > 1:
        b = np.sort(boundary[n - kk:]) - 1
        out[1:, 0] = pos[b]
        out[:-1, 1] = pos[b - 1]
    return out


def _assemble(res, bad_idx1) -> Tadpole:
    n = len(res["good"])
    good1 = np.asarray(res["good"])
    dendro = Chclust(merge=res["merge"], height=res["height"], order=np.arange(1, n + 1),
                     label_ids=good1, boundary=res["boundary"])
    t = Tadpole(n_pcs=res["n_pcs"], optimal_n_clusters=res["n_clusters"], dendro=dendro,
                scores=res["scores"], bad_columns=bad_idx1, timings_ms=res["timings"])
    row = res["scores"][res["n_pcs"] - 1]
    levels = np.flatnonzero(~np.isnan(row)) + 1
    if bad_idx1 is None or len(bad_idx1) == 0:
        pos = np.arange(1, n + 1, dtype=np.int64)
    else:
        names = np.concatenate([good1, np.asarray(bad_idx1)]).astype(np.float64)
        if not np.all(np.diff(good1.astype(np.float64)) > 0):
            return _assemble_rle(t, dendro, levels, good1, bad_idx1)
        tot = len(names)
        seen = np.zeros(tot + 1, bool)
        ok = names.min() >= 1 and names.max() <= tot
        if ok:
            seen[names.astype(np.int64)] = True
        if ok and seen[1:].all():
            # the names are 1..N (a full matrix's good + bad bins): the rank of
            # each good bin in order(c(good, bad)) is its own name
            pos = good1.astype(np.int64)
        else:
            order = np.argsort(names, kind="stable")
            rank = np.empty(tot, np.int64)
            rank[order] = np.arange(1, tot + 1)
            pos = rank[:n]
    t.clusters.update(zip(map(str, levels.tolist()), _all_level_coords(res["boundary"], n, levels, pos)))
    return t


def _all_level_coords(boundary, n, levels, pos):
    """``_level_coords`` of every level at once (the cuts are nested: the cut
    into kk clusters is the cut into kk - 1 plus boundary[n - kk]): one stable
    sort of the deepest level's boundaries in the library
    (``tp_level_coords``), each level's rows a view of one int64 block."""
    levels = np.ascontiguousarray(levels, np.int32)
    if len(levels) == 0:
        return []
    bnd = np.ascontiguousarray(boundary[:max(n - 1, 0)], np.int32)
    pos32 = np.ascontiguousarray(pos, np.int32)
    off = np.zeros(len(levels) + 1, np.int64)
    np.cumsum(levels, out=off[1:])
    out = np.empty((int(off[-1]), 2), np.int32)
    st = _lib.cint(0)
    _lib.load().tp_level_coords(_lib.ip(bnd), ctypes.byref(_lib.cint(n)), _lib.ip(levels),
                                ctypes.byref(_lib.cint(len(levels))), _lib.ip(pos32), _lib.ip(out), ctypes.byref(st))
    _lib.check(st)
    out = out.astype(np.int64)
    offl = off.tolist()
    return [out[offl[l]:offl[l + 1]] for l in range(len(levels))]


def _assemble_rle(t, dendro, levels, good1, bad_idx1) -> Tadpole:
    """Literal R/TADpole.R:470-488 (cutree, c(good, bad), order, rle,
    fix_values, inverse.rle, runs): used when the good names are not
    ascending, and by the tests as the reference for ``_level_coords``."""
    for kk in levels:
        lab = dendro.cutree(int(kk))
        if bad_idx1 is not None and len(bad_idx1):
            fixed, _ = _fixed_clusters(lab, good1, bad_idx1)
            t.clusters[str(int(kk))] = _coords(fixed)
        else:
            eb = np.cumsum(np.bincount(lab)[1:])
            t.clusters[str(int(kk))] = np.stack([np.concatenate([[1], eb[:-1] + 1]), eb], axis=1)
    return t


def TADpole(mat_file, max_pcs: int = 200, min_clusters: int = 2, bad_frac: float = 0.01,
            chr=None, start=None, end=None, resol=None, centromere_search: bool = False,
            device: int = 0, sharded: bool = False, stream=None, fixed_centromere: bool = False,
            verbose: bool = False, inplace: bool = False, arm_groups=None) -> Tadpole:
    """``TADpole()`` (R/TADpole.R:344-501).  ``mat_file`` may be a path to a
    tab-separated matrix or an in-memory square array.  ``sharded``: split this
    matrix over the ranks of the communicator made by
    ``tadpole_amd.multi.init_comm`` (every rank calls with the same matrix).
    ``stream``: a torch.cuda.Stream to run on (concurrent pipelines per GPU).
    ``fixed_centromere``: the centromere split without the reference's q-arm
    index bug (R/TADpole.R:78-80), and the single-matrix path where R would
    fail on a plain matrix (:66-70,356).  ``verbose``: R's message() lines on
    stderr (always logged on the ``tadpole_amd`` logger).

    A GPU-resident ``mat_file`` (a torch tensor) is left untouched: the
    pipeline cleans (NA -> 0, forceSymmetric, R/TADpole.R:19-20) a device copy.
    ``inplace=True`` skips that copy (N0^2 doubles of HBM) and cleans the
    caller's float64 tensor in place.  ``stream`` contexts: see
    ``tadpole_amd.release_stream``.  ``arm_groups`` (from
    ``tadpole_amd.multi.init_arm_comms``, with ``centromere_search`` and
    ``sharded``): each rank computes only its group's arm, sharded over that
    group, and the arms' results are exchanged -- the two arms on disjoint
    GPUs at the same time."""
    if _is_device(mat_file):
        raw = mat_file
        if not inplace:
            import torch
            raw = raw.to(torch.float64).contiguous()
            if raw.data_ptr() == mat_file.data_ptr():
                raw = raw.clone()
    elif _is_path(mat_file):
        try:
            import torch  # noqa: F401  (device memory for the direct-to-device parse)
        except ImportError:   # R-like hosts without torch: the host parse, then tp_pipeline
            raw = read_matrix(mat_file)
        else:
            raw = _read_to_device(mat_file, device, stream)   # ours: cleaned in place on the device
    else:
        raw = _as_matrix(mat_file)
    shard_flag = _lib.TP_FLAG_SHARDED if sharded else 0
    if arm_groups is not None and not (centromere_search and sharded):
        raise ValueError("arm_groups: the two-group schedule is for centromere_search=True, sharded=True")
    if not centromere_search:
        res = _pipeline(raw, max_pcs, min_clusters, bad_frac, shard_flag, device, stream)
        bad_idx1 = np.flatnonzero(res["bad"]) + 1
        _message(f"{len(bad_idx1)} bad columns found at position(s):", verbose)
        _message(" ".join(str(int(b)) for b in bad_idx1), verbose)
        ta = time.perf_counter()
        t = _assemble(res, bad_idx1)
        t.host_s = dict(res["host_s"], assemble=time.perf_counter() - ta)
        _message(f"Optimal number of PCs: {t.n_pcs}", verbose)
        _message(f"Optimal number of clusters: {t.optimal_n_clusters}", verbose)
        return t
    if _is_device(raw):
        import torch
        raw = raw.to(torch.float64).contiguous()
        bad, _, _ = mask_dev(raw, bad_frac, stream)   # raw is clean and symmetric from here on
    else:
        bad, _, _ = mask(raw, bad_frac, device)
    bad_idx1 = np.flatnonzero(bad) + 1
    _message(f"{len(bad_idx1)} bad columns found at position(s):", verbose)
    _message(" ".join(str(int(b)) for b in bad_idx1), verbose)
    plan = _arm_plan(bad, fixed_centromere, verbose) if bad.any() else None
    if plan is None:
        if not fixed_centromere:
            # R/TADpole.R:356: `mat$centromer` on a matrix is an error in R
            raise TypeError("$ operator is invalid for atomic vectors (no centromere split: no bad bin, or the "
                            "longest bad run touches an end of the matrix; R/TADpole.R:66-70,87-90,356)")
        if arm_groups is not None:
            raise ValueError("arm_groups: no centromere split (the group communicators cover one arm each)")
        return TADpole(raw, max_pcs, min_clusters, bad_frac, device=device, sharded=sharded, stream=stream,
                       verbose=verbose, inplace=True)
    return _tadpole_arms(raw, plan, max_pcs, min_clusters, device, shard_flag, stream, verbose, arm_groups)


_ARM_STREAMS: Dict[int, tuple] = {}


def _arm_streams(device: int):
    """Two persistent HIP streams per device for the concurrent arms (the
    library keeps one context per stream: reusing them reuses its scratch):
    (high priority, normal) -- the larger arm takes the first (see
    _tadpole_arms); TADPOLE_ARMS_PRIO=0 makes both normal."""
    s = _ARM_STREAMS.get(device)
    if s is None:
        import torch
        hi = -1 if os.environ.get("TADPOLE_ARMS_PRIO", "1") != "0" else 0
        s = _ARM_STREAMS[device] = (torch.cuda.Stream(device=f"cuda:{device}", priority=hi),
                                    torch.cuda.Stream(device=f"cuda:{device}"))
    return s


def _arms_concurrent(raw, shard_flag: int, stream) -> bool:
    """The two arms are independent matrices (R/TADpole.R:357-432 runs them
    one after the other): on one GPU they run on two streams at once, so one
    arm's latency-bound CONISS sweep (~200 of 256 CUs, mostly idle SIMDs)
    overlaps the other arm's MFMA-bound correlation and PCA.  Not for sharded
    calls (one communicator per device serialises them) or when the caller
    chose the stream."""
    if shard_flag or stream is not None or os.environ.get("TADPOLE_ARMS_SERIAL") == "1":
        return False
    try:
        import torch
    except ImportError:
        return False
    return torch.cuda.is_available()


def _run_arm(raw, plan, arm, max_pcs, min_clusters, device, shard_flag: int = 0, stream=None) -> Tadpole:
    """One centromere arm (R/TADpole.R:362-408): the raw principal submatrix
    of its kept bins; NA->0 and forceSymmetric(uplo='U') commute with taking
    it, so the device cleans it (TP_FLAG_NO_MASK: the arm matrices are
    correlated as given, R/TADpole.R:362)."""
    names, bad_cols = plan[arm]
    if _is_device(raw):
        # already cleaned by tp_mask_dev: the pipeline reads the arm's rows and
        # columns straight from it (TP_FLAG_SUBSET; an index_select copy of the
        # two C5 arms cost 16.5 ms of HBM traffic before either could start)
        res = _pipeline(raw, max_pcs, min_clusters, 0.0, _lib.TP_FLAG_CLEAN | shard_flag, device, stream,
                        subset=names)
    else:
        sub = raw[np.ix_(names - 1, names - 1)]
        res = _pipeline(sub, max_pcs, min_clusters, 0.0, _lib.TP_FLAG_NO_MASK | shard_flag, device, stream)
        del sub
    res["good"] = names.astype(np.int32)   # rownames inherited from the full matrix
    return _assemble(res, np.asarray(bad_cols))


def _merge_arms(plan, subs, verbose: bool = False) -> Tadpole:
    """R/TADpole.R:404-442: the per-arm objects, R's message() lines in the
    sequential loop's order, and merging_arms (p labels, a zero pad of the
    centromere's length after each arm, the trailing pad dropped, RLE)."""
    tad = Tadpole()
    centromer = plan["centromere"]
    fixed_arms: List[np.ndarray] = []
    for arm in ("p", "q"):
        names, bad_cols = plan[arm]
        sub_t = subs[arm]
        _message(f"Processing arm {arm}", verbose)
        _message(f"Optimal number of PCs: {sub_t.n_pcs}", verbose)
        _message(f"Optimal number of clusters: {sub_t.optimal_n_clusters}", verbose)
        setattr(tad, arm, sub_t)
        lab = sub_t.dendro.cutree(sub_t.optimal_n_clusters)
        fixed, _ = _fixed_clusters(lab, names, np.asarray(bad_cols))
        fixed_arms.append(fixed)
        fixed_arms.append(np.zeros(len(centromer)))
    allv = np.concatenate(fixed_arms)
    allv = allv[: len(allv) - len(centromer)]
    tad.merging_arms = _coords(allv)
    return tad


def _tadpole_arms(raw, plan, max_pcs, min_clusters, device, shard_flag: int = 0, stream=None,
                  verbose: bool = False, arm_groups=None) -> Tadpole:
    """R/TADpole.R:351-442 (arm loop and arm merge).  On one GPU the two arms
    run concurrently on two streams (``_arms_concurrent``); with ``arm_groups``
    each rank runs its group's arm sharded over the group and the results are
    exchanged (``multi.exchange_arms``); results and R's message() lines are
    those of the sequential loop, in its order."""
    if _is_device(raw):
        device = raw.device.index if raw.device.index is not None else device

    def run_arm(arm, arm_stream, hint=0):
        return _run_arm(raw, plan, arm, max_pcs, min_clusters, device, shard_flag | hint, arm_stream)

    if arm_groups is not None:
        from . import multi
        # a failing arm (a data error, or a communicator abort) must not leave
        # the other group blocked in the result exchange: the status goes to
        # every rank first and all of them raise together
        try:
            mine, err = run_arm(arm_groups.arm, stream), None
        except Exception as e:   # noqa: BLE001 -- re-raised by exchange_arms on every rank
            mine, err = None, e
        subs = multi.exchange_arms(arm_groups, mine, err)
    elif _arms_concurrent(raw, shard_flag, stream):
        # both arms start at once (0.305 s for C5 on one MI355X, 0.33 s one
        # after the other).  Both arms' CONISS trees keep only their link
        # array in LDS (TP_FLAG_LDS_LEAN: 48.6 + 43 KB a tree instead of 97 +
        # 86) so a tree of each arm fits on one CU: c5_full 0.207 -> 0.190 s.
        # With only the smaller arm lean ("smaller") it was 0.182 or 0.216 s
        # run to run: a CU's LDS is allocated contiguously, and a lean tree
        # placed mid-LDS (above a workgroup still resident when it started)
        # leaves no 97 KB gap for the other arm's full tree, which then waits
        # for a CU; with both lean any placement leaves a >= 58 KB gap.  (The
        # library also makes a sweep lean by itself while another pipeline is
        # in flight on the device, knob 47.)  TADPOLE_ARMS_Q_AT=s (1..3) holds q back until p's
        # progress word reaches stage s (2: p's correlation queued, 3: p's
        # sweep): measured slower (0.32-0.34 s at s = 3: q's int8 X'X, 160 KiB
        # of LDS a workgroup, cannot share a CU with p's CONISS trees).
        import time
        from concurrent.futures import ThreadPoolExecutor
        # the larger arm's sweep ends last: its stream goes first when both
        # arms' correlation and PCA kernels compete for the CUs
        s_hi, s_lo = _arm_streams(device)
        sp, sq = (s_hi, s_lo) if len(plan["p"][0]) >= len(plan["q"][0]) else (s_lo, s_hi)
        q_at = int(os.environ.get("TADPOLE_ARMS_Q_AT", "0"))
        L = _lib.load() if q_at > 0 else None
        prog = np.zeros(1, np.int32)
        st = cint(0)
        if L is not None:
            L.tp_progress_attach(ctypes.byref(cint(device)), ctypes.c_void_p(sp.cuda_stream),
                                 prog.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st))
            _lib.check(st)
        try:
            with ThreadPoolExecutor(max_workers=2) as ex:
                lean = {"p": _lib.TP_FLAG_LDS_LEAN, "q": _lib.TP_FLAG_LDS_LEAN}
                fp = ex.submit(run_arm, "p", sp, lean["p"])

                def run_q():
                    while q_at > 0 and prog[0] < q_at and not fp.done():
                        time.sleep(2e-4)
                    return run_arm("q", sq, lean["q"])

                fq = ex.submit(run_q)
                subs = {"p": fp.result(), "q": fq.result()}
        finally:
            if L is not None:
                L.tp_progress_attach(ctypes.byref(cint(device)), ctypes.c_void_p(sp.cuda_stream), None,
                                     ctypes.byref(st))
    else:
        subs = {}
        for arm in ("p", "q"):
            subs[arm] = run_arm(arm, stream)
    return _merge_arms(plan, subs, verbose)


# ------------------------------------------------------------------ diffT

def _bed_rows(bed):
    if hasattr(bed, "itertuples"):
        return [(r[1], int(r[2]), int(r[3])) for r in bed.itertuples()]
    return [(r[0], int(r[1]), int(r[2])) for r in bed]


def bin_index(bed, size: int) -> np.ndarray:
    """``bin_index`` (R/DiffT.R:1-9)."""
    rows = _bed_rows(bed)
    out = np.zeros(size, np.int64)
    first = rows[0][1]
    for t, (_, s, e) in enumerate(rows, start=1):
        lo, hi = s - first, e - first
        if hi >= lo:
            out[lo:hi + 1] = t
        else:  # R's seq(s, e) counts down when e < s
            out[hi:lo + 1] = t
    return out


def diffT(bed_x, bed_y) -> np.ndarray:
    """``diffT`` (R/DiffT.R:19-50), O(L) instead of R's O(L^2) loop; identical
    integer counts, so the normalised profile is identical."""
    rx, ry = _bed_rows(bed_x), _bed_rows(bed_y)
    if len(rx) != len(ry):
        raise ValueError("Both calls must have the same number of TADs.")
    sx, sy = rx[0][1], ry[0][1]
    ex, ey = rx[-1][2], ry[-1][2]
    tx = bin_index(rx, ex - sx + 1)
    ty = bin_index(ry, ey - sy + 1)
    tx = np.concatenate([np.ones(max(0, sx - sy), np.int64), tx, np.full(max(0, ey - ex), tx.max())])
    ty = np.concatenate([np.ones(max(0, sy - sx), np.int64), ty, np.full(max(0, ex - ey), ty.max())])
    if len(tx) != len(ty):
        raise ValueError("length(tad_x) == length(tad_y) is not TRUE")
    # count_b = #{c : (tx[c]==tx[b]) xor (ty[c]==ty[b])} for nonzero ids
    _, ix, cx = np.unique(tx, return_inverse=True, return_counts=True)
    _, iy, cy = np.unique(ty, return_inverse=True, return_counts=True)
    pair = ix.astype(np.int64) * (iy.max() + 1) + iy
    _, ip_, cp = np.unique(pair, return_inverse=True, return_counts=True)
    A, B, AB = cx[ix], cy[iy], cp[ip_]
    L_ = len(tx)
    scores = A + B - 2 * AB
    zx, zy = tx == 0, ty == 0
    scores = np.where(zx & ~zy, B, scores)      # x all TRUE: xor = !y
    scores = np.where(~zx & zy, A, scores)      # y all TRUE: xor = !x
    scores = np.where(zx & zy, 0, scores)
    del L_
    s = np.cumsum(scores)
    if scores.max() == 0:
        return s
    return s / s.max()


def random_bed(bed, bad_columns=None, rng=None):
    """``random_bed`` (R/DiffT.R:61-73): same construction, numpy RNG."""
    rows = _bed_rows(bed)
    rng = np.random.default_rng(rng)
    start, end = rows[0][1], rows[-1][2]
    size = end - start + 1
    bins = np.arange(start, end + 1)
    if bad_columns is not None:
        bins = np.delete(bins, np.asarray(bad_columns, np.int64) - 1)
    borders = np.sort(rng.choice(bins[1:], len(rows) - 1, replace=False))
    import pandas as pd
    return pd.DataFrame({"chrom": [r[0] for r in rows],
                         "start": np.concatenate([[start], borders - 1]),
                         "end": np.concatenate([borders - 2, [start + size - 1]])})
