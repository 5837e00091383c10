"""Seeded synthetic Hi-C matrices.

The reference ships no matrix for its own example (``README.md:65-68`` names
``inst/extdata/raw_chr18_300_500_30kb.tsv``, which is absent), so every test and
bench input is generated here:

* TAD sizes ~ U{10..60} bins, grouped into meta-TADs of 3-6 TADs;
* ``E_ij = 1000 (1+|i-j|)^-1 (1 + 2[same TAD] + [same meta-TAD])``;
* ``M_ij ~ Poisson(E_ij)`` for ``i <= j``, mirrored (upper wins);
* ``zero_frac`` of the bins zeroed (row and column), i.e. bad via ``diag == 0``;
* optionally a zero run at ``[0.4875 N0, 0.572 N0)`` standing in for a centromere.

Seeds follow the survey: ``20261015 + config index``.
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 20261015

#: Config shapes of BASELINE.json (index -> raw bins).  C4/C5 are described in
#: SURVEY.md §8; C4 uses the hg19 chromosome sizes at 25 kb.
CONFIG_BINS = {1: 200, 2: 2000, 3: 7808, 5: 49851}

#: hg19 chromosome lengths (bp) for the whole-genome config C4 (@25 kb).
HG19_BP = {
    "chr1": 249250621, "chr2": 243199373, "chr3": 198022430, "chr4": 191154276,
    "chr5": 180915260, "chr6": 171115067, "chr7": 159138663, "chr8": 146364022,
    "chr9": 141213431, "chr10": 135534747, "chr11": 135006516, "chr12": 133851895,
    "chr13": 115169878, "chr14": 107349540, "chr15": 102531392, "chr16": 90354753,
    "chr17": 81195210, "chr18": 78077248, "chr19": 59128983, "chr20": 63025520,
    "chr21": 48129895, "chr22": 51304566, "chrX": 155270560,
}


def tad_layout(n0: int, rng: np.random.Generator):
    """Per-bin TAD and meta-TAD ids."""
    tad = np.empty(n0, np.int64)
    meta = np.empty(n0, np.int64)
    pos = t = m = 0
    while pos < n0:
        for _ in range(int(rng.integers(3, 7))):
            if pos >= n0:
                break
            e = min(n0, pos + int(rng.integers(10, 61)))
            tad[pos:e] = t
            meta[pos:e] = m
            pos = e
            t += 1
        m += 1
    return tad, meta


def synth_hic(n0: int, seed: int, zero_frac: float = 0.005,
              centromere: bool = False, dtype=np.float64) -> np.ndarray:
    """Symmetric n0 x n0 synthetic contact matrix (C-contiguous)."""
    rng = np.random.default_rng(seed)
    tad, meta = tad_layout(n0, rng)
    out = np.empty((n0, n0), dtype=dtype)
    # Row blocks keep the peak memory at a few rows of n0 at a time.
    blk = max(1, min(n0, (1 << 24) // max(n0, 1)))
    idx = np.arange(n0)
    for r0 in range(0, n0, blk):
        r1 = min(n0, r0 + blk)
        i = idx[r0:r1, None]
        e = 1000.0 / (1.0 + np.abs(i - idx[None, :]))
        e = e * (1.0 + 2.0 * (tad[r0:r1, None] == tad[None, :])
                 + 1.0 * (meta[r0:r1, None] == meta[None, :]))
        e[idx[None, :] < i] = 0.0          # draw the upper triangle only
        out[r0:r1] = rng.poisson(e)
    for r0 in range(0, n0, blk):           # mirror: upper wins (row blocks, no N^2 index arrays)
        r1 = min(n0, r0 + blk)
        out[r0:r1, :r0] = out[:r0, r0:r1].T
        sub = out[r0:r1, r0:r1]
        il = np.tril_indices(r1 - r0, -1)
        sub[il] = sub.T[il]
    nz = max(1, int(round(zero_frac * n0))) if zero_frac > 0 else 0
    if nz:
        z = rng.choice(n0, nz, replace=False)
        out[z, :] = 0
        out[:, z] = 0
    if centromere:
        a, b = int(0.4875 * n0), int(0.572 * n0)
        out[a:b, :] = 0
        out[:, a:b] = 0
    return out


PAR_BLOCK = 256   # rows per independently seeded block of synth_hic_par


def synth_hic_par(n0: int, seed: int, zero_frac: float = 0.005, centromere: bool = False,
                  threads: int = 0) -> np.ndarray:
    """The same model as ``synth_hic`` with the Poisson draws of every
    ``PAR_BLOCK``-row block taken from its own generator
    (``default_rng([seed, 1, block])``), so the blocks are drawn in parallel
    threads (numpy's generators release the GIL) and the matrix does not depend
    on the thread count.  Layout and zeroed bins come from ``default_rng(seed)``
    as in ``synth_hic``; the values differ from ``synth_hic(n0, seed)``.  Used for
    the large matrices (C4 chromosomes, C5-arm shapes): ~8 M cells/s serially."""
    from concurrent.futures import ThreadPoolExecutor
    import os

    rng = np.random.default_rng(seed)
    tad, meta = tad_layout(n0, rng)
    out = np.empty((n0, n0), dtype=np.float64)
    idx = np.arange(n0)
    nblk = -(-n0 // PAR_BLOCK)

    def draw(b):
        r0, r1 = b * PAR_BLOCK, min(n0, (b + 1) * PAR_BLOCK)
        i = idx[r0:r1, None]
        c = idx[None, r0:]                     # upper triangle of the block rows only
        e = 1000.0 / (1.0 + np.abs(c - i))
        e = e * (1.0 + 2.0 * (tad[r0:r1, None] == tad[None, r0:])
                 + 1.0 * (meta[r0:r1, None] == meta[None, r0:]))
        e[c < i] = 0.0
        out[r0:r1, r0:] = np.random.default_rng([seed, 1, b]).poisson(e)

    def mirror(b):
        r0, r1 = b * PAR_BLOCK, min(n0, (b + 1) * PAR_BLOCK)
        out[r0:r1, :r0] = out[:r0, r0:r1].T
        sub = out[r0:r1, r0:r1]
        il = np.tril_indices(r1 - r0, -1)
        sub[il] = sub.T[il]

    nt = threads or min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(max_workers=nt) as ex:
        list(ex.map(draw, range(nblk)))
        list(ex.map(mirror, range(nblk)))      # reads only the upper blocks, all drawn above
    nz = max(1, int(round(zero_frac * n0))) if zero_frac > 0 else 0
    if nz:
        z = rng.choice(n0, nz, replace=False)
        out[z, :] = 0
        out[:, z] = 0
    if centromere:
        a, b = int(0.4875 * n0), int(0.572 * n0)
        out[a:b, :] = 0
        out[:, a:b] = 0
    return out


def synth_hic_par_stream(n0: int, seed: int, put, zero_frac: float = 0.005, centromere: bool = False,
                         threads: int = 0) -> np.ndarray:
    """``synth_hic_par`` without its n0 x n0 host array: the same draws (bit
    for bit), handed to ``put(r0, r1, U)`` block by block in row order, U = the
    block's upper rows ``[r0, r1) x [r0, n0)`` (zero below the diagonal; the
    consumer mirrors them, e.g. with ``place_upper_block``).  Blocks are drawn
    in parallel threads, at most one per thread ahead of the consumer.  Returns
    the bins the caller zeroes afterwards (rows and columns): the random bad
    bins and the centromere run.  Every rank of a multi-GPU run can fill its
    own device copy of the C5 matrix this way (no broadcast)."""
    from concurrent.futures import ThreadPoolExecutor
    import os

    rng = np.random.default_rng(seed)
    tad, meta = tad_layout(n0, rng)
    idx = np.arange(n0)
    nblk = -(-n0 // PAR_BLOCK)

    def draw(b):
        r0, r1 = b * PAR_BLOCK, min(n0, (b + 1) * PAR_BLOCK)
        i = idx[r0:r1, None]
        c = idx[None, r0:]
        e = 1000.0 / (1.0 + np.abs(c - i))
        e = e * (1.0 + 2.0 * (tad[r0:r1, None] == tad[None, r0:])
                 + 1.0 * (meta[r0:r1, None] == meta[None, r0:]))
        e[c < i] = 0.0
        return np.random.default_rng([seed, 1, b]).poisson(e).astype(np.float64)

    nt = threads or min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(max_workers=nt) as ex:
        pend = {}
        nxt = 0
        for b in range(nblk):
            while nxt < nblk and nxt < b + nt + 1:
                pend[nxt] = ex.submit(draw, nxt)
                nxt += 1
            U = pend.pop(b).result()
            put(b * PAR_BLOCK, min(n0, (b + 1) * PAR_BLOCK), U)
    zero = []
    nz = max(1, int(round(zero_frac * n0))) if zero_frac > 0 else 0
    if nz:
        zero.append(rng.choice(n0, nz, replace=False))
    if centromere:
        zero.append(np.arange(int(0.4875 * n0), int(0.572 * n0)))
    return np.unique(np.concatenate(zero)) if zero else np.zeros(0, np.int64)


def place_upper_block(M, r0: int, r1: int, U) -> None:
    """Write one block of ``synth_hic_par_stream`` into the symmetric M (numpy
    or torch, either device): rows [r0, r1) from column r1 on, their mirror
    below, and the diagonal block symmetrised (upper wins, as the generators
    mirror)."""
    w = r1 - r0
    R = U[:, w:]
    M[r0:r1, r1:] = R
    M[r1:, r0:r1] = R.T
    D = U[:, :w]
    if hasattr(D, "triu"):            # torch
        M[r0:r1, r0:r1] = D.triu() + D.triu(1).T
    else:
        M[r0:r1, r0:r1] = np.triu(D) + np.triu(D, 1).T


def config_matrix(config: int, **kw) -> np.ndarray:
    return synth_hic(CONFIG_BINS[config], SEED_BASE + config,
                     centromere=(config == 5), **kw)


def genome_bins(resol: int = 25000):
    """Bins per chromosome for C4 (whole genome @resol)."""
    return {c: -(-bp // resol) for c, bp in HG19_BP.items()}


def genome_seed(name: str) -> int:
    """Seed of chromosome ``name``'s C4 matrix: SEED_BASE + 4 + 100 * (its index
    in HG19_BP)."""
    return SEED_BASE + 4 + 100 * list(HG19_BP).index(name)


def genome_matrix(name: str, resol: int = 25000) -> np.ndarray:
    """C4: the synthetic matrix of one chromosome at ``resol`` (the parallel
    generator: 757 M cells for the whole genome)."""
    return synth_hic_par(genome_bins(resol)[name], genome_seed(name))


def early_centromere_matrix(n0: int, seed: int, lo: int, hi: int) -> np.ndarray:
    """A synthetic matrix whose centromere (zero run) is bins [lo, hi) of the
    first half, so the reference's q-arm removal by original index
    (R/TADpole.R:78-80) drops bins inside the arm (the C5 layout, centromere
    past the middle, drops none)."""
    m = synth_hic(n0, seed)
    m[lo:hi, :] = 0
    m[:, lo:hi] = 0
    return m


def matrix_checksum(m: np.ndarray) -> np.ndarray:
    """Two exact integers that pin a count matrix's values (the committed large
    fixtures store them instead of the matrix): the sum of the counts and
    sum (row + 1) (column + 1) m mod 2^61 - 1 (exact Python integers)."""
    from concurrent.futures import ThreadPoolExecutor
    import os
    n = m.shape[0]
    P = (1 << 61) - 1
    w = np.arange(n, dtype=np.int64) + 1

    def part(r0):   # exact integers per 1024-row block; summed in Python ints
        blk = np.asarray(m[r0:r0 + 1024], np.float64).astype(np.int64)
        rows = (blk * w[None, :]).sum(axis=1)      # < 2^43 per row at counts < 2^13, n < 2^16
        return int(blk.sum()), sum(int(v) * (r0 + q + 1) for q, v in enumerate(rows))

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        parts = list(ex.map(part, range(0, n, 1024)))
    total = sum(p[0] for p in parts)
    acc = sum(p[1] for p in parts)
    return np.array([total, acc % P], np.int64)


def _tsv_block(v: np.ndarray, ncol: int) -> bytes:
    v = v.astype(np.int64).ravel()
    if v.size == 0:
        return b""
    if v.min() < 0:
        raise ValueError("write_tsv: counts must be non-negative")
    nd = np.ones(v.size, np.int64)
    p = 10
    vmax = v.max()
    while p <= vmax:
        nd += v >= p
        p *= 10
    ends = np.cumsum(nd + 1)
    starts = ends - (nd + 1)
    buf = np.empty(int(ends[-1]), np.uint8)
    sep = np.full(v.size, 9, np.uint8)          # '\t'
    sep[ncol - 1::ncol] = 10                    # '\n' ends every row
    buf[ends - 1] = sep
    d, q = 0, v.copy()
    while True:
        sel = nd > d
        if not sel.any():
            break
        buf[(starts + nd - 1 - d)[sel]] = (q[sel] % 10 + 48).astype(np.uint8)
        q //= 10
        d += 1
    return buf.tobytes()


def write_tsv(m: np.ndarray, path: str, block_rows: int = 256, threads: int = 0) -> int:
    """Write a non-negative integer matrix as a headerless tab-separated file
    (``read.big.matrix``'s input, R/TADpole.R:17): vectorised digit formatting
    of row blocks in parallel threads, written in order.  Returns the bytes."""
    from concurrent.futures import ThreadPoolExecutor
    import os
    n, ncol = m.shape
    nt = threads or min(16, os.cpu_count() or 1)
    total = 0
    with open(path, "wb") as f, ThreadPoolExecutor(max_workers=nt) as ex:
        for b in ex.map(lambda r0: _tsv_block(np.asarray(m[r0:r0 + block_rows]), ncol),
                        range(0, n, block_rows)):
            f.write(b)
            total += len(b)
    return total
