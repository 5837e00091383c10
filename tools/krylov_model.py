"""CPU model of the block Krylov PCA variants (numpy fp64, not product code).

  python tools/krylov_model.py [n0] [k]

Builds the C3-style correlation matrix C (synthetic Hi-C, masked, Pearson),
then compares, at equal Krylov dimension D, the worst relative Ritz residual
||G v - theta v|| / theta_1 over the top k pairs of G = Xc'Xc = C^2 - n m m'
(the acceptance the device applies, 1e-11):

  G p s : block Krylov in G (two products with C per block, the round-2/3 path)
  C p s : block Krylov in C with 1 in the start block (one product per block);
          the next block is Xc K_t = C K_t - 1 (m'K_t), which spans the same new
          directions once 1 is in the basis; T = (Xc K)'(Xc K)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tadpole_oracle as O  # noqa: E402
from tadpole_amd.synth import SEED_BASE, synth_hic  # noqa: E402


def orth(w, basis=None):
    for _ in range(2):
        if basis is not None:
            w = w - basis @ (basis.T @ w)
    q, _ = np.linalg.qr(w)
    if basis is not None:
        q = q - basis @ (basis.T @ q)
        q, _ = np.linalg.qr(q)
    return q


def orth_pip2(w, basis):
    """BCGS-PIP2: per pass one product [K W]'W, R = chol(W'W - H'H), W <- (W - K H) R^-1."""
    for _ in range(2):
        if basis is None:
            h = None
            g = w.T @ w
        else:
            z = np.hstack([basis, w]).T @ w
            h = z[:basis.shape[1]]
            g = z[basis.shape[1]:] - h.T @ h
        r = np.linalg.cholesky(0.5 * (g + g.T)).T
        ri = np.linalg.inv(r)
        w = (w - basis @ h) @ ri if h is not None else w @ ri
    return w


def run(C, m, k, mode, p, s, seed=1):
    n = C.shape[0]
    rng = np.random.default_rng(seed)
    x0 = rng.standard_normal((n, p))
    if mode in "CP":
        x0[:, 0] = 1.0
    blocks = [orth(x0)]
    prod = []
    for t in range(s):
        kt = blocks[-1]
        if mode == "G":
            xk = C @ kt - np.outer(np.ones(n), m @ kt)
            gk = C @ xk - np.outer(m, xk.sum(axis=0))
            prod.append(gk)
            nxt = gk
        else:
            xk = C @ kt - np.outer(np.ones(n), m @ kt)
            prod.append(xk)
            nxt = xk
        if t + 1 < s:
            blocks.append(orth_pip2(nxt, np.hstack(blocks)) if mode == "P" else orth(nxt, np.hstack(blocks)))
    K = np.hstack(blocks)
    P = np.hstack(prod)
    T = K.T @ P if mode == "G" else P.T @ P
    orth_err = np.abs(K.T @ K - np.eye(K.shape[1])).max()
    T = 0.5 * (T + T.T)
    th, Y = np.linalg.eigh(T)
    th, Y = th[::-1][:k], Y[:, ::-1][:, :k]
    V = K @ Y
    XV = C @ V - np.outer(np.ones(n), m @ V)
    GV = C @ XV - np.outer(m, XV.sum(axis=0))
    r = np.linalg.norm(GV - V * th[None, :], axis=0) / th[0]
    return r.max(), th, orth_err


def main():
    n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 7808
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    t0 = time.time()
    from tadpole_amd.synth import synth_hic_par
    mat = synth_hic(n0, SEED_BASE + 3) if n0 < 12000 else synth_hic_par(n0, SEED_BASE + 5)
    bad, _, _ = O.bad_mask(mat, 0.01)
    x = mat[~bad][:, ~bad]
    C = O.sparse_cor(x)
    n = C.shape[0]
    m = C.mean(axis=0)
    print(f"n={n} C built {time.time() - t0:.1f} s", flush=True)
    runs = [("G", 64, 16), ("P", 32, 32), ("P", 32, 33), ("P", 32, 34), ("P", 32, 36)]
    if len(sys.argv) > 3:
        runs = [(a[0], int(a[1:].split("x")[0]), int(a.split("x")[1])) for a in sys.argv[3].split(",")]
    for mode, p, s in runs:
        t1 = time.time()
        w, th, oe = run(C, m, k, mode, p, s)
        nprod = 2 * s if mode == "G" else s
        print(f"{mode} p={p:3d} s={s:3d} D={p * s:5d} C-products {nprod:3d} x {p:3d} cols: worst {w:.2e} orth {oe:.1e}"
              f"  ({time.time() - t1:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
