"""CPU model (numpy fp64, not product code) of the C-Krylov PCA planned for the
device: block Krylov in C itself (start block [1 | random], one product
P_t = Xc K_t per block), BCGS-PIP2 orthogonalisation written as the device
will run it (Z = [K W]'W, R = chol(Z_w - H'H), W <- [K W] [-H R^-1; R^-1]),
T = P'P, and the Ritz residual of G = Xc'Xc from one extra block:
Xc v lies in span(K_0..K_s), so G v = (Xc'Q) (Q'Xc v) with
Xc'Q = P_Q + 1 (m'Q) - m (1'Q) -- no product with a k-column block.

  python tools/krylov_c_model.py [n0] [k] [p1xs1,p2xs2,...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tadpole_oracle as O  # noqa: E402
from tadpole_amd.synth import SEED_BASE, synth_hic, synth_hic_par  # noqa: E402


def pip_pass(K, W, shift=1e-14):
    if K is None:
        S = W.T @ W
        H = None
    else:
        Z = np.hstack([K, W]).T @ W
        H = Z[:K.shape[1]]
        S = Z[K.shape[1]:] - H.T @ H
    S = 0.5 * (S + S.T)
    d = np.sqrt(np.diag(S))
    Sj = S / np.outer(d, d) + shift * np.eye(S.shape[0])
    R = np.linalg.cholesky(Sj).T * d[None, :]       # S ~ R'R
    Ri = np.linalg.inv(R)
    return (W @ Ri) if H is None else (W - K @ H) @ Ri


def run(C, m, k, p, s):
    n = C.shape[0]
    rng = np.random.default_rng(1)
    x0 = rng.uniform(-1, 1, (n, p))
    x0[:, 0] = 1.0
    K = pip_pass(None, pip_pass(None, x0))
    blocks, prods = [K], []
    xc = lambda B: C @ B - np.outer(np.ones(n), m @ B)
    for t in range(s + 1):                     # P_0..P_s (P_s: residual block)
        prods.append(xc(blocks[t]))
        if t < s:
            Kb = np.hstack(blocks)
            W = pip_pass(Kb, pip_pass(Kb, prods[t]))
            blocks.append(W)
    Kall = np.hstack(blocks)                   # Q: s + 1 blocks
    Pall = np.hstack(prods)
    D = s * p
    K, P = Kall[:, :D], Pall[:, :D]
    T = P.T @ P
    th, Y = np.linalg.eigh(0.5 * (T + T.T))
    th, Y = th[::-1][:k], Y[:, ::-1][:, :k]
    V = K @ Y
    S = P @ Y                                  # scores Xc V
    z = Kall.T @ S
    GV = Pall @ z + np.outer(np.ones(n), m @ Kall @ z) - np.outer(m, Kall.sum(axis=0) @ z)
    r_cheap = np.linalg.norm(GV - V * th[None, :], axis=0) / th[0]
    XV = xc(V)
    GVt = C @ XV - np.outer(m, XV.sum(axis=0))
    r_true = np.linalg.norm(GVt - V * th[None, :], axis=0) / th[0]
    orth = np.abs(Kall.T @ Kall - np.eye(Kall.shape[1])).max()
    return r_cheap.max(), r_true.max(), orth, th


def main():
    n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 7808
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    t0 = time.time()
    mat = synth_hic(n0, SEED_BASE + 3) if n0 < 12000 else synth_hic_par(n0, SEED_BASE + 5)
    bad, _, _ = O.bad_mask(mat, 0.01)
    x = mat[~bad][:, ~bad]
    del mat
    C = O.sparse_cor(x)
    del x
    n = C.shape[0]
    m = C.mean(axis=0)
    print(f"n={n} C built {time.time() - t0:.1f} s", flush=True)
    runs = [(32, 33), (32, 34), (48, 23), (64, 22)]
    if len(sys.argv) > 3:
        runs = [(int(a.split("x")[0]), int(a.split("x")[1])) for a in sys.argv[3].split(",")]
    for p, s in runs:
        t1 = time.time()
        rc, rt, oe, th = run(C, m, k, p, s)
        print(f"C-Krylov p={p:3d} s={s:3d} D={p * s:5d} products {s + 1:3d} x {p:3d}: resid cheap {rc:.2e} "
              f"true {rt:.2e} orth {oe:.1e} ({time.time() - t1:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
