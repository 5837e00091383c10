"""CPU functional model of the candidate-list CONISS argmin (design study for
k_coniss, not product code).  Wave A keeps a sorted list L of at most 64
(cost, position) entries, one per lane, complete below a bound T: every
current adjacent cost (c, p) <lex T is a live entry of L.  A merge kills the
entries at its three touched positions (ls, a, b) and inserts its two new
costs when they are <lex T (a full list drops its last entry, which lowers T);
the next merge is the first live entry.  An exhausted list is rebuilt from the
cost array: T = the lexicographic minimum over lanes of each lane's second
smallest (cost, position) over its strided positions (p % 64 == lane), so at
most one entry per lane is below T.  Checks the merge sequence against the
oracle's CONISS (R/TADpole.R:108, rioja::chclust) and reports rebuild rates.
usage: python tools/coniss_llist_model.py [N0]"""
import bisect
import sys

import numpy as np

sys.path[:0] = ['/root/repo', '/root/repo/oracle']
import tadpole_oracle as O  # noqa: E402
from tadpole_amd.synth import synth_hic  # noqa: E402

INF = float('inf')


def ward(sa, na, sb, nb):
    e = sa * nb - sb * na
    return float(np.sum(e * e)) / (na * nb * (na + nb))


def rebuild(cost, n):
    """(sorted entries, T) from the current costs (NaN = no candidate)."""
    best = {}
    for p in range(n - 1):
        c = cost[p]
        if c != c:
            continue
        lane = p % 64
        lst = best.setdefault(lane, [])
        lst.append((c, p))
        lst.sort()
        del lst[2:]
    seconds = [v[1] for v in best.values() if len(v) == 2]
    T = min(seconds) if seconds else (INF, 1 << 40)
    ent = sorted((cost[p], p) for p in range(n - 1) if cost[p] == cost[p] and (cost[p], p) < T)
    return ent, T


def llist(p, cap=64):
    n = p.shape[0]
    nxt = list(range(1, n)) + [-1]
    prv = list(range(-1, n - 1))
    sums = {i: p[i].copy() for i in range(n)}
    size = {i: 1 for i in range(n)}
    cost = [ward(p[i], 1, p[i + 1], 1) for i in range(n - 1)] + [float('nan')]
    L, T = rebuild(cost, n)
    live = [True] * len(L)
    merges, rebuilds, drops = [], 0, 0
    while len(merges) < n - 1:
        f = next((j for j in range(len(L)) if live[j]), None)
        if f is None:
            L, T = rebuild(cost, n)
            live = [True] * len(L)
            rebuilds += 1
            continue
        c, a = L[f]
        b = nxt[a]
        ls, r = prv[a], nxt[b]
        merges.append((a, b))
        sums[a] = sums[a] + sums[b]
        size[a] += size[b]
        nxt[a] = r
        if r >= 0:
            prv[r] = a
        cost[a] = cost[b] = float('nan')
        kill = {a, b}
        new = []
        if ls >= 0:
            kill.add(ls)
            cost[ls] = ward(sums[ls], size[ls], sums[a], size[a])
            new.append((cost[ls], ls))
        if r >= 0:
            cost[a] = ward(sums[a], size[a], sums[r], size[r])
            new.append((cost[a], a))
        for j, (_, q) in enumerate(L):
            if q in kill:
                live[j] = False
        for e in new:
            if not e < T:
                continue
            if len(L) == cap:   # compact dead entries first, then drop the last
                keep = [j for j in range(len(L)) if live[j]]
                L = [L[j] for j in keep]
                live = [True] * len(L)
            if len(L) == cap:
                T = L.pop()
                live.pop()
                drops += 1
                if not e < T:
                    continue
            k = bisect.bisect_left(L, e)
            L.insert(k, e)
            live.insert(k, True)
    return merges, rebuilds, drops


if __name__ == "__main__":
    n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    m = synth_hic(n0, 20261017)
    cm = O.clean_symmetrize(m)
    bad, _, _ = O.bad_mask(cm, 0.01)
    g = np.flatnonzero(~bad)
    x = cm[np.ix_(g, g)]
    P = O.prcomp_x(O.sparse_cor(x), 200, method="eigh")
    for i in (1, 2, 20, 100, 200):
        ma, mb, co, he = O.coniss(np.ascontiguousarray(P[:, :i]))
        mg, rb, dr = llist(P[:, :i])
        ok = np.array_equal(np.array(mg)[:, 0], ma)
        print(f"tree {i:3d}: same merges {ok}  rebuilds {rb}  merges/rebuild {(len(mg)) / max(rb, 1):.1f}  drops {dr}",
              flush=True)
