"""CPU functional model of a batched CONISS (design study, not product code):
candidate list = the K smallest (cost, position) pairs, merged in that order
while no new cost made inside the batch undercuts the next valid candidate.
Checks the merge sequence against the oracle's CONISS (R/TADpole.R:108,
rioja::chclust) and reports batch lengths.
usage: python tools/coniss_batch_model.py N0 [indep]"""
import sys, numpy as np
sys.path[:0]=['/root/repo','/root/repo/oracle']
import tadpole_oracle as O
from tadpole_amd.synth import synth_hic

def ward(sa, na, sb, nb):
    e = sa * nb - sb * na
    return float(np.sum(e * e)) / (na * nb * (na + nb))

def batched(p, K):
    n = p.shape[0]
    start = list(range(n)); end = {i: i for i in range(n)}
    nxt = {i: (i + 1 if i + 1 < n else -1) for i in range(n)}
    prv = {i: (i - 1) for i in range(n)}
    sums = {i: p[i].copy() for i in range(n)}
    size = {i: 1 for i in range(n)}
    cost = {}
    for i in range(n - 1):
        cost[i] = ward(sums[i], 1, sums[i + 1], 1)
    merges = []; batches = []
    while len(merges) < n - 1:
        L = sorted(cost.items(), key=lambda kv: (kv[1], kv[0]))[:K]
        touched = set(); pending = {}; cnt = 0
        for pos, c in L:
            if pos in touched:
                continue
            if pending:
                pm = min(pending.items(), key=lambda kv: (kv[1], kv[0]))
                if (pm[1], pm[0]) < (c, pos):
                    break
            # merge pair at pos
            a = pos; b = nxt[a]; ls = prv[a]; r = nxt[b]
            merges.append((a, b))
            sums[a] = sums[a] + sums[b]; size[a] += size[b]
            del sums[b]; del size[b]
            nxt[a] = r
            if r >= 0: prv[r] = a
            del cost[a]
            if b in cost: del cost[b]
            touched |= {a, b}
            pending.pop(a, None); pending.pop(b, None)
            if ls >= 0:
                touched.add(ls); pending.pop(ls, None)
                cost[ls] = ward(sums[ls], size[ls], sums[a], size[a]); pending[ls] = cost[ls]
            if r >= 0:
                cost[a] = ward(sums[a], size[a], sums[r], size[r]); pending[a] = cost[a]
            cnt += 1
            if len(merges) == n - 1: break
        batches.append(cnt)
    return merges, batches

m = synth_hic(int(sys.argv[1]) if len(sys.argv) > 1 else 600, 20261017)
cm = O.clean_symmetrize(m); bad,_,_ = O.bad_mask(cm, 0.01); g = np.flatnonzero(~bad)
x = cm[np.ix_(g,g)]; c = O.sparse_cor(x); P = O.prcomp_x(c, 200, method="eigh")
for i in (() if len(sys.argv) > 2 else (1, 20, 100, 200)):
    ma, mb, co, he = O.coniss(np.ascontiguousarray(P[:, :i]))
    for K in (8, 16, 32):
        mg, bt = batched(P[:, :i], K)
        ok = np.array_equal(np.array(mg)[:, 0], ma)
        bt = np.array(bt)
        print(f"tree {i:3d} K {K:2d}: same merges {ok}  batches {len(bt)}  mean len {bt.mean():.2f}  merges/batch p10 {np.percentile(bt,10):.0f}", flush=True)

def batched_indep(p, K):
    """Batches of pairwise-independent candidates (no shared or neighbouring
    cluster), cut at the first conflict or the first pending cost that wins."""
    n = p.shape[0]
    nxt = {i: (i + 1 if i + 1 < n else -1) for i in range(n)}
    prv = {i: (i - 1) for i in range(n)}
    sums = {i: p[i].copy() for i in range(n)}
    size = {i: 1 for i in range(n)}
    cost = {i: ward(sums[i], 1, sums[i + 1], 1) for i in range(n - 1)}
    merges = []; batches = []
    while len(merges) < n - 1:
        L = sorted(cost.items(), key=lambda kv: (kv[1], kv[0]))[:K]
        used = set(); acc = []
        for pos, c in L:
            a = pos; b = nxt[a]; ls = prv[a]; r = nxt[b]
            cl = {x for x in (ls, a, b, r) if x >= 0}
            if cl & used: break
            used |= cl; acc.append((pos, c, a, b, ls, r))
        # precompute new costs with pre-batch rows, then scan
        cnt = 0; pend = []
        for (pos, c, a, b, ls, r) in acc:
            if pend and min(pend) < (c, pos): break
            sm = sums[a] + sums[b]; nm = size[a] + size[b]
            if ls >= 0: pend.append((ward(sums[ls], size[ls], sm, nm), ls))
            if r >= 0: pend.append((ward(sm, nm, sums[r], size[r]), a))
            cnt += 1
        for (pos, c, a, b, ls, r) in acc[:cnt]:
            merges.append((a, b))
            sums[a] = sums[a] + sums[b]; size[a] += size[b]; del sums[b]; del size[b]
            nxt[a] = r
            if r >= 0: prv[r] = a
            del cost[a]
            if b in cost: del cost[b]
            if ls >= 0: cost[ls] = ward(sums[ls], size[ls], sums[a], size[a])
            if r >= 0: cost[a] = ward(sums[a], size[a], sums[r], size[r])
        batches.append(cnt)
    return merges, batches

if __name__ == "__main__" and len(sys.argv) > 2:
    for i in (1, 20, 100, 200):
        ma, mb, co, he = O.coniss(np.ascontiguousarray(P[:, :i]))
        for K in (8, 16, 32):
            mg, bt = batched_indep(P[:, :i], K)
            ok = np.array_equal(np.array(mg)[:, 0], ma)
            bt = np.array(bt)
            print(f"INDEP tree {i:3d} K {K:2d}: same merges {ok}  batches {len(bt)}  mean len {bt.mean():.2f}", flush=True)
