"""CPU emulation of k_coniss_b's control flow (tp_sweep.hip: the candidate
scan, the waves' segments, slot_of, ranks, windows, conflicts, runs, the
block-minimum refresh) with range assertions on every LDS / slab index,
checked merge for merge against a sequential CONISS with the same cost
function.  Design tool and regression check of the batched kernel's indexing
(it found the slot_of prefix-search bug that faulted the first build): python
tools/coniss_batch_emu.py"""
import sys, numpy as np
NAN = float('nan')
W, CAP, FMAX, SEG = 8, 16, 16, 8   # SEG: positions <= T a wave may contribute (CB_SEG)
NMIN = 2                           # rescan when the maintained set holds fewer (CB_NMIN)

def ward(sa, na, sb, nb):
    e = sa * nb - sb * na
    return float(np.sum(e * e)) / (na * nb * (na + nb))

def seq_coniss(p):
    n = p.shape[0]
    starts = list(range(n)); sums = [p[i].copy() for i in range(n)]; size = [1]*n
    merges = []
    while len(starts) > 1:
        best = None
        for t in range(len(starts) - 1):
            c = ward(sums[t], size[t], sums[t+1], size[t+1])
            if c != c: c = float('inf')
            if best is None or c < best[0]: best = (c, t)
        c, t = best
        merges.append((starts[t], starts[t+1], c))
        sums[t] = sums[t] + sums[t+1]; size[t] += size[t+1]
        del starts[t+1]; del sums[t+1]; del size[t+1]
    return merges

def kernel(p):
    n = p.shape[0]
    nbk = (n + 63) // 64; BS = (nbk + 63) // 64
    cst = nbk * 64 + 64; lst = n + 64; DC = nbk * 64; DL = n
    cost = np.full(cst, NAN); link = np.full(lst, -1, np.int64); rn = np.full(lst, -1, np.int64)
    bmin = np.full(nbk, NAN)
    rows = {}                      # slab rows of merged clusters: start -> (sums, size)
    def row(start, single):
        if single: return p[start].copy()
        assert start in rows, ("slab row never written", start)
        return rows[start].copy()
    for q in range(n - 1):
        c = ward(p[q], 1, p[q+1], 1); cost[q] = c if c == c else float('inf')
    for q in range(n):
        link[q] = q; rn[q] = q + 1 if q + 1 < n else -1
    for bk in range(nbk):
        bmin[bk] = np.nanmin(cost[bk*64:bk*64+64]) if not np.all(np.isnan(cost[bk*64:bk*64+64])) else NAN
    def lds_cost(i):
        assert 0 <= i < cst, ("cost index", i); return cost[i]
    def lds_link(i):
        assert 0 <= i < lst, ("link index", i); return int(link[i])
    def lds_rn(i):
        assert 0 <= i < lst, ("rn index", i); return int(rn[i])
    merges = []; s = 0; gap = -1.0; h = 0.0; nbatch = 0; Sset = None; Tset = None; nscan = 0
    sgc = [NAN] * (W * SEG); sgp = [-(10**9)] * (W * SEG)
    while s < n - 1:
        nbatch += 1
        bm = [[bmin[64*q+l] if 64*q+l < nbk else NAN for l in range(64)] for q in range(BS)]
        allv = [x for row_ in bm for x in row_ if x == x]
        gq = min(allv)
        if not (gap > 0.0): gap = 0.5 * gq if (gq > 0.0 and gq < 1e300) else 1e-300
        tries = 0; C = 0; cands = None
        rescan = Sset is None or len(Sset) < NMIN
        if not rescan:
            cands = list(Sset); C = len(cands); T = Tset
        nscan += rescan
        while rescan:
            T = gq + gap
            if not (T >= gq) or tries >= 6: T = gq
            segn = [0] * W
            F = 0
            waves = [[-1, -1] for _ in range(W)]
            for q in range(BS):
                f = [bm[q][l] <= T for l in range(64)]
                idxs = []; cntb = 0
                for l in range(64):
                    idxs.append(F + cntb)
                    if f[l]: cntb += 1
                for w in range(W):
                    mine = [l for l in range(64) if f[l] and (idxs[l] & (W - 1)) == w]
                    i0 = 64*q + mine[0] if len(mine) > 0 else -1
                    i1 = 64*q + mine[1] if len(mine) > 1 else -1
                    mb0, mb1 = waves[w]
                    if i0 >= 0:
                        if mb0 < 0: mb0 = i0
                        elif mb1 < 0: mb1 = i0
                    if i1 >= 0 and mb1 < 0: mb1 = i1
                    waves[w] = [mb0, mb1]
                F += cntb
            ent = []
            for w in range(W):
                mb0, mb1 = waves[w]
                if F <= FMAX:
                    v0 = [lds_cost((mb0 if mb0 >= 0 else 0) * 64 + l) for l in range(64)]
                    v1 = [lds_cost((mb1 if mb1 >= 0 else 0) * 64 + l) for l in range(64)]
                    sel = [(v0[l], mb0*64+l) for l in range(64) if mb0 >= 0 and v0[l] <= T] + \
                          [(v1[l], mb1*64+l) for l in range(64) if mb1 >= 0 and v1[l] <= T]
                    segn[w] = len(sel)
                    if len(sel) <= SEG: ent += sel
                else:
                    segn[w] = SEG + 1
            if max(segn) <= SEG and CAP >= sum(segn) >= 1:
                C = sum(segn); cands = ent; Tset = T
                if tries <= 5: gap *= 1.3 if C < 12 else (0.8 if C > 15 else 1.0)   # TP_CB_LO / TP_CB_HI
                break
            if tries >= 6:                                 # the exact argmin alone
                pos = min([q_ for q_ in range(n) if cost[q_] == gq])
                cands = [(gq, pos)]; C = 1; T = None; Tset = None
                break
            gap *= 0.5; tries += 1
        for (cc, pp) in cands: assert 0 <= pp < n and cost[pp] == cc, ("cand", pp, cc)
        if T is not None:
            allpos = sorted([q_ for q_ in range(n) if cost[q_] <= T], key=lambda q_: (cost[q_], q_))
            assert len(allpos) == C, "incomplete set"
        srt = sorted(cands, key=lambda kv: (kv[0], kv[1]))
        Kc = min(C, W); slots = srt[:Kc]
        # A2
        rec = []
        for w in range(Kc):
            key, a = slots[w]
            lsv = lds_link(a - 1 if a > 0 else DL); ea = lds_link(a); eb = lds_rn(a)
            b = ea + 1; ls = lsv if a > 0 else -1; r = eb + 1 if eb + 1 < n else -1
            er = lds_rn(b) if r >= 0 else -1
            assert 0 <= a < n and a <= ea < n - 1 and b <= eb < n, ("window", a, ea, b, eb)
            assert ls < 0 or (0 <= ls < a and lds_link(a - 1) == ls), ("ls", ls)
            assert r < 0 or (eb < r <= er < n), ("r", r, er)
            sa = row(a, ea == a); sb = row(b, eb == b)
            sl = row(ls, ls == a - 1) if ls >= 0 else sa; sr = row(r, er == r) if r >= 0 else sa
            sm = sa + sb; fm = eb - a + 1; fl = a - ls; fr = er - r + 1
            cl = ward(sl, fl, sm, fm) if ls >= 0 else NAN
            cr = ward(sm, fm, sr, fr) if r >= 0 else NAN
            if ls >= 0 and cl != cl: cl = float('inf')
            if r >= 0 and cr != cr: cr = float('inf')
            lo = ls if ls >= 0 else a; hi = er if r >= 0 else eb
            rec.append(dict(a=a, key=key, ea=ea, b=b, eb=eb, ls=ls, r=r, er=er, lo=lo, hi=hi, cl=cl, cr=cr, sm=sm))
        # A3
        kacc = Kc
        for i in range(Kc):
            if any(not (rec[i]['hi'] < rec[j]['lo'] or rec[j]['hi'] < rec[i]['lo']) for j in range(i)):
                kacc = i; break
        cnt = kacc
        for i in range(kacc):
            ki, ai = rec[i]['key'], rec[i]['a']
            und = False
            for j in range(i):
                rj = rec[j]
                if rj['ls'] >= 0 and (rj['cl'], rj['ls']) < (ki, ai): und = True
                if rj['r'] >= 0 and (rj['cr'], rj['a']) < (ki, ai): und = True
            if und: cnt = i; break
        assert cnt >= 1 and s + cnt <= n - 1
        for j in range(cnt):
            x = rec[j]
            cost[x['b']] = NAN; cost[x['a']] = x['cr']; link[x['a']] = x['eb']; link[x['eb']] = x['a']; rn[x['a']] = x['er']
            if x['ls'] >= 0: cost[x['ls']] = x['cl']; rn[x['ls']] = x['eb']
        # the maintained set: drop the changed positions, add the new costs <= T
        if T is None:
            Sset = None
        else:
            chg = set()
            for j in range(cnt):
                chg |= {rec[j]['a'], rec[j]['b']} | ({rec[j]['ls']} if rec[j]['ls'] >= 0 else set())
            ns = [(cc, pp) for (cc, pp) in cands if pp not in chg]
            for j in range(cnt):
                x = rec[j]
                if x['ls'] >= 0 and x['cl'] <= Tset: ns.append((x['cl'], x['ls']))
                if x['r'] >= 0 and x['cr'] <= Tset: ns.append((x['cr'], x['a']))
            Sset = ns if len(ns) <= CAP else None
            if Sset is not None:
                exact = sorted([q_ for q_ in range(n) if cost[q_] <= Tset])
                assert sorted(pp for _, pp in Sset) == exact, "maintained set not exact"
        for j in range(cnt):
            x = rec[j]
            rows[x['a']] = x['sm']
            merges.append((x['a'], x['b'], x['key']))
            for blk in (x['a'] >> 6, x['b'] >> 6, (x['ls'] >> 6) if x['ls'] >= 0 else x['a'] >> 6):
                seg = cost[blk*64:blk*64+64]
                bmin[blk] = NAN if np.all(np.isnan(seg)) else np.nanmin(seg)
        s += cnt
    return merges, (nbatch, nscan)

def structured(n, k, seed):
    r = np.random.default_rng(seed)
    cuts = np.cumsum(r.integers(10, 60, size=n)); seg = np.searchsorted(cuts, np.arange(n), side="right")
    means = r.standard_normal((seg.max() + 1, k)) * (1.0 / (1 + np.arange(k)))
    return means[seg] + 0.05 * r.standard_normal((n, k))


if __name__ == "__main__":
    cases = [(150, 5, 31), (150, 1, 3), (70, 2, 5), (300, 3, 7), (1000, 1, 9), (1000, 4, 11), (3, 1, 1), (64, 1, 2), (65, 2, 4), (129, 1, 6)]
    for n, k, seed in cases:
        p = structured(n, k, seed)
        ref = seq_coniss(p)
        got, nb = kernel(p)
        ok = [(a, b) for a, b, _ in got] == [(a, b) for a, b, _ in ref]
        print(f"n={n} k={k}: same merges {ok}, batches {nb[0]} ({(n-1)/nb[0]:.2f} merges each), scans {nb[1]}", flush=True)
        assert ok
    # ties: duplicate rows
    p = np.repeat(structured(40, 2, 3), 5, axis=0)
    ref = seq_coniss(p); got, nb = kernel(p)
    print("ties:", [(a, b) for a, b, _ in got] == [(a, b) for a, b, _ in ref], nb)
