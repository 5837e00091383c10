"""Which library switch breaks V=1 vs V=8 bit-identity of the sharded pipeline?
python tools/shard_bits.py N0 'which=value,...' ..."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "tests")]
import gpu_helpers as G  # noqa: E402
import tadpole_amd as tp  # noqa: E402
from tadpole_amd import multi  # noqa: E402
from tadpole_amd.synth import synth_hic  # noqa: E402

n0 = int(sys.argv[1])
if n0 < 0:   # the C5 test's arms: a |n0|-bin matrix generated in HBM (tests/test_gpu_configs.py)
    import torch
    from tadpole_amd.synth import SEED_BASE
    n0 = -n0
    gen = torch.Generator(device="cuda").manual_seed(SEED_BASE + 5)
    idx = torch.arange(n0, device="cuda", dtype=torch.float64)
    m = torch.empty((n0, n0), dtype=torch.float64, device="cuda")
    for r0 in range(0, n0, 2048):
        r1 = min(n0, r0 + 2048)
        m[r0:r1] = torch.poisson(1000.0 / (1.0 + (idx[r0:r1, None] - idx[None, :]).abs()), generator=gen)
    for r0 in range(0, n0, 2048):
        r1 = min(n0, r0 + 2048)
        m[r0:r1, :r0] = m[:r0, r0:r1].T
        m[r0:r1, r0:r1] = torch.triu(m[r0:r1, r0:r1]) + torch.triu(m[r0:r1, r0:r1], 1).T
    m = m.cpu().numpy()
else:
    m = synth_hic(n0, 20261099)
for cfg in sys.argv[2:]:
    sets = [tuple(int(v) for v in kv.split("=")) for kv in cfg.split(",") if kv]
    olds = [(w, G.knob(w, v)) for w, v in sets]
    outs = []
    Ps = []
    import ctypes
    from tadpole_amd import _lib
    L = _lib.load()

    def lastP(t):
        nn = int(np.asarray(t.timings_ms)[14])
        P = np.zeros((nn, 200), order="F")
        st = ctypes.c_int(0)
        L.tp_debug_last_scores(ctypes.byref(ctypes.c_int(nn)), ctypes.byref(ctypes.c_int(200)),
                               P.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(st))
        return P
    for v in (1, 8):
        multi.set_virtual_shards(v)
        outs.append(tp.TADpole(m, max_pcs=200, sharded=True))
        Ps.append(lastP(outs[-1]))
    multi.set_virtual_shards(1)
    un = tp.TADpole(m, max_pcs=200)
    for w, v in olds:
        G.knob(w, v)
    a, b = outs
    same = lambda x, y: np.array_equal(np.asarray(x.scores).view(np.uint64), np.asarray(y.scores).view(np.uint64))  # noqa: E731
    print(f"{cfg or 'default'}: V1==V8 {same(a, b)}  V1==unsharded {same(a, un)}", flush=True)
    for name, t in (("V1", a), ("V8", b), ("un", un)):
        tm = np.asarray(t.timings_ms)
        print(f"   {name}: n_pcs {t.n_pcs} ncl {t.optimal_n_clusters} iters {int(tm[11])} block {int(tm[12])} "
              f"resid {tm[13]!r} krylov {int(tm[16])}x{int(tm[17])}", flush=True)
    sa, sb = np.asarray(a.scores), np.asarray(b.scores)
    d = np.flatnonzero((sa.view(np.uint64) != sb.view(np.uint64)).any(axis=1))
    print("   rows (PC prefixes) with differing CH bits:", d[:20], len(d), flush=True)
    dP = Ps[0] != Ps[1]
    print("   P differs:", int(dP.sum()), "entries; columns", np.flatnonzero(dP.any(axis=0))[:10],
          "max abs", float(np.abs(Ps[0] - Ps[1]).max()), flush=True)
