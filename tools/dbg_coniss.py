import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
import gpu_helpers as G, tadpole_oracle as O
for (n, c, seed) in [(400, 200, 6), (300, 65, 5), (513, 256, 7)]:
    rng = np.random.default_rng(seed)
    p = rng.standard_normal((n, c)) * rng.random(c)[None, :] * 10
    ma, mb, co, he = O.coniss(p)
    for mode in (0,):
        old = 0
        _, h, bnd = G.coniss(p)
        pass
        bad = np.flatnonzero(bnd != mb)
        print(n, c, 'mode', mode, 'ok' if len(bad) == 0 else f'first diff at merge {bad[0]}', flush=True)
