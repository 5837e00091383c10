"""Where the end-to-end TADpole(path) time goes at 10k bins: the call timed
whole, then under cProfile (top entries by cumulative time)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tadpole_amd as tp  # noqa: E402
from tadpole_amd.synth import SEED_BASE, synth_hic_par, write_tsv  # noqa: E402

n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"e2e_prof_{os.getpid()}.tsv")
write_tsv(synth_hic_par(n0, SEED_BASE + 3), path)
try:
    tp.TADpole(path)
    for _ in range(3):
        t0 = time.perf_counter()
        tp.TADpole(path)
        print(f"TADpole({n0}) {time.perf_counter() - t0:.4f} s", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    tp.TADpole(path)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(18)
finally:
    os.remove(path)
