"""C4 alone (the 23 hg19 chromosomes @25 kb through run_genome, 8 streams on
one GPU, host matrices), for kernel traces: python tools/c4_time.py [reps]
[streams] [knob=value ...]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE]
import torch  # noqa: E402,F401

from tadpole_amd.genome import run_genome  # noqa: E402
from tadpole_amd.synth import genome_bins, genome_matrix  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
streams = int(sys.argv[2]) if len(sys.argv) > 2 else 8
from tadpole_amd import _lib  # noqa: E402
for kv in sys.argv[3:]:
    w, v = (int(x) for x in kv.split("="))
    _lib.debug_knob(w, v)
sizes = genome_bins()
mats = {c: genome_matrix(c) for c in sizes}
run_genome(mats, sizes=sizes, streams=streams, max_pcs=200)   # warm-up
for _ in range(reps):
    ph = {}
    t0 = time.perf_counter()
    res, secs = run_genome(mats, sizes=sizes, streams=streams, max_pcs=200, phases=ph)
    print(f"c4 {time.perf_counter() - t0:.4f} s  slowest chromosome {max(secs.values()):.4f} s", flush=True)
