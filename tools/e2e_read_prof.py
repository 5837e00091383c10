"""Times tp_read_tsv_dev (via tadpole_amd.api._read_to_device) alone and
inside TADpole(path) on a 10k-bin TSV in several orders, with TADpole's own
steps timed separately, to find where an interleaved call loses time (GPU box)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tadpole_amd as tp  # noqa: E402
from tadpole_amd.api import _assemble, _pipeline, _read_to_device  # noqa: E402
from tadpole_amd.synth import SEED_BASE, synth_hic_par, write_tsv  # noqa: E402

n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"e2e_read_{os.getpid()}.tsv")
write_tsv(synth_hic_par(n0, SEED_BASE + 3), path)


def steps(tag):
    t0 = time.perf_counter()
    raw = _read_to_device(path, 0)
    t1 = time.perf_counter()
    r = _pipeline(raw, 200, 2, 0.01, 0, 0)
    t2 = time.perf_counter()
    _assemble(r, np.flatnonzero(r["bad"]) + 1)
    t3 = time.perf_counter()
    del raw
    t4 = time.perf_counter()
    print(f"{tag}: read {1e3 * (t1 - t0):.1f} pipeline {1e3 * (t2 - t1):.1f} (device {r['timings'][4]:.1f}) "
          f"assemble {1e3 * (t3 - t2):.1f} del {1e3 * (t4 - t3):.1f} ms", flush=True)


print("cpu.max:", open("/sys/fs/cgroup/cpu.max").read().strip() if os.path.exists("/sys/fs/cgroup/cpu.max") else None, "affinity:", len(os.sched_getaffinity(0)), flush=True)
try:
    tp.TADpole(path)
    for rep in range(3):
        t0 = time.perf_counter()
        tp.TADpole(path)
        print(f"TADpole back to back: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    for rep in range(3):
        steps("steps back to back")
    for rep in range(3):
        t0 = time.perf_counter()
        d = _read_to_device(path, 0)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        del d
        print(f"read alone {1e3 * (t1 - t0):.1f} ms", flush=True)
        steps("steps after a read alone")
    for rep in range(3):
        t0 = time.perf_counter()
        d = _read_to_device(path, 0)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        del d
        print(f"read {1e3 * (t1 - t0):.1f} ms then device sync {1e3 * (t2 - t1):.1f} ms", flush=True)
    for rep in range(3):
        t0 = time.perf_counter()
        d = _read_to_device(path, 0)
        t1 = time.perf_counter()
        torch.cuda.current_stream(0).synchronize()
        t2 = time.perf_counter()
        del d
        print(f"read {1e3 * (t1 - t0):.1f} ms then null-stream sync {1e3 * (t2 - t1):.1f} ms", flush=True)
finally:
    os.remove(path)
