"""Library context lifetime and concurrency (include/tadpole_hip.h,
tp_release_stream): one context of ~N^2 scratch per caller stream, retired
least-recently-used past TP_MAX_STREAM_CONTEXTS (default 8) or freed by
tadpole_amd.release_stream; every entry locks its context for the whole call,
so callers sharing the library stream serialise instead of racing."""
import threading

import numpy as np
import pytest

from tadpole_amd.synth import synth_hic

pytestmark = pytest.mark.gpu


def _used():
    import torch
    torch.cuda.synchronize()
    torch.cuda.empty_cache()     # torch caches blocks per stream: not the library's memory
    free, total = torch.cuda.mem_get_info(0)
    return total - free


def _same(a, b):
    return (a.n_pcs == b.n_pcs and a.optimal_n_clusters == b.optimal_n_clusters
            and np.array_equal(np.asarray(a.scores).view(np.uint64), np.asarray(b.scores).view(np.uint64))
            and a.clusters.keys() == b.clusters.keys()
            and all(np.array_equal(a.clusters[q], b.clusters[q]) for q in a.clusters))


def test_fresh_streams_keep_device_memory_bounded(gpu):
    """50 TADpole(stream=new) calls: the library keeps at most 8 stream
    contexts, so device memory stops growing; release_stream frees them."""
    import torch
    import tadpole_amd as tp
    m = synth_hic(3000, 61)
    ref = tp.TADpole(m, max_pcs=60)
    gpu.tp_shutdown()            # earlier tests' stream contexts out of the baseline
    base = _used()
    streams, used = [], []
    for i in range(50):
        s = torch.cuda.Stream()
        got = tp.TADpole(m, max_pcs=60, stream=s)
        assert _same(got, ref), i
        streams.append(s)
        used.append(_used() - base)
    per_ctx = max(used[0], 1)
    print("device memory above baseline after 1, 8, 16, 50 stream calls (MB):",
          [round(used[q] / 2**20) for q in (0, 7, 15, 49)])
    assert max(used) <= 8 * per_ctx + (256 << 20)         # bounded by the cap, not by the 50 calls
    assert used[-1] <= used[15] + (256 << 20)             # flat past the cap
    for s in streams:
        tp.release_stream(s)
    assert _used() - base <= (256 << 20)


def test_failed_scratch_allocation_then_smaller_call(gpu):
    """a scratch regrowth whose allocation fails (injected
    out-of-memory, knob 51) leaves that buffer empty, not a null block that
    still claims its old size: a smaller call on the same stream context then
    allocates it again and gives the same result (before the fix it wrote
    through a null pointer)."""
    import torch
    import tadpole_amd as tp
    import gpu_helpers as G
    small, large = synth_hic(900, 67), synth_hic(2200, 68)
    s = torch.cuda.Stream()
    ref = tp.TADpole(small, max_pcs=60, stream=s)
    old = G.knob(51, 1)
    try:
        with pytest.raises(Exception, match="injected out-of-memory"):
            tp.TADpole(large, max_pcs=60, stream=s)
    finally:
        G.knob(51, 0)
    assert _same(tp.TADpole(small, max_pcs=60, stream=s), ref)
    assert _same(tp.TADpole(large, max_pcs=60, stream=s), tp.TADpole(large, max_pcs=60))
    tp.release_stream(s)
    assert old == 0


_POOL_SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import tadpole_amd as tp
from tadpole_amd import _lib
from tadpole_amd.synth import synth_hic
def used():
    torch.cuda.synchronize(); torch.cuda.empty_cache()
    f, t = torch.cuda.mem_get_info(0)
    return t - f
m = synth_hic(4000, 69)
torch.zeros(1, device="cuda")
base = used()                       # before the library's first allocation
s = torch.cuda.Stream()
tp.TADpole(m, max_pcs=60, stream=s)
tp.TADpole(m, max_pcs=60)
peak = used()
tp.release_stream(s)
_lib.load().tp_shutdown()
after = used()
print("POOL", base, peak, after)
"""


def test_library_pool_returns_memory(gpu, tmp_path):
    """scratch comes from the library's own stream-ordered pool (not
    the device's default pool with its release threshold raised), and retiring
    the contexts trims it: in a fresh process, device memory after
    release_stream + tp_shutdown is back to its level before the library's
    first allocation (code objects aside)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _POOL_SCRIPT, root], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("POOL")][-1]
    base, peak, after = (int(v) for v in line.split()[1:])
    print(f"device memory: before {base >> 20} MB, two contexts {peak >> 20} MB, after shutdown {after >> 20} MB")
    assert peak - base > (512 << 20)                  # the scratch was really there
    assert after - base <= (96 << 20), (base, peak, after)


def test_default_stream_callers_serialise(gpu):
    """Two host threads on the library stream of one device (no stream given)
    get the same results as one caller: the context lock serialises them."""
    import tadpole_amd as tp
    mats = [synth_hic(1500, 62), synth_hic(1700, 63)]
    refs = [tp.TADpole(m, max_pcs=80) for m in mats]
    out = [[None] * 3, [None] * 3]
    errs = []

    def run(w):
        try:
            for r in range(3):
                out[w][r] = tp.TADpole(mats[w], max_pcs=80)
        except Exception as e:   # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(w,)) for w in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for w in range(2):
        for r in range(3):
            assert _same(out[w][r], refs[w]), (w, r)


def test_release_stream_while_in_use(gpu):
    """Releasing a stream's context while a call runs on it lets that call
    finish (it holds the context); the next call gets a fresh one."""
    import torch
    import tadpole_amd as tp
    m = synth_hic(2500, 64)
    s = torch.cuda.Stream()
    ref = tp.TADpole(m, max_pcs=100, stream=s)
    res = [None]
    t = threading.Thread(target=lambda: res.__setitem__(0, tp.TADpole(m, max_pcs=100, stream=s)))
    t.start()
    tp.release_stream(s)
    t.join()
    assert _same(res[0], ref)
    assert _same(tp.TADpole(m, max_pcs=100, stream=s), ref)
    tp.release_stream(s)


def test_device_input_not_modified(gpu):
    """TADpole() on a GPU tensor leaves the caller's tensor as it was (the
    pipeline cleans a device copy); inplace=True cleans it in place."""
    import torch
    import tadpole_amd as tp
    m = synth_hic(400, 65)
    m[3, 10] = np.nan
    m[20, 5] = 7.0                       # asymmetric entry (the upper triangle wins)
    d = torch.from_numpy(m).cuda()
    before = d.clone()
    a = tp.TADpole(d, max_pcs=50)
    assert torch.equal(torch.nan_to_num(d, nan=-1.0), torch.nan_to_num(before, nan=-1.0))
    b = tp.TADpole(d, max_pcs=50, inplace=True)
    assert _same(a, b)
    assert not torch.isnan(d).any() and torch.equal(d, d.T)


def test_run_genome_reuses_stream_contexts(gpu):
    """Consecutive run_genome calls draw their streams from a persistent pool,
    so the second call creates no library context (no N^2 scratch allocated
    or retired inside it) and gives bit-identical results."""
    from tadpole_amd import _lib
    from tadpole_amd.genome import run_genome
    mats = {f"c{i}": synth_hic(600 + 40 * i, 70 + i) for i in range(6)}
    a, _ = run_genome(mats, streams=4, max_pcs=60)
    live0, made0 = _lib.context_stats(0)
    b, _ = run_genome(mats, streams=4, max_pcs=60)
    live1, made1 = _lib.context_stats(0)
    assert made1 == made0, (made0, made1)
    assert live1 == live0
    for c in mats:
        assert _same(a[c], b[c]), c


def test_progress_word_reports_stages(gpu):
    """tp_progress_attach: a host word the pipeline on that stream's context
    advances 0 -> 1 (mask read back) -> 2 (correlation queued) -> 3 (PCA done)
    -> 4 (returned), polled from another thread while the call runs (what the
    concurrent centromere arms use to start the q arm under the p arm's sweep)."""
    import ctypes
    import time
    import torch
    from tadpole_amd import _lib
    m = synth_hic(2500, 66)
    s = torch.cuda.Stream()
    L = _lib.load()
    prog = np.full(1, -1, np.int32)
    st = ctypes.c_int(0)
    L.tp_progress_attach(ctypes.byref(ctypes.c_int(0)), ctypes.c_void_p(s.cuda_stream),
                         prog.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st))
    _lib.check(st)
    seen, done = [], [False]

    def run():
        try:
            import tadpole_amd as tp
            tp.TADpole(m, max_pcs=100, stream=s)
        finally:
            done[0] = True

    th = threading.Thread(target=run)
    th.start()
    while not done[0]:
        v = int(prog[0])
        if not seen or seen[-1] != v:
            seen.append(v)
        time.sleep(5e-5)
    th.join()
    seen.append(int(prog[0]))
    L.tp_progress_attach(ctypes.byref(ctypes.c_int(0)), ctypes.c_void_p(s.cuda_stream), None, ctypes.byref(st))
    _lib.check(st)
    vals = [v for v in seen if v >= 0]
    assert vals == sorted(vals) and vals[-1] == 4 and 3 in vals, seen
    import tadpole_amd as tp
    tp.release_stream(s)


def test_run_genome_presized_contexts_do_not_regrow(gpu):
    """Verdict r5 item 7: run_genome sizes its pool's stream contexts for the
    largest chromosome once (presize), so later calls regrow no scratch
    whichever stream receives which chromosome (knob 41 counts regrowths)."""
    from tadpole_amd import _lib
    from tadpole_amd.genome import run_genome
    mats = {f"c{i}": synth_hic(500 + 150 * i, 80 + i) for i in range(6)}
    a, _ = run_genome(mats, streams=3, max_pcs=60)
    _lib.debug_knob(41, 0)
    for _ in range(2):
        b, _ = run_genome(mats, streams=3, max_pcs=60)
    grows = _lib.debug_knob(41, 0)
    assert grows == 0, grows
    for c in mats:
        assert _same(a[c], b[c]), c
