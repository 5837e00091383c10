"""One matrix sharded over several GPUs on the one-GPU box:

* virtual shards (tp_set_virtual_shards): the sharded schedule -- column-tile
  split of X'X / Xc'Xc, row split of G Q / Xc V, tree split of the sweep -- as
  V shards on one device.  Bar: bit-identical tadpole objects for V = 1, 2, 3,
  and, at a size where the unsharded products run without split-K (N >= 3072),
  bit-identical to the unsharded pipeline too;
* a real RCCL communicator of one rank (tp_comm_unique_id / tp_comm_init):
  the same schedule through ncclBroadcast; bit-identical to V = 1.
True multi-rank runs need several GPUs (bench.py --sharded under
torch.distributed.run); the exchange of the unique id is covered on CPU
(tests/test_multi.py)."""
import numpy as np
import pytest

import tadpole_amd as tp
from tadpole_amd import multi
from tadpole_amd.synth import synth_hic

pytestmark = pytest.mark.gpu


def _same(a, b):
    assert a.n_pcs == b.n_pcs and a.optimal_n_clusters == b.optimal_n_clusters
    assert set(a.clusters) == set(b.clusters)
    for k in a.clusters:
        assert np.array_equal(a.clusters[k], b.clusters[k]), k
    sa, sb = np.asarray(a.scores), np.asarray(b.scores)
    assert sa.shape == sb.shape
    assert np.array_equal(sa.view(np.uint64), sb.view(np.uint64))   # bit for bit, NA patterns included


@pytest.mark.parametrize("n0,seed", [(600, 31), (3300, 32)])
def test_virtual_shards_bit_identical(gpu, n0, seed):
    m = synth_hic(n0, seed)
    try:
        multi.set_virtual_shards(1)
        ref = tp.TADpole(m, max_pcs=200, sharded=True)
        for v in (2, 3):
            multi.set_virtual_shards(v)
            _same(tp.TADpole(m, max_pcs=200, sharded=True), ref)
    finally:
        multi.set_virtual_shards(1)
    if n0 >= 3100:
        _same(tp.TADpole(m, max_pcs=200), ref)


def test_virtual_shards_row_sharded_c(gpu):
    """C5's row-sharded C (knob 24, default): on the Krylov path each shard
    computes only its columns of C (the int8 X'X tiles that touch them) and
    their means, and the Krylov products read only those columns -- C is never
    gathered.  Bit-identical to the gathered schedule (knob 24 = 0) and to one
    shard, for both Krylov spaces (knob 20) and both X'X tile kernels (knob 44:
    k_xtx_i8_w's 256 x 128 slab tiles or the 128-tiles)."""
    import gpu_helpers as G
    m = synth_hic(2600, 35)
    old8 = G.knob(8, 0)            # the Krylov path at this size
    try:
        for space in (0, 1):
            old20 = G.knob(20, space)
            try:
                multi.set_virtual_shards(1)
                ref = tp.TADpole(m, max_pcs=160, sharded=True)
                assert ref.timings_ms[16] > 0
                for slab, wide in ((1, 1), (1, 0), (0, 1)):
                    old24, old44 = G.knob(24, slab), G.knob(44, wide)
                    try:
                        multi.set_virtual_shards(3)
                        _same(tp.TADpole(m, max_pcs=160, sharded=True), ref)
                    finally:
                        G.knob(24, old24)
                        G.knob(44, old44)
            finally:
                G.knob(20, old20)
                multi.set_virtual_shards(1)
    finally:
        G.knob(8, old8)


def test_virtual_shards_centromere_arms(gpu):
    m = synth_hic(700, 33, centromere=True)
    try:
        multi.set_virtual_shards(1)
        ref = tp.TADpole(m, max_pcs=60, centromere_search=True, sharded=True)
        multi.set_virtual_shards(4)
        got = tp.TADpole(m, max_pcs=60, centromere_search=True, sharded=True)
    finally:
        multi.set_virtual_shards(1)
    assert np.array_equal(got.merging_arms, ref.merging_arms)
    _same(got.p, ref.p)
    _same(got.q, ref.q)


def test_rccl_one_rank_communicator(gpu):
    m = synth_hic(500, 34)
    multi.set_virtual_shards(1)
    ref = tp.TADpole(m, max_pcs=100, sharded=True)
    uid = multi.comm_unique_id()
    assert len(uid) == 128
    import ctypes
    from tadpole_amd import _lib
    L = _lib.load()
    st = ctypes.c_int(0)
    L.tp_comm_init(uid, ctypes.byref(ctypes.c_int(1)), ctypes.byref(ctypes.c_int(0)),
                   ctypes.byref(ctypes.c_int(0)), ctypes.byref(st))
    _lib.check(st)
    try:
        _same(tp.TADpole(m, max_pcs=100, sharded=True), ref)
    finally:
        multi.destroy_comm(0)


def test_concurrent_streams_same_results(gpu):
    """Pipelines on several HIP streams at once (one library context per
    stream): each result equals the one-at-a-time result, bit for bit."""
    import threading

    import torch
    mats = [synth_hic(n, 40 + i) for i, n in enumerate((700, 640, 580, 700))]
    ref = [tp.TADpole(m, max_pcs=120) for m in mats]
    out = [None] * len(mats)
    streams = [torch.cuda.Stream() for _ in range(3)]

    def run(i):
        for j in range(i, len(mats), 3):
            out[j] = tp.TADpole(mats[j], max_pcs=120, stream=streams[i])

    th = [threading.Thread(target=run, args=(i,)) for i in range(3)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for a, b in zip(out, ref):
        _same(a, b)


def test_genome_driver_streams(gpu):
    from tadpole_amd.genome import run_genome
    mats = {f"chr{i}": synth_hic(n, 50 + i) for i, n in enumerate((500, 420, 460))}
    res, secs = run_genome(mats, streams=3, max_pcs=80)
    for name, m in mats.items():
        _same(res[name], tp.TADpole(m, max_pcs=80))


def _one_rank_comm():
    import ctypes
    from tadpole_amd import _lib
    uid = multi.comm_unique_id()
    L = _lib.load()
    st = ctypes.c_int(0)
    L.tp_comm_init(uid, ctypes.byref(ctypes.c_int(1)), ctypes.byref(ctypes.c_int(0)),
                   ctypes.byref(ctypes.c_int(0)), ctypes.byref(st))
    _lib.check(st)


def test_sharded_failure_on_caller_stream_aborts_device_communicator(gpu):
    """A device failure inside a sharded call on a caller stream (injected:
    knob 30) aborts the DEVICE's communicator, not just that stream
    context's copy: the next sharded call on any stream fails loudly (no
    silent unsharded run, no use of the freed communicator), tp_comm_destroy
    does not free it a second time, and a new communicator works again."""
    import torch
    import gpu_helpers as G
    from tadpole_amd._lib import TadpoleError, TP_ERR_HIP
    m = synth_hic(500, 36)
    multi.set_virtual_shards(1)
    ref = tp.TADpole(m, max_pcs=80, sharded=True)
    ref_u = tp.TADpole(m, max_pcs=80)
    _one_rank_comm()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        _same(tp.TADpole(m, max_pcs=80, sharded=True, stream=s1), ref)   # s1's context copies the comm
        G.knob(30, 1)
        with pytest.raises(TadpoleError) as e:
            tp.TADpole(m, max_pcs=80, sharded=True, stream=s1)
        assert e.value.status == TP_ERR_HIP and "injected" in str(e.value)
        for s in (s1, s2, None):      # the device's communicator is gone for every stream
            with pytest.raises(TadpoleError) as e:
                tp.TADpole(m, max_pcs=80, sharded=True, stream=s)
            assert "aborted" in str(e.value)
        _same(tp.TADpole(m, max_pcs=80, stream=s2), ref_u)                # unsharded calls are unaffected
    finally:
        G.knob(30, 0)
        multi.destroy_comm(0)          # no second free of the aborted communicator
    _same(tp.TADpole(m, max_pcs=80, sharded=True, stream=s1), ref)       # destroyed on purpose: one shard
    _one_rank_comm()
    try:
        _same(tp.TADpole(m, max_pcs=80, sharded=True, stream=s2), ref)
    finally:
        multi.destroy_comm(0)
    tp.release_stream(s1)
    tp.release_stream(s2)


def test_sharded_data_error_keeps_communicator(gpu):
    """A data error in a sharded call (fewer than 3 good bins: every rank
    sees it at the same point) fails that call only; the communicator stays
    alive and the next sharded call runs on it."""
    from tadpole_amd._lib import TadpoleError, TP_ERR_NO_BSTICK
    m = synth_hic(400, 37)
    multi.set_virtual_shards(1)
    ref = tp.TADpole(m, max_pcs=60, sharded=True)
    bad = np.zeros((50, 50))
    bad[0, 0] = bad[1, 1] = 5.0
    _one_rank_comm()
    try:
        with pytest.raises(TadpoleError) as e:
            tp.TADpole(bad, max_pcs=10, sharded=True)
        assert e.value.status == TP_ERR_NO_BSTICK
        _same(tp.TADpole(m, max_pcs=60, sharded=True), ref)
    finally:
        multi.destroy_comm(0)
