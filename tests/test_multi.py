"""CPU, world_size 2 over gloo: the whole-genome driver shards independent
chromosome matrices with LPT, runs each on its owner, and gathers results on
rank 0 (no data-path collective).  The per-matrix runner here is the CPU
oracle (the GPU path is covered by the gpu-marked tests)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tadpole_amd.genome import lpt_assign, matrix_cost, run_genome
from tadpole_amd.synth import genome_bins


def test_lpt_plan_balanced_and_deterministic():
    bins = genome_bins(25000)
    costs = {c: matrix_cost(n) for c, n in bins.items()}
    for w in (1, 2, 4, 8):
        plan = lpt_assign(costs, w)
        assert sorted(sum(plan, [])) == sorted(bins)
        assert plan == lpt_assign(dict(reversed(list(costs.items()))), w)
        loads = [sum(costs[c] for c in p) for p in plan]
        assert max(loads) <= 2 * (sum(loads) / w) or w >= len(bins) // 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    import tadpole_oracle as O
    from tadpole_amd.synth import synth_hic
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sizes = {"chrA": 120, "chrB": 90, "chrC": 70, "chrD": 60}
    mats = {c: (lambda n=n, s=i: synth_hic(n, 100 + s)) for i, (c, n) in enumerate(sizes.items())}

    def runner(name, m, device):
        r = O.tadpole(m, max_pcs=30, nthreads=1)
        return (rank, r.n_pcs, r.optimal_n_clusters)

    res, secs = run_genome(mats, sizes=sizes, runner=runner)
    if rank == 0:
        out.put((sorted(res.items()), sorted(secs)))
    dist.barrier()
    dist.destroy_process_group()


def test_genome_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    items, names = q.get(timeout=300)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    got = dict(items)
    assert sorted(got) == ["chrA", "chrB", "chrC", "chrD"]
    owners = {c: v[0] for c, v in got.items()}
    assert set(owners.values()) == {0, 1}          # both ranks did work
    assert owners["chrA"] != owners["chrB"]         # LPT: two largest split
    # same answers as a single-process run
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import tadpole_oracle as O
    from tadpole_amd.synth import synth_hic
    r = O.tadpole(synth_hic(120, 100), max_pcs=30, nthreads=1)
    assert got["chrA"][1:] == (r.n_pcs, r.optimal_n_clusters)


def _flaky_worker(rank, world, port, out, always):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sizes = {"chrA": 120, "chrB": 90, "chrC": 70, "chrD": 60}
    mats = {c: np.full((n, n), 1.0) for c, n in sizes.items()}

    def runner(name, m, device):
        # "one": chrB fails on whichever rank first gets it (rank 1 under LPT);
        # "rank1": everything fails on rank 1 (a lost device: all of its
        # chromosomes must move to rank 0); "always": chrB on every rank
        if (always == "rank1" and rank == 1) or (name == "chrB" and (always == "always" or rank == 1)):
            raise RuntimeError(f"device lost on rank {rank}")
        return (rank, m.shape[0])

    try:
        res, _ = run_genome(mats, sizes=sizes, runner=runner, retries=1)
        msg = None
    except RuntimeError as e:
        res, msg = {}, str(e)
    if rank == 0:
        out.put((sorted(res.items()), msg))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("always", ["one", "rank1", "always"])
def test_genome_failed_chromosome_requeued_on_other_rank(always):
    """a chromosome that fails on one rank is re-planned onto
    another rank; one that fails everywhere is reported by name."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_flaky_worker, args=(r, 2, port, q, always)) for r in range(2)]
    for p in ps:
        p.start()
    items, msg = q.get(timeout=300)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    if always == "always":
        assert msg is not None and "chrB" in msg and "device lost" in msg
    else:
        got = dict(items)
        assert msg is None and sorted(got) == ["chrA", "chrB", "chrC", "chrD"]
        assert got["chrB"] == (0, 90)          # re-run by rank 0 after rank 1 failed it
        if always == "rank1":                  # every chromosome ends on the healthy rank
            assert all(r == 0 for r, _ in got.values())


# ------------------------------------------- one matrix over several GPUs
# (SURVEY.md §8(e)2).  The split is host logic of the library (tp_shard_plan,
# no device needed); the unique-id exchange runs over gloo with the library
# calls replaced (no RCCL device here); the sharded arithmetic itself is
# covered on the GPU by tests/test_gpu_shard.py.

@pytest.mark.parametrize("n", [64, 65, 1000, 7808, 24300, 49851])
@pytest.mark.parametrize("R", [1, 2, 3, 4, 8])
def test_shard_plan_tile_columns_balanced(n, R):
    from tadpole_amd import multi
    b = multi.shard_plan(n, R, multi.PLAN_TILE_COLUMNS)
    tn = (n + 63) // 64
    assert b[0] == 0 and b[-1] == tn and np.all(np.diff(b) >= 0)
    w = np.array([sum(j + 1 for j in range(b[r], b[r + 1])) for r in range(R)])
    assert w.sum() == tn * (tn + 1) // 2
    # every rank within one tile column of the ideal share
    assert np.all(np.abs(w - w.sum() / R) <= tn + 1)


@pytest.mark.parametrize("n,R", [(24300, 8), (3300, 3), (100, 4), (7808, 2)])
def test_shard_plan_rows_and_trees(n, R):
    from tadpole_amd import multi
    r = multi.shard_plan(n, R, multi.PLAN_ROWS)
    assert r[0] == 0 and r[-1] == n and np.all(np.diff(r) >= 0)
    assert all(x % 64 == 0 for x in r[:-1])
    t = multi.shard_plan(200, R, multi.PLAN_TREES)
    assert t[0] == 0 and t[-1] == 200 and np.all(np.diff(t) >= 0) and np.diff(t).max() - np.diff(t).min() <= 1


def _comm_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tadpole_amd import multi
    seen = []
    uid = bytes(range(128))

    def uid_fn():
        assert dist.get_rank() == 0, "only rank 0 makes the id"
        return uid

    def init_fn(u, nranks, r, device):
        seen.append((u == uid, nranks, r, device))

    rr, ww = multi.init_comm(device=rank, uid_fn=uid_fn, init_fn=init_fn)
    out.put((rank, rr, ww, seen))
    dist.barrier()
    dist.destroy_process_group()


def test_comm_unique_id_exchange_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, rr, ww, seen in got:
        assert (rr, ww) == (rank, 2)
        assert seen == [(True, 2, rank, rank)]
