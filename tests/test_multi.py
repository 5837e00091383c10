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
