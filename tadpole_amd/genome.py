"""Whole-genome driver: independent chromosome matrices sharded over the GPUs
of one node (BASELINE.json configs[3]).

One process per GPU (``torch.distributed.run``), each rank owning the
chromosomes that LPT (longest processing time first, cost ~ N^3) assigns to it.
There is no data-path collective: each matrix is processed entirely on its
rank's GPU, and only the small per-chromosome results are gathered to rank 0
(``gather_object``).  The reference has no equivalent (it runs one matrix per
R call, R/TADpole.R:344); this replaces a shell loop over chromosomes.
"""
from __future__ import annotations

import heapq
import os
import time
from typing import Callable, Dict, List, Mapping, Optional, Sequence, Tuple


def lpt_assign(costs: Mapping[str, float], n_workers: int) -> List[List[str]]:
    """Greedy LPT: biggest job first onto the least-loaded worker.  Ties are
    broken by name and worker index so every rank computes the same plan."""
    if n_workers < 1:
        raise ValueError("n_workers must be >= 1")
    heap = [(0.0, w) for w in range(n_workers)]
    plan: List[List[str]] = [[] for _ in range(n_workers)]
    for name in sorted(costs, key=lambda c: (-costs[c], c)):
        load, w = heapq.heappop(heap)
        plan[w].append(name)
        heapq.heappush(heap, (load + float(costs[name]), w))
    return plan


def matrix_cost(n_bins: int) -> float:
    """Relative cost of one matrix: the N^3 products dominate."""
    return float(n_bins) ** 3


def run_genome(matrices: Mapping[str, object], sizes: Optional[Mapping[str, int]] = None,
               runner: Optional[Callable[[str, object, int], object]] = None, streams: int = 8,
               **tadpole_kwargs) -> Tuple[Dict[str, object], Dict[str, float]]:
    """Process every chromosome once across the ranks of the default process
    group (or locally when torch.distributed is not initialised).

    matrices: name -> path / array / zero-arg loader callable (only the
    owner of a chromosome materialises it).  sizes: name -> bins (for the
    plan; read from the arrays when absent).  runner(name, matrix, device)
    defaults to ``TADpole(matrix, device=device, **tadpole_kwargs)``.
    Returns (results, seconds per chromosome) on rank 0 (empty dicts elsewhere
    unless every rank asked for them).
    """
    import torch.distributed as dist

    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size() if dist_on else 1
    rank = dist.get_rank() if dist_on else 0
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if sizes is None:
        sizes = {}
        for name, m in matrices.items():
            shape = getattr(m, "shape", None)
            if shape is None:
                raise ValueError(f"sizes[{name!r}] is needed when the matrix is not an array")
            sizes[name] = int(shape[0])
    plan = lpt_assign({c: matrix_cost(sizes[c]) for c in matrices}, world)
    mine: Dict[str, object] = {}
    secs: Dict[str, float] = {}

    def one(name, run):
        m = matrices[name]
        if callable(m):
            m = m()
        t0 = time.perf_counter()
        mine[name] = run(name, m, local)
        secs[name] = time.perf_counter() - t0

    if runner is None and streams > 1 and len(plan[rank]) > 1:
        # this rank's chromosomes, up to `streams` in flight on one GPU (one
        # HIP stream and library context each): the latency-bound stages of a
        # pipeline leave most CUs idle
        import threading
        from concurrent.futures import ThreadPoolExecutor

        import torch

        from .api import TADpole
        tls = threading.local()

        def run_stream(name, m, device):
            if getattr(tls, "stream", None) is None:
                tls.stream = torch.cuda.Stream(device=f"cuda:{device}")
            return TADpole(m, device=device, stream=tls.stream, **tadpole_kwargs)

        with ThreadPoolExecutor(max_workers=streams) as ex:
            for f in [ex.submit(one, name, run_stream) for name in plan[rank]]:
                f.result()
    else:
        if runner is None:
            from .api import TADpole

            def runner(name, m, device):
                return TADpole(m, device=device, **tadpole_kwargs)

        for name in plan[rank]:
            one(name, runner)
    if not dist_on:
        return mine, secs
    gathered = [None] * world if rank == 0 else None
    dist.gather_object((mine, secs), gathered, dst=0)
    if rank != 0:
        return {}, {}
    res: Dict[str, object] = {}
    tim: Dict[str, float] = {}
    for part in gathered:
        res.update(part[0])
        tim.update(part[1])
    return res, tim
