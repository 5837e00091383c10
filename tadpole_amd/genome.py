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
import queue
import threading
import time
from typing import Callable, Dict, List, Mapping, Optional, Sequence, Tuple

# persistent per-(device, width) pools: a worker executor and `width` HIP
# streams handed out one per running chromosome.  The library keeps one
# context (~N^2 of scratch) per caller stream, so reusing the same streams
# call after call reuses those contexts instead of building fresh ones (and
# retiring old ones) inside every run_genome call.
_POOLS: Dict[Tuple[int, int], tuple] = {}
_POOLS_LOCK = threading.Lock()


def _stream_pool(device: int, width: int):
    key = (device, width)
    with _POOLS_LOCK:
        pool = _POOLS.get(key)
        if pool is None:
            import torch
            from concurrent.futures import ThreadPoolExecutor
            free = queue.SimpleQueue()
            for _ in range(width):
                free.put(torch.cuda.Stream(device=f"cuda:{device}"))
            pool = (ThreadPoolExecutor(max_workers=width, thread_name_prefix=f"tadpole-genome{device}"), free)
            _POOLS[key] = pool
    return pool


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
               retries: int = 1, phases: Optional[Dict[str, Dict[str, float]]] = None,
               presize: bool = True, **tadpole_kwargs) -> Tuple[Dict[str, object], Dict[str, float]]:
    """Process every chromosome once across the ranks of the default process
    group (or locally when torch.distributed is not initialised).

    matrices: name -> path / array / zero-arg loader callable (only the
    owner of a chromosome materialises it).  sizes: name -> bins (for the
    plan; read from the arrays when absent).  runner(name, matrix, device)
    defaults to ``TADpole(matrix, device=device, **tadpole_kwargs)``.

    Failure handling: a chromosome whose run raises is
    re-queued up to ``retries`` times; the failures of all ranks are gathered
    and re-planned (LPT) onto the OTHER ranks when there are any, one matrix at
    a time.  What still fails afterwards raises a RuntimeError on every rank,
    naming the chromosomes and their last errors.
    Returns (results, seconds per chromosome) on rank 0 (empty dicts elsewhere).
    ``phases`` (optional, filled on this rank): per chromosome the seconds it
    waited for a stream worker (``wait``), then the result's ``host_s``
    (``upload``, ``call``, ``assemble``) when the runner reports them.
    ``presize``: with several streams any stream may receive any chromosome,
    so after the chromosomes have run, every context of the pool is sized
    like the largest (``_lib.reserve_streams``: each scratch buffer to its
    largest size over the pool, allocation only): later calls on the same
    genome regrow no scratch whichever stream receives which chromosome (each
    regrowth re-allocates a buffer on the stream).
    """
    import torch.distributed as dist

    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size() if dist_on else 1
    rank = dist.get_rank() if dist_on else 0
    local = int(os.environ.get("LOCAL_RANK", "0"))
    try:   # ranks beyond the visible GPUs wrap onto them (as bench.py's ranks do)
        import torch
        nd = torch.cuda.device_count()
        if nd > 0:
            local %= nd
    except ImportError:
        pass
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
    failed: Dict[str, str] = {}

    t_submit = time.perf_counter()

    def one(name, run):
        m = matrices[name]
        try:
            if callable(m):
                m = m()
            t0 = time.perf_counter()
            mine[name] = run(name, m, local)
            secs[name] = time.perf_counter() - t0
            if phases is not None:
                phases[name] = dict(wait=t0 - t_submit, **dict(getattr(mine[name], "host_s", {}) or {}))
            failed.pop(name, None)
        except Exception as e:   # noqa: BLE001 -- recorded, re-queued below
            failed[name] = f"{type(e).__name__}: {e}"

    if runner is None:
        from .api import TADpole

        def runner(name, m, device):
            return TADpole(m, device=device, **tadpole_kwargs)

        if streams > 1 and len(plan[rank]) > 1:
            # this rank's chromosomes, up to `streams` in flight on one GPU (one
            # HIP stream and library context each, from the persistent pool):
            # the latency-bound stages of a pipeline leave most CUs idle.
            # (Hardware queues: see tadpole_amd.use_hw_queues.)
            ex, free = _stream_pool(local, streams)

            def run_stream(name, m, device):
                s = free.get()
                try:
                    return TADpole(m, device=device, stream=s, **tadpole_kwargs)
                finally:
                    free.put(s)

            for f in [ex.submit(one, name, run_stream) for name in plan[rank]]:
                f.result()
            if presize:
                # every chromosome has now run on some stream of the pool: size
                # all of its contexts alike (each buffer to its largest size
                # over the pool), so later calls regrow no scratch whichever
                # stream receives which chromosome
                from . import _lib
                held = [free.get() for _ in range(streams)]
                try:
                    _lib.reserve_streams(held, device=local)
                finally:
                    for st in held:
                        free.put(st)
        else:
            for name in plan[rank]:
                one(name, runner)
    else:
        for name in plan[rank]:
            one(name, runner)

    def gather_failed():
        if not dist_on:
            return {c: (rank, e) for c, e in failed.items()}
        parts = [None] * world
        dist.all_gather_object(parts, {c: (rank, e) for c, e in failed.items()})
        out = {}
        for p in parts:
            out.update(p)
        return out

    for _ in range(max(0, retries)):
        all_failed = gather_failed()
        if not all_failed:
            break
        # re-plan onto the other ranks (a rank that failed a matrix may have a
        # bad device): LPT over world - 1 bins, bin w of a matrix that failed on
        # rank r going to rank (r + 1 + w) % world, never r; alone, retry locally
        replan = lpt_assign({c: matrix_cost(sizes[c]) for c in all_failed}, max(1, world - 1))
        failed.clear()   # every failure is re-owned below (and re-recorded if it fails again)
        for w, names in enumerate(replan):
            for name in names:
                owner = (all_failed[name][0] + 1 + w) % world if world > 1 else 0
                if owner == rank:
                    one(name, runner)
    still = gather_failed()
    if still:
        raise RuntimeError("chromosomes failed after %d retr%s: %s" % (
            retries, "y" if retries == 1 else "ies",
            "; ".join(f"{c} (rank {r}): {e}" for c, (r, e) in sorted(still.items()))))
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
