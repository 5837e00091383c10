"""One matrix over the GPUs of one node (BASELINE.json
configs[4]: chr1 @5kb, arms of ~24k bins).

One process per GPU (``torch.distributed.run``).  Rank 0 asks the library for
an RCCL unique id (``tp_comm_unique_id``), the 128 bytes travel over the
default process group (gloo or nccl), and every rank binds the library's own
RCCL communicator to its device (``tp_comm_init``).  ``TADpole(...,
sharded=True)`` then passes ``TP_FLAG_SHARDED``: every rank holds the same
matrix, the O(N^3) / O(N^2 b) products are split by column tiles / rows and
all-gathered over xGMI inside the library, the sweep is split by PC prefix,
and every rank returns the same ``tadpole`` object, bit-identical for any rank
count.  The reference has no multi-GPU path (it forks over PC prefixes on one
host, R/TADpole.R:104).
"""
from __future__ import annotations

import ctypes
from typing import Callable, List, NamedTuple, Optional, Tuple

import numpy as np

from . import _lib


def comm_unique_id() -> bytes:
    """RCCL unique id (128 bytes) from the library (needs RCCL, not a GPU)."""
    L = _lib.load()
    buf = ctypes.create_string_buffer(128)
    st = ctypes.c_int(0)
    L.tp_comm_unique_id(buf, ctypes.byref(st))
    _lib.check(st)
    return buf.raw


def _lib_init(uid: bytes, nranks: int, rank: int, device: int) -> None:
    L = _lib.load()
    st = ctypes.c_int(0)
    L.tp_comm_init(uid, ctypes.byref(ctypes.c_int(nranks)), ctypes.byref(ctypes.c_int(rank)),
                   ctypes.byref(ctypes.c_int(device)), ctypes.byref(st))
    _lib.check(st)


def init_comm(device: int, group=None, uid_fn: Optional[Callable[[], bytes]] = None,
              init_fn: Optional[Callable[[bytes, int, int, int], None]] = None) -> Tuple[int, int]:
    """Create the library's communicator for this rank over the ranks of
    ``group`` (default: the default process group).  ``uid_fn`` / ``init_fn``
    replace the library calls (tests on hosts without RCCL devices)."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    obj = [(uid_fn or comm_unique_id)() if rank == 0 else None]
    src = 0 if group is None else dist.get_global_rank(group, 0)
    dist.broadcast_object_list(obj, src=src, group=group)
    uid = obj[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != 128:
        raise RuntimeError("bad RCCL unique id from rank 0")
    (init_fn or _lib_init)(bytes(uid), world, rank, device)
    return rank, world


class ArmGroups(NamedTuple):
    """The C5 schedule over R >= 2 ranks (``init_arm_comms``): the p arm on
    ``p_ranks``, the q arm on ``q_ranks``, each group one communicator."""
    arm: str              # this rank's arm, "p" or "q"
    p_ranks: List[int]    # global ranks of the p group (its root first)
    q_ranks: List[int]
    rank: int             # global rank
    world: int


def arm_group_ranks(world: int) -> Tuple[List[int], List[int]]:
    """p on ranks [0, ceil(R/2)), q on the rest: the two centromere arms are
    independent matrices (R/TADpole.R:357-436) of similar size (C5: ~24.3k and
    ~21.3k bins), so each group takes one and their unshardable CONISS merge
    chains run at the same time instead of one after the other."""
    if world < 2:
        raise ValueError("arm groups need at least two ranks")
    npr = (world + 1) // 2
    return list(range(npr)), list(range(npr, world))


def init_arm_comms(device: int, uid_fn: Optional[Callable[[], bytes]] = None,
                   init_fn: Optional[Callable[[bytes, int, int, int], None]] = None) -> ArmGroups:
    """Split the default process group into the p and q arm groups
    (``arm_group_ranks``) and bind this rank's library communicator over its
    group: ``TADpole(..., centromere_search=True, sharded=True,
    arm_groups=<this>)`` then shards each arm over its own group only.  Every
    rank calls this (``new_group`` is collective)."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    p_ranks, q_ranks = arm_group_ranks(world)
    gp = dist.new_group(p_ranks)
    gq = dist.new_group(q_ranks)
    arm = "p" if rank in p_ranks else "q"
    init_comm(device, group=gp if arm == "p" else gq, uid_fn=uid_fn, init_fn=init_fn)
    return ArmGroups(arm, p_ranks, q_ranks, rank, world)


class ArmGroupError(RuntimeError):
    """An arm failed on another rank's group (raised on every rank that did
    not fail itself, so no rank is left waiting for that arm's result)."""


def exchange_arms(groups: ArmGroups, mine, error: Optional[BaseException] = None) -> dict:
    """Every rank gets both arms' results: each group's root broadcasts its
    arm's ``tadpole`` object over the default (control) group.

    ``error``: this rank's arm raised (``mine`` is then ignored).  Every rank
    first all-gathers its status, so when any arm failed all ranks raise at once
    -- the failing ranks their own exception, the others ``ArmGroupError``
    naming the first failing rank -- instead of the healthy group blocking in
    the result broadcast until the process-group timeout."""
    import torch.distributed as dist

    status: List[Optional[str]] = [None] * groups.world
    msg = None if error is None else f"{type(error).__name__}: {error}"
    dist.all_gather_object(status, msg)
    failed = [(r, m) for r, m in enumerate(status) if m is not None]
    if failed:
        if error is not None:
            raise error
        r, m = failed[0]
        raise ArmGroupError(f"the {'p' if r in groups.p_ranks else 'q'} arm failed on rank {r}: {m}")
    out = {}
    for arm, ranks in (("p", groups.p_ranks), ("q", groups.q_ranks)):
        obj = [mine if (groups.arm == arm and groups.rank == ranks[0]) else None]
        dist.broadcast_object_list(obj, src=ranks[0])
        out[arm] = obj[0]
    return out


def destroy_comm(device: int = 0) -> None:
    _lib.load().tp_comm_destroy(ctypes.byref(ctypes.c_int(device)))


def set_virtual_shards(nvirt: int, device: int = 0) -> None:
    """Test hook: run sharded calls as ``nvirt`` shards on one device."""
    L = _lib.load()
    st = ctypes.c_int(0)
    L.tp_set_virtual_shards(ctypes.byref(ctypes.c_int(device)), ctypes.byref(ctypes.c_int(nvirt)),
                            ctypes.byref(st))
    _lib.check(st)


PLAN_TILE_COLUMNS, PLAN_ROWS, PLAN_TREES = 0, 1, 2


def shard_plan(n: int, nranks: int, kind: int) -> np.ndarray:
    """The library's split (host only): bounds[r]..bounds[r+1] for rank r.
    kind 0: 64-column tiles of X'X / Xc'Xc; 1: rows of G Q / Xc V; 2: trees."""
    L = _lib.load()
    b = np.zeros(nranks + 1, np.int32)
    st = ctypes.c_int(0)
    L.tp_shard_plan(ctypes.byref(ctypes.c_int(n)), ctypes.byref(ctypes.c_int(nranks)),
                    ctypes.byref(ctypes.c_int(kind)), _lib.ip(b), ctypes.byref(st))
    _lib.check(st)
    return b
