"""bench.py's `--gpus N` launcher (CPU): outside torch.distributed it runs N
ranks under torch.distributed.run and returns their exit code; inside, it
refuses a WORLD_SIZE that differs from --gpus (the driver's SCALE runs must
measure the rank count they claim)."""
import json
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STUB = r'''
import json, os, sys
out = sys.argv[sys.argv.index("--out") + 1]
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({"rank": int(os.environ["RANK"]), "world": int(os.environ["WORLD_SIZE"]),
               "local": int(os.environ["LOCAL_RANK"]), "master": os.environ["MASTER_ADDR"]}, f)
'''


def _args(gpus):
    return types.SimpleNamespace(gpus=gpus)


def test_relaunch_runs_n_ranks(tmp_path, monkeypatch):
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    rc = bench.relaunch_if_needed(_args(3), script=str(stub), argv=["--out", str(tmp_path)])
    assert rc == 0
    seen = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    assert [s["rank"] for s in seen] == [0, 1, 2]
    assert all(s["world"] == 3 and s["master"] == "127.0.0.1" for s in seen)


def test_relaunch_propagates_failure(tmp_path, monkeypatch):
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    stub = tmp_path / "bad.py"
    stub.write_text("import sys; sys.exit(3)\n")
    assert bench.relaunch_if_needed(_args(2), script=str(stub), argv=[]) != 0


def test_no_relaunch_single_gpu(monkeypatch):
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.relaunch_if_needed(_args(1)) is None


@pytest.mark.parametrize("world,gpus,expect", [("2", 2, None), ("4", 2, 2), ("1", 1, None)])
def test_world_size_must_match(monkeypatch, world, gpus, expect):
    import bench
    monkeypatch.setenv("WORLD_SIZE", world)
    assert bench.relaunch_if_needed(_args(gpus)) == expect


def test_bench_cli_refuses_mismatch():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=3" in p.stderr


def _dist_worker(rank, world, port, out):
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n0 = 37
    host = np.arange(n0 * n0, dtype=np.float64).reshape(n0, n0) if rank == 0 else None
    got = torch.full((n0, n0), -1.0, dtype=torch.float64)
    bench.distribute_rows(host, n0, world, rank, lambda r0, r1, t: got[r0:r1].copy_(t), chunk_rows=8)
    want = torch.arange(n0 * n0, dtype=torch.float64).reshape(n0, n0)
    out.put((rank, bool(torch.equal(got, want)), bench.c5_mode(world)))
    dist.barrier()
    dist.destroy_process_group()


def test_c5_full_multi_rank_path_gloo(monkeypatch):
    """The c5_full line at world 2 (what `bench.py --gpus 2` selects): the
    sharded mode with a device per rank (skipped when ranks would share a
    GPU), and the C5 matrix reaching every rank intact through the chunked
    gloo broadcast (rank 0 holds the only host copy)."""
    import socket
    import torch
    import torch.multiprocessing as mp
    import bench
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert bench.c5_mode(1) == "one_gpu" and bench.c5_mode(8) == "sharded"
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert bench.c5_mode(2) == "skipped"
    monkeypatch.undo()
    want_mode = "sharded" if torch.cuda.device_count() >= 2 else "skipped"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert res == [(0, True, want_mode), (1, True, want_mode)]
