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
    from tadpole_amd import multi
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seen = []
    g = multi.init_arm_comms(0, uid_fn=lambda: bytes(range(128)),
                             init_fn=lambda uid, n, r, dev: seen.append((len(uid), n, r)))
    # each rank computes only its arm; every rank ends with both
    mine = {"arm": g.arm, "by": rank, "data": np.arange(3) + (0 if g.arm == "p" else 10)}
    got = multi.exchange_arms(g, mine)
    out.put((rank, g.arm, g.p_ranks, g.q_ranks, seen, got["p"]["by"], got["q"]["by"],
             int(got["p"]["data"][0]), int(got["q"]["data"][0])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_c5_arm_groups_gloo(world, monkeypatch):
    """The c5_full line at N > 1 ranks (what `bench.py --gpus N` selects with a
    device per rank): the p arm on ranks [0, ceil(N/2)), the q arm on the rest,
    each group binding one communicator of its own size (rank within the
    group), and every rank receiving both arms' results from the group roots
    (SURVEY §8(e)2, R/TADpole.R:357-442)."""
    import socket
    import torch
    import torch.multiprocessing as mp
    import bench
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert bench.c5_mode(1) == "one_gpu" and bench.c5_mode(8) == "arm_groups"
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert bench.c5_mode(2) == "skipped"
    monkeypatch.undo()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    npr = (world + 1) // 2
    for rank, arm, pr, qr, seen, by_p, by_q, d_p, d_q in res:
        assert pr == list(range(npr)) and qr == list(range(npr, world))
        assert arm == ("p" if rank < npr else "q")
        grp = pr if arm == "p" else qr
        assert seen == [(128, len(grp), grp.index(rank))]
        assert (by_p, by_q, d_p, d_q) == (0, npr, 0, 10)


def _fail_worker(rank, world, port, out, bad_arm):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from tadpole_amd import multi
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = multi.init_arm_comms(0, uid_fn=lambda: bytes(range(128)), init_fn=lambda uid, n, r, dev: None)
    try:
        if g.arm == bad_arm:
            raise ValueError("TP_ERR_NO_BSTICK on this arm")
        mine, err = {"arm": g.arm}, None
    except ValueError as e:
        mine, err = None, e
    try:
        multi.exchange_arms(g, mine, err)
        out.put((rank, "ok", ""))
    except multi.ArmGroupError as e:
        out.put((rank, "group", str(e)))
    except ValueError as e:
        out.put((rank, "own", str(e)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bad_arm", [(2, "q"), (3, "p")])
def test_c5_arm_group_failure_reaches_every_rank(world, bad_arm):
    """an arm that raises on its group (a data error or a
    communicator abort) makes every rank raise at once -- its own ranks their
    exception, the other group's ranks ArmGroupError naming the failing rank --
    instead of the healthy group blocking in the result broadcast until the
    process-group timeout."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_fail_worker, args=(r, world, port, q, bad_arm)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    npr = (world + 1) // 2
    bad = list(range(npr)) if bad_arm == "p" else list(range(npr, world))
    for rank, kind, msg in res:
        if rank in bad:
            assert kind == "own" and "NO_BSTICK" in msg
        else:
            assert kind == "group" and f"rank {bad[0]}" in msg and "NO_BSTICK" in msg


def test_matrix_checksum_dev_matches_host():
    """The on-device checksum every rank takes of its own C5 copy equals the
    fixture's host checksum (synth.matrix_checksum)."""
    import numpy as np
    import torch
    import bench
    from tadpole_amd.synth import matrix_checksum, synth_hic_par
    m = synth_hic_par(1500, 7, centromere=True)
    assert np.array_equal(bench.matrix_checksum_dev(torch.from_numpy(m)), matrix_checksum(m))


@pytest.mark.parametrize("n0,cen", [(700, True), (513, False), (256, True)])
def test_synth_stream_equals_synth_hic_par(n0, cen):
    """synth_hic_par_stream + place_upper_block (numpy and torch sinks) give
    synth_hic_par's matrix bit for bit (the C5 input each rank draws itself)."""
    import numpy as np
    import torch
    from tadpole_amd.synth import place_upper_block, synth_hic_par, synth_hic_par_stream
    ref = synth_hic_par(n0, 99, centromere=cen)
    M = np.full((n0, n0), -1.0)
    z = synth_hic_par_stream(n0, 99, lambda r0, r1, U: place_upper_block(M, r0, r1, U), centromere=cen)
    M[z, :] = 0
    M[:, z] = 0
    assert np.array_equal(M, ref)
    T = torch.full((n0, n0), -1.0, dtype=torch.float64)
    z = synth_hic_par_stream(n0, 99, lambda r0, r1, U: place_upper_block(T, r0, r1, torch.from_numpy(U)),
                             centromere=cen, threads=3)
    zi = torch.as_tensor(z)
    T.index_fill_(0, zi, 0.0)
    T.index_fill_(1, zi, 0.0)
    assert np.array_equal(T.numpy(), ref)
