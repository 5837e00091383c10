"""Headline benchmark (BASELINE.json metric "bins/sec (NxN matrix)").

A step = one TADpole()-equivalent pipeline over one synthetic N0 x N0 Hi-C
matrix already resident in HBM: NA->0 + symmetrise, bad-column mask, Pearson
correlation, PCA to max_pcs, CONISS sweep over every PC prefix, broken stick,
Calinski-Harabasz, parameter choice, TAD coordinates of every significant level
(host assembly of the `tadpole` object included).

Workload: BASELINE.json configs[2], C3 (chr18 @10kb shape: 7808 x 7808,
max_pcs = 200), the largest configuration that is one matrix on one GPU (C4 is
23 matrices, C5 two arms over 8 GPUs).  value = N0 x K / wall time of K
pipelines run one after another on one stream (N0 over one
pipeline's wall time).  The throughput of S matrices in flight on S streams is
reported beside it (`throughput`), never as `value`.

Multi-GPU: one process per GPU.  `--gpus N` without a torch.distributed
environment re-launches this script under torch.distributed.run with N ranks
(as a child process, before anything touches the GPU) and exits with its
code; under torch.distributed.run WORLD_SIZE must equal --gpus.  Each rank
processes its own C3 matrix (independent chromosomes): weak
scaling, no data-path collective, value = bins of all ranks / max-over-ranks
time; `ranks_seen` is counted over the process group.
--sharded: one matrix split over all ranks (RCCL all-gathers, strong scaling).
--e2e-tsv N: only the north_star end-to-end line: TADpole() on an N-bin
tab-separated file (native parse + upload + pipeline + assembly).

North-star lines (same JSON object, after the C3 headline; --no-extras skips):
  "e2e_10k"    TADpole() on a 10 000-bin TSV file, median of 3, stage breakdown
               (rank 0 at N=1);
  "c5_arm"     one 24 300-bin matrix (the C5 p-arm shape) on one GPU, with its
               parity against tests/golden/c5arm.npz (rank 0 at N=1);
  "c4_genome"  the 23 hg19 chromosomes @25 kb through run_genome over all
               ranks (LPT, 8 streams a GPU), parity of four chromosomes
               against their golden fixtures;
  "c5_full"    BASELINE config 5: TADpole(centromere_search=TRUE) on the
               49 851-bin chr1 @5kb matrix, one GPU at N=1 (plus a one-rank
               RCCL sharded run checked bit for bit), every arm sharded over
               all ranks at N > 1 (--no-c5 skips), parity against
               tests/golden/c5full.npz.

Extra fields: "roofline" for the kernel class with the largest time per
pipeline (HIP events recorded inside the library on the stream the kernels run
on, averaged over the timed steps; the Krylov products' class, 32 launches a
pipeline, from a few untimed pipelines after them, since an event per launch
costs ~0.4 ms a pipeline), "cpu_baseline" (the CPU oracle on this
host, rank 0, N=1), "parity" (rank 0's result vs the committed oracle fixture
and vs the CPU oracle run on the same matrix).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

FP64_MFMA_PEAK_TFLOPS = 78.6     # MI355X FP64 matrix, dense (AMD spec)
FP32_MFMA_PEAK_TFLOPS = 157.3    # MI355X FP32 matrix, dense (MI355X_MICROARCH.md: 155 TF measured)
INT8_MFMA_PEAK_TOPS = 5000.0     # MI355X I8 MFMA, dense: 2x the BF16 rate per clock (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E (MI355X_MICROARCH.md)
METRIC = "bins/sec (NxN matrix) at 1/2/4/8 GPUs; TAD boundary bit-match vs R ref"


def _pmc_traffic(kernel_class, n0, k):
    """HBM bytes per launch of a kernel class (the kernels one launch runs,
    summed) from the newest committed PMC summary (profiles/*_traffic.json,
    written by tools/prof_summary.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this bench) for the same workload; null when absent."""
    import glob
    for path in sorted(glob.glob(os.path.join(HERE, "profiles", "*_traffic.json")), reverse=True):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("n0") != n0 or t.get("k") != k:
            continue
        rec = t.get("classes", {}).get(kernel_class)
        if isinstance(rec, dict) and rec.get("hbm_bytes") is not None:
            return round(rec["hbm_bytes"]), os.path.relpath(path, HERE)
    return None, None


def _config_name(n0, max_pcs):
    """BASELINE.json config this run corresponds to."""
    if max_pcs == 200 and n0 == 7808:
        return "C3"
    if max_pcs == 200 and n0 == 2000:
        return "C2"
    if max_pcs == 200 and n0 in (24300, 21300):
        return "C5 arm shape"
    if n0 == 200:
        return "C1 shape"
    return "custom"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n0", type=int, default=7808)
    ap.add_argument("--max-pcs", type=int, default=200)
    ap.add_argument("--min-clusters", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--throughput-streams", type=int, default=8,
                    help="after the timed region: S matrices in flight on S streams (0/1 = skip)")
    ap.add_argument("--throughput-steps", type=int, default=16)
    ap.add_argument("--sharded", action="store_true",
                    help="one matrix split over all ranks (SURVEY §8(e)2, C5 arms): strong scaling")
    ap.add_argument("--e2e-tsv", type=int, default=0,
                    help="end-to-end TADpole() on an N-bin TSV file (parse included) instead of the HBM bench")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the north-star lines (e2e_10k, c5_arm, c4_genome)")
    ap.add_argument("--extras-reps", type=int, default=3)
    ap.add_argument("--no-c5", action="store_true", help="skip the c5_full line (49 851-bin config 5)")
    return ap.parse_args()


def relaunch_if_needed(args, script=None, argv=None):
    """`--gpus N` outside torch.distributed: run N ranks under
    torch.distributed.run as a child process (nothing here has touched the
    GPU) and return its exit code; None when this process is a rank already.
    ``script``/``argv`` (tests): what the ranks run instead of this file."""
    import socket
    import subprocess
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
            return 2
        return None
    if args.gpus <= 1:
        return None
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__)]
    cmd += list(sys.argv[1:] if argv is None else argv)
    return subprocess.call(cmd)


STAGES = ["mask", "cor", "pca", "sweep", "total"]


def torch_device() -> int:
    import torch
    return torch.cuda.current_device()


def _stages(timings):
    return {q: round(float(timings[i]), 3) for i, q in enumerate(STAGES)}


def run_e2e_tsv(n0, max_pcs, reps):
    """north_star: end-to-end TADpole() on an n0-bin matrix file (native parse
    + upload + device pipeline + host assembly), median of `reps`, and the
    same call split into its parts (R/TADpole.R:344-349,444-497)."""
    import tadpole_amd as tp
    from tadpole_amd.api import _assemble, _pipeline, _read_to_device
    from tadpole_amd.synth import SEED_BASE, synth_hic_par, write_tsv
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"tadpole_e2e_{n0}_{os.getpid()}.tsv")
    t0 = time.perf_counter()
    size = write_tsv(synth_hic_par(n0, SEED_BASE + 3), path)
    t_write = time.perf_counter() - t0
    try:
        tp.TADpole(path, max_pcs=max_pcs)            # warm-up (device context, code objects)
        t_all, parts = [], []
        res = None
        for _ in range(max(1, reps)):
            t0 = time.perf_counter()
            res = tp.TADpole(path, max_pcs=max_pcs)
            t_all.append(time.perf_counter() - t0)
        for _ in range(max(1, reps)):               # the same call, piece by piece
            t0 = time.perf_counter()
            raw = _read_to_device(path, 0)          # parse, each row block's upload under the next one's parse
            t1 = time.perf_counter()
            r = _pipeline(raw, max_pcs, 2, 0.01, 0, 0)
            t2 = time.perf_counter()
            _assemble(r, np.flatnonzero(r["bad"]) + 1)
            t3 = time.perf_counter()
            parts.append((t1 - t0, t2 - t1, t3 - t2, float(r["timings"][4]) * 1e-3))
            del raw
    finally:
        os.remove(path)
    med = float(np.median(t_all))
    pm = np.median(np.array(parts), axis=0)
    return {"metric": "end-to-end TADpole() seconds on an N-bin TSV file (north_star: < 1 s at 10k bins)",
            "value": round(med, 4), "unit": "s", "higher_is_better": False, "n0": n0, "reps": len(t_all),
            "all_s": [round(x, 4) for x in t_all], "bins_per_s": round(n0 / med, 1),
            "breakdown_s": {"parse_and_overlapped_upload": round(pm[0], 4), "pipeline_call": round(pm[1], 4),
                            "device_pipeline": round(pm[3], 4), "host_sync_and_readback": round(pm[1] - pm[3], 4),
                            "host_assembly": round(pm[2], 4)},
            "tsv_bytes": size, "tsv_write_s": round(t_write, 2), "n_pcs": res.n_pcs,
            "optimal_n_clusters": res.optimal_n_clusters, "device_stages_ms": _stages(res.timings_ms),
            "data": "synthetic (tadpole_amd/synth.py synth_hic_par, seed 20261015+3) written as an integer TSV"}


def _golden_check(got, z, prefix=""):
    """Parity of a tadpole object against a committed oracle fixture: TAD
    coordinates of every level, n_pcs, optimal_n_clusters, bad columns, merge
    order (bit-exact) and CH scores (max relative error)."""
    lev = z[prefix + "levels"]
    co = z[prefix + "coords"]
    ok = (got.n_pcs == int(z[prefix + "n_pcs"]) and got.optimal_n_clusters == int(z[prefix + "optimal_n_clusters"])
          and set(got.clusters) == {str(int(q)) for q in lev}
          and all(np.array_equal(got.clusters[str(int(q))], co[co[:, 0] == q][:, 1:]) for q in lev)
          and np.array_equal(got.dendro.boundary - 1, z[prefix + "merge_b"]))
    if (prefix + "bad_idx1") in z and got.bad_columns is not None:
        ok = ok and np.array_equal(got.bad_columns, z[prefix + "bad_idx1"])
    a, b = got.scores, z[prefix + "scores"]
    fin = ~np.isnan(b)
    rel = float(np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin]))) if a.shape == b.shape else None
    return bool(ok and rel is not None and rel < 1e-6), rel


def run_c5_arm(device, max_pcs, reps):
    """One C5-arm-shape matrix (24 300 bins, the p arm of chr1 @5kb) resident
    in HBM, pipelines one after another on one stream; parity against the
    oracle fixture tests/golden/c5arm.npz."""
    import torch
    from tadpole_amd.api import TADpole
    from tadpole_amd.synth import SEED_BASE, synth_hic_par
    n0 = 24300
    gold = os.path.join(HERE, "tests", "golden", "c5arm.npz")
    host = synth_hic_par(n0, SEED_BASE + 5)
    dm = torch.from_numpy(host).to(f"cuda:{device}")
    del host
    TADpole(dm, max_pcs=max_pcs, inplace=False)          # warm-up (scratch of this size)
    ts, res = [], None
    for _ in range(max(1, reps)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = TADpole(dm, max_pcs=max_pcs, inplace=True)   # clean in place: no device copy in the timing
        ts.append(time.perf_counter() - t0)
    del dm
    torch.cuda.empty_cache()
    med = float(np.median(ts))
    out = {"n0": n0, "n_good": int(res.timings_ms[14]), "k": int(res.timings_ms[15]), "reps": len(ts),
           "s_median": round(med, 4), "bins_per_s": round(n0 / med, 1), "stages_ms": _stages(res.timings_ms),
           "coniss_ms": round(float(res.timings_ms[9]), 3), "xtx_ms": round(float(res.timings_ms[5]), 3),
           "krylov_steps": int(res.timings_ms[16]), "pca_resid": float(res.timings_ms[13]),
           "n_pcs": res.n_pcs, "optimal_n_clusters": res.optimal_n_clusters,
           "workload": "C5 arm shape: synthetic 24300x24300 Hi-C (synth_hic_par, seed 20261015+5), max_pcs=%d, "
                       "one GPU, resident in HBM" % max_pcs}
    if os.path.exists(gold) and max_pcs == 200:
        ok, rel = _golden_check(res, np.load(gold))
        out["parity"] = {"golden_fixture": "tests/golden/c5arm.npz", "match": ok, "ch_max_rel_err": rel}
    return out


def pipeline_roofline(n, k, ms):
    """SURVEY.md §8(d)'s whole-pipeline roofline time of one n-bin, k-PC
    pipeline, T_roof = (N^3 + 2 N^2 k) / P_mfma + (3 * 8 N^2 + 4 N k^2 + 3000 * 8 N k)
    / BW_hbm, against the fp32 and the fp64 MFMA peaks (north_star asks for
    the fp32 one) and 8 TB/s of HBM, and the measured ms_per_step's fraction of
    it (T_roof / T_measured: 1.0 = at the roofline)."""
    flops = float(n) ** 3 + 2.0 * float(n) ** 2 * k
    bytes_ = 3 * 8.0 * float(n) ** 2 + 4.0 * n * k * k + 3000 * 8.0 * n * k
    t_hbm = bytes_ / (HBM_PEAK_GBS * 1e9) * 1e3
    out = {"formula": "T_roof = (N^3 + 2N^2k)/P_mfma + (3*8N^2 + 4Nk^2 + 3000*8Nk)/BW_hbm (SURVEY.md §8(d))",
           "n": n, "k": k, "flops": flops, "hbm_bytes": bytes_, "hbm_ms": round(t_hbm, 4)}
    for name, peak in (("fp32_mfma", FP32_MFMA_PEAK_TFLOPS), ("fp64_mfma", FP64_MFMA_PEAK_TFLOPS)):
        t = flops / (peak * 1e12) * 1e3 + t_hbm
        out[name] = {"peak_tflops": peak, "t_roof_ms": round(t, 4),
                     "frac_of_roofline": round(t / ms, 4) if ms > 0 else None}
    return out


def run_c2(device, max_pcs, steps, warmup):
    """BASELINE.json configs[1], C2: one synthetic 2000 x 2000 Hi-C matrix
    (synth_hic, seed 20261015+2, the input of tests/golden/c2.npz) resident in
    HBM, pipelines one after another on one stream, TADpole()'s whole call with
    the host assembly; stage times from the library's events; parity against
    the golden fixture; the whole-pipeline roofline fraction."""
    import torch
    from tadpole_amd.api import TADpole
    from tadpole_amd.synth import SEED_BASE, synth_hic
    n0 = 2000
    dm = torch.from_numpy(synth_hic(n0, SEED_BASE + 2)).to(f"cuda:{device}")
    for _ in range(max(1, warmup)):
        TADpole(dm, max_pcs=max_pcs, inplace=True)   # symmetric, NaN-free: cleaning in place is idempotent
    ts, tms, res = [], [], None
    torch.cuda.synchronize()
    for _ in range(max(1, steps)):
        t0 = time.perf_counter()
        res = TADpole(dm, max_pcs=max_pcs, inplace=True)
        ts.append(time.perf_counter() - t0)
        tms.append(res.timings_ms)
    torch.cuda.synchronize()
    del dm
    tm = np.mean(np.stack(tms), axis=0)
    ms = float(np.sum(ts)) / len(ts) * 1e3
    n, k = int(tm[14]), int(tm[15])
    out = {"n0": n0, "n_good": n, "k": k, "steps": len(ts), "ms_per_step": round(ms, 3),
           "ms_median": round(float(np.median(ts)) * 1e3, 3), "bins_per_s": round(n0 / (ms * 1e-3), 1),
           "stages_ms": _stages(tm), "coniss_ms": round(float(tm[9]), 3), "ch_ms": round(float(tm[10]), 3),
           "pca": {"path": "block Krylov" if int(tm[16]) else "G = Xc'Xc + subspace iteration",
                   "chebyshev_degrees": int(tm[11]), "block": int(tm[12]), "resid": float(tm[13])},
           "pipeline_roofline": pipeline_roofline(n, k, ms),
           "workload": "C2 (BASELINE configs[1]): synthetic 2000x2000 Hi-C (synth_hic, seed 20261015+2), "
                       "max_pcs=%d, one GPU, resident in HBM, TADpole() incl. host assembly" % max_pcs}
    gold = os.path.join(HERE, "tests", "golden", "c2.npz")
    if os.path.exists(gold) and max_pcs == 200:
        z = np.load(gold)
        ok, rel = _golden_check(res, z)
        ok = ok and np.array_equal(res.dendro.merge, z["merge"])
        out["parity"] = {"golden_fixture": "tests/golden/c2.npz", "match": bool(ok), "ch_max_rel_err": rel}
    return out


C4_GOLDEN = ("chr21", "chr22", "chr19", "chr1")


def _phase_summary(ph):
    tot = {}
    for d in ph.values():
        for k, v in d.items():
            tot[k] = tot.get(k, 0.0) + v
    out = {k: round(v, 4) for k, v in sorted(tot.items())}
    if ph:
        c = max(ph, key=lambda q: sum(v for k, v in ph[q].items() if k != "wait"))
        out["slowest"] = {"chrom": c, **{k: round(v, 4) for k, v in sorted(ph[c].items())}}
    return out


def run_c4_genome(world, rank, max_pcs, reps, streams=8):
    """C4: the 23 hg19 chromosomes @25 kb (synthetic counts of the real bin
    numbers) through run_genome over every rank of the default process group:
    LPT over ranks, `streams` pipelines in flight per GPU, host-resident
    matrices (the H2D copies and the host assembly are inside the time).  Each
    rank builds only its own chromosomes.  Median of `reps` whole runs."""
    import torch.distributed as dist
    from tadpole_amd.genome import lpt_assign, matrix_cost, run_genome
    from tadpole_amd.synth import genome_bins, genome_matrix
    sizes = genome_bins()
    plan = lpt_assign({c: matrix_cost(sizes[c]) for c in sizes}, world)
    t0 = time.perf_counter()
    mats = {c: (genome_matrix(c) if c in plan[rank] else (lambda c=c: genome_matrix(c))) for c in sizes}
    t_gen = time.perf_counter() - t0
    from tadpole_amd import _lib
    run_genome(mats, sizes=sizes, streams=streams, max_pcs=max_pcs)     # warm-up (contexts, code objects)
    walls, res, rep_secs = [], None, []
    ctx0 = _lib.context_stats(torch_device())[1]
    rep_phases = []
    grows0 = _lib.debug_knob(41, 0)
    for _ in range(max(1, reps)):
        if world > 1:
            dist.barrier()
        ph = {}
        t0 = time.perf_counter()
        res, secs = run_genome(mats, sizes=sizes, streams=streams, max_pcs=max_pcs, phases=ph)
        if world > 1:
            dist.barrier()
        walls.append(time.perf_counter() - t0)
        rep_secs.append(secs)
        rep_phases.append(ph)
    ctx_new = _lib.context_stats(torch_device())[1] - ctx0
    grows = _lib.debug_knob(41, 0)   # scratch regrowths (each a device-wide sync) during the timed reps
    if rank != 0:
        return None
    bins = sum(sizes.values())
    wall = float(np.median(walls))
    out = {"chromosomes": len(sizes), "bins": bins, "ranks": world, "streams_per_rank": streams,
           "wall_s_median": round(wall, 4), "all_s": [round(x, 4) for x in walls],
           "bins_per_s": round(bins / wall, 1), "matrix_build_s_rank0": round(t_gen, 2),
           # seconds of each chromosome's TADpole() call (every rank's, gathered) per timed rep,
           # and the library contexts rank 0 created during the timed reps (0: the stream pool reuses them)
           "chrom_s_per_rep": [{c: round(v, 4) for c, v in sorted(sc.items())} for sc in rep_secs],
           "contexts_created_in_timed_reps_rank0": ctx_new,
           "scratch_regrowths_in_timed_reps_rank0": grows,
           "scratch_regrowths_before_rank0": grows0,
           # rank 0's chromosomes, per timed rep: summed seconds of each phase (queue wait for a
           # stream worker, upload through the pinned staging, library call, Python assembly)
           # and the slowest chromosome's split
           "phases_rank0": [_phase_summary(ph) for ph in rep_phases],
           "workload": "C4: 23 hg19 chromosomes @25 kb (synthetic, synth_hic_par), max_pcs=%d, one run_genome "
                       "call; host-resident matrices (H2D copies and host assembly included)" % max_pcs}
    par = {}
    for c in C4_GOLDEN:
        gold = os.path.join(HERE, "tests", "golden", f"genome_{c}.npz")
        if os.path.exists(gold) and max_pcs == 200 and c in res:
            ok, rel = _golden_check(res[c], np.load(gold))
            par[c] = {"match": ok, "ch_max_rel_err": rel}
    if par:
        out["parity"] = par
    return out


C5_BINS = 49851
C5_CHUNK_ROWS = 4096


def matrix_checksum_dev(dm):
    """``synth.matrix_checksum`` of a device-resident count matrix: exact int64
    row sums on the GPU (< 2^43 a row at counts < 2^13, n < 2^16), the two
    integers accumulated on the host in Python ints."""
    import torch
    n = dm.shape[0]
    P = (1 << 61) - 1
    w = torch.arange(1, n + 1, dtype=torch.int64, device=dm.device)
    total, acc = 0, 0
    for r0 in range(0, n, 1024):
        blk = dm[r0:r0 + 1024].to(torch.int64)
        total += int(blk.sum().item())
        rows = (blk * w[None, :]).sum(dim=1).cpu().numpy()
        acc += sum(int(v) * (r0 + q + 1) for q, v in enumerate(rows))
    return np.array([total, acc % P], np.int64)


def _c5_resident(world, rank, local):
    """BASELINE config 5's matrix (chr1 @5kb: synth_hic_par(49 851, seed
    20261015+5, centromere=True), the input of tests/golden/c5full.npz) resident
    in HBM on every rank.  Every rank draws it itself, block by block straight
    into its device copy (``synth_hic_par_stream``: the same bits, no n0 x n0
    host array, no broadcast between ranks), and checks its checksum against
    the fixture on the device.  Setup, outside every timing."""
    import torch
    from tadpole_amd.synth import SEED_BASE, place_upper_block, synth_hic_par_stream
    n0 = C5_BINS
    info = {}
    dm = torch.empty((n0, n0), dtype=torch.float64, device=f"cuda:{local}")
    t0 = time.perf_counter()
    zero = synth_hic_par_stream(n0, SEED_BASE + 5, lambda r0, r1, U: place_upper_block(
        dm, r0, r1, torch.from_numpy(U).to(dm.device, non_blocking=False)), centromere=True)
    zi = torch.as_tensor(zero, device=dm.device)
    dm.index_fill_(0, zi, 0.0)
    dm.index_fill_(1, zi, 0.0)
    torch.cuda.synchronize()
    info["matrix_build_s"] = round(time.perf_counter() - t0, 2)
    gold = os.path.join(HERE, "tests", "golden", "c5full.npz")
    if os.path.exists(gold):
        ok = bool(np.array_equal(matrix_checksum_dev(dm), np.load(gold)["matrix_checksum"]))
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([0 if ok else 1], dtype=torch.int64)
            dist.all_reduce(t)
            ok = int(t.item()) == 0
        info["matrix_checksum_match"] = ok
    return dm, info


def c5_mode(world):
    """How the c5_full line runs at this rank count: one GPU unsharded (plus a
    one-rank RCCL check); N ranks in two groups, the p arm sharded over ranks
    [0, ceil(N/2)) and the q arm over the rest at the same time
    (``multi.init_arm_comms``); or skipped when ranks share a GPU (a rehearsal
    with more ranks than devices: RCCL needs one device per rank)."""
    if world == 1:
        return "one_gpu"
    import torch
    return "arm_groups" if torch.cuda.device_count() >= world else "skipped"


def run_c5_full(world, rank, local, max_pcs, reps):
    """BASELINE config 5 end to end: TADpole(centromere_search=TRUE) on the
    49 851-bin chr1 @5kb matrix resident in HBM (R/TADpole.R:58-85,351-442:
    mask, centromere split, the p (~24.3k bins) and q (~21.3k, bug-compatible)
    arms, merging_arms).  One GPU: the plain pipeline per arm.  N ranks: every
    arm's products split over all ranks through the library's RCCL
    communicator (column slabs of C, row-split Krylov products, tree-split
    sweep), the time the max over ranks.  Parity: bit-exact
    TAD coordinates / merge order / n_pcs / optimal_n_clusters of both arms
    and merging_arms, CH <= 1e-6, against tests/golden/c5full.npz (the CPU
    oracle on the same matrix); one GPU also checks a one-rank sharded run
    against the unsharded one bit for bit."""
    import torch
    import torch.distributed as dist
    from tadpole_amd import multi
    from tadpole_amd.api import TADpole
    dm, info = _c5_resident(world, rank, local)
    sharded = c5_mode(world) == "arm_groups"
    comm_size = groups = None
    if sharded:
        groups = multi.init_arm_comms(device=local)
        comm_size = {"p": len(groups.p_ranks), "q": len(groups.q_ranks)}

    def once():
        return TADpole(dm, max_pcs=max_pcs, centromere_search=True, sharded=sharded, inplace=True,
                       arm_groups=groups)

    try:
        once()                                     # warm-up (scratch of these sizes)
        ts, res = [], None
        for _ in range(max(1, reps)):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = once()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([el], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = float(t.item())
            ts.append(el)
        one_rank = None
        if world == 1:
            # the sharded schedule through a real one-rank RCCL communicator
            # must give the unsharded bits
            uid = multi.comm_unique_id()
            multi._lib_init(uid, 1, 0, local)
            try:
                sh = TADpole(dm, max_pcs=max_pcs, centromere_search=True, sharded=True, inplace=True)
            finally:
                multi.destroy_comm(local)
            one_rank = bool(np.array_equal(sh.merging_arms, res.merging_arms) and all(
                np.array_equal(getattr(sh, a).scores.view(np.uint64), getattr(res, a).scores.view(np.uint64))
                and np.array_equal(getattr(sh, a).dendro.boundary, getattr(res, a).dendro.boundary)
                and np.array_equal(getattr(sh, a).dendro.height.view(np.uint64),
                                   getattr(res, a).dendro.height.view(np.uint64))
                for a in ("p", "q")))
    finally:
        if sharded:
            multi.destroy_comm(local)
        del dm
        torch.cuda.empty_cache()
    if rank != 0:
        return None
    med = float(np.median(ts))
    out = {"n0": C5_BINS, "ranks": world, "reps": len(ts), "s_median": round(med, 4),
           "all_s": [round(x, 4) for x in ts], "bins_per_s": round(C5_BINS / med, 1),
           "workload": ("C5: chr1 @5kb shape, synthetic 49851x49851 Hi-C (synth_hic_par, seed 20261015+5, "
                        "centromere run at [0.4875, 0.572) N0), TADpole(centromere_search=TRUE) bug-compatible, "
                        "max_pcs=%d, resident in HBM, " % max_pcs +
                        (f"p arm sharded over GPUs {groups.p_ranks}, q arm over {groups.q_ranks} at the same "
                         f"time (RCCL, one communicator a group)" if sharded else "one GPU")),
           "arms": {}}
    out.update(info)
    if comm_size is not None:
        out["rccl_comm_size"] = comm_size   # ranks of each arm's group
    if one_rank is not None:
        out["sharded_1rank_bit_identical"] = one_rank
    for a in ("p", "q"):
        r = getattr(res, a)
        out["arms"][a] = {"n": int(r.timings_ms[14]), "k": int(r.timings_ms[15]), "stages_ms": _stages(r.timings_ms),
                          "xtx_ms": round(float(r.timings_ms[5]), 3), "coniss_ms": round(float(r.timings_ms[9]), 3),
                          "krylov_steps": int(r.timings_ms[16]), "pca_resid": float(r.timings_ms[13]),
                          "n_pcs": r.n_pcs, "optimal_n_clusters": r.optimal_n_clusters}
    gold = os.path.join(HERE, "tests", "golden", "c5full.npz")
    if os.path.exists(gold) and max_pcs == 200:
        z = np.load(gold)
        par = {"golden_fixture": "tests/golden/c5full.npz",
               "merging_arms_match": bool(np.array_equal(res.merging_arms, z["bug_merging_arms"]))}
        for a in ("p", "q"):
            ok, rel = _golden_check(getattr(res, a), z, f"bug_{a}_")
            par[a] = {"match": ok and np.array_equal(getattr(res, a).dendro.label_ids, z[f"bug_{a}_names"]),
                      "ch_max_rel_err": rel}
        par["match"] = bool(par["merging_arms_match"] and par["p"]["match"] and par["q"]["match"])
        out["parity"] = par
    return out


def e2e_tsv(args):
    out = run_e2e_tsv(args.e2e_tsv, args.max_pcs, max(1, args.steps))
    line = json.dumps(out)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")


def main():
    args = parse()
    rc = relaunch_if_needed(args)
    if rc is not None:
        sys.exit(rc)
    if args.throughput_streams > 1 and not args.sharded:
        # concurrent pipelines need one hardware queue per stream (HIP's default
        # is 4 and streams sharing a queue serialise); only before HIP starts
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
            os.environ["GPU_MAX_HW_QUEUES"] = "16"
    # a first-time collective hang in a sharded line fails that line within a
    # minute (the library's watchdog aborts its communicator), not the run
    os.environ.setdefault("TP_SHARD_TIMEOUT_S", "60")
    if args.e2e_tsv:
        return e2e_tsv(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # control only (barriers, the max of the elapsed times, the sharded
        # path's RCCL id, the C5 matrix's distribution): no data-path
        # collective, so gloo over TCP; a bounded timeout, so a rank that died
        # ends the run instead of parking the others for gloo's default 30 min
        import datetime
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
    # one GPU per rank; more ranks than GPUs (a rehearsal on a smaller box)
    # share devices round-robin
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev
    torch.cuda.set_device(local)
    seen = [(rank, local)]
    if world > 1:
        seen = [None] * world
        dist.all_gather_object(seen, (rank, local))
    if len({r for r, _ in seen}) != args.gpus:
        raise SystemExit(f"bench.py: {len(seen)} ranks seen, --gpus {args.gpus}")
    comm_size = None

    from tadpole_amd import _lib
    from tadpole_amd.api import _assemble
    from tadpole_amd.synth import SEED_BASE, synth_hic

    L = _lib.load()
    n0 = args.n0
    cfg = {7808: 3, 2000: 2}.get(n0, 3)
    seed = SEED_BASE + cfg + (0 if args.sharded else 1000 * rank)   # sharded: every rank holds the same matrix
    host = synth_hic(n0, seed)
    flags = _lib.TP_FLAG_ROW_MAJOR
    if args.sharded:
        from tadpole_amd import multi
        if world > 1:
            comm_size = multi.init_comm(device=local)[1]
        flags |= _lib.TP_FLAG_SHARDED
    k_cap = max(1, min(args.max_pcs, n0))
    w_cap = n0
    I = ctypes.c_int

    class Lane:
        """One pipeline in flight: its own stream (hence its own library context
        and scratch), its own resident copy of the matrix, its own host outputs."""

        def __init__(self, idx):
            self.stream = torch.cuda.current_stream() if idx == 0 else torch.cuda.Stream(device=f"cuda:{local}")
            self.dev_m = torch.from_numpy(host).to(f"cuda:{local}")
            self.bufs = dict(bad=np.zeros(n0, np.int32), good=np.zeros(n0, np.int32),
                             nclu=np.zeros(k_cap, np.int32), scores=np.zeros(k_cap * w_cap),
                             merge=np.zeros(2 * (n0 - 1), np.int32), height=np.zeros(n0 - 1),
                             boundary=np.zeros(n0 - 1, np.int32), timings=np.zeros(32))

    lane0 = Lane(0)
    torch.cuda.synchronize()

    host_t = {"call": 0.0, "assemble": 0.0, "n": 0}   # wall of the C call / of the host assembly

    def step(lane, want_timings=True):
        b, dev_m, stream = lane.bufs, lane.dev_m, lane.stream
        outs = [I(0) for _ in range(6)]
        tc0 = time.perf_counter()
        n_good, k, w, n_pcs, n_clusters, st = outs
        L.tp_pipeline_dev(ctypes.c_void_p(dev_m.data_ptr()), ctypes.byref(I(n0)), ctypes.byref(I(args.max_pcs)),
                          ctypes.byref(I(args.min_clusters)), ctypes.byref(ctypes.c_double(0.01)),
                          ctypes.byref(I(flags)), ctypes.byref(I(local)),
                          ctypes.c_void_p(stream.cuda_stream), ctypes.byref(I(k_cap)), ctypes.byref(I(w_cap)),
                          _lib.ip(b["bad"]), ctypes.byref(n_good), _lib.ip(b["good"]), ctypes.byref(k),
                          _lib.ip(b["nclu"]), _lib.dp(b["scores"]), ctypes.byref(w), ctypes.byref(n_pcs),
                          ctypes.byref(n_clusters), _lib.ip(b["merge"]), _lib.dp(b["height"]),
                          _lib.ip(b["boundary"]), _lib.dp(b["timings"]) if want_timings else None,
                          ctypes.byref(st))
        _lib.check(st)
        tc1 = time.perf_counter()
        n = n_good.value
        kk, ww = k.value, w.value
        res = dict(bad=b["bad"].astype(bool), good=b["good"][:n].copy(), k=kk, w=ww,
                   scores=b["scores"][:kk * ww].reshape(ww, kk).T.copy(), n_pcs=n_pcs.value,
                   n_clusters=n_clusters.value,
                   merge=b["merge"][:2 * (n - 1)].reshape(2, n - 1).T.copy(), height=b["height"][:n - 1].copy(),
                   boundary=b["boundary"][:n - 1].copy(), timings=b["timings"].copy())
        out = _assemble(res, np.flatnonzero(res["bad"]) + 1)
        host_t["call"] += tc1 - tc0
        host_t["assemble"] += time.perf_counter() - tc1
        host_t["n"] += 1
        return out

    for _ in range(args.warmup):
        step(lane0)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def fine_events(on):
        """knob 25: HIP events around every Krylov product (off in the timed
        region: each hipEventRecord opens a few-us gap on the stream, ~0.4 ms
        over a pipeline's 32 products)."""
        old, st = I(0), I(0)
        L.tp_debug_knob(ctypes.byref(I(25)), ctypes.byref(I(1 if on else 0)), ctypes.byref(old), ctypes.byref(st))
        _lib.check(st)

    # ---- timed region: K pipelines, one after another, on one stream; the
    # library records HIP events per stage and around its one-launch kernel
    # classes (int8 X'X, CONISS, CH) on that stream
    fine_events(False)
    tms = []
    barrier()
    host_t.update(call=0.0, assemble=0.0, n=0)
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = step(lane0)
        tms.append(last.timings_ms)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    host_call = dict(host_t)
    tm = np.mean(np.stack(tms), axis=0)
    # the Krylov products' class (32 launches a pipeline) from separate
    # untimed pipelines with their events on
    fine_events(True)
    tmf = np.mean(np.stack([step(lane0).timings_ms for _ in range(max(2, min(5, args.steps)))]), axis=0)
    torch.cuda.synchronize()
    tm[7], tm[8] = tmf[7], tmf[8]
    n, k = int(tm[14]), int(tm[15])
    # the int8 MACs the last whole-triangle X'X executed (its high slice runs only
    # on the k-blocks the block-nonzero map lists): read back after the timing
    xexec = np.zeros(5)
    st_x = I(0)
    L.tp_debug_xtx_exec(ctypes.byref(I(local)), ctypes.c_void_p(lane0.stream.cuda_stream), _lib.dp(xexec),
                        ctypes.byref(st_x))
    _lib.check(st_x)
    nh = max(1, host_call["n"])
    host_ms = {"c_call": round(host_call["call"] / nh * 1e3, 3), "device_stages": round(float(tm[4]), 3),
               "c_call_minus_device": round(host_call["call"] / nh * 1e3 - float(tm[4]), 3),
               "python_assembly": round(host_call["assemble"] / nh * 1e3, 3)}

    # ---- throughput with S matrices in flight (not `value`)
    thr = None
    S = 1 if args.sharded else args.throughput_streams
    if S > 1:
        import threading
        lanes = [lane0] + [Lane(i) for i in range(1, S)]
        for ln in lanes[1:]:
            step(ln, False)
        done = [0] * S
        errs = []
        outs = [None] * S

        def run(i):
            try:
                for _ in range(i, args.throughput_steps, S):
                    outs[i] = step(lanes[i], False)
                    done[i] += 1
            except Exception as e:   # noqa: BLE001 -- collected; the run fails below
                errs.append(repr(e))

        barrier()
        t1 = time.perf_counter()
        th = [threading.Thread(target=run, args=(i,)) for i in range(S)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        barrier()
        el2 = time.perf_counter() - t1
        if errs:
            raise RuntimeError(f"throughput lanes failed: {errs[:3]}")
        same = all(o is not None and o.n_pcs == last.n_pcs and o.optimal_n_clusters == last.optimal_n_clusters
                   and np.array_equal(o.scores.view(np.uint64), last.scores.view(np.uint64))
                   and all(np.array_equal(o.clusters[q], last.clusters[q]) for q in last.clusters)
                   for o in outs)
        thr = {"streams": S, "matrices": int(sum(done)), "bins_per_s": round(n0 * sum(done) / el2, 1),
               "ms_per_matrix": round(el2 / sum(done) * 1e3, 3), "lanes_identical": bool(same),
               "note": "S matrices in flight on S streams (own library context each); not `value`"}
        del lanes

    # ---- north-star lines (C3 timing above is untouched by them)
    extras = {}
    if not args.no_extras and not args.sharded:
        if world == 1:
            extras["c2"] = run_c2(local, args.max_pcs, max(5, args.steps), 2)
            extras["e2e_10k"] = run_e2e_tsv(10000, args.max_pcs, args.extras_reps)
            extras["c5_arm"] = run_c5_arm(local, args.max_pcs, args.extras_reps)
        c4 = run_c4_genome(world, rank, args.max_pcs, args.extras_reps)
        if rank == 0:
            extras["c4_genome"] = c4
        if not args.no_c5 and c5_mode(world) == "skipped":
            if rank == 0:
                extras["c5_full"] = {"skipped": "ranks share a GPU (RCCL needs one device per rank)"}
        elif not args.no_c5:
            try:
                c5 = run_c5_full(world, rank, local, args.max_pcs, args.extras_reps)
            except Exception as e:   # noqa: BLE001 -- reported in the line; the C3 headline stands
                c5 = {"error": f"{type(e).__name__}: {e}"}
            if rank == 0:
                extras["c5_full"] = c5

    if rank == 0:
        value = n0 * (1 if args.sharded else world) * args.steps / elapsed
        share = 1.0 / world if args.sharded else 1.0   # sharded: this rank's part of each product
        krylov_steps, krylov_d, block = int(tm[16]), int(tm[17]), int(tm[12])
        gq_launches = max(1, int(round(tm[8])))
        if krylov_steps:   # one record = one product with C (C K_t or C (Xc K_t)): 2 N^2 p flops
            p = krylov_d // max(1, krylov_steps)
            gq_flops = share * 2.0 * n * n * p
        else:              # one record = G Q: 2 N^2 b flops
            gq_flops = share * 2.0 * n * n * block
        ns = int(tm[18])   # int8 slices of the exact X'X (0: fp64 product)
        pairs = int(tm[19])   # int8 digit pairs of each product with C (0: fp64 products)
        kern = {   # class: (ms per pipeline, bound, launches per pipeline, algorithmic work per launch, peak)
            # X'X on the int8 MFMA: the int8 ops the kernel executed (2 x MACs: slice 0 over every
            # upper 256 x 128 tile and k-block, the three high-slice products on the k-blocks the
            # map lists; tp_debug_xtx_exec); the dense-equivalent ns^2 N^3 figure is a labelled extra
            "xtx_gemm": ((tm[5], "mfma", 1, share * 2.0 * xexec[0] if xexec[0] > 0 else share * ns * ns * float(n) ** 3,
                          INT8_MFMA_PEAK_TOPS) if ns else
                         (tm[5], "mfma", 1, share * float(n) ** 3, FP64_MFMA_PEAK_TFLOPS)),
            "xcxc_gemm": (tm[6], "mfma", 1, share * float(n) ** 3, FP64_MFMA_PEAK_TFLOPS),
            # products with C on the int8 MFMA: `pairs` digit products of 2 N^2 p int8 ops each
            "gq_gemm": ((tm[7], "mfma", gq_launches, gq_flops * pairs, INT8_MFMA_PEAK_TOPS) if pairs else
                        (tm[7], "mfma", gq_launches, gq_flops, FP64_MFMA_PEAK_TFLOPS)),
            "coniss": (tm[9], "hbm", 1, 40.0 * (n - 1) * k * (k + 1) / 2.0, HBM_PEAK_GBS),   # 5 sum rows/merge
            "ch": (tm[10], "hbm", 1, 16.0 * n * k, HBM_PEAK_GBS),   # the scores twice (segment statistics shared by the trees)
        }
        dom = max(kern, key=lambda q: kern[q][0])

        def rate(q):
            ms_tot, bound, launches, per_launch, peak = kern[q]
            avg_ms = ms_tot / launches
            if not avg_ms > 0:   # a class this path does not run (e.g. G = Xc'Xc on the Krylov path)
                return float("nan"), peak, "TFLOP/s" if bound == "mfma" else "GB/s", avg_ms
            if bound == "mfma":
                unit = "TOP/s (int8)" if ((q == "xtx_gemm" and ns) or (q == "gq_gemm" and pairs)) else "TFLOP/s"
                return per_launch / (avg_ms * 1e-3) / 1e12, peak, unit, avg_ms
            return per_launch / (avg_ms * 1e-3) / 1e9, peak, "GB/s", avg_ms

        ms_tot, bound, launches, per_launch, _ = kern[dom]
        achieved, peak, unit, avg_ms = rate(dom)
        traffic, tsrc = _pmc_traffic(dom, n0, k)
        roof = {"kernel": dom, "bound": bound, "achieved": round(achieved, 3), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 5), "traffic": traffic, "traffic_source": tsrc,
                "algorithmic_per_launch": per_launch, "avg_launch_ms": round(avg_ms, 4),
                "launches_per_step": launches,
                "dominance": "largest kernel-class time of one pipeline (events over the timed steps)",
                "classes": {q: {"ms_per_step": round(kern[q][0], 4),
                                "achieved": round(rate(q)[0], 3) if kern[q][0] > 0 else None, "unit": rate(q)[2],
                                "frac_of_peak": round(rate(q)[0] / rate(q)[1], 5) if kern[q][0] > 0 else None}
                            for q in kern},
                "xtx": {"int8_slices": ns,
                        "fp64_equivalent_tflops": (round(share * float(n) ** 3 / (tm[5] * 1e-3) / 1e12, 2)
                                                   if tm[5] > 0 else None),
                        "executed_int8_macs": xexec[0] if xexec[0] > 0 else None,
                        "slice0_macs": xexec[1] if xexec[0] > 0 else None,
                        "high_slice_blocks_executed": int(xexec[2]) if xexec[0] > 0 else None,
                        "high_slice_blocks_dense": int(xexec[3] * xexec[4]) if xexec[0] > 0 else None,
                        "dense_equivalent_tops": (round(share * ns * ns * float(n) ** 3 / (tm[5] * 1e-3) / 1e12, 2)
                                                  if tm[5] > 0 and ns else None),
                        "note": ("xtx_gemm.achieved counts the int8 ops k_xtx_i8_w executed (2 x MACs over its "
                                 "256x128 upper tiles: slice 0 on every 64-deep k-block, the three high-slice "
                                 "products only on the blocks the nonzero map lists); dense_equivalent_tops "
                                 "counts all ns^2 slice products whole (a labelled extra, not the roofline)")
                        if ns == 2 else None},
                "gq": {"int8_digit_pairs": pairs,
                       "fp64_equivalent_tflops": (round(gq_flops * gq_launches / (tm[7] * 1e-3) / 1e12, 2)
                                                  if tm[7] > 0 else None),
                       "note": ("the products with C on the int8 MFMA from digit images (6 digits of C, 7 of "
                                "the block, pairs s + t <= 6; tp_prod_i8.hip); achieved counts the int8 ops")
                       if pairs else None},
                "stages_ms": {"mask": round(tm[0], 3), "cor": round(tm[1], 3), "pca": round(tm[2], 3),
                              "sweep": round(tm[3], 3), "total": round(tm[4], 3)},
                "pca": {"path": "block Krylov (G never formed)" if krylov_steps else "G = Xc'Xc + subspace iteration",
                        "krylov_steps": krylov_steps, "krylov_dim": krylov_d, "chebyshev_degrees": int(tm[11]),
                        "block": block, "resid": float(tm[13])}}
        if dom == "coniss":
            roof["note"] = "one dependent merge chain per tree: latency-bound (merges/s below)"
            roof["merges_per_s"] = round(k * (n - 1) / (avg_ms * 1e-3), 1)
        out = {"metric": METRIC,
               "value": round(value, 2), "unit": "bins/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "strong" if args.sharded else "weak", "vs_baseline": None,
               "dtype": "f64",
               # what "f64" covers: every result is fp64; two products run on integer matrix cores
               # without changing that (exact, or within fp64 rounding of the fp64 product)
               "dtype_detail": ("f64 results; X'X of integer counts exact on the int8 MFMA (7-bit slices, "
                                "int32 accumulation, one rounding); the G-space Krylov products with C on the "
                                "int8 MFMA from base-256 digit images (6 digits of C, 7 of each block, 27 digit "
                                "pairs, within ~1e-15 of sum |A||B|), and from 10 000 bins (the c5 lines) the "
                                "C-space Krylov products of 32 columns on the same 6-digit image of C (not "
                                "bit-equal to the fp64 products: heights within 1e-9, same TADs); everything "
                                "else fp64 VALU / MFMA"),
               "data": "synthetic (SURVEY.md §8(d) Hi-C generator, seed 20261015+%d" % cfg +
                       ("" if args.sharded else "+1000*rank") + ")",
               "ranks_seen": len(seen), "devices_seen": sorted({d for _, d in seen}),
               "config": {"workload": (f"{_config_name(n0, args.max_pcs)}: synthetic {n0}x{n0} Hi-C matrix "
                                       + ("sharded over all GPUs" if args.sharded else "per GPU")
                                       + f", max_pcs={args.max_pcs}, one pipeline at a time on one stream"),
                          "n0": n0, "n_good": n, "k": k, "max_pcs": args.max_pcs,
                          "parallelism": (f"one matrix over {world} GPU(s): column/row-split products, "
                                          "RCCL all-gather" if args.sharded else f"one matrix per GPU x{world}")},
               "roofline": roof, "host_ms_per_step": host_ms,
               "pipeline_roofline": pipeline_roofline(n, k, elapsed / args.steps * 1e3)}
        if comm_size is not None:
            out["rccl_comm_size"] = comm_size
        if thr:
            out["throughput"] = thr
        out.update(extras)
        # parity vs the committed oracle fixture of this workload (R-faithful SVD PCA)
        par = {}
        gold = os.path.join(HERE, "tests", "golden", f"c{cfg}.npz")
        if not args.sharded and os.path.exists(gold) and n0 == {3: 7808, 2: 2000}[cfg] and args.max_pcs == 200:
            z = np.load(gold)
            lev = z["levels"]
            co = z["coords"]
            ok = (last.n_pcs == int(z["n_pcs"]) and last.optimal_n_clusters == int(z["optimal_n_clusters"])
                  and set(last.clusters) == {str(int(q)) for q in lev}
                  and all(np.array_equal(last.clusters[str(int(q))], co[co[:, 0] == q][:, 1:]) for q in lev)
                  and np.array_equal(last.dendro.merge, z["merge"]))
            a, b = last.scores, z["scores"]
            fin = ~np.isnan(b)
            par["golden_fixture"] = os.path.relpath(gold, HERE)
            par["boundaries_match_golden"] = bool(ok)
            par["ch_max_rel_err_golden"] = (float(np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin])))
                                            if a.shape == b.shape else None)
        if not args.no_cpu_baseline and world == 1 and not args.sharded:   # CPU baseline: rank 0 at N=1 only
            sys.path.insert(0, os.path.join(HERE, "oracle"))
            import tadpole_oracle as O
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
            t1 = time.perf_counter()
            ref = O.tadpole(host, max_pcs=args.max_pcs, min_clusters=args.min_clusters, nthreads=threads,
                            pca="eigh")
            cpu_s = time.perf_counter() - t1
            out["cpu_baseline"] = {"value": round(n0 / cpu_s, 2), "unit": "bins/s", "cores": threads,
                                   "kind": "port",
                                   "sample": (f"one full {_config_name(n0, args.max_pcs)} pipeline of the CPU oracle "
                                              f"({cpu_s:.2f} s): numpy mask + X'X correlation, LAPACK dsyevr top-"
                                              f"{k} eigenpairs of Xc'Xc (cheaper than R's full gesdd SVD), OpenMP C "
                                              "CONISS/CH sweep over all PC prefixes")}
            same = (last.n_pcs == ref.n_pcs and last.optimal_n_clusters == ref.optimal_n_clusters
                    and set(last.clusters) == {str(q) for q in ref.clusters}
                    and all(np.array_equal(last.clusters[str(q)], v) for q, v in ref.clusters.items()))
            a, b = last.scores, ref.scores
            fin = ~np.isnan(b)
            par["boundaries_match_cpu_oracle"] = bool(same)
            par["n_pcs"] = [last.n_pcs, ref.n_pcs]
            par["n_clusters"] = [last.optimal_n_clusters, ref.optimal_n_clusters]
            par["ch_max_rel_err_cpu_oracle"] = (float(np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin])))
                                                if a.shape == b.shape else None)
        if par:
            out["parity"] = par
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        if args.sharded:
            from tadpole_amd import multi
            multi.destroy_comm(local)
        dist.destroy_process_group()
    L.tp_shutdown()


if __name__ == "__main__":
    main()
