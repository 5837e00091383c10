"""Headline benchmark (BASELINE.json metric "bins/sec (NxN matrix)").

A step = one TADpole()-equivalent pipeline over one synthetic N0 x N0 Hi-C
matrix already resident in HBM: NA->0 + symmetrise, bad-column mask, Pearson
correlation, PCA to max_pcs, CONISS sweep over every PC prefix, broken stick,
Calinski-Harabasz, parameter choice, TAD coordinates of every significant level.
Workload = BASELINE.json configs[1] (C2: synthetic 2000 x 2000, max_pcs=200).

Throughput: up to --streams (default 12) matrices in flight per GPU, each on
its own HIP stream / library context / host thread -- the latency-bound stages
of one pipeline (CONISS merges, the one-workgroup Cholesky and
tridiagonalisation) leave most of the 256 CUs idle, and a stream of matrices (a
genome is 23 of them) fills them.  HIP maps streams onto GPU_MAX_HW_QUEUES
hardware queues (4 by default); streams sharing a queue serialise, so the bench
raises it to 16.  value = bins of all matrices / wall time; the one-matrix
latency is reported next to it (config.single_stream_ms_per_matrix).

Multi-GPU: one process per GPU (torch.distributed.run); each rank processes its
own matrices (independent chromosomes): weak scaling, no
data-path collective.  value = bins of all ranks / max-over-ranks time.

Extra fields: "roofline" for the dominant kernel (HIP events inside the
library, same stream), "cpu_baseline" (the CPU oracle on this host, rank 0),
"parity" (rank 0's TAD boundaries vs the oracle on the same matrix).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

# before HIP initialises (torch import / first device call): one hardware queue
# per concurrent pipeline (see the docstring); raises a lower setting (HIP's
# default, 4, is often exported explicitly)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

FP64_MFMA_PEAK_TFLOPS = 78.6     # MI355X FP64 matrix, dense (AMD spec)
# what v_mfma_f64_16x16x4_f64 sustains on this chip: back-to-back, independent
# accumulators, 4 waves/SIMD on every CU (tools/mfma_rate.hip; 33 TF/s at 1
# wave/SIMD, 43 at 2)
FP64_MFMA_MEASURED_TFLOPS = 45.0
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E (MI355X_MICROARCH.md)


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
    if max_pcs == 200 and n0 == 2000:
        return "C2"
    if max_pcs == 200 and n0 == 7808:
        return "C3 shape (chr18 @10kb)"
    if max_pcs == 200 and n0 in (24300, 21300):
        return "C5 arm shape (chr1 @5kb)"
    if n0 == 200:
        return "C1 shape"
    return "custom"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n0", type=int, default=2000)
    ap.add_argument("--max-pcs", type=int, default=200)
    ap.add_argument("--min-clusters", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--streams", type=int, default=12,
                    help="matrices in flight per GPU (one stream + host thread each; the single-CU stages of one "
                         "pipeline leave most of the chip idle); 1 = one matrix at a time")
    ap.add_argument("--sharded", action="store_true",
                    help="one matrix split over all ranks (SURVEY §8(e)2, C5 arms): strong scaling")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)

    import tadpole_amd as tp
    from tadpole_amd import _lib
    from tadpole_amd.api import _assemble
    from tadpole_amd.synth import SEED_BASE, synth_hic

    L = _lib.load()
    n0 = args.n0
    seed = SEED_BASE + 2 + (0 if args.sharded else 1000 * rank)   # sharded: every rank holds the same matrix
    host = synth_hic(n0, seed)
    flags = _lib.TP_FLAG_ROW_MAJOR
    if args.sharded:
        from tadpole_amd import multi
        if world > 1:
            multi.init_comm(device=local)
        flags |= _lib.TP_FLAG_SHARDED
    k_cap = max(1, min(args.max_pcs, n0))
    w_cap = n0
    I = ctypes.c_int
    # one pipeline at a time when sharded: the ranks' collectives must be issued
    # in the same order, one communicator per device
    S = 1 if args.sharded else max(1, args.streams)

    class Lane:
        """One pipeline in flight: its own stream (hence its own library context
        and scratch), its own resident copy of the matrix, its own host outputs."""

        def __init__(self, idx):
            self.stream = torch.cuda.current_stream() if idx == 0 else torch.cuda.Stream(device=f"cuda:{local}")
            self.dev_m = torch.from_numpy(host).to(f"cuda:{local}")
            self.bufs = dict(bad=np.zeros(n0, np.int32), good=np.zeros(n0, np.int32),
                             nclu=np.zeros(k_cap, np.int32), scores=np.zeros(k_cap * w_cap),
                             merge=np.zeros(2 * (n0 - 1), np.int32), height=np.zeros(n0 - 1),
                             boundary=np.zeros(n0 - 1, np.int32), timings=np.zeros(16))

    lanes = [Lane(i) for i in range(S)]
    torch.cuda.synchronize()

    def step(want_timings: bool, lane=None):
        lane = lane or lanes[0]
        b, dev_m, stream = lane.bufs, lane.dev_m, lane.stream
        outs = [I(0) for _ in range(6)]
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
        n = n_good.value
        kk, ww = k.value, w.value
        res = dict(bad=b["bad"].astype(bool), good=b["good"][:n].copy(), k=kk, w=ww,
                   scores=b["scores"][:kk * ww].reshape(ww, kk).T.copy(), n_pcs=n_pcs.value,
                   n_clusters=n_clusters.value,
                   merge=b["merge"][:2 * (n - 1)].reshape(2, n - 1).T.copy(), height=b["height"][:n - 1].copy(),
                   boundary=b["boundary"][:n - 1].copy(), timings=b["timings"].copy())
        return _assemble(res, np.flatnonzero(res["bad"]) + 1)

    for _ in range(args.warmup):
        for ln in lanes:
            step(False, ln)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    last = None
    if S == 1:
        for _ in range(args.steps):
            last = step(False)
    else:
        # S host threads, one stream each, the K steps dealt round-robin (ctypes
        # releases the GIL inside the library call)
        import threading
        outs = [None] * S

        def run(i):
            for _ in range(i, args.steps, S):
                outs[i] = step(False, lanes[i])

        th = [threading.Thread(target=run, args=(i,)) for i in range(S)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        last = outs[0]
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # latency of one matrix on its own (one stream), for reference next to the
    # S-stream throughput in `value`
    single_ms = None
    if S > 1:
        barrier()
        t1 = time.perf_counter()
        reps = max(3, min(10, args.steps // S))
        for _ in range(reps):
            step(False)
        barrier()
        single_ms = (time.perf_counter() - t1) / reps * 1e3

    # one more instrumented step for the per-kernel breakdown (not in `value`)
    prof = step(True)
    tm = prof.timings_ms
    n = int(tm[14])
    k = int(tm[15])

    if rank == 0:
        value = n0 * (1 if args.sharded else world) * args.steps / elapsed
        # ---- roofline of the dominant kernel
        share = 1.0 / world if args.sharded else 1.0   # sharded: this rank's part of each product
        kern = {
            "xtx_gemm": (tm[5], "mfma", 1, share * float(n) ** 3),              # N^3 (symmetric half)
            "xcxc_gemm": (tm[6], "mfma", 1, share * float(n) ** 3),
            "gq_gemm": (tm[7], "mfma", max(1, int(tm[8])), share * 2.0 * n * n * int(tm[12]) if tm[12] else 0.0),
            "coniss": (tm[9], "hbm", 1, 40.0 * (n - 1) * k * (k + 1) / 2.0),    # bytes: 5 sum vectors/merge
            "ch": (tm[10], "hbm", 1, 16.0 * n * k * k),                         # bytes: 2 passes/tree
        }
        # Dominant kernel.  With S > 1 matrices in flight `value` is bound by
        # how much of the chip each kernel class occupies, not by one
        # pipeline's critical path: weight each class's time by the share of
        # the 1024 SIMDs its grid fills (GEMMs: all; CONISS: 2 waves per tree;
        # CH: 4 waves per tree).  With one stream: the longest class.
        simd_share = {"xtx_gemm": 1.0, "xcxc_gemm": 1.0, "gq_gemm": 1.0,
                      "coniss": min(1.0, 2.0 * k / 1024), "ch": min(1.0, 4.0 * k / 1024)}
        chip_ms = {q: kern[q][0] * simd_share[q] for q in kern}
        longest = max(kern, key=lambda q: kern[q][0])
        dom = max(chip_ms, key=chip_ms.get) if S > 1 else longest

        def rate(q):
            ms_tot, bound, launches, per_launch = kern[q]
            avg_ms = ms_tot / launches
            if bound == "mfma":
                return per_launch / (avg_ms * 1e-3) / 1e12, FP64_MFMA_PEAK_TFLOPS, "TFLOP/s", avg_ms
            return per_launch / (avg_ms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s", avg_ms

        ms_tot, bound, launches, per_launch = kern[dom]
        achieved, peak, unit, avg_ms = rate(dom)
        traffic, tsrc = _pmc_traffic(dom, n0, k)
        roof = {"kernel": dom, "bound": bound, "achieved": round(achieved, 3), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 5), "traffic": traffic, "traffic_source": tsrc,
                "algorithmic_per_launch": per_launch, "avg_launch_ms": round(avg_ms, 4),
                "launches_per_step": launches,
                "dominance": ("largest SIMD-time share per matrix with %d matrices in flight" % S if S > 1
                              else "longest kernel class of one pipeline"),
                "chip_ms_per_matrix": {q: round(v, 4) for q, v in chip_ms.items()},
                "breakdown_ms": {q: round(kern[q][0], 4) for q in kern},
                "stages_ms": {"mask": round(tm[0], 3), "cor": round(tm[1], 3), "pca": round(tm[2], 3),
                              "sweep": round(tm[3], 3), "total": round(tm[4], 3)},
                "pca": {"iters": int(tm[11]), "block": int(tm[12]), "resid": float(tm[13])}}
        if bound == "mfma":
            roof["measured_mfma_ceiling"] = FP64_MFMA_MEASURED_TFLOPS
            roof["frac_of_measured_ceiling"] = round(achieved / FP64_MFMA_MEASURED_TFLOPS, 4)
        if longest != dom:   # the one-pipeline critical path (latency), beside it
            a2, p2, u2, m2 = rate(longest)
            t2, ts2 = _pmc_traffic(longest, n0, k)
            roof["latency_critical"] = {"kernel": longest, "bound": kern[longest][1], "achieved": round(a2, 3),
                                        "peak": p2, "unit": u2, "frac": round(a2 / p2, 5), "avg_launch_ms": round(m2, 4),
                                        "traffic": t2, "traffic_source": ts2}
            if longest == "coniss":
                roof["latency_critical"]["note"] = "one dependent merge chain per tree: latency-bound"
                roof["latency_critical"]["merges_per_s"] = round(k * (n - 1) / (m2 * 1e-3), 1)
        out = {"metric": "bins/sec (NxN matrix) at 1/2/4/8 GPUs; TAD boundary bit-match vs R ref",
               "value": round(value, 2), "unit": "bins/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "strong" if args.sharded else "weak", "vs_baseline": None,
               "dtype": "f64",
               "data": "synthetic (SURVEY.md §8(d) Hi-C generator, seed 20261015+2" +
                       ("" if args.sharded else "+1000*rank") + ")",
               "config": {"workload": (f"{_config_name(n0, args.max_pcs)}: synthetic {n0}x{n0} Hi-C matrix "
                                       + ("sharded over all GPUs" if args.sharded else "per GPU")
                                       + f", max_pcs={args.max_pcs}"),
                          "n0": n0, "n_good": n, "k": k, "max_pcs": args.max_pcs,
                          "parallelism": (f"one matrix over {world} GPU(s): column/row-split products, "
                                          "RCCL all-gather" if args.sharded else f"one matrix per GPU x{world}"),
                          "streams_per_gpu": S,
                          "single_stream_ms_per_matrix": round(single_ms, 3) if single_ms else None},
               "roofline": roof}
        if not args.no_cpu_baseline and world == 1 and not args.sharded:   # CPU baseline: rank 0 at N=1 only
            sys.path.insert(0, os.path.join(HERE, "oracle"))
            import tadpole_oracle as O
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
            t1 = time.perf_counter()
            ref = None
            for _ in range(args.cpu_reps):
                ref = O.tadpole(host, max_pcs=args.max_pcs, min_clusters=args.min_clusters, nthreads=threads)
            cpu_s = (time.perf_counter() - t1) / args.cpu_reps
            out["cpu_baseline"] = {"value": round(n0 / cpu_s, 2), "unit": "bins/s", "cores": threads,
                                   "kind": "port",
                                   "sample": f"{args.cpu_reps} full C2 pipelines (numpy LAPACK SVD + C sweep, "
                                             f"OpenMP over PC prefixes), {cpu_s:.3f} s each"}
            same = (last.n_pcs == ref.n_pcs and last.optimal_n_clusters == ref.optimal_n_clusters
                    and set(last.clusters) == {str(q) for q in ref.clusters}
                    and all(np.array_equal(last.clusters[str(q)], v) for q, v in ref.clusters.items()))
            a, b = last.scores, ref.scores
            fin = ~np.isnan(b)
            rel = float(np.max(np.abs(a[fin] - b[fin]) / np.abs(b[fin]))) if a.shape == b.shape else None
            out["parity"] = {"boundaries_match_oracle": bool(same), "n_pcs": [last.n_pcs, ref.n_pcs],
                             "n_clusters": [last.optimal_n_clusters, ref.optimal_n_clusters],
                             "ch_max_rel_err": rel}
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
