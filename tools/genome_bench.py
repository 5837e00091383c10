"""C4 timing (BASELINE configs[3]): the 23 hg19 chromosomes @25 kb (synthetic
Hi-C of the real bin counts) through tadpole_amd.genome.run_genome on this
process's GPU(s).  Under torch.distributed.run each rank owns a share of the
chromosomes (LPT, no data-path collective); rank 0 prints one JSON line with
the whole-genome wall time and bins/s.  usage:
  python tools/genome_bench.py [--streams S] [--reps R]
  python -m torch.distributed.run --nproc-per-node N tools/genome_bench.py"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    from tadpole_amd.genome import run_genome
    from tadpole_amd.synth import genome_bins, genome_matrix
    sizes = genome_bins()
    mats = {c: genome_matrix(c) for c in sizes}   # built before the timed runs
    run_genome(mats, sizes=sizes, streams=args.streams, max_pcs=200)   # warm-up (contexts, code objects)
    walls = []
    for _ in range(args.reps):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        res, secs = run_genome(mats, sizes=sizes, streams=args.streams, max_pcs=200)
        if world > 1:
            dist.barrier()
        walls.append(time.perf_counter() - t0)
    if int(os.environ.get("RANK", "0")) == 0:
        bins = sum(sizes.values())
        wall = float(np.median(walls))
        print(json.dumps({"workload": "C4: 23 hg19 chromosomes @25 kb, max_pcs=200, one run_genome call",
                          "ranks": world, "streams_per_rank": args.streams, "chromosomes": len(sizes),
                          "bins": bins, "wall_s": round(wall, 4), "bins_per_s": round(bins / wall, 1),
                          "note": "host-resident matrices: the wall time includes the host-to-device copies "
                                  "and the host assembly of every tadpole object"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
