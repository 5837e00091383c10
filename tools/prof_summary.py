"""Summarise a gpu_prof.sh run (rocprofv3 CSVs under gpurun_out/) into
profiles/<tag>_kernel_stats.csv (copy), profiles/<tag>_summary.md and
profiles/<tag>_traffic.json (per-launch HBM bytes from the two PMC passes).

Traffic per the MI355X guide: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reads half the bytes of a wide coalesced stream, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (raw values are kept too).

usage: python tools/prof_summary.py <tag> [steps_per_run]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")

# bench.py kernel class -> name prefixes of the kernels one launch of that class
# runs; per prefix the variant with the largest total time in the trace is taken
# (the CONISS block size and the GEMM tile are chosen per problem size)
CLASSES = {"coniss": ["tp::k_coniss_"],   # k_coniss_b (batched, round 6) or k_coniss_t
           "ch": ["tp::k_ch_cut", "tp::k_ch_segstat", "tp::k_ch<"],
           "xtx_gemm": ["tp::k_xtx_i8_"]}


def pick(stats, prefix):
    cand = [r for r in stats if r["Name"].replace("void ", "").startswith(prefix)]
    return short(max(cand, key=lambda r: float(r["TotalDurationNs"]))["Name"]) if cand else None


def short(name):
    return name.split("(")[0].replace("void ", "")[:90]


def main():
    tag = sys.argv[1]
    bench = json.load(open(os.path.join(OUT, "prof_bench.json")))
    # timed + warmup pipelines + the untimed ones bench.py runs after the timed
    # region with per-product events on (max(2, min(5, steps)))
    steps = bench["steps"] + bench["warmup"] + max(2, min(5, bench["steps"]))
    stats = list(csv.DictReader(open(os.path.join(OUT, "prof", "run_kernel_stats.csv"))))
    shutil.copy(os.path.join(OUT, "prof", "run_kernel_stats.csv"),
                os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    tot = sum(float(r["TotalDurationNs"]) for r in stats)
    lines = [f"# {tag}: rocprofv3 --kernel-trace --stats, `python bench.py --steps {bench['steps']} "
             f"--warmup {bench['warmup']} --throughput-streams 0 --no-cpu-baseline` "
             f"({steps} pipelines, {bench['config']['workload']})",
             "", f"bench line of the profiled run: value {bench['value']} bins/s, "
                 f"{bench['ms_per_step']} ms/step (profiler attached)", "",
             "| kernel | calls/pipeline | ms/pipeline | avg us | % |", "|---|---|---|---|---|"]
    for r in stats:
        lines.append(f"| `{short(r['Name'])}` | {int(r['Calls']) / steps:.1f} | "
                     f"{float(r['TotalDurationNs']) / steps / 1e6:.3f} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['Percentage']):.2f} |")
    lines += ["", f"GPU kernel time per pipeline: {tot / steps / 1e6:.3f} ms", ""]
    # ---- PMC passes
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for tagc, cnt in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        path = os.path.join(OUT, tagc, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            pmc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    traffic = {}
    if pmc:
        lines += ["## HBM traffic (separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes)", "",
                  "hbm bytes/launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE counts half of a "
                  "wide coalesced read: MI355X_MICROARCH.md, HBM)", "",
                  "| kernel | launches | FETCH_SIZE KiB | WRITE_SIZE KiB | hbm MB/launch |", "|---|---|---|---|---|"]
        for name, cs in sorted(pmc.items()):
            f = cs.get("FETCH_SIZE", [0.0])
            w = cs.get("WRITE_SIZE", [0.0])
            fa, wa = sum(f) / len(f), sum(w) / len(w)
            hb = (2 * fa + wa) * 1024
            traffic[short(name)] = {"launches": len(f), "fetch_kib": fa, "write_kib": wa, "hbm_bytes": hb}
            lines.append(f"| `{short(name)}` | {len(f)} | {fa:.0f} | {wa:.0f} | {hb / 1e6:.2f} |")
    # per-class figures: kernels of one class launch, summed (avg duration from
    # the trace stats, HBM bytes from the PMC passes)
    avg_us = {short(r["Name"]): float(r["AverageNs"]) / 1e3 for r in stats}
    classes = {}
    for cls, prefixes in CLASSES.items():
        names = [pick(stats, pf) for pf in prefixes]
        if all(nm is not None and nm in avg_us for nm in names):
            classes[cls] = {"kernels": names, "avg_us": sum(avg_us[nm] for nm in names),
                            "hbm_bytes": (sum(traffic[nm]["hbm_bytes"] for nm in names)
                                          if all(nm in traffic for nm in names) else None)}
    if classes:
        lines += ["", "## Bench kernel classes (one launch = these kernels)", "",
                  "| class | kernels | avg us | hbm MB |", "|---|---|---|---|"]
        for cls, rec in classes.items():
            hb = f"{rec['hbm_bytes'] / 1e6:.2f}" if rec["hbm_bytes"] is not None else "-"
            lines.append(f"| {cls} | {' + '.join('`%s`' % k for k in rec['kernels'])} | {rec['avg_us']:.1f} | {hb} |")
    with open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    if traffic:
        cfg = bench["config"]
        with open(os.path.join(ROOT, "profiles", f"{tag}_traffic.json"), "w") as fh:
            json.dump({"tag": tag, "n0": cfg["n0"], "k": cfg["k"], "kernels": traffic,
                       "classes": classes}, fh, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
