#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench workload (no counters).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps ${STEPS:-3} --warmup 1 --throughput-streams 0 --no-cpu-baseline ${BARGS} --json-out gpurun_out/prof_bench.json > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; cut -c1-300 gpurun_out/prof_bench.json
exit $rc
