#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (csv), then bench json
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --json-out gpurun_out/prof_bench.json > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof_bench.json | cut -c1-300
exit $rc
