#!/bin/bash
# C3 baseline: one-stream bench with the PCA round log, then a rocprofv3 kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TP_TRACE_PCA=1 timeout -k 10 300 python bench.py --n0 7808 --steps 3 --warmup 1 --streams 1 --no-cpu-baseline > gpurun_out/c3_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/c3_bench.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/c3prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3prof -o run -- python3 bench.py --n0 7808 --steps 2 --warmup 1 --streams 1 --no-cpu-baseline > gpurun_out/c3_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
