#!/bin/bash
# Bench latency (one stream) at the C3 shape / 10k / C5 arm shape, and C3
# throughput with 4 matrices in flight.  NOTEST=1 skips the parity suite.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for cfg in "7808 3 1 --throughput-streams 0" "10000 3 1 --throughput-streams 0" "24300 2 1 --sharded" "7808 8 1 --throughput-streams 4"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --n0 $1 --steps $2 --warmup $3 $4 $5 --no-cpu-baseline > gpurun_out/bench_$1_$2.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"; tail -1 gpurun_out/bench_$1_$2.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"single_stream_ms_per_matrix": [0-9.a-z]*'; tail -1 gpurun_out/bench_$1_$2.log | grep -o '"stages_ms[^}]*}'
  [ $rc -eq 0 ] || exit $rc
done
exit 0
