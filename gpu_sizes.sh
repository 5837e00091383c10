#!/bin/bash
# Full GPU parity suite, then bench at C2 / C3 shape / 10k / C5 arm shape.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in "2000 10 2" "7808 5 1" "10000 5 1" "24300 2 1 --sharded"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --n0 $1 --steps $2 --warmup $3 $4 --no-cpu-baseline > gpurun_out/bench_$1.log 2>&1
  rc=$?; echo "bench $1 rc=$rc"; tail -1 gpurun_out/bench_$1.log | cut -c1-300; tail -1 gpurun_out/bench_$1.log | grep -o '"stages_ms[^}]*}'
  [ $rc -eq 0 ] || exit $rc
done
exit 0
