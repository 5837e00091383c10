#!/bin/bash
# GPU round trip: (K=expr) parity tests -> bench (ARGS) -> (PROF=1) rocprof.
# Every GPU step has its own time limit; a failing step ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -8
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py ${ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  ./tools/gpu_prof.sh; exit $?
fi
exit 0
