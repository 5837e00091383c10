#!/bin/bash
# One GPU round trip: optional pytest selection ($TESTS, -k filter $K), then
# optional bench ($BENCH args).  Every GPU step has its own time limit; a
# failing step ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -x -v -s -m gpu --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_LIMIT:-400} python bench.py $BENCH > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -c 3000
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
