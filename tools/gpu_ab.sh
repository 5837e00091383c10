#!/bin/bash
# A/B of library knobs on C3 (tools/ab_knobs.py, one config per argument),
# then the GPU suite unless NOTEST is set.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TP_TRACE_PCA=1 timeout -k 10 300 python -u tools/ab_knobs.py ${N0:-7808} "$@" > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | grep -v "^\[pca\] n=" | tail -30
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
