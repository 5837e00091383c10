#!/bin/bash
# C-Krylov A/B (G path vs C path, split counts), then the GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TP_TRACE_PCA=1 timeout -k 10 300 python -u tools/ab_knobs.py 7808 '20=0' '20=1' '20=1,23=16' '20=1,21=256' '20=1,21=1024' > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | tail -40
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
