#!/bin/bash
# GPU round trip: parity tests -> bench -> (PROF=1) rocprofv3 trace + PMC passes.
# Every GPU step has its own time limit; a crash/timeout code ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2  > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-1800
[ $rc -eq 0 ] || exit $rc
if [ -n "$DIAG" ]; then
  timeout -k 10 300 python tools/diag_kernels.py > gpurun_out/diag.log 2>&1
  rc=$?; echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/diag.log
  fatal $rc && exit $rc
fi
if [ -n "$PROF" ]; then
  ./tools/gpu_prof.sh; exit $?
fi
exit 0
