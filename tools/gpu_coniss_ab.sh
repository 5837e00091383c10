#!/bin/bash
# CONISS change check: stamps at C3, sweep bit-exactness tests, C3 stage timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_kernels.py coniss3 > gpurun_out/diag.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/diag.log | head -9
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sweep.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_sweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_knobs.py 7808 '' '' > gpurun_out/ab.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/ab.log; exit $rc
