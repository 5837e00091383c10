#!/bin/bash
# limits tests first (new kernels), then the GEMM microbenchmark, then the full GPU suite
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_limits.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_limits.log 2>&1
rc=$?; echo "limits rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|Error" gpurun_out/pytest_limits.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/gemm_ts_bench > gpurun_out/gemm_ts.log 2>&1; rc=$?; cat gpurun_out/gemm_ts.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/mfma_valu_mix > gpurun_out/mix.log 2>&1; rc=$?; cat gpurun_out/mix.log; [ $rc -eq 0 ] || exit $rc
NOBENCH=1 ./tools/gpu_round.sh
