cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemm_ts_bench > gpurun_out/gemm_ts.log 2>&1; rc=$?; cat gpurun_out/gemm_ts.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/gemm_ts_bench 24057 > gpurun_out/gemm_ts24.log 2>&1; rc=$?; cat gpurun_out/gemm_ts24.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/mfma_valu_mix > gpurun_out/mix.log 2>&1; rc=$?; cat gpurun_out/mix.log; exit $rc
