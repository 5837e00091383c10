#!/bin/bash
# rocprofv3 evidence for bench.py (default workload, C3): kernel trace + stats, then two separate
# PMC passes (FETCH_SIZE, WRITE_SIZE) on the sweep/GEMM kernels -- counters are
# never combined with trace domains.  Each GPU step has its own time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
B="bench.py --steps ${STEPS:-5} --warmup 1 --throughput-streams 0 --no-cpu-baseline --no-extras"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 $B --json-out gpurun_out/prof_bench.json > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cut -c1-400 gpurun_out/prof_bench.json
[ -n "$TRACE_ONLY" ] && exit 0
RX="k_coniss|k_gemm|k_splitk|k_ch|k_seed|k_xtx|k_cor|k_mask|k_sytrd|k_trS|k_pd_"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 $B > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc_write -o run -- python3 $B > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"
exit $rc
