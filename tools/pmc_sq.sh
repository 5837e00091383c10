#!/bin/bash
# One SQ/GRBM counter pass (no trace domains) over the Krylov GEMM and CONISS
# of the default bench workload: MFMA busy, wait/issue breakdown, LDS conflicts.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_sq
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  --kernel-include-regex "${RX:-k_gemm_ts|k_coniss}" --output-format csv -d gpurun_out/pmc_sq -o run -- \
  python3 bench.py --steps 2 --warmup 1 --throughput-streams 0 --no-cpu-baseline > gpurun_out/pmc_sq.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
