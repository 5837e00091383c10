#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
for B in 16 256; do
  timeout -s KILL 90 rocprofv3 --pmc $C1 --kernel-include-regex k_sytrd_reg --output-format csv -d gpurun_out/pmc/s$B -o run -- python3 tools/run_kernel.py sytrd $B 1 > gpurun_out/pmc/s$B.log 2>&1
  echo "b=$B rc=$?"
done
find gpurun_out/pmc -name "*counter_collection.csv" | head
