#!/bin/bash
# C-Krylov: kernel trace of one pipeline configuration, then the A/B timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
./tools/gpu_trace_ab.sh || exit $?
timeout -k 10 300 python -u tools/ab_knobs.py 7808 '20=0' '20=1' ${ABX} > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | tail -12
exit $rc
