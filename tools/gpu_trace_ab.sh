#!/bin/bash
# rocprofv3 kernel trace of tools/ab_knobs.py (one configuration) -> gpurun_out/prof
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 tools/ab_knobs.py ${N0:-7808} "${CFG:-20=1}" > gpurun_out/trace_ab.log 2>&1
rc=$?; echo "trace rc=$rc"; grep -v amdgpu.ids gpurun_out/trace_ab.log | tail -3
exit $rc
