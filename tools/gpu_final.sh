#!/bin/bash
# One call: GPU suite -> knob A/B (ARGS, default the Gram kernel on/off) -> bench + rocprof passes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_knobs.py 7808 ${AB:-29=1 29=0 29=1} > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | grep -v "^\[pca\]" | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
./tools/gpu_prof.sh
