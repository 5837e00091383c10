#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_kernels.py > gpurun_out/diag.log 2>&1
rc=$?; echo "diag rc=$rc"; cat gpurun_out/diag.log | grep -v amdgpu.ids
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-reps 1 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-1500
exit 0
