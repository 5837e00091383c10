#!/bin/bash
# first GPU pass: parity tests, then a short bench; stop on any crash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --cpu-reps 1 > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -5 gpurun_out/bench.log
exit $rc2
