#!/bin/bash
# Quick GPU iteration: selected parity tests (-k "$K"), then the C2 bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -s -m gpu --timeout 300 --timeout-method thread -k "${K:-chol_inv or pca or pipeline}" > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "chol_inv b=|passed|failed|Error|error" gpurun_out/pytest_quick.log | tail -30
[ $rc -eq 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_quick.log | cut -c1-1500
exit $rc
