cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q -k "two_stage or krylov" --timeout 200 --timeout-method thread > gpurun_out/ab12.log 2>&1 &&
timeout -k 10 400 python tools/ab_knobs.py 24300 '' '35=1' '' '35=1' >> gpurun_out/ab12.log 2>&1
