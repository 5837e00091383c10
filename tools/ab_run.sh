cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tiles128 or xtx" --timeout 120 --timeout-method thread -s > gpurun_out/ab6.log 2>&1 &&
timeout -k 10 200 python tools/xtx_ab.py 24300 0 >> gpurun_out/ab6.log 2>&1 &&
timeout -k 10 200 python tools/xtx_ab.py 24300 0 34=0 >> gpurun_out/ab6.log 2>&1 &&
timeout -k 10 100 python tools/xtx_ab.py 7808 0 >> gpurun_out/ab6.log 2>&1 &&
timeout -k 10 100 python tools/xtx_ab.py 7808 0 34=0 >> gpurun_out/ab6.log 2>&1 &&
timeout -k 10 100 python tools/xtx_ab.py 7808 >> gpurun_out/ab6.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread >> gpurun_out/ab6.log 2>&1
