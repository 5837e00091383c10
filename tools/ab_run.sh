cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_limits.py -x -q -k "sweep or coniss" --timeout 200 --timeout-method thread > gpurun_out/ab13.log 2>&1 &&
for n in 7808 24300; do
  for v in "" _rb0 "" _rb0; do
    TADPOLE_LIB=$PWD/tadpole_amd/libtadpole_hip$v.so timeout -k 10 150 python tools/coniss_ab.py $n 5 >> gpurun_out/ab13.log 2>&1 || exit 1
  done
done
