cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in nodma nomfma; do
TADPOLE_LIB=$PWD/tadpole_amd/libtadpole_hip_$v.so timeout -k 10 200 python tools/xtx_ab.py 24300 > gpurun_out/ab5_$v.log 2>&1 || exit 1
TADPOLE_LIB=$PWD/tadpole_amd/libtadpole_hip_$v.so timeout -k 10 200 python tools/xtx_ab.py 7808 >> gpurun_out/ab5_$v.log 2>&1 || exit 1
done
