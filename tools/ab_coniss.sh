# A/B of library variants on the GPU box (tools/build_variant.sh builds them)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TADPOLE_LIB=$PWD/tadpole_amd/libtadpole_hip.so timeout -k 10 60 python tools/sytrd_ab.py base 256 224 160 >> gpurun_out/ab.log 2>&1 || exit 1
TADPOLE_LIB=$PWD/tadpole_amd/libtadpole_hip_sy1.so timeout -k 10 60 python tools/sytrd_ab.py sy1 256 224 160 >> gpurun_out/ab.log 2>&1 || exit 1
python -c "
import numpy as np
for b in (256, 224, 160):
    x = np.load(f'gpurun_out/sytrd_base_{b}.npz'); y = np.load(f'gpurun_out/sytrd_sy1_{b}.npz')
    print(b, 'bit-identical' if all(np.array_equal(x[k], y[k]) for k in x.files) else 'DIFFERENT')
" >> gpurun_out/ab.log 2>&1 || exit 1
for n in 7808 24300; do
  for v in "" v100 v010 v001 v111; do
    lib=tadpole_amd/libtadpole_hip${v:+_$v}.so
    TADPOLE_LIB=$PWD/$lib timeout -k 10 120 python tools/coniss_ab.py $n 5 >> gpurun_out/ab.log 2>&1 || exit 1
  done
done
