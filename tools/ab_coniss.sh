cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for n in 7808 24300; do
  for v in "" v100 v010 v001 v111; do
    lib=tadpole_amd/libtadpole_hip${v:+_$v}.so
    TADPOLE_LIB=$PWD/$lib timeout -k 10 120 python tools/coniss_ab.py $n 5 >> gpurun_out/ab_coniss.log 2>&1 || exit 1
  done
done
