#!/bin/bash
# X'X diagnostics on the GPU box: device time of the base build and of the
# DMA-only / MFMA-only diagnostic builds (tools/build_variant.sh nodma / nomfma
# with -DTP_XG_DIAG_NODMA / -DTP_XG_DIAG_NOMFMA), then PMC passes on the base
# build, each pass its own run.  N defaults to the C5 arm size.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/xtx
export TMPDIR=/tmp
N=${N:-24300}
O=gpurun_out/xtx
for v in "" _nodma _nomfma; do
  [ -f tadpole_amd/libtadpole_hip$v.so ] || continue
  TADPOLE_LIB=$PWD/tadpole_amd/libtadpole_hip$v.so timeout -k 10 240 python3 -u tools/xtx_time.py $N 2 >> $O/time.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "time$v rc=$rc"; exit $rc; }
done
cat $O/time.log
[ -n "$TIME_ONLY" ] && exit 0
pass() {   # name counters...
  local nm=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "${KRX:-k_xtx_i8}" --output-format csv -d $O/pmc_$nm -o run -- python3 tools/xtx_time.py $N 1 > $O/pmc_$nm.log 2>&1
  local rc=$?; echo "pmc $nm rc=$rc"; return $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE &&
pass tcc TCC_HIT_sum TCC_MISS_sum &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE
