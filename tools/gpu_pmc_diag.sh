#!/bin/bash
# Diagnostic PMC passes (one rocprofv3 --pmc pass per counter group, each under its own time limit)
# over one tools/bench_kernels.py mode: per-dispatch counters of every kernel it launches.
#   tools/gpu_pmc_diag.sh OUTDIR MODE [ENV=VAL ...]     e.g. tools/gpu_pmc_diag.sh gpurun_out/pmc_v2 logsimple
# Groups stay within one block's limits (<= 8 SQ, FETCH_SIZE 3 TCC, WRITE_SIZE 2 TCC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; MODE=$2; shift 2
mkdir -p $OUT
for part in ${PARTS:-write issue stall lds mix}; do
  case $part in
    fetch) grp="FETCH_SIZE" ;;
    write) grp="WRITE_SIZE" ;;
    issue) grp="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE" ;;
    stall) grp="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_WR" ;;
    lds)   grp="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_WAVE_CYCLES" ;;
    mix)   grp="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64" ;;
  esac
  env "$@" timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/$part -o p -- \
    python3 tools/bench_kernels.py $MODE > $OUT/$part.log 2>&1
  rc=$?
  echo "$OUT $part rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
