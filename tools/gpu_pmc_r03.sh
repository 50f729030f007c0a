#!/bin/bash
# PMC passes for bench.py's roofline (profiles/pmc_summary.json via tools/pmc_summary.py): one
# rocprofv3 --pmc pass per counter group over `bench.py --env-id ID --global-envs N` for every case
# (the strong-scaling shard sizes of the metric, 65536 / G for G = 1, 2, 4, 8, and config 3); the
# 65536-env metric run also carries the basis-GEMM launch (k_traj_mfma) for the MFMA counters.
# Counter groups stay within one block's limits (<= 8 SQ, FETCH_SIZE 3 TCC, WRITE_SIZE 2 TCC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_r03
mkdir -p $OUT
METRIC=fancy_ProMP/LongSimpleReacher-v0
for case in ${CASES:-65536:$METRIC 32768:$METRIC 16384:$METRIC 8192:$METRIC 65536_hole:fancy_ProDMP/HoleReacher-v0}; do
  tag=${case%%:*}; env=${case#*:}; n=${tag%%_*}
  d=$OUT/n$tag
  mkdir -p $d
  echo "$env" > $d/workload.txt
  parts="fetch write issue busy mix"
  [ "$tag" = "65536" ] && parts="$parts mfma"
  for part in $parts; do
    case $part in
      fetch) grp="FETCH_SIZE" ;;
      write) grp="WRITE_SIZE" ;;
      issue) grp="SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE" ;;
      busy)  grp="VALUBusy" ;;
      mix)   grp="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64" ;;
      mfma)  grp="SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES" ;;
    esac
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $d/$part -o p -- \
      python3 bench.py --env-id $env --global-envs $n --steps 10 --warmup 2 --no-cpu-baseline > $d/$part.log 2>&1
    rc=$?
    echo "n=$tag $part rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
