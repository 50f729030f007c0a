#!/bin/bash
# PMC passes for bench.py's roofline (profiles/pmc_summary.json via tools/pmc_summary.py): one
# rocprofv3 --pmc pass per counter group over `bench.py --env-id ID --global-envs N` for every case
# (the strong-scaling shard sizes of the metric, 65536 / G for G = 1, 2, 4, 8, config 3, and the
# info_level=2 step of the metric env and of config 3); the
# 65536-env metric run also carries the basis-GEMM launch (k_traj_mfma) for the MFMA counters.
# Counter groups stay within one block's limits (<= 8 SQ, FETCH_SIZE 3 TCC, WRITE_SIZE 2 TCC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_r03}
mkdir -p $OUT
METRIC=fancy_ProMP/LongSimpleReacher-v0
# a tag ending in _log runs the info_level=2 step (tools/bench_kernels.py log{simple,hole}) instead
for case in ${CASES:-65536:$METRIC 32768:$METRIC 16384:$METRIC 8192:$METRIC 65536_hole:fancy_ProDMP/HoleReacher-v0 65536_log:$METRIC 65536_holelog:fancy_ProDMP/HoleReacher-v0}; do
  tag=${case%%:*}; env=${case#*:}; n=${tag%%_*}
  d=$OUT/n$tag
  mkdir -p $d
  echo "$env" > $d/workload.txt
  parts=${PARTS:-fetch write issue busy mix stall}
  [ "$tag" = "65536" ] && [ -z "$PARTS" ] && parts="$parts mfma"
  cmd="bench.py --env-id $env --global-envs $n --steps 10 --warmup 2 --no-cpu-baseline"
  case $tag in
    *holelog) cmd="tools/bench_kernels.py loghole"; parts=${PARTS:-fetch write stall} ;;
    *log) cmd="tools/bench_kernels.py logsimple"; parts=${PARTS:-fetch write stall} ;;
  esac
  for part in $parts; do
    case $part in
      fetch) grp="FETCH_SIZE" ;;
      write) grp="WRITE_SIZE" ;;
      issue) grp="SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE" ;;
      busy)  grp="VALUBusy" ;;
      mix)   grp="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64" ;;
      mfma)  grp="SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES" ;;
      stall) grp="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_WR" ;;
    esac
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $d/$part -o p -- \
      python3 $cmd > $d/$part.log 2>&1
    rc=$?
    echo "n=$tag $part rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
