#!/bin/bash
# PMC passes of config 3 (fancy_ProDMP/HoleReacher-v0, 65536 envs): k_episode_hp against k_episode
# (FGX_EPISODE_KERNEL=classic).  Output: gpurun_out/${TAG}_pmc/<variant>/<pass>/.  One --pmc pass per group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05hp}
OUT=gpurun_out/${TAG}_pmc
mkdir -p $OUT
for variant in ${VARIANTS:-hp classic}; do
  if [ "$variant" = classic ]; then export FGX_EPISODE_KERNEL=classic; else unset FGX_EPISODE_KERNEL; fi
  for part in ${PARTS:-issue mix}; do
    case $part in
      issue) grp="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" ;;
      mix)   grp="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU" ;;
      icache) grp="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" ;;
      ifetch) grp="SQ_IFETCH SQ_INSTS SQ_INSTS_BRANCH SQ_INSTS_SMEM" ;;
      hbm)   grp="FETCH_SIZE" ;;
      wr)    grp="WRITE_SIZE" ;;
    esac
    d=$OUT/$variant/$part
    mkdir -p $d
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $d -o p -- \
      python3 bench.py --env-id fancy_ProDMP/HoleReacher-v0 --global-envs 65536 --steps 5 --warmup 1 --no-cpu-baseline > $d.log 2>&1
    rc=$?
    echo "$variant $part rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
