#!/bin/bash
# PMC passes of config 3 (65536 envs) for several library builds (LIBS: name=path relative to the repo;
# "intree" = the in-tree library).  Output: gpurun_out/${TAG}_pmc/<name>/<pass>/.  One --pmc pass per group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-libs}
OUT=gpurun_out/${TAG}_pmc
mkdir -p $OUT
for spec in ${LIBS:-intree}; do
  name=${spec%%=*}; path=${spec#*=}
  if [ "$name" = intree ]; then unset FGX_LIB; else export FGX_LIB=$PWD/$path; fi
  for part in ${PARTS:-issue mix icache}; do
    case $part in
      issue) grp="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" ;;
      mix)   grp="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU" ;;
      icache) grp="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" ;;
      ifetch) grp="SQ_IFETCH SQ_INSTS SQ_INSTS_BRANCH SQ_INSTS_SMEM" ;;
    esac
    d=$OUT/$name/$part
    mkdir -p $d
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $d -o p -- \
      python3 bench.py --env-id fancy_ProDMP/HoleReacher-v0 --global-envs 65536 --steps 5 --warmup 1 --no-cpu-baseline > $d.log 2>&1
    rc=$?
    echo "$name $part rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
