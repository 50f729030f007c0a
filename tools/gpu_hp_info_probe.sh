#!/bin/bash
# Where k_episode_hp's verbose-2 (INFO) launch spends its cycles: config 3's public step() at
# info_level 2 (tools/bench_kernels.py loghole) with FGX_HP=1 (k_episode_hp) and FGX_HP=0
# (k_episode_v2h): a kernel-trace pass and two SQ counter passes each.  Output gpurun_out/${TAG}_hpi/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06}
OUT=gpurun_out/${TAG}_hpi
mkdir -p $OUT
for hp in 1 0; do
  export FGX_HP=$hp
  d=$OUT/hp$hp
  mkdir -p $d
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o p -- \
    python3 tools/bench_kernels.py loghole > $d/trace.log 2>&1
  rc=$?; echo "hp=$hp trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for part in a b; do
    case $part in
      a) grp="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" ;;
      b) grp="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" ;;
    esac
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $d/$part -o p -- \
      python3 tools/bench_kernels.py loghole > $d/$part.log 2>&1
    rc=$?; echo "hp=$hp $part rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
