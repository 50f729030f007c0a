#!/bin/bash
# Issue-side PMC counters of the metric workload (tools/bench_kernels.py metric), one rocprofv3
# --pmc pass per group; OUT names the directory under gpurun_out/ (FGX_EPISODE_KERNEL selects).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in ${PMC_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT -o g$i -- python3 tools/bench_kernels.py metric > $OUT/g$i.log 2>&1; rc=$?
  echo "group $i ($grp) rc=$rc"; tail -2 $OUT/g$i.log
  [ $rc -ge 124 ] && exit $rc
done
exit 0
