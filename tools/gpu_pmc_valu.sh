#!/bin/bash
# Issue-side PMC counters of the metric kernel (one rocprofv3 --pmc pass per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_valu
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_valu/avail.txt 2>&1; rc=$?
echo "list rc=$rc"; [ $rc -ge 124 ] && exit $rc
i=0
for grp in ${PMC_GROUPS:-"SQ_WAVES SQ_INSTS_VALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_ANY SQ_WAIT_ANY" "GRBM_GUI_ACTIVE SQ_INSTS_SALU" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64" "SQ_INSTS_LDS SQ_INST_CYCLES_VALU"}; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_valu -o g$i -- python3 tools/bench_kernels.py metric > gpurun_out/pmc_valu/g$i.log 2>&1; rc=$?
  echo "group $i ($grp) rc=$rc"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
