#!/bin/bash
# Round-3 session 12: counters of the SimpleReacher info_level=2 step's two kernels (the logging
# k_episode and k_info_obs): instruction mix and wave stall cycles, one rocprofv3 --pmc pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_s12
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_WR" \
           "WRITE_SIZE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_s12/g$i -o p -- \
    python3 tools/bench_kernels.py logsimple > gpurun_out/pmc_s12/g$i.log 2>&1; rc=$?
  echo "group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
