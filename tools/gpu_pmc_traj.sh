#!/bin/bash
# PMC passes (one counter each) over the trajectory kernels (tools/bench_kernels.py traj).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_traj
export TMPDIR=/tmp
i=0
for ctr in ${PMC_CTRS:-WRITE_SIZE FETCH_SIZE VALUBusy MemUnitStalled TCC_EA0_WRREQ_64B TCC_EA0_WRREQ GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES}; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_traj -o c$i -- python3 tools/bench_kernels.py traj > gpurun_out/pmc_traj/c$i.log 2>&1; rc=$?
  echo "counter $ctr rc=$rc"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
