#!/bin/bash
# Round-3 session 18: where the SimpleReacher logging kernel's wait cycles go -- the counter list of
# the box, then one --pmc pass per group of the available LDS / scalar-memory / vector-memory wait
# counters over tools/bench_kernels.py logsimple (final build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_s18
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_s18/avail.txt 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  ok=""
  for c in $grp; do grep -qw "$c" gpurun_out/pmc_s18/avail.txt && ok="$ok $c"; done
  echo "group $i: $ok"
  [ -z "$ok" ] && continue
  timeout -s KILL 150 rocprofv3 --pmc $ok --output-format csv -d gpurun_out/pmc_s18/g$i -o p -- \
    python3 tools/bench_kernels.py logsimple > gpurun_out/pmc_s18/g$i.log 2>&1; rc=$?
  echo "group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
