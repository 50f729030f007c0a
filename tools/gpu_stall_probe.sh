#!/bin/bash
# Where the episode kernels' cycles go (tools/bench_kernels.py probe: ProMP LongSimpleReacher at
# 65536 and 32768 envs) for each forced kernel: timing, then two rocprofv3 --pmc passes of SQ
# wave-state / instruction counters (each <= 8 SQ counters, one pass each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/stall
mkdir -p $OUT
for k in ${KERNELS:-classic jl}; do
  FGX_EPISODE_KERNEL=$k timeout -k 10 200 python tools/bench_kernels.py probe > $OUT/time_$k.jsonl 2> $OUT/time_$k.err || exit $?
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    FGX_EPISODE_KERNEL=$k timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/$k/g$i -o p -- \
      python3 tools/bench_kernels.py probe > $OUT/${k}_g$i.log 2>&1
    rc=$?; echo "$k g$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
cat $OUT/time_*.jsonl
exit 0
