#!/bin/bash
# Round-3 session 13: the GPU suite on the build whose InfoStage stores each array's rows from SGPR row bases
# (no LDS address table), the info_level=2 step A/B against tools/ab/libfgx_prev.so (the k_info_obs
# build), kernel stats and the stall counters of the logging kernel (one --pmc pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab13.log
for i in 1 2; do
  for v in new prev; do
    lib=""; [ $v = prev ] && lib=$PWD/tools/ab/libfgx_prev.so
    FGX_LIB=$lib timeout -k 10 300 python -u tools/bench_kernels.py log > gpurun_out/ab13_run.log 2>&1 || { tail -5 gpurun_out/ab13_run.log; exit 1; }
    grep '^{' gpurun_out/ab13_run.log | sed "s/^/$v /" >> gpurun_out/ab13.log
  done
done
cut -c1-220 gpurun_out/ab13.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_log -o log -- \
  python3 tools/bench_kernels.py log > gpurun_out/prof_log.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_WR \
  --output-format csv -d gpurun_out/pmc_s13 -o s -- python3 tools/bench_kernels.py logsimple > gpurun_out/pmc_s13.log 2>&1 || exit 1
exit 0
