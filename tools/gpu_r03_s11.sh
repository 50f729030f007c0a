#!/bin/bash
# Round-3 session 11: the GPU suite on the k_info_obs build (SimpleReacher observation trigonometry of
# the logged rows at full occupancy), then the info_level=2 step A/B against tools/ab/libfgx_prev.so (the
# InfoStage build), the kernel stats of the logging kernels and their HBM write traffic (one --pmc pass each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab11.log
for i in 1 2; do
  for v in new prev; do
    lib=""; [ $v = prev ] && lib=$PWD/tools/ab/libfgx_prev.so
    FGX_LIB=$lib timeout -k 10 300 python -u tools/bench_kernels.py log > gpurun_out/ab11_run.log 2>&1 || { tail -5 gpurun_out/ab11_run.log; exit 1; }
    grep '^{' gpurun_out/ab11_run.log | sed "s/^/$v /" >> gpurun_out/ab11.log
  done
done
cut -c1-220 gpurun_out/ab11.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_log -o log -- \
  python3 tools/bench_kernels.py log > gpurun_out/prof_log.log 2>&1 || exit 1
for case in logsimple loghole; do
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_$case -o w -- \
    python3 tools/bench_kernels.py $case > gpurun_out/pmc_$case.log 2>&1 || exit 1
done
exit 0
