#!/bin/bash
# Round-3 session 8: the GPU suite; A/B of this build against tools/ab/libfgx_prev.so (the previous
# commit's library: runtime-slot pairwise pushes, 64-bit info-store addresses) on the info_level=2
# step, config 3 (k_episode forced) and the metric kernel; PMC issue / stall of the logging kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab8.log
for i in 1 2; do
  for v in new prev; do
    lib=""; [ $v = prev ] && lib=$PWD/tools/ab/libfgx_prev.so
    FGX_LIB=$lib timeout -k 10 300 python -u tools/bench_kernels.py log | grep '^{' | sed "s/^/$v /" >> gpurun_out/ab8.log || exit 1
    FGX_LIB=$lib timeout -k 10 300 python -u tools/kernel_scan.py fancy_ProDMP/HoleReacher-v0 classic 65536 | grep '^{' | sed "s/^/$v /" >> gpurun_out/ab8.log || exit 1
    FGX_LIB=$lib timeout -k 10 300 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 classic 65536 | grep '^{' | sed "s/^/$v /" >> gpurun_out/ab8.log || exit 1
  done
done
cut -c1-200 gpurun_out/ab8.log
CASES="65536_log:fancy_ProMP/LongSimpleReacher-v0 65536_holelog:fancy_ProDMP/HoleReacher-v0" PARTS="issue stall write" \
  OUT=gpurun_out/pmc_s8 bash tools/gpu_pmc_r03.sh
