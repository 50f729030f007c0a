#!/bin/bash
# Round-3 session 6: the GPU suite, the info_level=2 step (wave-walked NaN padding) with its kernel
# stats, and PMC passes of config 3 and of the two info_level=2 kernels (traffic, stalls, lanes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_kernels.py hole log > gpurun_out/hole_log.log 2>&1; rc=$?
grep '^{' gpurun_out/hole_log.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_log -o run -- \
  python3 tools/bench_kernels.py log > gpurun_out/prof_log.log 2>&1; rc=$?
head -3 gpurun_out/prof_log/run_kernel_stats.csv | cut -c1-160; [ $rc -eq 0 ] || exit $rc
CASES="65536_hole:fancy_ProDMP/HoleReacher-v0 65536_log:fancy_ProMP/LongSimpleReacher-v0 65536_holelog:fancy_ProDMP/HoleReacher-v0" \
  bash tools/gpu_pmc_r03.sh
