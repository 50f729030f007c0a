#!/bin/bash
# Round-3 session 5: the GPU suite, the kernel scan, the HoleReacher split and the info_level=2 step
# with its kernel stats (component-major per-step arrays).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SKIP_BENCH=1 bash tools/gpu_r03_scan.sh || exit 1
timeout -k 10 400 python -u tools/bench_kernels.py hole log > gpurun_out/hole_log.log 2>&1; rc=$?
grep '^{' gpurun_out/hole_log.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_log -o run -- \
  python3 tools/bench_kernels.py log > gpurun_out/prof_log.log 2>&1; rc=$?
head -4 gpurun_out/prof_log/run_kernel_stats.csv | cut -c1-160
exit $rc
