#!/bin/bash
# Round-3 session 4: A/B of the sincos / ProDMP-pair changes against their toggled-off variant builds,
# the HoleReacher cost split, the info_level=2 step, and the kernel stats of the latter.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SKIP_TESTS=1 SKIP_BENCH=1 ROUNDS=2 AB_LIBS="ocml=tools/ab/libfgx_ocml.so nopkd=tools/ab/libfgx_nopkd.so" \
  bash tools/gpu_r03_scan.sh || exit 1
timeout -k 10 400 python -u tools/bench_kernels.py hole log > gpurun_out/hole_log.log 2>&1; rc=$?
cat gpurun_out/hole_log.log | grep '^{'; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_log -o run -- \
  python3 tools/bench_kernels.py log > gpurun_out/prof_log.log 2>&1; rc=$?
head -6 gpurun_out/prof_log/run_kernel_stats.csv | cut -c1-220
exit $rc
