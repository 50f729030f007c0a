#!/bin/bash
# Round-3 session 15: the public step() of the metric env at info_level 0 / 1 / 2 and the kernel
# stats of the same command (info_level 1 runs the logging kernel with two f64 rows per sample
# instead of the 2.2 GB of per-step arrays: what its stores cost).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_levels -o lv -- \
  python3 tools/bench_kernels.py levels > gpurun_out/levels.log 2>&1 || exit 1
grep '^{' gpurun_out/levels.log
