#!/bin/bash
# Round-3 session 17: section clocks of the final build's shard and metric kernels (FGX_STAMPS
# diagnostics variant, tools/ab/libfgx_stamps.so) and a second bench line of the final build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/stamps.log
STAMP_RUNS="jl:8192 jl:16384 classic:65536" bash tools/gpu_stamps.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench2.log 2>&1 || exit 1
grep '^{' gpurun_out/bench2.log | cut -c1-300
