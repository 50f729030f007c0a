#!/bin/bash
# Round-3 session 9 (re-entry): the GPU suite, smoke, bench line and rocprofv3 kernel stats of this
# build, plus the info_level=2 step timings and the torch write / copy rates of the box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGES="tests smoke bench prof" bash tools/gpu_r03.sh || exit $?
timeout -k 10 300 python -u tools/bench_kernels.py bw log > gpurun_out/logbw.log 2>&1 || exit $?
cut -c1-300 gpurun_out/logbw.log
