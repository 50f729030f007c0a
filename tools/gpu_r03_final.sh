#!/bin/bash
# Round-3 final evidence on the committed build: the GPU suite, smoke, the bench line (with the CPU
# baseline), rocprofv3 kernel stats of the bench command, every PMC pass bench.py's roofline reads
# (tools/gpu_pmc_r03.sh: the strong-scaling shards 65536 / 32768 / 16384 / 8192, config 3, the
# info_level=2 steps, the basis GEMM's MFMA counters) and the info_level=2 step timings.
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGES="tests smoke bench prof" TEST_TIMEOUT=900 bash tools/gpu_r03.sh || exit $?
OUT=gpurun_out/pmc_r03 bash tools/gpu_pmc_r03.sh > gpurun_out/pmc_run.log 2>&1; rc=$?
tail -3 gpurun_out/pmc_run.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_kernels.py log shards > gpurun_out/kernels.log 2>&1 || exit 1
grep '^{' gpurun_out/kernels.log | cut -c1-250
