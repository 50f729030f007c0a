#!/bin/bash
# k_episode_jl after a change: its bit-identity tests, a forced-kernel scan of the metric env and
# of the other 5-link / 2-link workloads, then the SQ stall counters of the probe sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_jl.py tests/test_gpu_configs.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/jl_tests.log 2>&1; rc=$?; tail -2 gpurun_out/jl_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/jl_scan.log
run() { timeout -k 10 300 python -u tools/kernel_scan.py "$@" >> gpurun_out/jl_scan.log 2>&1 || exit 1; }
run fancy_ProMP/LongSimpleReacher-v0 classic,jl 8192,16384,32768,49152,65536,98304,131072
run fancy_DMP/LongSimpleReacher-v0 classic,jp,jl 32768,65536
run fancy_ProDMP/LongSimpleReacher-v0 classic,jl 32768,65536
run fancy_ProMP/SimpleReacher-v0 classic,jl 4096,65536
grep '^{' gpurun_out/jl_scan.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['env'], d['envs'], d['kernel'], d['us_per_bb_step'])"
KERNELS=jl bash tools/gpu_stall_probe.sh
