#!/bin/bash
# jl tests on the in-tree build, then the metric env's forced-kernel scan on the in-tree build and on
# the amdgpu_waves_per_eu(4) variant of k_episode_jl (tools/ab/libfgx_jlw4.so, 128 VGPRs + spills).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_jl.py tests/test_gpu_ws.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/jl_tests.log 2>&1; rc=$?; tail -2 gpurun_out/jl_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/jlw4_scan.log
run() { timeout -k 10 300 python -u tools/kernel_scan.py "$@" >> gpurun_out/jlw4_scan.log 2>&1 || exit 1; }
run fancy_ProMP/LongSimpleReacher-v0 classic,jp,jl 8192,32768,65536,98304
FGX_LIB=tools/ab/libfgx_jlw4.so run fancy_ProMP/LongSimpleReacher-v0 jl 8192,32768,49152,65536,98304
FGX_LIB=tools/ab/libfgx_jlw4.so run fancy_ProMP/SimpleReacher-v0 jl 4096,65536
run fancy_ProMP/SimpleReacher-v0 jl 4096,65536
grep '^{' gpurun_out/jlw4_scan.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['env'], d['envs'], d['kernel'], d['us_per_bb_step'])"
