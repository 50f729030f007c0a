#!/bin/bash
# k_episode_jl A/B (round 3): jl / config tests, then forced-kernel scans of the metric workload at
# the strong-scaling shard sizes, alternating the previous library (tools/ab/libfgx_prev.so) and the
# in-tree one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_jl.py tests/test_gpu_configs.py tests/test_gpu_ws.py tests/test_gpu_bench.py \
  tests/test_gpu_edges.py -x -q --timeout 300 --timeout-method thread > gpurun_out/jl_tests.log 2>&1; rc=$?
tail -2 gpurun_out/jl_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/jl_ab.log
SIZES=${AB_SIZES:-8192,16384,32768,49152}
for i in 1 2 3; do
  FGX_LIB=$PWD/tools/ab/libfgx_prev.so timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 jl $SIZES | sed 's/^/prev /' >> gpurun_out/jl_ab.log || exit 1
  timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 jl $SIZES | sed 's/^/new /' >> gpurun_out/jl_ab.log || exit 1
done
grep '{' gpurun_out/jl_ab.log | python -c "
import sys, json
for l in sys.stdin:
    tag, js = l.split(' ', 1); d = json.loads(js); print(tag, d['envs'], d['kernel'], d['us_per_bb_step'])"
