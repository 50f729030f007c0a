#!/bin/bash
# k_episode_jl producer / consumer A/B (round 3): the jl bit-identity tests with the PC form forced on,
# then forced-kernel scans of the metric workload at the strong-scaling shard sizes, alternating the
# previous library (tools/ab/libfgx_prev.so: jl before the reset waves), the in-tree library with
# FGX_JL_PC=0 (reset waves) and with FGX_JL_PC=1 (reset waves + producer waves).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FGX_JL_PC=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread ${AB_TESTS:+-k "$AB_TESTS"} > gpurun_out/jl_pc_tests.log 2>&1; rc=$?
tail -2 gpurun_out/jl_pc_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/jl_pc_ab.log
SIZES=${AB_SIZES:-8192,16384,32768,49152}
for i in 1 2; do
  FGX_LIB=$PWD/tools/ab/libfgx_prev.so timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 jl $SIZES | sed 's/^/prev /' >> gpurun_out/jl_pc_ab.log || exit 1
  FGX_JL_PC=0 timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 jl $SIZES | sed 's/^/rw /' >> gpurun_out/jl_pc_ab.log || exit 1
  FGX_JL_PC=1 timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 jl $SIZES | sed 's/^/pc /' >> gpurun_out/jl_pc_ab.log || exit 1
  FGX_LIB=$PWD/tools/ab/libfgx_prev.so timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProDMP/HoleReacher-v0 classic 65536 | sed 's/^/prev /' >> gpurun_out/jl_pc_ab.log || exit 1
  timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProDMP/HoleReacher-v0 classic 65536 | sed 's/^/new /' >> gpurun_out/jl_pc_ab.log || exit 1
done
grep '{' gpurun_out/jl_pc_ab.log | python -c "
import sys, json
for l in sys.stdin:
    tag, js = l.split(' ', 1); d = json.loads(js); print(tag, d['envs'], d['kernel'], d['us_per_bb_step'])"
