#!/bin/bash
# Round-3 session: the GPU suite, then A/B of the previous library (tools/ab/libfgx_prev.so, ABI 6)
# against the in-tree one over the configs the last changes touch (device counter spread over
# lines; ProDMP contraction on joint pairs; HoleReacher wall-check estimates), with the counter on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab2.log
M=fancy_ProMP/LongSimpleReacher-v0
for i in 1 2; do
  for lib in prev new; do
    if [ $lib = prev ]; then export FGX_LIB=$PWD/tools/ab/libfgx_prev.so FGX_LIB_ABI6=1; else unset FGX_LIB FGX_LIB_ABI6; fi
    timeout -k 10 200 python -u tools/kernel_scan.py $M classic 65536 | sed "s/^/$lib /" >> gpurun_out/ab2.log || exit 1
    timeout -k 10 200 python -u tools/kernel_scan.py $M jl 8192,16384,32768 | sed "s/^/$lib /" >> gpurun_out/ab2.log || exit 1
    timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProDMP/HoleReacher-v0 classic 65536 | sed "s/^/$lib /" >> gpurun_out/ab2.log || exit 1
    timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProDMP/LongSimpleReacher-v0 classic 65536 | sed "s/^/$lib /" >> gpurun_out/ab2.log || exit 1
    SCAN_OVER=replan25 timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProDMP/SimpleReacher-v0 jl,classic 8192 | sed "s/^/$lib /" >> gpurun_out/ab2.log || exit 1
  done
done
grep '{' gpurun_out/ab2.log | python -c "
import sys, json
for l in sys.stdin:
    tag, js = l.split(' ', 1); d = json.loads(js); print(tag, d['env'].split('/')[0][6:], d['envs'], d['kernel'], d['us_per_bb_step'])"
