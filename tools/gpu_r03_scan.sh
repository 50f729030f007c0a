#!/bin/bash
# Round-3 session: the GPU suite, the episode-kernel scan of the configs the latest changes touch
# (optionally A/B against variant libraries, AB_LIBS="name=path ..."), and the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1; rc=$?
  tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
: > gpurun_out/scan.log
M=fancy_ProMP/LongSimpleReacher-v0
scan() {   # tag
  timeout -k 10 200 python -u tools/kernel_scan.py $M classic 65536 | sed "s/^/$1 /" >> gpurun_out/scan.log || return 1
  timeout -k 10 200 python -u tools/kernel_scan.py $M jl 8192,16384,32768 | sed "s/^/$1 /" >> gpurun_out/scan.log || return 1
  timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProDMP/HoleReacher-v0 classic 65536 | sed "s/^/$1 /" >> gpurun_out/scan.log || return 1
  timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProDMP/LongSimpleReacher-v0 classic 65536 | sed "s/^/$1 /" >> gpurun_out/scan.log || return 1
  SCAN_OVER=replan25 timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProDMP/SimpleReacher-v0 jl 8192 | sed "s/^/$1 /" >> gpurun_out/scan.log || return 1
}
for i in $(seq ${ROUNDS:-1}); do
  scan new || exit 1
  for ab in $AB_LIBS; do
    FGX_LIB=$PWD/${ab#*=} scan ${ab%%=*} || exit 1
  done
done
grep '{' gpurun_out/scan.log | python -c "
import sys, json
for l in sys.stdin:
    tag, js = l.split(' ', 1); d = json.loads(js); print(tag, d['env'].split('/')[0][6:], d['env'].split('/')[1][:6], d['envs'], d['kernel'], d['us_per_bb_step'])"
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -c 600 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
fi
