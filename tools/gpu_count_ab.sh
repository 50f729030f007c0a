#!/bin/bash
# Is the device inner-step counter (one atomicAdd per wave on one address) visible in the kernel
# time?  jl shard sizes and the metric's k_episode, previous and in-tree library, with / without it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/count_ab.log
for i in 1 2; do
  for lib in prev new; do
    for cnt in 1 0; do
      if [ $lib = prev ]; then L=$PWD/tools/ab/libfgx_prev.so; else L=; fi
      if [ $cnt = 0 ]; then NC=1; else NC=; fi
      FGX_LIB=$L SCAN_NO_COUNT=$NC timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 jl 8192,16384,49152 | sed "s/^/$lib /" >> gpurun_out/count_ab.log || exit 1
      FGX_LIB=$L SCAN_NO_COUNT=$NC timeout -k 10 200 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 classic 65536 | sed "s/^/$lib /" >> gpurun_out/count_ab.log || exit 1
    done
  done
done
grep '{' gpurun_out/count_ab.log | python -c "
import sys, json
for l in sys.stdin:
    tag, js = l.split(' ', 1); d = json.loads(js); print(tag, d['envs'], d['kernel'], 'count' if d['counter'] else 'nocount', d['us_per_bb_step'])"
