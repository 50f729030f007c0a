#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out; : > gpurun_out/scan_all.log
run() { timeout -k 10 300 python -u tools/kernel_scan.py "$@" >> gpurun_out/scan_all.log 2>&1 || exit 1; }
run fancy_DMP/LongSimpleReacher-v0 classic,jp,jl 8192,16384,32768,65536
run fancy_ProDMP/LongSimpleReacher-v0 classic,jp,jl 8192,32768,65536
run fancy_ProMP/SimpleReacher-v0 classic,jp,ws,jl 4096,8192,32768,65536
run fancy_DMP/SimpleReacher-v0 classic,jp,ws,jl 8192,65536
SCAN_OVER=replan25 run fancy_ProDMP/SimpleReacher-v0 classic,jp,ws,jl 8192,65536
SCAN_OVER=replan25 run fancy_ProMP/LongSimpleReacher-v0 classic,jp,jl 8192,65536
grep '^{' gpurun_out/scan_all.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['env'], d['envs'], d['kernel'], d['us_per_bb_step'])"
