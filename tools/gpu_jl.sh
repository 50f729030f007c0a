#!/bin/bash
# k_episode_jl bring-up: its parity tests, then the kernel scan over the strong-scaling shard sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jl.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/jl_tests.log 2>&1
rc=$?; echo "jl tests rc=$rc"; tail -3 gpurun_out/jl_tests.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/jl_scan.log
timeout -k 10 300 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 ${SCAN_KERNELS:-jp,jl} ${SCAN_SIZES:-8192,16384,32768,65536} >> gpurun_out/jl_scan.log 2>&1
rc=$?; echo "scan rc=$rc"; [ $rc -eq 0 ] || exit $rc
for gw in ${GW_SWEEP:-}; do
  FGX_JL_GW=$gw timeout -k 10 120 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 jl ${GW_SIZES:-8192,16384} | sed "s/^{/{\"gw\": $gw, /" >> gpurun_out/jl_scan.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
done
grep '^{' gpurun_out/jl_scan.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('gw', '-'), d['envs'], d['kernel'], d['us_per_bb_step'])"
