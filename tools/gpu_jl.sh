#!/bin/bash
# k_episode_jl bring-up: its parity tests, then the kernel scan over the strong-scaling shard sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jl.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/jl_tests.log 2>&1
rc=$?; echo "jl tests rc=$rc"; tail -5 gpurun_out/jl_tests.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kernel_scan.py fancy_ProMP/LongSimpleReacher-v0 classic,jp,jl 8192,16384,32768,65536 > gpurun_out/jl_scan.log 2>&1
rc=$?; echo "scan rc=$rc"; cat gpurun_out/jl_scan.log | cut -c1-300
exit $rc
