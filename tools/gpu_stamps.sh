#!/bin/bash
# Section clocks of the episode kernels from the FGX_STAMPS diagnostics build (tools/stamps.py).
# STAMP_RUNS: kernel:envs[:env_id] ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${STAMP_RUNS:-jl:8192 jl:65536 classic:8192 classic:65536}; do
  IFS=: read -r k n env <<< "$spec"
  env=${env:-fancy_ProMP/LongSimpleReacher-v0}
  FGX_LIB=$PWD/tools/ab/libfgx_stamps.so FGX_EPISODE_KERNEL=$k timeout -k 10 120 python tools/stamps.py $env $n >> gpurun_out/stamps.log 2>&1
  rc=$?; echo "$spec rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
tail -4 gpurun_out/stamps.log | cut -c1-900
