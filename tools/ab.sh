#!/bin/bash
# A/B of the metric kernel: tools/ab/libfgx_prev.so (FGX_LIB) against the in-tree library,
# alternated in one session (tools/bench_kernels.py metric; µs per BB step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.log
for i in 1 2 3; do
  FGX_LIB=$PWD/tools/ab/libfgx_prev.so timeout -k 5 120 python tools/bench_kernels.py ${AB_WHAT:-metric} | sed 's/^/prev /' >> gpurun_out/ab.log || exit 1
  timeout -k 5 120 python tools/bench_kernels.py ${AB_WHAT:-metric} | sed 's/^/new  /' >> gpurun_out/ab.log || exit 1
done
