#!/bin/bash
# A/B of two library builds, both loaded through FGX_LIB (AB_A, AB_B: paths relative to the repo),
# alternated three times in one session (tools/bench_kernels.py ${AB_WHAT:-metric}; µs per BB step).
# Summary: python tools/ab_summary.py gpurun_out/ab.log ("prev" = AB_A, "new" = AB_B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.log
for i in 1 2 3; do
  FGX_LIB=$PWD/${AB_A:-tools/ab/libfgx_prev.so} timeout -k 5 150 python tools/bench_kernels.py ${AB_WHAT:-metric} | sed 's/^/prev /' >> gpurun_out/ab.log || exit 1
  FGX_LIB=$PWD/$AB_B timeout -k 5 150 python tools/bench_kernels.py ${AB_WHAT:-metric} | sed 's/^/new  /' >> gpurun_out/ab.log || exit 1
done
python tools/ab_summary.py gpurun_out/ab.log
