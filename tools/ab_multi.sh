#!/bin/bash
# A/B/C of the metric kernel across library builds, alternated in one session
# (tools/bench_kernels.py metric; µs per BB step).  Usage: AB_LIBS="tools/ab/libfgx_x.so ..." tools/ab_multi.sh
# ("tree" = the in-tree library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab_multi.log
for i in 1 2 3; do
  for lib in tree ${AB_LIBS}; do
    if [ "$lib" = tree ]; then
      timeout -k 5 120 python tools/bench_kernels.py ${AB_WHAT:-metric} | sed "s|^|tree |" >> gpurun_out/ab_multi.log || exit 1
    else
      FGX_LIB=$PWD/$lib timeout -k 5 120 python tools/bench_kernels.py ${AB_WHAT:-metric} | sed "s|^|$(basename $lib) |" >> gpurun_out/ab_multi.log || exit 1
    fi
  done
done
