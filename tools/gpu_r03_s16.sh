#!/bin/bash
# Round-3 session 16: the GPU suite on the build with DPP wave reductions and the jl state loads
# issued ahead of the segment; the shard kernels A/B against tools/ab/libfgx_prev.so (the final-evidence
# build 7b93bf80), three alternations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab16.log
for i in 1 2 3; do
  for v in new prev; do
    lib=""; [ $v = prev ] && lib=$PWD/tools/ab/libfgx_prev.so
    FGX_LIB=$lib timeout -k 10 300 python -u tools/bench_kernels.py shards > gpurun_out/ab16_run.log 2>&1 || { tail -5 gpurun_out/ab16_run.log; exit 1; }
    grep '^{' gpurun_out/ab16_run.log | sed "s/^/$v /" >> gpurun_out/ab16.log
  done
done
cut -c1-160 gpurun_out/ab16.log
exit 0
