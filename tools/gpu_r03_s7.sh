#!/bin/bash
# Round-3 session 7: the GPU suite; the info_level=2 step (rows padded inside the sample loop) A/B
# against non-temporal info stores (tools/ab/libfgx_nt.so, FGX_INFO_NT) with WRITE_SIZE passes;
# the MFMA plan A/B (k_traj_mfma + k_episode<MP_GIVEN> vs the fused VALU contraction).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/log_ab.log
for i in 1 2; do
  for v in new nt; do
    lib=""; [ $v = nt ] && lib=$PWD/tools/ab/libfgx_nt.so
    FGX_LIB=$lib timeout -k 10 300 python -u tools/bench_kernels.py log | grep '^{' | sed "s/^/$v /" >> gpurun_out/log_ab.log || exit 1
  done
done
cat gpurun_out/log_ab.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_kernels.py mfmaab > gpurun_out/mfma_ab.log 2>&1; rc=$?
grep '^{' gpurun_out/mfma_ab.log; [ $rc -eq 0 ] || exit $rc
CASES="65536_log:fancy_ProMP/LongSimpleReacher-v0 65536_holelog:fancy_ProDMP/HoleReacher-v0" PARTS="fetch write stall" \
  OUT=gpurun_out/pmc_s7 bash tools/gpu_pmc_r03.sh
