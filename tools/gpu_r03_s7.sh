#!/bin/bash
# Round-3 session 7: the new pair-kernel tests first, then the GPU suite; HoleReacher k_episode_pair vs
# k_episode (config 3 and sizes around it); the info_level=2 step (rows padded inside the sample loop)
# A/B against non-temporal info stores (tools/ab/libfgx_nt.so, FGX_INFO_NT); the MFMA plan A/B
# (k_traj_mfma + k_episode<MP_GIVEN> vs the fused VALU contraction); PMC of the pair kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pair_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pair_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/pair_scan.log
H=fancy_ProDMP/HoleReacher-v0
for i in 1 2; do
  timeout -k 10 300 python -u tools/kernel_scan.py $H pair,classic 16384,32768,65536,131072 >> gpurun_out/pair_scan.log || exit 1
done
grep '^{' gpurun_out/pair_scan.log | cut -c1-200
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
cut -c1-200 gpurun_out/log_ab.log
timeout -k 10 300 python -u tools/bench_kernels.py mfmaab > gpurun_out/mfma_ab.log 2>&1; rc=$?
grep '^{' gpurun_out/mfma_ab.log; [ $rc -eq 0 ] || exit $rc
CASES="65536_hole:$H 65536_log:fancy_ProMP/LongSimpleReacher-v0 65536_holelog:$H" PARTS="fetch write issue stall" \
  OUT=gpurun_out/pmc_s7 bash tools/gpu_pmc_r03.sh
