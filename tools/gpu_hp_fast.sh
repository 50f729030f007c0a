#!/bin/bash
# k_episode_hp's approximate-FK consumers: the hp tests and config 3's full-batch check, then config 3
# timed against the previous consumer (tools/ab/libfgx_hp_base.so), alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_hp.py \
  "tests/test_gpu_configs.py::test_config3_full_batch_flags_and_lengths" \
  "tests/test_gpu_configs.py::test_config_full_size_vs_oracle_subset" -k "hp or config3" > gpurun_out/hp_fast_tests.log 2>&1
rc=$?
tail -5 gpurun_out/hp_fast_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/hp_fast_ab.log
for i in 1 2; do
  FGX_LIB=$PWD/tools/ab/libfgx_hp_base.so timeout -k 5 120 python tools/bench_kernels.py hp3 | sed "s/^/base /" >> gpurun_out/hp_fast_ab.log || exit 1
  timeout -k 5 120 python tools/bench_kernels.py hp3 | sed "s/^/new  /" >> gpurun_out/hp_fast_ab.log || exit 1
done
cat gpurun_out/hp_fast_ab.log
