#!/bin/bash
# k_episode_v2h storing waves' observation trigonometry (fgx_sincos_fast + f32 checks, exact fallback):
# the info-rows tests on the new build, then config 3's verbose-2 public step() A/B against the
# previous build (tools/ab/libfgx_prev.so), alternated three times.  Outputs gpurun_out/r06c_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_info_rows.py tests/test_gpu_edges.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06c_tests.log 2>&1 || { tail -30 gpurun_out/r06c_tests.log; exit 1; }
tail -1 gpurun_out/r06c_tests.log
AB_A=tools/ab/libfgx_prev.so AB_B=fancy_gym_crowd_amd/libfgx.so AB_WHAT=loghole bash tools/ab_libs.sh || exit $?
cp gpurun_out/ab.log gpurun_out/r06c_ab.log
