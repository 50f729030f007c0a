#!/bin/bash
# k_episode_jl's reset wave (the auto-resets beside the joint waves instead of after the gather): the jl
# tests and every full-size config on the new build, then the shard sizes A/B against the previous
# build (tools/ab/libfgx_prev.so), alternated three times.  Outputs gpurun_out/${TAG:-r06d}_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_jl.py tests/test_gpu_jp.py tests/test_gpu_configs.py tests/test_gpu_dist.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG:-r06d}_tests.log 2>&1 \
  || { tail -40 gpurun_out/${TAG:-r06d}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG:-r06d}_tests.log
AB_A=tools/ab/libfgx_prev.so AB_B=fancy_gym_crowd_amd/libfgx.so AB_WHAT=shards bash tools/ab_libs.sh || exit $?
cp gpurun_out/ab.log gpurun_out/${TAG:-r06d}_ab.log
# the graph's inter-kernel gaps at the 8-GPU shard size (kernel trace of the bench's timed graph)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG:-r06d}_trace8192 -o t -- \
  python3 bench.py --global-envs 8192 --no-cpu-baseline --steps 50 > gpurun_out/${TAG:-r06d}_trace8192.log 2>&1 || exit $?
echo "trace ok"
