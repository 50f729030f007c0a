#!/bin/bash
# k_traj_run DMP shape check + sweep (tools/gpu_dmp_shape.sh), then three more bench lines of the final build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_dmp_shape.sh || exit $?
bash tools/gpu_bench_repeats_r06.sh || exit $?
