#!/bin/bash
# PMC passes of the round-6 final build: tools/gpu_pmc_r03.sh's cases (metric shard sizes, config 3, the
# verbose-2 steps, the basis GEMM) into gpurun_out/r06f_pmc, then k_traj_run's traffic
# (tools/gpu_pmc_traj.sh) into gpurun_out/r06f_traj.  Summaries: tools/pmc_summary.py / traj_pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06f_pmc bash tools/gpu_pmc_r03.sh || exit $?
bash tools/gpu_pmc_traj.sh r06f || exit $?
echo "pmc done"
