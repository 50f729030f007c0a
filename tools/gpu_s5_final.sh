#!/bin/bash
# Round-2 session 5 evidence on HEAD's build: section clocks (FGX_STAMPS diagnostics build), PMC
# passes of the strong-scaling shard sizes (profiles/pmc_summary.json), then GPU tests, smoke, the
# bench line and the rocprofv3 kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAMP_RUNS="${STAMP_RUNS:-classic:65536 jl:8192 jl:32768}" bash tools/gpu_stamps.sh || exit $?
bash tools/gpu_pmc_r02.sh || exit $?
STAGES="${STAGES:-tests smoke bench prof}" bash tools/gpu_round.sh
