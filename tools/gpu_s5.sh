#!/bin/bash
# Round-2 session 5: A/B of the scalar-cache warm-up (tools/ab/libfgx_prev.so = the build before it)
# over the metric's strong-scaling shards and configs 2/4/5, SQ wave-state counters of k_episode on
# the new build, then the round stages (GPU tests, smoke, bench, rocprofv3 kernel stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_WHAT=shards bash tools/ab.sh || exit $?
python tools/ab_summary.py gpurun_out/ab.log
KERNELS=${PROBE_KERNELS:-classic} bash tools/gpu_stall_probe.sh || exit $?
STAGES="${STAGES:-tests smoke bench prof}" bash tools/gpu_round.sh
