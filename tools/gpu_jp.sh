#!/bin/bash
# k_episode_jp vs k_episode: the whole GPU suite, then both kernels forced over the envs-per-GPU
# scans (tools/bench_kernels.py scan / scanmp) -> gpurun_out/scan_{jp,classic}.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 ${T:-600} "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
run gpu_tests python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
FGX_EPISODE_KERNEL=jp run scan_jp python tools/bench_kernels.py scan scanmp
FGX_EPISODE_KERNEL=classic run scan_classic python tools/bench_kernels.py scan scanmp
run kbench python tools/bench_kernels.py episode
exit 0
