#!/bin/bash
# k_episode_ws session: ws-vs-classic equality tests, then the three kernels forced over the scans.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 ${T:-600} "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
run ws_tests python -u -m pytest tests/test_gpu_ws.py -x -v -m gpu --timeout 120 --timeout-method thread
FGX_EPISODE_KERNEL=ws run scan_ws python tools/bench_kernels.py ${SCANS:-scan scanmp}
exit 0
