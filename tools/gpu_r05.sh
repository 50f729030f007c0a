#!/bin/bash
# Round-5 GPU session: selected -m gpu tests, then tools/bench_kernels.py modes.  Outputs under
# gpurun_out/<TAG>_*; every GPU step under its own time limit; a fault / abort / timeout of the tests
# ends the session.  Usage: tools/gpu_r05.sh TAG "<pytest files / -k args>" "<bench_kernels modes>"
set -o pipefail
TAG=${1:-s}
TESTS=${2:-}
MODES=${3:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?
  tail -3 gpurun_out/${TAG}_pytest.log
  grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -30
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ -n "$MODES" ]; then
  timeout -k 10 600 python tools/bench_kernels.py $MODES > gpurun_out/${TAG}_kernels.jsonl 2> gpurun_out/${TAG}_kernels.err
  echo "kernels rc=$?"
  cut -c1-260 gpurun_out/${TAG}_kernels.jsonl
fi
exit ${rc:-0}
