#!/bin/bash
# Round-6 GPU session: selected -m gpu tests, then tools/bench_kernels.py modes, then extra bench.py
# lines.  Outputs under gpurun_out/<TAG>_*; every GPU step under its own time limit; a fault / abort /
# timeout ends the session.
# Usage: tools/gpu_r06.sh TAG "<pytest files / -k args>" "<bench_kernels modes>" "<bench.py args;...>"
set -o pipefail
TAG=${1:-s}
TESTS=${2:-}
MODES=${3:-}
BENCHES=${4:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rc=0
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
  krc=$?
  echo "kernels rc=$krc"
  cut -c1-260 gpurun_out/${TAG}_kernels.jsonl
  if [ $krc -ne 0 ]; then tail -5 gpurun_out/${TAG}_kernels.err; exit $krc; fi
fi
if [ -n "$BENCHES" ]; then
  i=0
  IFS=';' read -ra BL <<< "$BENCHES"
  for b in "${BL[@]}"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py $b > gpurun_out/${TAG}_bench$i.json 2> gpurun_out/${TAG}_bench$i.err
    brc=$?
    echo "bench $i ($b) rc=$brc"
    cut -c1-400 gpurun_out/${TAG}_bench$i.json
    if [ $brc -ne 0 ]; then tail -5 gpurun_out/${TAG}_bench$i.err; exit $brc; fi
  done
fi
exit $rc
