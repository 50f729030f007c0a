#!/bin/bash
# GPU session script: the whole -m gpu suite (no -x: every failure listed), then a default bench
# line.  Output under gpurun_out/<tag>_*.  Usage: tools/gpu_suite.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-s}
K=${2:-}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "${KARG[@]}" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest.log
grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -40
# a fault / abort / timeout ends the session here (no further GPU work)
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo "bench rc=$?"
cat gpurun_out/${TAG}_bench.json | cut -c1-600
# optional: per-kernel timings (tools/bench_kernels.py modes, e.g. "episode hole")
if [ -n "$3" ]; then
  timeout -k 10 400 python tools/bench_kernels.py $3 > gpurun_out/${TAG}_kernels.jsonl 2> gpurun_out/${TAG}_kernels.err
  echo "kernels rc=$?"
  cut -c1-300 gpurun_out/${TAG}_kernels.jsonl
fi
