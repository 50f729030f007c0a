#!/bin/bash
# Round-6 re-entry check of the current build: the whole -m gpu suite, smoke(), the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06b_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r06b_pytest.log
grep -E "FAILED|ERROR" gpurun_out/r06b_pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06b_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r06b_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err || exit $?
cut -c1-600 gpurun_out/r06b_bench.json
exit $rc
