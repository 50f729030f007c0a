#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprof kernel stats.
# Stops at the first GPU fault / abort / segfault / timeout (rc not in {0,1}).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
STAGES="${STAGES:-tests smoke bench prof}"
for st in $STAGES; do
  case $st in
    tests) timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$? ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$? ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$? ;;
    prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$? ;;
    kbench) timeout -k 10 600 python tools/bench_kernels.py episode traj raw > gpurun_out/kbench.log 2>&1; rc=$? ;;
    *) echo "unknown stage $st"; rc=2 ;;
  esac
  echo "stage $st rc=$rc"
  tail -3 gpurun_out/*${st}*.log 2>/dev/null | tail -4 | cut -c1-400
  ok $rc || { echo "stopping after stage $st (rc=$rc)"; exit $rc; }
  [ $rc -eq 0 ] || { echo "stage $st failed"; exit 1; }
done
exit 0
