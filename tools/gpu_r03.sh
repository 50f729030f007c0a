#!/bin/bash
# Round-3 GPU session: counter list, parity tests, smoke, bench line, rocprof kernel stats.
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES="${STAGES:-list tests smoke bench prof}"
for st in $STAGES; do
  case $st in
    list)  timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1; rc=$?
           grep -o "SQ_INSTS_VALU[A-Z0-9_]*\|SQ_INSTS_[A-Z0-9_]*\|SQ_VALU_MFMA[A-Z0-9_]*" gpurun_out/avail.txt | sort -u > gpurun_out/sq_counters.txt || true ;;
    tests) timeout -k 10 ${TEST_TIMEOUT:-1100} python -u -m pytest tests -v -m gpu --maxfail=10 --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$? ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$? ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$? ;;
    stamps) STAMP_RUNS="${STAMP_RUNS:-jl:8192 jl:16384 classic:65536}" bash tools/gpu_stamps.sh > gpurun_out/stamps_run.log 2>&1; rc=$? ;;
    prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$? ;;
    *) echo "unknown stage $st"; rc=2 ;;
  esac
  echo "stage $st rc=$rc"
  tail -3 gpurun_out/*${st}*.log 2>/dev/null | tail -4 | cut -c1-600
  [ $rc -eq 0 ] || { echo "stopping after stage $st (rc=$rc)"; exit $rc; }
done
exit 0
