#!/bin/bash
# Kernel benchmarks + rocprofv3 kernel stats and PMC HBM counters (separate passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_pmc
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
run() { local name=$1; shift; timeout -k 10 ${T:-400} "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; ok $rc || exit $rc; }
run kbench python tools/bench_kernels.py ${KB:-episode traj raw}
run prof_kern rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kern -o k -- python3 tools/bench_kernels.py ${KB:-episode traj raw}
run pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_pmc -o fetch -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
run pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_pmc -o write -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
exit 0
