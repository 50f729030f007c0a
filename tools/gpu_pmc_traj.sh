#!/bin/bash
# k_traj_run's HBM traffic and kernel times: FETCH_SIZE and WRITE_SIZE passes and
# one kernel-trace pass over tools/bench_kernels.py trajrun1 (65536 envs: DMP LongSimpleReacher, DMP
# HoleReacher, ProMP LongSimpleReacher and ProDMP HoleReacher with replanning schedules).
# Output: gpurun_out/${TAG}_traj/{fetch,write,trace}/.  Summary: python tools/traj_pmc_summary.py DIR.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05}
OUT=gpurun_out/${TAG}_traj
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o p -- \
  python3 tools/bench_kernels.py trajrun1 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for part in fetch write; do
  grp=FETCH_SIZE; [ $part = write ] && grp=WRITE_SIZE
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/$part -o p -- \
    python3 tools/bench_kernels.py trajrun1 > $OUT/$part.log 2>&1
  rc=$?; echo "$part rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
