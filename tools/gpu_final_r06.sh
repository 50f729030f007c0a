#!/bin/bash
# Round-6 evidence session on the final build: the whole -m gpu suite, smoke(), the default bench
# line (its roofline reads profiles/pmc_summary.json of this build), the 8192-env shard through the
# one-rank RCCL branch (per-step return gather), and the rocprofv3 kernel-trace summaries of the bench
# command, the verbose-2 steps and config 3.  Outputs under gpurun_out/r06f_*; each GPU step under its
# own time limit, a fault / abort / timeout ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06f_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r06f_pytest.log
grep -E "FAILED|ERROR" gpurun_out/r06f_pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06f_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r06f_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06f_bench.json 2> gpurun_out/r06f_bench.err || exit $?
cut -c1-400 gpurun_out/r06f_bench.json
timeout -k 10 300 python bench.py --force-dist --no-cpu-baseline --global-envs 8192 --steps 50 \
  > gpurun_out/r06f_bench_rccl8192.json 2> gpurun_out/r06f_bench_rccl8192.err || exit $?
timeout -k 10 300 python bench.py --force-dist --no-cpu-baseline --steps 50 \
  > gpurun_out/r06f_bench_rccl65536.json 2> gpurun_out/r06f_bench_rccl65536.err || exit $?
echo "rccl benches ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06f_rocprof -o bench -- \
  python3 bench.py --no-cpu-baseline > gpurun_out/r06f_rocprof.log 2>&1 || exit $?
echo "rocprof ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06f_rocprof_log -o log -- \
  python3 tools/bench_kernels.py logsimple levels > gpurun_out/r06f_rocprof_log.log 2>&1 || exit $?
echo "rocprof log ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06f_rocprof_hp -o hp -- \
  python3 bench.py --env-id fancy_ProDMP/HoleReacher-v0 --global-envs 65536 --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r06f_rocprof_hp.log 2>&1 || exit $?
echo "rocprof hp ok"
timeout -k 10 600 python tools/bench_kernels.py shards hpinfo > gpurun_out/r06f_kernels.jsonl 2> gpurun_out/r06f_kernels.err || exit $?
echo "kernels ok"
exit $rc
