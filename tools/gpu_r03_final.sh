#!/bin/bash
# Round-3 final evidence on the committed build: the GPU suite and smoke, every PMC pass bench.py's
# roofline reads (tools/gpu_pmc_r03.sh: the strong-scaling shards 65536 / 32768 / 16384 / 8192,
# config 3, the info_level=2 steps, the basis GEMM's MFMA counters) summarised for this build, then
# the bench line (with the CPU baseline and the PMC-backed roofline), rocprofv3 kernel stats of the
# bench command, and the info_level=2 / shard kernel timings.
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGES="tests smoke" TEST_TIMEOUT=900 bash tools/gpu_r03.sh || exit $?
OUT=gpurun_out/pmc_r03 bash tools/gpu_pmc_r03.sh > gpurun_out/pmc_run.log 2>&1; rc=$?
tail -3 gpurun_out/pmc_run.log; [ $rc -eq 0 ] || exit $rc
python tools/pmc_summary.py gpurun_out/pmc_r03 --no-copy > gpurun_out/pmc_summary_run.log 2>&1 || exit 1
cp profiles/pmc_summary.json gpurun_out/pmc_summary_box.json
STAGES="bench prof" bash tools/gpu_r03.sh || exit $?
timeout -k 10 300 python -u tools/bench_kernels.py log shards > gpurun_out/kernels.log 2>&1 || exit 1
grep '^{' gpurun_out/kernels.log | cut -c1-250
# info_level=2 A/B against tools/ab/libfgx_prev.so (the previous build)
: > gpurun_out/abf.log
for i in 1 2; do
  for v in new prev; do
    lib=""; [ $v = prev ] && lib=$PWD/tools/ab/libfgx_prev.so
    FGX_LIB=$lib timeout -k 10 300 python -u tools/bench_kernels.py log > gpurun_out/abf_run.log 2>&1 || { tail -5 gpurun_out/abf_run.log; exit 1; }
    grep '^{' gpurun_out/abf_run.log | sed "s/^/$v /" >> gpurun_out/abf.log
  done
done
cut -c1-200 gpurun_out/abf.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_log -o log -- \
  python3 tools/bench_kernels.py log > gpurun_out/prof_log.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_WR \
  --output-format csv -d gpurun_out/pmc_logstall -o s -- python3 tools/bench_kernels.py logsimple > gpurun_out/pmc_logstall.log 2>&1 || exit 1
exit 0
