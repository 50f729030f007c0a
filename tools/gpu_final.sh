#!/bin/bash
# Round evidence on the current build: bench line (with CPU baseline), rocprofv3 kernel stats of the
# same command, PMC HBM traffic (FETCH_SIZE, WRITE_SIZE) and issue counters of the metric kernel,
# each rocprofv3 --pmc group in its own pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 ${T:-600} "$@" > gpurun_out/final/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/final/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run bench python bench.py
run prof rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o bench -- python3 bench.py --no-cpu-baseline
run pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/final/pmc_hbm -o fetch -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
run pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/final/pmc_hbm -o write -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT" "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F64" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE" "VALUBusy" "VALUUtilization"; do
  i=$((i+1))
  T=180 run pmc_issue$i rocprofv3 --pmc $grp --output-format csv -d gpurun_out/final/pmc_issue -o g$i -- python3 tools/bench_kernels.py metric
done
exit 0
