cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for v in base ablobs abldyn; do
  FGX_LIB=exp/libfgx_$v.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r04s13_pmc_$v -o p -- python3 tools/bench_kernels.py logsimple > gpurun_out/r04s13_pmc_$v.log 2>&1 || exit $?
  echo "$v ok"
done
