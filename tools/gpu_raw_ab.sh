#!/bin/bash
# A/B of k_step_raw: the LDS-staged kernel (in-tree libfgx.so) vs round 1's per-lane AoS rows
# (tools/ab/libfgx_rawdirect.so = _build.build_variant(..., ["FGX_STEP_RAW_DIRECT"])): kernel time
# of every step id at 1M envs, then FETCH_SIZE / WRITE_SIZE passes of config 1 (SimpleReacher) for both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/raw_ab
mkdir -p $OUT
timeout -k 10 300 python tools/bench_kernels.py raw > $OUT/lds.jsonl 2> $OUT/lds.err || exit $?
FGX_LIB=tools/ab/libfgx_rawdirect.so timeout -k 10 300 python tools/bench_kernels.py raw > $OUT/direct.jsonl 2> $OUT/direct.err || exit $?
for v in lds direct; do
  lib=""; [ $v = direct ] && lib=tools/ab/libfgx_rawdirect.so
  for grp in FETCH_SIZE WRITE_SIZE; do
    FGX_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$v/$grp -o p -- \
      python3 tools/bench_kernels.py raw1 > $OUT/pmc_${v}_$grp.log 2>&1
    rc=$?; echo "pmc $v $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
cat $OUT/lds.jsonl $OUT/direct.jsonl
exit 0
