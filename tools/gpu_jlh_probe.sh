#!/bin/bash
# k_episode_jl's helper form (FGX_JL_HELPER=1/2) against the plain joint-lane kernel at the 8-GPU shard
# size (8192 envs): section clocks of the joint waves (FGX_STAMPS build, tools/stamps.py) and one PMC
# pass of issue counters per variant.  Output: gpurun_out/${TAG}_jlh/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05}
OUT=gpurun_out/${TAG}_jlh
mkdir -p $OUT
for h in 0 1 2; do
  FGX_LIB=$PWD/tools/ab/libfgx_stamps.so FGX_EPISODE_KERNEL=jl FGX_JL_HELPER=$h timeout -k 10 120 \
    python tools/stamps.py fancy_ProMP/LongSimpleReacher-v0 8192 > $OUT/stamps_h$h.json 2> $OUT/stamps_h$h.err
  rc=$?; echo "stamps h=$h rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for h in 0 1; do
  d=$OUT/pmc_h$h
  mkdir -p $d
  FGX_EPISODE_KERNEL=jl FGX_JL_HELPER=$h timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $d -o p -- \
    python3 bench.py --env-id fancy_ProMP/LongSimpleReacher-v0 --global-envs 8192 --steps 10 --warmup 2 --no-cpu-baseline \
    > $d.log 2>&1
  rc=$?; echo "pmc h=$h rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
