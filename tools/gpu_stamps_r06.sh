#!/bin/bash
# Section clocks of k_episode_jl at the 8-GPU shard (8192 envs) with the reset wave (default) and without
# (FGX_JL_RW=0), and at 16384 envs, from the FGX_STAMPS variant of the final build (tools/ab/libfgx_stamps.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06i_stamps.jsonl
for spec in 1:8192 0:8192 1:8192 0:8192 auto:16384; do
  IFS=: read -r rw n <<< "$spec"
  if [ "$rw" = auto ]; then unset FGX_JL_RW; else export FGX_JL_RW=$rw; fi
  FGX_LIB=$PWD/tools/ab/libfgx_stamps.so FGX_EPISODE_KERNEL=jl timeout -k 10 120 python tools/stamps.py \
    fancy_ProMP/LongSimpleReacher-v0 $n > gpurun_out/r06i_one.json 2> gpurun_out/r06i_stamps.err
  rc=$?; echo "$spec rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open('gpurun_out/r06i_one.json')); d['FGX_JL_RW']='$rw'; print(json.dumps(d))" >> gpurun_out/r06i_stamps.jsonl
done
python -c "
import json
for l in open('gpurun_out/r06i_stamps.jsonl'):
    d=json.loads(l); print(d['FGX_JL_RW'], d['envs'], d['kernel_us_events'], d['wave_total_median'], d['total_cycles_pctl'], d['cycles_median'], d['slowest10pct_cycles_median'])
"
