#!/bin/bash
# Config-3 ablations of k_episode_hp's consumer (tools/unit_variant.py builds under tools/ab/,
# FGX_HP_ONLY_CFG3): each library's config-3 step at 65536 / 32768 envs, alternated twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/hp_abl.log
for i in 1 2; do
  for v in ${HP_VARIANTS:-base fast noself nowall fastnoself nocons}; do
    FGX_LIB=$PWD/tools/ab/libfgx_hp_$v.so timeout -k 5 120 python tools/bench_kernels.py hp3 | sed "s/^/$v /" >> gpurun_out/hp_abl.log || exit 1
  done
done
cat gpurun_out/hp_abl.log
