#!/bin/bash
# Round-3 session 19: bench.py --gpus 2 on the one-GPU box (rehearsal: both ranks on cuda:0, gloo) with
# the final build -- the driver's multi-GPU invocation, spawned by bench.py itself.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/dist2.log 2>&1 || { tail -20 gpurun_out/dist2.log; exit 1; }
grep '^{' gpurun_out/dist2.log | cut -c1-400
