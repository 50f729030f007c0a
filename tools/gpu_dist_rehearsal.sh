#!/bin/bash
# bench.py --gpus 2 through torch.distributed.run on a 1-GPU box: rehearsal mode (both ranks on
# cuda:0, gloo collectives) exercises the sharding, barriers, max-over-ranks timing and the
# return gather of the multi-GPU path (strong scaling: the 65536 global envs split 32768 per rank,
# plus the secondary weak-scaling leg at 65536 per rank).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dist2.log 2>&1
rc=$?; echo "dist2 rc=$rc"; grep '^{' gpurun_out/dist2.log | cut -c1-400; exit $rc
