#!/bin/bash
# Full default bench (with cpu_baseline) + a 2-rank rehearsal of the multi-GPU path on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_full.log
ok $rc || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_2rank.log 2>&1; rc=$?; echo "bench2 rc=$rc"; tail -2 gpurun_out/bench_2rank.log
exit $rc
