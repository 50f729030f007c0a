#!/bin/bash
# bench.py with the HIP-graph timed region vs eager launches, the rocprofv3 kernel stats of the
# graph run (its k_episode average must agree with the bench's roofline.kernel_ms), and a 2-rank
# rehearsal of the multi-GPU path on the one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
run() { local name=$1; shift; timeout -k 10 ${T:-600} "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/$name.log; ok $rc || exit $rc; }
run bench_graph python bench.py
run bench_eager python bench.py --no-graph --no-cpu-baseline
run prof_graph rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_graph -o run -- python3 bench.py --no-cpu-baseline
run bench_2rank python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3
exit 0
