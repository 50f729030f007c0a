#!/bin/bash
# k_traj_run DMP shapes: bit-identity of the alternative shapes, then the shape sweep (bench_kernels dmpshape)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/dmp_shape_check.py > gpurun_out/r06h_dmp_check.log 2>&1 || { tail -20 gpurun_out/r06h_dmp_check.log; exit 1; }
tail -3 gpurun_out/r06h_dmp_check.log
timeout -k 10 300 python tools/bench_kernels.py dmpshape > gpurun_out/r06h_dmp_shapes.jsonl 2> gpurun_out/r06h_dmp_shapes.err || exit $?
python -c "
import json
for l in open('gpurun_out/r06h_dmp_shapes.jsonl'):
    d=json.loads(l); print(d['traj_ge'], d['traj_rc'], round(d['kernel_us'],1), round(d['GBps']))
"
