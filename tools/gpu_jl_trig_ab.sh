#!/bin/bash
# k_episode_jl gather trigonometry variants, linked out of tree against the final build's other objects:
# A = the restated small-argument sincos (no -DFGX_OCML_SINCOS), B = the observation's cos / sin of q on the
# checked fast path, AB = both.  Bit-identity through the jl tests (jl vs k_episode in the same library),
# then the shard sizes against the in-tree library, alternated three times.  Output gpurun_out/r06j_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in A B AB; do
  FGX_LIB=$PWD/tools/ab/libfgx_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_jl.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06j_tests_$v.log 2>&1 \
    || { echo "tests $v failed"; tail -30 gpurun_out/r06j_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06j_tests_$v.log)"
done
: > gpurun_out/r06j_ab.log
for i in 1 2 3; do
  for v in prev A B AB; do
    lib=$PWD/fancy_gym_crowd_amd/libfgx.so; [ $v = prev ] || lib=$PWD/tools/ab/libfgx_$v.so
    FGX_LIB=$lib timeout -k 5 150 python tools/bench_kernels.py shards | sed "s/^/$(printf '%-4s' $v) /" >> gpurun_out/r06j_ab.log || exit 1
  done
done
python - <<'PY'
import collections, json
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/r06j_ab.log"):
    tag, js = l[:4].strip(), l[5:]
    j = json.loads(js); d[(j["config"], j["envs"])][tag].append(j["kernel_us"])
for k in sorted(d):
    print(k, " ".join(f"{t}: {min(v):.1f}-{max(v):.1f}" for t, v in sorted(d[k].items())))
PY
