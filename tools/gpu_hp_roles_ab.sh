#!/bin/bash
# k_episode_hp role order by wave age (the SIMD's issue arbitration favours older waves): v1 = C0, C1, P,
# v2 = C1, C0, P (the kept build: P, C0, C1), linked out of tree against the final build's other objects.
# hp tests on each, then config 3 at 65536 / 32768 envs against the in-tree library, three alternations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in v1 v2; do
  FGX_LIB=$PWD/tools/ab/libfgx_hp$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_hp.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06k_tests_$v.log 2>&1 \
    || { echo "tests $v failed"; tail -30 gpurun_out/r06k_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06k_tests_$v.log)"
done
: > gpurun_out/r06k_ab.log
for i in 1 2 3; do
  for v in prev v1 v2; do
    lib=$PWD/fancy_gym_crowd_amd/libfgx.so; [ $v = prev ] || lib=$PWD/tools/ab/libfgx_hp$v.so
    FGX_LIB=$lib timeout -k 5 150 python tools/bench_kernels.py config3 | sed "s/^/$(printf '%-4s' $v) /" >> gpurun_out/r06k_ab.log || exit 1
  done
done
python - <<'PY'
import collections, json
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/r06k_ab.log"):
    tag, js = l[:4].strip(), l[5:]
    j = json.loads(js); d[(j["config"], j["envs"])][tag].append(j["kernel_us"])
for k in sorted(d):
    print(k, " ".join(f"{t}: {min(v):.1f}-{max(v):.1f}" for t, v in sorted(d[k].items())))
PY
