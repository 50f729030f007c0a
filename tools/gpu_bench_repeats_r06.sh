#!/bin/bash
# Three more default bench lines of the final build (box-to-box / run-to-run spread of the metric).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/r06g_bench_repeats.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline >> gpurun_out/r06g_bench_repeats.jsonl 2> gpurun_out/r06g_bench_$i.err || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/r06g_bench_repeats.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])
PY
