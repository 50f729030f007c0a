"""Summarise gpurun_out/ab_multi.log (tools/ab_multi.sh): kernel µs per (config, envs) and build."""
import collections
import json
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_multi.log"):
    tag, js = line.split(" ", 1)
    j = json.loads(js)
    d[(j["config"], j["envs"])][tag].append(j["kernel_us"])
for k in sorted(d):
    print(k, " | ".join(f"{t}: {min(v):.1f}-{max(v):.1f}" for t, v in sorted(d[k].items())))
