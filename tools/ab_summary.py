"""Summarise gpurun_out/ab.log (tools/ab.sh): kernel µs per (config, envs, build)."""
import collections
import json
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    tag, js = line[:4].strip(), line[5:]
    j = json.loads(js)
    d[(j["config"], j["envs"])].append((tag, j.get("kernel_us", j.get("us_per_step"))))
for k in sorted(d):
    by = collections.defaultdict(list)
    for tag, us in d[k]:
        by[tag].append(us)
    print(k, " ".join(f"{t}: {min(v):.1f}-{max(v):.1f}" for t, v in sorted(by.items())))
