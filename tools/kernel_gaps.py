"""Inter-kernel gaps of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``): for the
launches of one kernel (name substring), the gap from each launch's end to the next launch's start on
the same queue, and the launch durations.  Used on the bench's timed HIP graph at the 8-GPU shard
size (tools/gpu_jl_rw_ab.sh), where consecutive BB steps are back-to-back graph nodes.

    python tools/kernel_gaps.py gpurun_out/r06d_trace8192 k_episode_jl
"""
import csv
import glob
import json
import os
import statistics
import sys


def trace_rows(path):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def gaps(rows, name):
    ks = [r for r in rows if name in r["Kernel_Name"]]
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks]
    # gaps between consecutive launches of any kernel that follow one of ours (graph order)
    allk = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    nxt = []
    for i, r in enumerate(allk[:-1]):
        if name in r["Kernel_Name"]:
            n = allk[i + 1]
            nxt.append((int(n["Start_Timestamp"]) - int(r["End_Timestamp"]), n["Kernel_Name"][:60]))
    return dur, nxt


def main():
    path, name = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_episode"
    dur, nxt = gaps(trace_rows(path), name)
    g = [x for x, _ in nxt]
    succ = {}
    for _, k in nxt:
        succ[k] = succ.get(k, 0) + 1
    # the timed graph: the longest run of back-to-back launches (gap < 20 us)
    out = dict(kernel=name, launches=len(dur), dur_us_median=statistics.median(dur) / 1e3 if dur else None,
               dur_us_min=min(dur) / 1e3 if dur else None,
               gap_us_median=statistics.median(g) / 1e3 if g else None,
               gap_us_p10=sorted(g)[len(g) // 10] / 1e3 if g else None,
               gap_us_p90=sorted(g)[(9 * len(g)) // 10] / 1e3 if g else None,
               gaps_below_20us=sum(1 for x in g if x < 20000), next_kernel=succ)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
