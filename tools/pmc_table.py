"""Per-dispatch medians of rocprofv3 --pmc counters for kernels matching a substring.

  python tools/pmc_table.py gpurun_out/pmc_jp k_episode_jp [gpurun_out/pmc_classic k_episode<]
"""
import collections
import csv
import glob
import os
import sys


def table(src, pat):
    vals, durs = collections.defaultdict(list), []
    for path in sorted(glob.glob(os.path.join(src, "*_counter_collection.csv"))):
        agg, dur = collections.defaultdict(float), {}
        for r in csv.DictReader(open(path)):
            if pat not in r["Kernel_Name"]:
                continue
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (d, c), v in agg.items():
            vals[c].append(v)
        durs += list(dur.values())
    med = {c: sorted(v)[len(v) // 2] for c, v in vals.items()}
    return med, (sorted(durs)[len(durs) // 2] if durs else None)


if __name__ == "__main__":
    args = sys.argv[1:]
    for src, pat in zip(args[::2], args[1::2]):
        med, ns = table(src, pat)
        print(f"== {src} [{pat}] kernel_ns={ns}")
        for k in sorted(med):
            print(f"  {k:28s} {med[k]:.6g}")
        if "SQ_WAVE_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
            print(f"  waves/SIMD (WAVE_CYCLES/GUI_ACTIVE/1024)  {med['SQ_WAVE_CYCLES'] / med['GRBM_GUI_ACTIVE'] / 1024:.3f}")
