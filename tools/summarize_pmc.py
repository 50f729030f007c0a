"""Summarise rocprofv3 --pmc counter CSVs (gpurun_out/...) for the metric kernel into profiles/.

  python tools/summarize_pmc.py hbm   gpurun_out/prof_pmc  -> profiles/pmc_k_episode.json
  python tools/summarize_pmc.py issue gpurun_out/pmc_valu  -> profiles/r01_pmc_issue_k_episode.json
"""
import collections
import csv
import glob
import json
import os
import sys

KERNEL = "k_episode<0, 1, 0, 5, 5, false>"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(paths):
    """counter -> median over dispatches of the per-dispatch sum over instances; kernel ns median."""
    vals, durs = collections.defaultdict(list), []
    for path in paths:
        agg, dur = collections.defaultdict(float), {}
        for r in csv.DictReader(open(path)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (d, c), v in agg.items():
            vals[c].append(v)
        durs += list(dur.values())
    med = {c: sorted(v)[len(v) // 2] for c, v in vals.items()}
    return med, (sorted(durs)[len(durs) // 2] if durs else None)


def main():
    mode, src = sys.argv[1], sys.argv[2]
    paths = sorted(glob.glob(os.path.join(src, "*_counter_collection.csv")))
    med, ns = per_dispatch(paths)
    if mode == "hbm":
        fetch_kib, write_kib = med["FETCH_SIZE"], med["WRITE_SIZE"]
        out = {"workload": "fancy_ProMP/LongSimpleReacher-v0", "envs": 65536,
               "kernel": "k_episode<SIMPLE,PROMP,PD,5,5,false>",
               "FETCH_SIZE_KiB": round(fetch_kib, 1), "WRITE_SIZE_KiB": round(write_kib, 1),
               "traffic_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024.0,
               "kernel_ns_median_under_pmc": ns,
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py "
                         "--steps 10; FETCH_SIZE doubled (gfx950 half-count, MI355X_MICROARCH.md §HBM), KiB->B",
               "source": "profiles/r01_pmc_hbm_k_episode.csv"}
        dst = os.path.join(ROOT, "profiles", "pmc_k_episode.json")
    else:
        waves = 1024.0
        samples = 200.0
        out = {"kernel": "k_episode<SIMPLE,PROMP,PD,5,5,false>, 65536 envs (1024 waves), T=200 "
                         "(tools/bench_kernels.py metric); one rocprofv3 --pmc pass per counter",
               "kernel_ns_median_under_pmc": ns, "counters_per_dispatch": med,
               "per_wave_sample": {c: v / waves / samples for c, v in med.items()
                                   if c.startswith("SQ_INSTS")}}
        dst = os.path.join(ROOT, "profiles", "r01_pmc_issue_k_episode.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
