"""Per-instantiation summary of tools/gpu_pmc_traj.sh: median kernel time (kernel trace), HBM bytes
per dispatch (2 * FETCH_SIZE + WRITE_SIZE KiB, MI355X_MICROARCH.md's gfx950 correction) and the
algorithmic bytes (params read + positions / velocities written, 65536 envs).

  python tools/traj_pmc_summary.py gpurun_out/r05_traj [--out profiles/r05_traj_run_pmc.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics

N = 65536
# (kernel instantiation substring, workload, T, dof, n_params): the trajrun1 cases in order
CASES = {"k_traj_run<2, 5": ("fancy_DMP/LongSimpleReacher-v0 | fancy_DMP/HoleReacher-v0", 200, 5, 30),
         "k_traj_run<1, 5": ("fancy_ProMP/LongSimpleReacher-v0 (replanning)", 200, 5, 25),
         "k_traj_run<3, 5": ("fancy_ProDMP/HoleReacher-v0 (replanning)", 200, 5, 30)}


def rows(d, name):
    out = []
    for p in glob.glob(os.path.join(d, "**", name), recursive=True):
        out += list(csv.DictReader(open(p)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {}
    durs = collections.defaultdict(list)
    for r in rows(os.path.join(a.src, "trace"), "*kernel_trace.csv"):
        durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = {}
    for part, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        agg = collections.defaultdict(float)
        names = {}
        for r in rows(os.path.join(a.src, part), "*counter_collection.csv"):
            if r["Counter_Name"] != ctr:
                continue
            agg[(r["Kernel_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        per = collections.defaultdict(list)
        for (k, _), v in agg.items():
            per[k].append(v)
        cnt[part] = {k: statistics.median(v) for k, v in per.items()}
    for key, (wl, T, dof, npar) in CASES.items():
        ks = [k for k in durs if key in k]
        if not ks:
            continue
        alg = N * (npar * 4 + 2 * T * dof * 4)
        for k in ks:
            us = statistics.median(durs[k]) / 1e3
            f = next((v for kk, v in cnt.get("fetch", {}).items() if kk == k), None)
            w = next((v for kk, v in cnt.get("write", {}).items() if kk == k), None)
            hbm = (2 * f + w) * 1024 if f is not None and w is not None else None
            res[k.split("(")[0]] = dict(workload=wl, envs=N, dispatches=len(durs[k]), median_us=round(us, 2),
                                        algorithmic_bytes=alg, achieved_TBps=round(alg / us / 1e6, 3),
                                        hbm_frac=round(alg / us / 1e6 / 8.0, 3),
                                        write_bytes=w * 1024 if w is not None else None,
                                        fetch_bytes_corrected=2 * f * 1024 if f is not None else None,
                                        traffic_over_algorithmic=round(hbm / alg, 3) if hbm else None)
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
