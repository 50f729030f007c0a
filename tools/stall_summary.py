"""Summarise tools/gpu_stall_probe.sh output: per kernel and grid size, the median per-dispatch SQ
counters and the wave-cycle split (active / parked on s_waitcnt or barrier / issue-stalled; quad-cycles).

  python tools/stall_summary.py gpurun_out/stall [kernels...]
"""
import collections
import csv
import glob
import json
import os
import sys


def summarise(root, kernel):
    out = {}
    for grp in sorted(glob.glob(os.path.join(root, kernel, "g*"))):
        f = glob.glob(os.path.join(grp, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        grid = {}
        for r in csv.DictReader(open(f[0])):
            if "k_episode" not in r["Kernel_Name"]:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
        by = collections.defaultdict(list)
        for d, v in per.items():
            by[grid[d]].append(v)
        for gs, lst in by.items():
            med = {c: sorted(x[c] for x in lst)[len(lst) // 2] for c in lst[0]}
            out.setdefault(gs, {}).update(med)
    for gs, m in out.items():
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            m["frac_active"] = m.get("SQ_ACTIVE_INST_ANY", 0) / wc
            m["frac_wait_any"] = m.get("SQ_WAIT_ANY", 0) / wc
            m["frac_wait_inst"] = m.get("SQ_WAIT_INST_ANY", 0) / wc
            m["frac_wait_inst_lds"] = m.get("SQ_WAIT_INST_LDS", 0) / wc
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
    return out


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stall"
    ks = sys.argv[2:] or sorted(os.path.basename(p) for p in glob.glob(os.path.join(root, "*")) if os.path.isdir(p))
    res = {k: summarise(root, k) for k in ks}
    print(json.dumps(res, indent=1, sort_keys=True))
