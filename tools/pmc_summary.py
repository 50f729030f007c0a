"""Build profiles/pmc_summary.json (read by bench.py's roofline) from rocprofv3 --pmc passes.

  python tools/pmc_summary.py gpurun_out/pmc_r02 [--round r02]

Expects, per profiled size, the sub-directories written by tools/gpu_pmc_r02.sh:
  <src>/n<ENVS>/fetch/*_counter_collection.csv    (--pmc FETCH_SIZE)
  <src>/n<ENVS>/write/*_counter_collection.csv    (--pmc WRITE_SIZE)
  <src>/n<ENVS>/issue/*_counter_collection.csv    (--pmc SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE)
  <src>/n<ENVS>/busy/*_counter_collection.csv     (--pmc VALUBusy)
each a separate rocprofv3 pass over `bench.py --global-envs ENVS --no-cpu-baseline`.

Per counter the value of one dispatch is the sum over its rows (instances / XCDs); the entry keeps
the median over the episode-kernel dispatches of the pass.  HBM traffic follows
MI355X_MICROARCH.md's HBM/rocprofv3 recipe: FETCH_SIZE and WRITE_SIZE in KiB, FETCH_SIZE doubled
(gfx950 counts half the fetched 64-B lines), bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOAD = "fancy_ProMP/LongSimpleReacher-v0"
T = 200


def kernel_family(name):
    """'fgx::k_episode_jp<1, 5, 5>(...)' -> 'k_episode_jp' (the name env.episode_kernel() reports)."""
    m = re.search(r"(k_episode(?:_jp|_ws|_jl)?)\b", name)
    return m.group(1) if m else None


def per_dispatch(src):
    """{counter: median per-dispatch value}, median kernel ns, kernel family, full kernel name."""
    vals, durs, fam, full = collections.defaultdict(list), [], None, None
    for path in sorted(glob.glob(os.path.join(src, "**", "*_counter_collection.csv"), recursive=True)):
        agg, dur = collections.defaultdict(float), {}
        for r in csv.DictReader(open(path)):
            f = kernel_family(r["Kernel_Name"])
            if f is None:
                continue
            fam, full = f, r["Kernel_Name"]
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (_, c), v in agg.items():
            vals[c].append(v)
        durs += list(dur.values())
    med = {c: sorted(v)[len(v) // 2] for c, v in vals.items()}
    return med, (sorted(durs)[len(durs) // 2] if durs else None), fam, full


def build_id():
    try:
        import sys
        sys.path.insert(0, ROOT)
        from fancy_gym_crowd_amd import _build
        return _build.source_hash()
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--round", default="r02")
    ap.add_argument("--build-id", default=None, help="build id of the profiled library (default: the "
                    "hash of the sources in this tree)")
    a = ap.parse_args()
    bid = a.build_id or build_id()
    entries = []
    for d in sorted(glob.glob(os.path.join(a.src, "n*"))):
        envs = int(os.path.basename(d)[1:])
        counters, ns, fam, full = {}, {}, None, None
        for part in ("fetch", "write", "issue", "busy"):
            med, kns, f, k = per_dispatch(os.path.join(d, part))
            counters.update(med)
            ns[part] = kns
            fam, full = fam or f, full or k
        if fam is None:
            continue
        e = {"workload": WORKLOAD, "envs": envs, "kernel": fam, "kernel_name": full,
             "build_id": bid, "kernel_ns_median_under_pmc": ns,
             "counters_per_dispatch": counters,
             "source": f"profiles/{a.round}_pmc/n{envs}"}
        if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
            e["FETCH_SIZE_KiB"] = counters["FETCH_SIZE"]
            e["WRITE_SIZE_KiB"] = counters["WRITE_SIZE"]
            e["traffic_bytes_per_launch"] = (2 * counters["FETCH_SIZE"] + counters["WRITE_SIZE"]) * 1024.0
        if "SQ_INSTS_VALU" in counters:
            e["valu_instr_per_launch"] = counters["SQ_INSTS_VALU"]
            e["waves"] = counters.get("SQ_WAVES")
            e["valu_instr_per_inner_step_per_env"] = counters["SQ_INSTS_VALU"] * 64 / envs / T
        if "VALUBusy" in counters:
            e["valu_busy_pct"] = counters["VALUBusy"]
        entries.append(e)
    out = {"method": "rocprofv3 --pmc, one pass per counter group (tools/gpu_pmc_r02.sh); median over "
                     "dispatches of the per-dispatch sum over instances; traffic = (2*FETCH_SIZE + "
                     "WRITE_SIZE) KiB (gfx950 FETCH_SIZE half-count)", "entries": entries}
    # the counter CSVs the entries come from travel with the summary
    for d in sorted(glob.glob(os.path.join(a.src, "n*"))):
        for path in glob.glob(os.path.join(d, "*", "**", "*_counter_collection.csv"), recursive=True):
            part = os.path.relpath(path, d).split(os.sep)[0]
            dd = os.path.join(ROOT, "profiles", f"{a.round}_pmc", os.path.basename(d), part)
            os.makedirs(dd, exist_ok=True)
            shutil.copy(path, os.path.join(dd, os.path.basename(path)))
    dst = os.path.join(ROOT, "profiles", "pmc_summary.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
