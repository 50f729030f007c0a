"""The committed measurement evidence is self-consistent (no GPU): the bench line's roofline can be
recomputed from profiles/pmc_summary.json, whose entries are of the library build in this tree, and
tools/pmc_summary.py rebuilds the summary from the committed counter CSVs (profiles/r05_pmc/)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from fancy_gym_crowd_amd import _build  # noqa: E402

BENCH_LINE = os.path.join(ROOT, "profiles", "r06_bench_n1_final.json")
KERNEL_STATS = os.path.join(ROOT, "profiles", "r06_kernel_stats_bench_final.csv")


def _line():
    with open(BENCH_LINE) as f:
        return json.loads(f.read())


def _current_or_skip(ids):
    """evidence of another build (sources changed since the PMC passes): nothing to check yet"""
    if ids != {_build.source_hash()}:
        pytest.skip(f"profiles are of build(s) {sorted(ids)}, the sources are {_build.source_hash()}: "
                    "re-run tools/gpu_pmc_r03.sh and tools/gpu_final_r06.sh")


def test_pmc_summary_is_of_this_tree():
    """every PMC entry bench.py may read carries one build id, and its shard / GEMM entries exist"""
    with open(bench.PMC_SUMMARY) as f:
        entries = json.load(f)["entries"]
    assert entries
    _current_or_skip({e["build_id"] for e in entries})
    have = {(e["kernel"], int(e["envs"])) for e in entries}
    for n, k in ((65536, "k_episode"), (32768, "k_episode_jl"), (16384, "k_episode_jl"), (8192, "k_episode_jl"),
                 (65536, "k_traj_mfma")):
        assert (k, n) in have, (k, n)


def test_bench_roofline_recomputes_from_profiles():
    """frac = (VALU wave-instructions per launch / SIMDs / kernel cycles) / mix-weighted issue peak"""
    line = _line()
    r = line["roofline"]
    _current_or_skip({r["build_id"]})
    assert r["bound"] == "valu_issue"
    pmc, note = bench.pmc_entry(line["config"]["workload"], line["config"]["envs_per_gpu"], r["kernel"], r["build_id"])
    assert pmc is not None, note
    simds = 1024   # 256 CUs x 4 SIMDs (MI355X)
    achieved = pmc["valu_instr_per_launch"] / simds / (r["kernel_ms"] * 1e-3 * bench.CLOCK_GHZ * 1e9)
    peak = bench.valu_issue_peak(pmc)[0]
    assert achieved == pytest.approx(r["achieved"], rel=1e-9)
    assert peak == pytest.approx(r["peak"], rel=1e-9)
    assert achieved / peak == pytest.approx(r["frac"], rel=1e-9)
    assert 0.0 < r["frac"] < 1.0
    # the kernel time the roofline divides by is the rocprofv3 average of the same build within 10%
    import csv
    with open(KERNEL_STATS) as f:
        avg = [float(row["AverageNs"]) for row in csv.DictReader(f) if "k_episode<0, 1, 0, 5, 5, false>" in row["Name"]]
    assert avg and abs(avg[0] * 1e-6 - r["kernel_ms"]) / r["kernel_ms"] < 0.1


def test_pmc_summary_rebuilds_from_committed_csvs(tmp_path):
    out = tmp_path / "s.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"),
                    os.path.join(ROOT, "profiles", "r06_pmc"), "--no-copy", "--out", str(out),
                    "--build-id", _build.source_hash()], check=True, capture_output=True)
    got = json.loads(out.read_text())["entries"]
    with open(bench.PMC_SUMMARY) as f:
        ref = json.load(f)["entries"]
    key = lambda e: (e["kernel"], e["envs"], e["workload"])   # noqa: E731
    g = {key(e): e for e in got}
    for e in ref:
        assert key(e) in g
        for fld in ("valu_instr_per_launch", "traffic_bytes_per_launch"):
            if fld in e:
                assert g[key(e)][fld] == e[fld]


def test_basis_gemm_accounting_from_pmc():
    """bench.py's basis-GEMM fields: ONE contraction per env is the algorithmic work (2 nb T dof N
    flops: ProMP's velocities are a forward difference, not a second GEMM), the PMC pass counts the
    MFMA-padded flops actually issued (K = 8 for 5 basis functions, 8 tiles of 28 rows for T = 200),
    and mfma_frac = issued flops / launch time / f32 matrix peak (round 4: 0.067, not 0.119)."""
    with open(bench.PMC_SUMMARY) as f:
        entries = json.load(f)["entries"]
    pmc = [e for e in entries if e["kernel"] == "k_traj_mfma" and int(e["envs"]) == 65536
           and e["workload"] == "fancy_ProMP/LongSimpleReacher-v0"]
    assert pmc
    pmc = pmc[0]
    N, T, n, nb = 65536, 200, 5, 5
    t = pmc["kernel_ns_median_under_pmc"]["mfma"] * 1e-9
    f = bench.basis_gemm_fields(N, T, n, nb, n * nb, t, pmc)
    assert f["flops_algorithmic"] == 2 * nb * T * n * N
    # issued = padded: K 8 / 5 and 224 rows / 200 (ProMP tiles of 28 of 32 rows)
    assert f["pmc"]["issued_over_algorithmic"] == pytest.approx(8 / 5 * 224 / 200, rel=1e-9)
    assert f["mfma_frac"] == pytest.approx(pmc["mfma_f32_flops"] / t / 1e12 / bench.FP32_VEC_PEAK_TF, rel=1e-12)
    assert 0.05 < f["mfma_frac"] < 0.09
    assert f["algorithmic_tflops"] < f["mfma_tflops"]
    line = _line()
    bg = line.get("basis_gemm", {})
    if "flops_algorithmic" in bg and bg.get("pmc"):   # a bench line of the corrected accounting
        g = bench.basis_gemm_fields(N, T, n, nb, n * nb, bg["us"] * 1e-6, pmc)
        for k in ("flops_algorithmic", "mfma_frac", "algorithmic_tflops", "hbm_GBps"):
            assert g[k] == pytest.approx(bg[k], rel=1e-9), k


def test_cpu_baseline_calibration_committed():
    """the CPU baseline worker bench.py runs on the GPU box is calibrated against the
    shimmed reference loop on one core of the build container (tools/cpu_calibration.py)."""
    import json
    p = os.path.join(ROOT, "profiles", "r06_cpu_calibration.json")
    d = json.load(open(p))
    assert d["reference_steps_per_s"] > 0 and d["port_steps_per_s"] > 0
    assert abs(d["port_over_reference"] - d["port_steps_per_s"] / d["reference_steps_per_s"]) < 1e-9
    assert 0.2 < d["port_over_reference"] < 5.0
