"""bench.py keeps the driver's contract: one JSON line with the metric of BASELINE.json, the
whole-job value, the roofline of the metric kernel (measured live) and the run's shape.  A short
run (4096 envs, 2 BB steps) in a child process, as the driver launches it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line():
    out = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--envs", "4096",
                          "--no-cpu-baseline"], cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["value"] > 0 and d["ms_per_step"] > 0
    r = d["roofline"]
    assert r["bound"] in ("hbm", "mfma") and r["peak"] > 0 and 0 < r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    assert r["kernel"].startswith("k_episode")
    # 4096 envs x 200 inner steps per BB step (SimpleReacher never terminates early)
    assert d["value"] == pytest.approx(4096 * 200 / (d["ms_per_step"] * 1e-3), rel=1e-6)
