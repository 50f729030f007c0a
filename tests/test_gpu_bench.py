"""bench.py keeps the driver's contract: one JSON line with the metric of BASELINE.json, the
whole-job value, the roofline of the metric kernel (measured live) and the run's shape.  Short
runs in a child process, as the driver launches them: `bench.py` (1 rank) and `bench.py --gpus 2`
without a launcher (bench.py starts the two ranks; on a one-GPU box they share cuda:0 over gloo)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:] + out.stderr[-2000:]
    return json.loads(lines[0])


def _check_roofline(r):
    assert r["kernel"].startswith("k_episode")
    assert r["bound"] in ("valu_issue", "hbm") and r["peak"] > 0
    assert 0 < r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    if r["bound"] == "valu_issue":   # PMC of this very build, architectural peak for its mix
        assert r["pmc"]["build_id"] == r["build_id"]
        assert 1 / 4.0 <= r["peak"] <= 1 / 2.0
    else:
        assert r["unit"] == "GB/s" and r["pmc_note"]


@pytest.mark.gpu
def test_bench_json_line():
    out = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--envs", "4096",
                          "--no-cpu-baseline"], cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    d = _line(out)
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["ranks_seen"] == 1
    assert d["higher_is_better"] is True and d["value"] > 0 and d["ms_per_step"] > 0
    _check_roofline(d["roofline"])
    # 4096 envs x 200 inner steps per BB step (SimpleReacher never terminates early)
    assert d["value"] == pytest.approx(4096 * 200 / (d["ms_per_step"] * 1e-3), rel=1e-6)
    assert d["timing"]["gathers"] == 0      # one rank, no process group: nothing to gather


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` (no torch.distributed.run) runs two ranks over the 65536 global envs."""
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--no-weak"], cwd=ROOT, capture_output=True, text=True, timeout=115)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["backend"] in ("nccl", "gloo")
    assert d["launcher"].startswith("torch.distributed.run")
    assert d["config"]["global_envs"] == 65536 and d["config"]["envs_per_gpu"] == 32768
    assert [s[:2] for s in d["shards"]] == [[0, 32768], [32768, 65536]]
    assert sum(s[2] for s in d["shards"]) == 65536 * 200 * 2
    assert d["value"] == pytest.approx(65536 * 200 / (d["ms_per_step"] * 1e-3), rel=1e-6)
    _check_roofline(d["roofline"])
    # the return all_gather runs after every timed BB step on every rank
    assert d["timing"]["gathers"] == 2
    assert [p["gathers"] for p in d["timing"]["per_rank"]] == [2, 2]


def test_bench_gpus_mismatch_is_refused():
    """A launcher that started a different number of ranks than --gpus asks for is an error
    (checked before anything touches torch or a GPU)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--no-cpu-baseline"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=60)
    assert out.returncode != 0
    assert "--gpus 4" in out.stderr and "WORLD_SIZE=2" in out.stderr
