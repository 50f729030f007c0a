"""The RCCL path runs: the `nccl` backend (RCCL on ROCm) with a one-rank process group on cuda:0.

On a one-GPU box two ranks cannot share a device under RCCL, so the multi-rank tests rehearse over
gloo (tests/test_gpu_dist.py, test_gpu_bench.py).  These run what the 8-GPU node runs, at one rank:
init_process_group("nccl", device_id=...) and every shard.py collective on device tensors
(tests/rccl_probe.py), then bench.py's own RCCL branch (--force-dist), whose line reports the
per-rank kernel / collective / barrier split the driver's multi-GPU points are decomposed with.
Reference concurrency being replaced: AsyncVectorEnv (examples/examples_general.py:68-110).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_collectives_on_device():
    env = dict(os.environ, FGX_PROBE_PORT=str(_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_probe.py")], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert d["backend"] == "nccl" and d["world"] == 1
    assert d["gather_ok"] and d["gather_device"] == "cuda:0"
    assert d["max"] == 3.25 and d["sum"] == 7
    assert d["ints"] == [[1, 2, 3]] and d["floats"] == [[0.5, 1.5]]


def test_bench_rccl_branch_one_rank():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run([sys.executable, "bench.py", "--force-dist", "--steps", "3", "--warmup", "1",
                          "--global-envs", "8192", "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert d["backend"] == "nccl" and d["ranks_seen"] == 1
    t = d["timing"]
    assert len(t["per_rank"]) == 1
    pr = t["per_rank"][0]
    assert pr["kernel_ms_per_step"] > 0 and pr["exposed_collective_ms_per_step"] >= 0 and pr["barrier_ms"] >= 0
    assert pr["step_ms"] * 3 <= pr["wall_ms"] * 1.001
    # one RCCL return all_gather per timed BB step, captured in the HIP graph
    assert pr["gathers"] == 3 and t["gathers"] == 3
    assert "capture_error" not in t, t.get("capture_error")
    assert "captured" in d["config"]["launch"]
    # --overlap auto: both schedules replayed once untimed, the faster one timed
    tr = t["schedule_trial"]
    assert tr["inline_ms_per_step"] > 0 and tr["overlap_ms_per_step"] > 0
    picked_overlap = "overlapped" in d["config"]["launch"]
    assert picked_overlap == (tr["overlap_ms_per_step"] < tr["inline_ms_per_step"])
    assert pr["gather_ms"] > 0      # the captured all_gather timed alone
