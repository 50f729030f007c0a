"""The oracle's unpinned MP table arithmetic, measured (no GPU): tools/mp_f32_exposure.py rebuilds
the basis tables with every operation in torch float32 (mp_pytorch's arithmetic, SURVEY.md Appendix
A) and runs the oracle on both table sets.  Here at a small size; the committed full-size result
(65536 envs x 2 BB steps of config 3 and of the metric) is profiles/r05_mp_f32_exposure.json,
quoted in DESIGN.md section 3."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import mp_f32_exposure as mx  # noqa: E402


def test_f32_tables_close_to_f64_tables():
    import fancy_gym_crowd_amd as fgx
    from oracle import mp
    for env_id in ("fancy_ProDMP/HoleReacher-v0", "fancy_ProMP/LongSimpleReacher-v0", "fancy_DMP/SimpleReacher-v0"):
        spec = mx.spec_from_cfg(fgx.resolve(env_id)[0])
        t64 = mp.build_tables(spec, spec.T + 2)
        t32 = mx.build_tables32(spec, spec.T + 2)
        assert set(t64) == set(t32)
        for k, d in mx.table_deviation(t64, t32).items():
            assert d["max_rel_to_max"] < 2e-5, (env_id, k, d)


def test_exposure_small_batch():
    r = mx.exposure("config3", 256, 1, workers=1, chunks=1)
    s = r["steps"][0]
    assert s["terminated_count"] > 0            # collisions took place
    assert s["length_flips"] == 0 and s["terminated_flips"] == 0 and s["truncated_flips"] == 0
    assert s["max_return_rel_dev"] < 1e-5


# committed bound per BB step on the observation values outside the north-star tolerance (rtol 1e-5,
# atol 1e-6) under f32 MP tables: config 3 <= 4, the metric <= 1 (profiles/r06_mp_f32_exposure.json)
OBS_OUTSIDE_TOL_MAX = {"config3": 4, "metric": 1}


def test_committed_full_size_result():
    with open(os.path.join(ROOT, "profiles", "r06_mp_f32_exposure.json")) as f:
        res = json.load(f)["results"]
    assert {r["config"] for r in res} == {"config3", "metric"}
    for r in res:
        assert r["envs"] == 65536 and r["bb_steps"] == 2
        for s in r["steps"]:
            assert s["length_flips"] == 0 and s["terminated_flips"] == 0 and s["truncated_flips"] == 0
            assert s["max_return_rel_dev"] < 1e-5 and np.isfinite(s["max_obs_abs_dev"])
            assert s["obs_outside_tol"] <= OBS_OUTSIDE_TOL_MAX[r["config"]]
            assert len(s["obs_outliers"]) == s["obs_outside_tol"]
            for o in s["obs_outliers"]:
                # every outlier is a small value where the absolute tolerance binds, off by < 5e-6
                assert o["atol_binds"] and abs(o["f64_tables"]) < 0.1 and o["abs_dev"] < 5e-6, o
                assert o["name"] in ("qdot0", "ee_minus_goal_y"), o


def test_outliers_are_named():
    """tools/mp_f32_exposure.obs_outliers names each value outside the tolerance and says whether the
    absolute tolerance binds there"""
    a = np.array([[0.05, 2.0, 1.0]], np.float32)
    b = np.array([[0.050003, 2.0, 1.00002]], np.float32)
    out = mx.obs_outliers(a, b, ["qdot0", "x", "y"])
    assert [(o["name"], o["atol_binds"]) for o in out] == [("qdot0", True), ("y", False)]
