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


def test_committed_full_size_result():
    with open(os.path.join(ROOT, "profiles", "r05_mp_f32_exposure.json")) as f:
        res = json.load(f)["results"]
    assert {r["config"] for r in res} == {"config3", "metric"}
    for r in res:
        assert r["envs"] == 65536 and r["bb_steps"] == 2
        for s in r["steps"]:
            assert s["length_flips"] == 0 and s["terminated_flips"] == 0 and s["truncated_flips"] == 0
            assert s["max_return_rel_dev"] < 1e-5 and np.isfinite(s["max_obs_abs_dev"])
