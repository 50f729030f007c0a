"""k_traj_run (csrc/fgx_traj_run.h: get_trajectory for DMP, replanning plans, condition_on_desired and
generic basis counts, written as whole env runs from LDS) against k_traj_valu (FGX_TRAJ_VALU=1, one env
per lane) bit for bit, and against the oracle's trajectory (oracle/mp.py) on the oracle's own tables:
every MP kind, plan starts s0 > 0 from a replanning schedule, partial last groups, chunked runs
(FGX_TRAJ_RC), other group sizes (FGX_TRAJ_GE), 2 / 3 / 5 links and a generic basis count."""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from oracle import mp
from test_gpu_parity import DEV, np_, spec_of

pytestmark = pytest.mark.gpu


def REPLAN(n):
    return {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(n)}}


CASES = [
    # (env id, mp_config_override, env kwargs, N, BB steps before the trajectory)
    ("fancy_DMP/LongSimpleReacher-v0", None, {}, 4099, 0),
    ("fancy_DMP/HoleReacher-v0", REPLAN(40), {}, 1000, 2),
    ("fancy_DMP/SimpleReacher-v0", None, {}, 777, 0),                  # 2 links
    ("fancy_ProMP/LongSimpleReacher-v0", REPLAN(50), {}, 4099, 1),     # s0 = 50
    ("fancy_ProDMP/HoleReacher-v0", REPLAN(60), {}, 2050, 2),          # s0 = 120
    ("fancy_ProMP/SimpleReacher-v0", REPLAN(25), {}, 333, 3),
    ("fancy_ProDMP/SimpleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25),
                                                            "condition_on_desired": True}}, {}, 511, 2),
    ("fancy_ProMP/LongSimpleReacher-v0", {"basis_generator_kwargs": {"num_basis": 7}}, {}, 300, 0),
    ("fancy_DMP/HoleReacher-v0", None, {"n_links": 3}, 129, 0),        # the n_links instantiations
    # T * dof not a multiple of 4: pieces stored as dwords (T = 201 / 199, 2 links)
    ("fancy_ProMP/SimpleReacher-v0", {"black_box_kwargs": {"duration": 2.01, "replanning_schedule": fgx.ReplanEvery(201)}},
     {}, 300, 0),
    ("fancy_DMP/SimpleReacher-v0", {"black_box_kwargs": {"duration": 1.99}}, {}, 97, 0),
]


def _traj(env_id, over, kw, N, n_bb, monkeypatch, env_vars):
    for k in ("FGX_TRAJ_VALU", "FGX_TRAJ_GE", "FGX_TRAJ_RC", "FGX_TRAJ_NT", "FGX_TRAJ_SEP", "FGX_TRAJ_ALIGN"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env_vars.items():
        monkeypatch.setenv(k, v)
    env = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=0, **kw)
    env.reset(seed=11)
    rng = np.random.default_rng(7)
    for _ in range(n_bb):
        env.step(torch.from_numpy(rng.standard_normal((N, env.n_params), dtype=np.float32)).to(DEV))
    params = rng.standard_normal((N, env.n_params), dtype=np.float32)
    params[5::97] = np.nan
    pos, vel = env.trajectory(torch.from_numpy(params).to(DEV))
    return env, params, np_(pos), np_(vel)


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_traj_run_equals_valu(ci, monkeypatch):
    env_id, over, kw, N, n_bb = CASES[ci]
    _, _, rp, rv = _traj(env_id, over, kw, N, n_bb, monkeypatch, {"FGX_TRAJ_VALU": "1"})
    for vars_ in ({}, {"FGX_TRAJ_RC": "36"}, {"FGX_TRAJ_GE": "3", "FGX_TRAJ_RC": "17"},
                  {"FGX_TRAJ_SEP": "1", "FGX_TRAJ_NT": "1", "FGX_TRAJ_GE": "5"},
                  {"FGX_TRAJ_SEP": "0", "FGX_TRAJ_RC": "64", "FGX_TRAJ_ALIGN": "0"}):
        _, _, p, v = _traj(env_id, over, kw, N, n_bb, monkeypatch, vars_)
        assert p.shape == rp.shape
        np.testing.assert_array_equal(p.view(np.uint32), rp.view(np.uint32), err_msg=str(vars_))
        np.testing.assert_array_equal(v.view(np.uint32), rv.view(np.uint32), err_msg=str(vars_))


@pytest.mark.parametrize("ci", [0, 1, 3, 4])
def test_traj_run_vs_oracle(ci, monkeypatch):
    """the oracle's trajectory (oracle/mp.py:243) on its own tables, per-env plan starts s0 = steps"""
    env_id, over, kw, N, n_bb = CASES[ci]
    env, params, p, v = _traj(env_id, over, kw, N, n_bb, monkeypatch, {})
    spec = spec_of(env)
    tabs = mp.build_tables(spec, np_(env.tables()).shape[0])
    st = env.get_state()
    s0 = np_(st["steps"]) if n_bb else 0
    rp, rv = mp.trajectory(spec, tabs, params, s0, np_(st["q"]), np_(st["qd"]))
    np.testing.assert_array_equal(p, rp)
    np.testing.assert_array_equal(v, rv)
