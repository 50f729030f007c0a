"""Reference options beyond the default path, the VectorEnv info contract and the fast path's
NaN-free-wave guard, on the device against the reference-generated fixtures and the oracle.

* reset(options={'random_start': ...}) sequences and SimpleReacher(target=...) vs
  tests/golden/options.npz (base_reacher.py:77-86, simple_reacher.py:19,93-94);
* reward_aggregation callables np.median / ``lambda x: np.mean(x[::2])`` vs options.npz
  (black_box_wrapper.py:252, test/test_black_box.py:139-150);
* info_level 1 (the env's per-step info lists without the verbose-2 arrays) and
  info['final_info'] / '_final_info' vs the goldens' info_a / info_b / info_ee
  (black_box_wrapper.py:170,218-227,244-249; gymnasium 0.29 SyncVectorEnv autoreset);
* the NaN-free-wave fast blocks of k_episode (fgx_kernels.h) vs the oracle for NaN / inf / 1e30
  weights, 1e200 gains and restored states with |q| = 1e250 (np.clip keeps NaN,
  black_box_wrapper.py:201-205);
* reset_mask rows of envs that are not reset, and argument-length checks.
"""
import os

import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from oracle import batched
from tests.test_gpu_parity import DEV, kernel_is, assert_ulps, close, ctrl_of, np_, oracle_kwargs, spec_of, split_tables
from tests.test_oracle_options import RESET_SEQ, TARGET

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLD, "options.npz"))


# ------------------------------------------------------------------------------ reset options
KIND_IDS = {"simple": ("fancy_ProMP/SimpleReacher-v0", {}), "long": ("fancy_ProMP/LongSimpleReacher-v0", {}),
            "hole": ("fancy/HoleReacher-v0", {}), "via": ("fancy_ProMP/ViaPointReacher-v0", {}),
            "target": ("fancy_ProMP/SimpleReacher-v0", {"target": TARGET}),
            "target_long": ("fancy/LongSimpleReacher-v0", {"target": TARGET})}


@pytest.mark.parametrize("kind", list(KIND_IDS))
def test_reset_options_golden(g, kind):
    """16 envs (env i seeded i) through the fixture's reset sequence; q, goal and the full
    observation after every reset."""
    env_id, kw = KIND_IDS[kind]
    env = fgx.make(env_id, num_envs=16, device=DEV, **kw)
    random_default = kind not in ("via",)   # registered HoleReacher: random_start=True
    for j, (sd, opt) in enumerate(RESET_SEQ):
        if opt is not None and opt.get("random_start") == "flip":
            opt = {"random_start": not random_default}
        env.reset(seed=0 if sd else None, options=opt)
        st = env.get_state()
        np.testing.assert_array_equal(np_(st["q"]), g[f"{kind}_reset_q0"][:, j])
        np.testing.assert_array_equal(np_(st["goal"]), g[f"{kind}_reset_goal"][:, j])
        # full observation: the env's obs of the current state via a no-op masked reset
        o, _ = env.reset(options={"reset_mask": np.zeros(16, bool)})
        ref = g[f"{kind}_reset_obs"][:, j]
        if o.shape[1] == ref.shape[1]:
            close(np_(o), ref)
        else:   # BB envs return the context-masked observation
            mask = batched.BatchedReacher({"simple": "SimpleReacher", "long": "LongSimpleReacher",
                                           "target": "SimpleReacher", "via": "ViaPointReacher",
                                           "hole": "HoleReacher"}[kind], 1).mask
            close(np_(o), ref[:, mask])


@pytest.mark.parametrize("kind", ["target", "target_long"])
def test_fixed_target_step_based_golden(g, kind):
    env_id = "fancy/SimpleReacher-v0" if kind == "target" else "fancy/LongSimpleReacher-v0"
    acts = g[f"{kind}_actions"]
    env = fgx.make(env_id, num_envs=acts.shape[1], device=DEV, target=TARGET)
    o0, _ = env.reset(seed=0)
    close(np_(o0), g[f"{kind}_obs0"])
    for t in range(acts.shape[0]):
        obs, rew, te, tr, info = env.step(torch.from_numpy(acts[t]))
        close(np_(info["final_observation"]), g[f"{kind}_obs"][t])
        close(np_(rew), g[f"{kind}_rew"][t])


# ------------------------------------------------------------------------------ reward aggregation
AGG = {"aggmedian": ("fancy_ProMP/LongSimpleReacher-v0", np.median),
       "aggeven": ("fancy_ProDMP/HoleReacher-v0", lambda x: np.mean(x[::2]))}


@pytest.mark.parametrize("case", list(AGG))
@pytest.mark.parametrize("info_level", [0, 2])
def test_reward_aggregation_callables_golden(g, case, info_level):
    env_id, agg = AGG[case]
    E, n_bb = g[f"{case}_ret"].shape
    env = fgx.make(env_id, num_envs=E, device=DEV, info_level=info_level,
                   mp_config_override={"black_box_kwargs": {"reward_aggregation": agg}})
    close(np_(env.reset(seed=[100 + i for i in range(E)])[0]), g[f"{case}_obs0"])
    for b in range(n_bb):
        P = np.ascontiguousarray(g[f"{case}_pos"][:, :200])
        V = np.ascontiguousarray(g[f"{case}_vel"][:, :200])
        obs, ret, te, tr, info = env.step_trajectory(torch.from_numpy(P), torch.from_numpy(V))
        np.testing.assert_array_equal(np_(info["trajectory_length"]), g[f"{case}_tlen"][:, b])
        assert_ulps(np_(ret), g[f"{case}_ret"][:, b], 16)
        close(np_(info["final_observation"]), g[f"{case}_obs"][:, b])
        assert ("step_rewards" in info) == (info_level >= 2)


# ------------------------------------------------------------------------------ info contract
INFO_CASES = {"bb_long": "fancy_ProMP/LongSimpleReacher-v0", "bb_hole_pd": "fancy_ProDMP/HoleReacher-v0"}


@pytest.mark.parametrize("case", list(INFO_CASES))
def test_info_level1_env_info_and_final_info(case):
    """info_level 1: the env info lists (reward_dist / reward_ctrl or is_collided / is_success /
    end_effector) without the verbose-2 arrays; final_info[i] holds env i's step info cut at its
    trajectory_length (gymnasium SyncVectorEnv moves a finished env's info there)."""
    gd = np.load(os.path.join(GOLD, case + ".npz"))
    E, n_bb = gd["ret"].shape
    env = fgx.make(INFO_CASES[case], num_envs=E, device=DEV, info_level=1)
    env.reset(seed=[100 + i for i in range(E)])
    hole = "hole" in case
    for b in range(n_bb):
        steps = np_(env.get_state()["steps"])
        P = np.stack([gd["pos"][i, steps[i]:steps[i] + 200] for i in range(E)])
        V = np.stack([gd["vel"][i, steps[i]:steps[i] + 200] for i in range(E)])
        obs, ret, te, tr, info = env.step_trajectory(torch.from_numpy(P), torch.from_numpy(V))
        assert "step_actions" not in info and "positions" not in info
        keys = ("is_collided", "is_success", "end_effector") if hole else ("reward_dist", "reward_ctrl")
        assert all(k in info for k in keys)
        tl = np_(info["trajectory_length"])
        np.testing.assert_array_equal(tl, gd["tlen"][:, b])
        done = gd["term"][:, b] | gd["trunc"][:, b]
        np.testing.assert_array_equal(np_(info["_final_info"]), done)
        np.testing.assert_array_equal(np_(info["_trajectory_length"]), ~done)
        fi = info["final_info"]
        assert len(fi) == E
        for i in range(E):
            L = tl[i]
            a, bb_ = (np_(info[keys[0]])[i, :L], np_(info[keys[1]])[i, :L])
            if hole:
                np.testing.assert_array_equal(a.astype(bool), gd["info_a"][i, b, :L].astype(bool))
                np.testing.assert_array_equal(bb_.astype(bool), gd["info_b"][i, b, :L].astype(bool))
                close(np_(info["end_effector"])[i, :L], gd["info_ee"][i, b, :L])
            else:
                close(a, gd["info_a"][i, b, :L])
                close(bb_, gd["info_b"][i, b, :L])
            if done[i]:
                assert fi[i]["trajectory_length"] == L
                for k in keys:
                    np.testing.assert_array_equal(fi[i][k], np_(info[k])[i, :L])
            else:
                assert fi[i] is None


def test_default_info_level_is_verbose2():
    """The reference's step(action, verbose=2) default (black_box_wrapper.py:170): a plain make()
    returns the verbose-2 arrays."""
    env = fgx.make("fancy_ProMP/SimpleReacher-v0", num_envs=8, device=DEV)
    env.reset(seed=0)
    _, _, _, _, info = env.step(torch.zeros((8, env.n_params)))
    for k in ("positions", "velocities", "step_actions", "step_observations", "step_rewards", "reward_dist",
              "reward_ctrl", "trajectory_length", "final_info", "_final_info"):
        assert k in info, k


# ------------------------------------------------------------------------------ NaN-free-wave guard
def _run_vs_oracle(env, name, params_list, setup=None, n_exact_frac=0.0):
    N = env.num_envs
    spec = spec_of(env)
    ob = batched.BatchedBB(name, N, ctrl_of(env), mp_spec=spec,
                           **oracle_kwargs(env))
    close(np_(env.reset(seed=300)[0]), ob.reset(seed=300))
    if setup is not None:
        setup(env, ob)
    with np.errstate(all="ignore"):
        for params in params_list:
            obs, ret, te, tr, info = env.step(torch.from_numpy(params).to(DEV))
            r_obs, r_ret, r_te, r_tr, r_info = ob.step(params)
            np.testing.assert_array_equal(np_(info["trajectory_length"]), r_info["trajectory_length"])
            np.testing.assert_array_equal(np_(te).astype(bool), r_te)
            np.testing.assert_array_equal(np_(tr).astype(bool), r_tr)
            assert_ulps(np_(ret), r_ret, 16)
            close(np_(info["final_observation"]), r_info["final_obs"])
            close(np_(obs), r_obs)
            st = env.get_state()
            np.testing.assert_array_equal(np_(st["q"]), ob.env.q)
            np.testing.assert_array_equal(np_(st["qd"]), ob.env.qd)


def test_fast_path_guard_extreme_weights(monkeypatch):
    """Waves with a NaN / inf / 1e30 weight in one lane leave the fast blocks; a wave of 1e29
    weights stays in them (controls clipped to +-1000, everything finite)."""
    monkeypatch.setenv("FGX_EPISODE_KERNEL", "classic")   # the fast blocks live in k_episode
    N = 320
    env = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=N, device=DEV, info_level=0)
    assert env.episode_kernel() == "k_episode"
    rng = np.random.default_rng(8)
    plist = []
    for b in range(2):
        p = rng.standard_normal((N, env.n_params), dtype=np.float32)
        p[64 + 3, 7] = np.nan
        p[128 + 10, 0] = np.inf
        p[128 + 11, 4] = -np.inf
        p[192 + 5, 12] = 1e30
        p[256:320] *= np.float32(1e29)
        plist.append(p)
    _run_vs_oracle(env, "LongSimpleReacher", plist)


@pytest.mark.parametrize("gain", [1e200, 1e149])
def test_fast_path_guard_extreme_gains(monkeypatch, gain):
    """Per-joint PD gains beyond the guard's 1e150 take the exact generic path — with a restored
    |q| = |qd| = 1e150 on that joint the two PD terms overflow to -inf and +inf, u = NaN, and
    np.clip keeps it; gains just inside the guard stay in the fast blocks."""
    monkeypatch.setenv("FGX_EPISODE_KERNEL", "classic")
    over = {"controller_kwargs": {"p_gains": (0.6, gain, 0.6, 0.6, 0.6), "d_gains": (0.075, gain, 0.075, 0.075, 0.075)}}
    N = 128
    env = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=N, device=DEV, info_level=0,
                   mp_config_override=over)

    def setup(env, ob):
        if gain < 1e150:
            return
        st = {k: np_(v) for k, v in env.get_state().items()}
        q, qd = st["q"].copy(), st["qd"].copy()
        q[3, 1], qd[3, 1] = 1e150, -1e150
        env.set_state(q=q, qd=qd)
        ob.env.q, ob.env.qd = q.copy(), qd.copy()
        ob.env._fk()
    rng = np.random.default_rng(9)
    _run_vs_oracle(env, "LongSimpleReacher", [rng.standard_normal((N, env.n_params), dtype=np.float32)
                                              for _ in range(2)], setup=setup)


def test_fast_path_guard_restored_extreme_state(monkeypatch):
    """set_state (checkpoint restore) with |q| = 1e250 and opposite-signed qd in some lanes (outside
    the guard: generic path), q = inf / qd = -inf in one (u = -inf + inf = NaN, np.clip keeps it)
    and |q| = 9e149 in others (inside the guard: fast blocks, finite, clipped)."""
    monkeypatch.setenv("FGX_EPISODE_KERNEL", "classic")
    N = 256
    env = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=N, device=DEV, info_level=0)

    def setup(env, ob):
        st = {k: np_(v) for k, v in env.get_state().items()}
        q, qd = st["q"].copy(), st["qd"].copy()
        q[5, 1], qd[5, 1] = 1e250, -1e250
        q[70, :], qd[70, :] = -1e250, 1e250
        q[9, 3], qd[9, 3] = np.inf, -np.inf          # u = -inf + inf = NaN
        q[130:140, 2], qd[130:140, 2] = 9e149, -9e149
        env.set_state(q=q, qd=qd)
        ob.env.q, ob.env.qd = q.copy(), qd.copy()
        ob.env._fk()
    rng = np.random.default_rng(10)
    _run_vs_oracle(env, "LongSimpleReacher", [rng.standard_normal((N, env.n_params), dtype=np.float32)
                                              for _ in range(2)], setup=setup)


@pytest.mark.parametrize("kernel", ["classic", "jl"])
def test_fast_path_guard_weights_scale(monkeypatch, kernel):
    """trajectory_generator_kwargs weights_scale = 1e12 is carried by the ProMP table
    (table = f32(weights_scale * phi)): a lane with |w| ~ 1e28 overflows its f32 position to inf
    (velocity NaN, u NaN, np.clip keeps it).  The NaN-free guard bounds |w| by 1e30 / (the table's
    largest row L1 norm), so that wave takes the exact path; waves of ordinary weights (positions
    ~1e12, controls clipped to +-1000) stay in the fast blocks.  k_episode and k_episode_jl."""
    monkeypatch.setenv("FGX_EPISODE_KERNEL", kernel)
    over = {"trajectory_generator_kwargs": {"weights_scale": 1e12}}
    N = 256
    env = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=N, device=DEV, info_level=0,
                   mp_config_override=over)
    assert kernel_is(env.episode_kernel(), {"classic": "k_episode", "jl": "k_episode_jl"}[kernel])
    assert float(np_(env.tables())[:, :5].max()) > 1e10
    rng = np.random.default_rng(12)
    plist = []
    for b in range(2):
        p = rng.standard_normal((N, env.n_params), dtype=np.float32)
        p[64 + 9, 3] = np.float32(1e28)
        p[130, 20] = np.float32(-3e27)
        p[192:256] *= np.float32(1e-9)
        plist.append(p)
    _run_vs_oracle(env, "LongSimpleReacher", plist)


# ------------------------------------------------------------------------------ reset_mask / checks
def test_reset_mask_rows_and_length_checks():
    N = 96
    env = fgx.make("fancy_ProMP/HoleReacher-v0", num_envs=N, device=DEV, info_level=0)
    o_all, _ = env.reset(seed=3)
    env.step(torch.zeros((N, env.n_params), device=DEV))
    o_cur, _ = env.reset(options={"reset_mask": np.zeros(N, bool)})   # nothing reset: current obs
    mask = np.zeros(N, bool)
    mask[::4] = True
    o_m, _ = env.reset(options={"reset_mask": mask})
    np.testing.assert_array_equal(np_(o_m)[~mask], np_(o_cur)[~mask])
    with pytest.raises(ValueError):
        env.reset(seed=[1, 2, 3])
    with pytest.raises(ValueError):
        env.reset(options={"reset_mask": np.ones(N - 1, bool)})
