"""The verbose-2 per-step info arrays row by row (black_box_wrapper.py:184-189,218-227,244-249),
written by the logging k_episode through the wave's LDS staging slots (InfoStage, fgx_device.h), and
for SimpleReacher + PD by k_episode_v2 (fgx_v2.h: dynamics and observation-trigonometry waves).

Every element of every array is checked, not only the rows before trajectory_length: rows < L
against the oracle, rows >= L as the host contract states (NaN; 0 for the flags), the desired plan
(positions / velocities) in full.  The batch sizes cover full waves, a partial last wave with
N % 4 == 0 and one with N % 4 != 0 (the element-wise tail of InfoStage::flush).
"""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from oracle import batched
from test_gpu_parity import NAME, close, ctrl_of, np_, oracle_kwargs, spec_of, split_tables, oracle_tables_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

CASES = [
    ("fancy_ProMP/LongSimpleReacher-v0", None),
    ("fancy_ProDMP/HoleReacher-v0", None),
    ("fancy_DMP/HoleReacher-v0", {"controller_kwargs": {"controller_type": "velocity"}}),
    ("fancy_ProDMP/SimpleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}}),
]


def _rows(dev, ref, L, name, T):
    """rows < L equal the oracle's, rows >= L are the padding (NaN, 0 for the u8 flags)"""
    d = np_(dev[name]).astype(np.float64)
    r = np.asarray(ref[name], np.float64)
    live = np.arange(T)[None, :] < L[:, None]
    close(d[live], r[live])
    pad = d[~live]
    if name in ("is_collided", "is_success"):
        assert (pad == 0).all(), name
    else:
        assert np.isnan(pad).all(), name


@pytest.mark.parametrize("N", [256, 1000, 203])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_info_rows_vs_oracle(ci, N, monkeypatch):
    env_id, over = CASES[ci]
    # SimpleReacher + PD: k_episode_v2 (fgx_v2.h); HoleReacher (simple reward, 5 links): k_episode_v2h,
    # and (N = 1000, FGX_HP=1) k_episode_hp's INFO instantiation (fgx_hp.h)
    hp = "Hole" in env_id and N == 1000
    if hp:
        monkeypatch.setenv("FGX_HP", "1")
    env = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=2)
    # (k_episode_v2h at a multiple of 256 envs, else the logging k_episode)
    hole = "k_episode_hp" if hp else ("k_episode_v2h" if N % 256 == 0 else "k_episode")
    want = hole if "Hole" in env_id else "k_episode_v2"
    assert env.episode_kernel(info_level=2) == want
    spec = spec_of(env)
    tabs = oracle_tables_dict(spec, env)   # the oracle's own tables (== the device's, bit for bit)
    ob = batched.BatchedBB(NAME[env_id.split("/")[1]], N, ctrl_of(env), mp_spec=spec, info_level=2, tables=tabs,
                           **oracle_kwargs(env))
    env.reset(seed=500)
    ob.reset(seed=500)
    rng = np.random.default_rng(ci * 1000 + N)
    for _ in range(2):
        params = rng.standard_normal((N, env.n_params), dtype=np.float32)
        _, _, _, _, info = env.step(torch.from_numpy(params).to(DEV))
        _, _, _, _, r_info = ob.step(params)
        L = r_info["trajectory_length"]
        np.testing.assert_array_equal(np_(info["trajectory_length"]), L)
        T = env.T
        np.testing.assert_array_equal(np_(info["positions"]), r_info["positions"])
        np.testing.assert_array_equal(np_(info["velocities"]), r_info["velocities"])
        for name in ("step_actions", "step_observations", "step_rewards"):
            _rows(info, r_info, L, name, T)
        keys = ("is_collided", "is_success", "end_effector") if "is_collided" in info else ("reward_dist",
                                                                                         "reward_ctrl")
        for name in keys:
            _rows(info, r_info, L, name, T)


REPLAN = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}}


@pytest.mark.parametrize("env_id,over", [("fancy_ProMP/LongSimpleReacher-v0", None),
                                         ("fancy_ProDMP/SimpleReacher-v0", REPLAN),
                                         ("fancy_ProDMP/HoleReacher-v0", None)])
def test_logging_step_equals_fast_step(env_id, over):
    """info_level=2 (the logging k_episode, + k_info_obs for SimpleReacher) and info_level=0 (the fast
    kernels) give bit-identical steps; the last logged observation row of an env is its final
    observation bit for bit (full observations: the replanning config has no context mask)."""
    N = 1061
    a = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=2)
    b = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=0)
    np.testing.assert_array_equal(np_(a.reset(seed=21)[0]), np_(b.reset(seed=21)[0]))
    rng = np.random.default_rng(5)
    full = a._eng.cfg.return_context == 0
    for _ in range(3):
        p = torch.from_numpy(rng.standard_normal((N, a.n_params), dtype=np.float32)).to(DEV)
        oa, ra, ta, ua, ia = a.step(p)
        ob, rb, tb, ub, ib = b.step(p)
        for x, y in ((oa, ob), (ra, rb), (ta, tb), (ua, ub), (ia["trajectory_length"], ib["trajectory_length"]),
                     (ia["final_observation"], ib["final_observation"])):
            np.testing.assert_array_equal(np_(x), np_(y))
        if full:
            L = np_(ia["trajectory_length"]).astype(np.int64)
            so = np_(ia["step_observations"])
            last = so[np.arange(N), L - 1]
            np.testing.assert_array_equal(last, np_(ia["final_observation"]))


V2_CASES = [
    ("fancy_ProMP/LongSimpleReacher-v0", None, {}),
    ("fancy_DMP/LongSimpleReacher-v0", None, {}),
    ("fancy_ProDMP/SimpleReacher-v0", REPLAN, {}),
    ("fancy_ProMP/SimpleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(30),
                                                           "condition_on_desired": True}}, {}),
    ("fancy_ProMP/LongSimpleReacher-v0", {"basis_generator_kwargs": {"num_basis": 7}}, {}),   # generic basis count
    ("fancy_ProMP/SimpleReacher-v0", None, {"target": (0.5, 1.0)}),
]


@pytest.mark.parametrize("N", [1000, 203])
@pytest.mark.parametrize("info_level", [1, 2])
@pytest.mark.parametrize("ci", range(len(V2_CASES)))
def test_v2_equals_logging_kernel(ci, info_level, N, monkeypatch):
    """k_episode_v2 (fgx_v2.h) against the logging k_episode + k_info_obs (FGX_V2=0, read at every
    launch): every per-step array, the step outputs and the whole device state bit for bit (NaN
    padding included), over steps that truncate and auto-reset (6 BB steps of up to 200 samples,
    TimeLimit 200), partial last waves (203, 1000) and replanning segments."""
    env_id, over, kw = V2_CASES[ci]
    a = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=info_level, **kw)
    b = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=info_level, **kw)
    assert a.episode_kernel() == "k_episode_v2"
    np.testing.assert_array_equal(np_(a.reset(seed=8)[0]), np_(b.reset(seed=8)[0]))
    rng = np.random.default_rng(ci + 10 * info_level)
    for _ in range(6):
        p = torch.from_numpy((rng.standard_normal((N, a.n_params)) * 3).astype(np.float32)).to(DEV)
        monkeypatch.delenv("FGX_V2", raising=False)
        ra = a.step(p)
        monkeypatch.setenv("FGX_V2", "0")
        rb = b.step(p)
        monkeypatch.delenv("FGX_V2")
        for x, y in zip(ra[:4], rb[:4]):
            np.testing.assert_array_equal(np_(x), np_(y))
        keys = [k for k in ra[4] if isinstance(ra[4][k], torch.Tensor) and not k.startswith("_")]
        assert "reward_dist" in keys and (info_level < 2 or "step_observations" in keys)
        for k in keys:
            np.testing.assert_array_equal(np_(ra[4][k]), np_(rb[4][k]), err_msg=k)
        sa, sb = a.get_state(), b.get_state()
        for k in sa:
            np.testing.assert_array_equal(np_(sa[k]), np_(sb[k]), err_msg=k)


@pytest.mark.parametrize("env_id", ["fancy_ProMP/LongSimpleReacher-v0", "fancy_ProMP/SimpleReacher-v0"])
def test_v2_observation_fallback_lanes(env_id, monkeypatch):
    """k_episode_v2's observation fast path (fgx_sincos_fast + angle-addition FK, each f32 result
    checked against its error bound) and its exact recompute, lane by lane: joint angles beyond the
    fast reduction's range (|q| >= 2^20), angles whose sin / cos round below f32 resolution of the
    margin (q ~ 1e-9, q0 = pi / 2) and ordinary lanes in the same waves; every observation row bit for
    bit against the logging k_episode + k_info_obs (exact sincos throughout)."""
    N = 640
    a = fgx.make(env_id, num_envs=N, device=DEV)
    b = fgx.make(env_id, num_envs=N, device=DEV)
    assert a.episode_kernel() == "k_episode_v2"
    a.reset(seed=3)
    b.reset(seed=3)
    rng = np.random.default_rng(7)
    st = a.get_state()
    q = np_(st["q"]).copy()
    q[0:N:5] = rng.choice([-1.0, 1.0], q[0:N:5].shape) * 10.0 ** rng.uniform(6.5, 9, q[0:N:5].shape)
    q[1:N:5] = rng.uniform(-1e-9, 1e-9, q[1:N:5].shape)
    q[2:N:5, 0] = np.pi / 2
    qd = np.zeros_like(q)
    for e in (a, b):
        e.set_state(q=q, qd=qd)
    p = torch.from_numpy((rng.standard_normal((N, a.n_params)) * 0.01).astype(np.float32)).to(DEV)
    monkeypatch.delenv("FGX_V2", raising=False)
    ra = a.step(p)
    monkeypatch.setenv("FGX_V2", "0")
    rb = b.step(p)
    monkeypatch.delenv("FGX_V2")
    np.testing.assert_array_equal(np_(ra[0]), np_(rb[0]))
    np.testing.assert_array_equal(np_(ra[4]["step_observations"]), np_(rb[4]["step_observations"]))
    assert np.isfinite(np_(ra[4]["step_observations"])[:, :10]).all()


V2H_CASES = [
    ("fancy_ProDMP/HoleReacher-v0", None, {}),
    ("fancy_DMP/HoleReacher-v0", None, {}),
    ("fancy_ProMP/HoleReacher-v0", None, {"allow_self_collision": True}),
    ("fancy_ProDMP/HoleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(50)}}, {}),
    ("fancy_ProMP/ViaPointReacher-v0", None, {}),
    ("fancy_DMP/HoleReacher-v0", None, {"n_links": 2}),
]


def _hp_or_v2h(a, kern, info_level=2):
    """the kernel under test: k_episode_hp where it applies (HoleReacher, simple reward, 5 links: info
    level 1 by default, level 2 with kern == "hp", FGX_HP=1), else k_episode_v2h; kern == "v2h" runs
    with FGX_HP=0 (k_episode_v2h everywhere)"""
    k = a.episode_kernel(info_level=info_level)
    if kern == "v2h" or (kern == "default" and info_level >= 2):
        assert k == "k_episode_v2h", k
    else:
        assert k in ("k_episode_v2h", "k_episode_hp"), k
    return k


# FGX_HP=1 only changes the level-2 dispatch, so "hp" runs at level 2 and one size only
V2H_KERNS = [(k, lvl, n) for k in ("default", "v2h") for lvl in (1, 2) for n in (512, 1024)] + [("hp", 2, 512)]


@pytest.mark.parametrize("kern,info_level,N", V2H_KERNS)
@pytest.mark.parametrize("ci", range(len(V2H_CASES)))
def test_v2h_equals_logging_kernel(ci, info_level, N, kern, monkeypatch):
    """k_episode_v2h (fgx_kernels.h: the logging body on waves 0..3, its per-step rows stored by waves
    4..7) against the logging k_episode (FGX_V2=0): every per-step array, the step outputs and the
    whole device state bit for bit over 6 BB steps with collisions (terminations at every sample),
    auto-resets and replanning segments."""
    env_id, over, kw = V2H_CASES[ci]
    if kern != "default":
        monkeypatch.setenv("FGX_HP", "0" if kern == "v2h" else "1")
    a = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=info_level, **kw)
    b = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=info_level, **kw)
    _hp_or_v2h(a, kern, info_level)
    np.testing.assert_array_equal(np_(a.reset(seed=5)[0]), np_(b.reset(seed=5)[0]))
    rng = np.random.default_rng(ci + 10 * info_level)
    lengths = set()
    for _ in range(6):
        p = torch.from_numpy((rng.standard_normal((N, a.n_params)) * 3).astype(np.float32)).to(DEV)
        monkeypatch.delenv("FGX_V2", raising=False)
        ra = a.step(p)
        monkeypatch.setenv("FGX_V2", "0")
        rb = b.step(p)
        monkeypatch.delenv("FGX_V2")
        for x, y in zip(ra[:4], rb[:4]):
            np.testing.assert_array_equal(np_(x), np_(y))
        keys = [k for k in ra[4] if isinstance(ra[4][k], torch.Tensor) and not k.startswith("_")]
        assert "is_collided" in keys and (info_level < 2 or "step_observations" in keys)
        for k in keys:
            np.testing.assert_array_equal(np_(ra[4][k]), np_(rb[4][k]), err_msg=k)
        sa, sb = a.get_state(), b.get_state()
        for k in sa:
            np.testing.assert_array_equal(np_(sa[k]), np_(sb[k]), err_msg=k)
        lengths |= set(np_(ra[4]["trajectory_length"]).tolist())
    if "Hole" in env_id:
        assert len(lengths) > 2   # collisions ended episodes at different samples


@pytest.mark.parametrize("kern", ["default", "v2h", "hp"])
@pytest.mark.parametrize("env_id,over", [("fancy_ProDMP/HoleReacher-v0", None),
                                         ("fancy_ProMP/ViaPointReacher-v0",
                                          {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(40)}})])
def test_v2h_nonfinite_lanes(env_id, over, kern, monkeypatch):
    """k_episode_v2h with NaN / inf parameters and NaN / huge joint angles mixed into ordinary waves:
    a NaN action passes np.clip, NaN positions never collide, so those envs keep running with NaN
    state and their observation rows carry NaN cos / sin (the storing wave's placeholder, as sincos(NaN)
    in the logging kernel); bit for bit against the logging k_episode (FGX_V2=0).  Also a grid larger
    than one round of workgroups (N = 66048) and ViaPointReacher with a replanning schedule."""
    if kern != "default":
        monkeypatch.setenv("FGX_HP", "0" if kern == "v2h" else "1")
    for N in (768, 66048):
        a = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over)
        b = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over)
        _hp_or_v2h(a, kern)
        a.reset(seed=9)
        b.reset(seed=9)
        rng = np.random.default_rng(N)
        if N == 768:
            st = a.get_state()
            q = np_(st["q"]).copy()
            q[5:N:23, 1] = np.nan
            q[9:N:29, 2] = 1e7
            for e in (a, b):
                e.set_state(q=q)
        for it in range(3):
            p = (rng.standard_normal((N, a.n_params)) * 2).astype(np.float32)
            p[it::7] = np.nan
            p[3 + it::11, 2] = np.inf
            p[4::13, 0] = -np.inf
            p = torch.from_numpy(p).to(DEV)
            monkeypatch.delenv("FGX_V2", raising=False)
            ra = a.step(p)
            monkeypatch.setenv("FGX_V2", "0")
            rb = b.step(p)
            monkeypatch.delenv("FGX_V2")
            for x, y in zip(ra[:4], rb[:4]):
                np.testing.assert_array_equal(np_(x), np_(y))
            for k in [k for k in ra[4] if isinstance(ra[4][k], torch.Tensor) and not k.startswith("_")]:
                np.testing.assert_array_equal(np_(ra[4][k]), np_(rb[4][k]), err_msg=k)
            sa, sb = a.get_state(), b.get_state()
            for k in sa:
                np.testing.assert_array_equal(np_(sa[k]), np_(sb[k]), err_msg=k)
        if N == 768:   # some NaN-parameter envs ran to the end with NaN rows
            so = np_(ra[4]["step_observations"])
            L = np_(ra[4]["trajectory_length"])
            assert (np.isnan(so[it::7, 0, 1]) & (L[it::7] > 1)).any()
        del a, b


@pytest.mark.parametrize("mode", ["step_trajectory", "validity"])
def test_v2h_given_plans_and_validity(mode, monkeypatch):
    """k_episode_v2h on the other logging paths: caller-supplied plans (fgx_step_traj, MP_GIVEN: no
    basis table, the rows from the given arrays) and trajectory-validity checks (invalid plans pad
    every row, then the artificial transition after the last barrier); bit for bit against the
    logging k_episode."""
    N = 512
    env_id = "fancy_ProDMP/HoleReacher-v0"
    monkeypatch.setenv("FGX_HP", "0")   # (k_episode_hp reports for the handle's own plans; v2h is tested here)
    kw = {}
    if mode == "validity":
        kw["traj_validity"] = fgx.TrajValidity(pos_low=[-1.2] * 5, pos_high=[1.2] * 5, invalid_return=-3.0,
                                               terminated=True, truncated=False, obs="current")
    a = fgx.make(env_id, num_envs=N, device=DEV, **kw)
    b = fgx.make(env_id, num_envs=N, device=DEV, **kw)
    assert a.episode_kernel() == "k_episode_v2h"
    np.testing.assert_array_equal(np_(a.reset(seed=2)[0]), np_(b.reset(seed=2)[0]))
    rng = np.random.default_rng(12)
    for _ in range(4):
        p = torch.from_numpy((rng.standard_normal((N, a.n_params)) * 2).astype(np.float32)).to(DEV)
        if mode == "step_trajectory":
            pos, vel = a.trajectory(p)
            pos = pos + torch.from_numpy(rng.standard_normal(pos.shape).astype(np.float32) * 0.05).to(DEV)
        monkeypatch.delenv("FGX_V2", raising=False)
        ra = a.step_trajectory(pos, vel) if mode == "step_trajectory" else a.step(p)
        monkeypatch.setenv("FGX_V2", "0")
        rb = b.step_trajectory(pos, vel) if mode == "step_trajectory" else b.step(p)
        monkeypatch.delenv("FGX_V2")
        for x, y in zip(ra[:4], rb[:4]):
            np.testing.assert_array_equal(np_(x), np_(y))
        for k in [k for k in ra[4] if isinstance(ra[4][k], torch.Tensor) and not k.startswith("_")]:
            np.testing.assert_array_equal(np_(ra[4][k]), np_(rb[4][k]), err_msg=k)
        sa, sb = a.get_state(), b.get_state()
        for k in sa:
            np.testing.assert_array_equal(np_(sa[k]), np_(sb[k]), err_msg=k)
    if mode == "validity":
        tl = np_(ra[4]["trajectory_length"])
        assert (tl == 0).any() and (tl > 0).any()   # both valid and invalid plans took part
