"""k_episode_hp (fgx_hp.h: HoleReacher as a producer wave of dynamics feeding two consumer waves of
FK / collision / reward through an LDS ring) against k_episode (FGX_EPISODE_KERNEL=classic): every
output and the whole device state bit for bit over several BB steps, at batch sizes with partial
workgroups, both workgroup shapes (one group of 64 envs per workgroup, four per workgroup), every MP
kind and controller, replanning segments, the allow_* switches, NaN / inf parameters, and envs whose
segments end by collision at every sample index (the return's pairwise split for every L)."""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from test_gpu_parity import DEV, np_

pytestmark = pytest.mark.gpu

REPLAN = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(50)}}
CASES = [
    # (env id, mp_config_override, env kwargs, N, BB steps, param scale)
    ("fancy_ProDMP/HoleReacher-v0", None, {}, 1000, 3, 1.0),            # config 3's env (PD)
    ("fancy_ProDMP/HoleReacher-v0", None, {}, 203, 3, 3.0),
    ("fancy_ProMP/HoleReacher-v0", None, {}, 777, 3, 1.0),              # velocity controller (f32 actions)
    ("fancy_DMP/HoleReacher-v0", None, {}, 512, 3, 0.3),
    ("fancy_ProDMP/HoleReacher-v0", REPLAN, {}, 640, 6, 1.0),           # replanning segments
    ("fancy_ProDMP/HoleReacher-v0", None, {"allow_self_collision": True}, 300, 3, 2.0),
    ("fancy_ProMP/HoleReacher-v0", None, {"allow_wall_collision": True}, 257, 3, 1.0),
    ("fancy_ProDMP/HoleReacher-v0", {"controller_kwargs": {"controller_type": "position"}}, {}, 129, 3, 1.0),
]


def _state(env):
    return {k: np_(v) for k, v in env.get_state().items()}


def _steps(env_id, over, kw, N, n_bb, plist, hp, monkeypatch, g=None, set_q=None):
    """(every output and state array in order, the trajectory lengths of each BB step)"""
    monkeypatch.delenv("FGX_HP", raising=False)
    monkeypatch.delenv("FGX_EPISODE_KERNEL", raising=False)
    monkeypatch.delenv("FGX_HP_G", raising=False)
    if not hp:
        monkeypatch.setenv("FGX_EPISODE_KERNEL", "classic")
    if g is not None:
        monkeypatch.setenv("FGX_HP_G", str(g))
    env = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=0, **kw)
    assert env.episode_kernel() == ("k_episode_hp" if hp else "k_episode")
    out = [np_(env.reset(seed=17)[0])]
    if set_q is not None:
        env.set_state(q=set_q)
    tls = []
    for b in range(n_bb):
        obs, ret, te, tr, info = env.step(torch.from_numpy(plist[b]).to(DEV))
        tls.append(np_(info["trajectory_length"]))
        out += [np_(obs), np_(ret), np_(te), np_(tr), tls[-1], np_(info["final_observation"])]
        out += list(_state(env).values())
    return out, tls


def _same(a, b):
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_array_equal(x, y, err_msg=f"output {i}")


@pytest.mark.parametrize("g", [1, 4])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_hp_equals_k_episode(ci, g, monkeypatch):
    env_id, over, kw, N, n_bb, scale = CASES[ci]
    probe = fgx.make(env_id, num_envs=8, device=DEV, mp_config_override=over, info_level=0, **kw)
    rng = np.random.default_rng(100 + ci)
    plist = [(rng.standard_normal((N, probe.n_params)) * scale).astype(np.float32) for _ in range(n_bb)]
    del probe
    a, _ = _steps(env_id, over, kw, N, n_bb, plist, True, monkeypatch, g=g)
    b, _ = _steps(env_id, over, kw, N, n_bb, plist, False, monkeypatch)
    _same(a, b)


def test_hp_every_length_and_nonfinite(monkeypatch):
    """Collisions at every sample index 1..200 (so every pairwise split of the return, L <= 128 and
    every second-half start 64..96), NaN / inf parameters (NaN states never collide: full-length
    segments) and huge joint angles (the joint-limit self-collision at the first sample)."""
    env_id, N = "fancy_ProDMP/HoleReacher-v0", 4096
    probe = fgx.make(env_id, num_envs=8, device=DEV, info_level=0)
    P = probe.n_params
    del probe
    rng = np.random.default_rng(5)
    plist = []
    for b in range(4):
        p = (rng.standard_normal((N, P)) * rng.uniform(0.2, 6.0, (N, 1))).astype(np.float32)
        p[b::37] = np.nan
        p[3 + b::41, 4] = np.inf
        plist.append(p)
    # joint angles past the limits on some envs: the self-collision test's joint-limit clause ends
    # those segments at the first sample (base_reacher.py:38-39,111)
    st = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
    st.reset(seed=17)
    q = np_(st.get_state()["q"]).copy()
    del st
    q[::53, 2] = 4.0
    a, tla = _steps(env_id, None, {}, N, 4, plist, True, monkeypatch, g=4, set_q=q)
    b, _ = _steps(env_id, None, {}, N, 4, plist, False, monkeypatch, set_q=q)
    _same(a, b)
    lengths = set(np.concatenate(tla).tolist())
    assert 1 in lengths and 200 in lengths
    assert len(lengths) > 150, len(lengths)   # collisions at most sample indices: every pairwise split


def test_hp_full_batch_and_counter(monkeypatch):
    """Config 3's size (65536 envs, four groups per workgroup): bit-identical to k_episode, and the
    device inner-step counter (one atomic per consumer wave) equals the sum of trajectory lengths."""
    env_id, N = "fancy_ProDMP/HoleReacher-v0", 65536
    rng = np.random.default_rng(1234)
    plist = [rng.standard_normal((N, 30), dtype=np.float32) for _ in range(2)]
    a, _ = _steps(env_id, None, {}, N, 2, plist, True, monkeypatch)
    b, _ = _steps(env_id, None, {}, N, 2, plist, False, monkeypatch)
    _same(a, b)
    monkeypatch.delenv("FGX_EPISODE_KERNEL", raising=False)
    env = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
    assert env.episode_kernel() == "k_episode_hp"
    env.reset(seed=0)
    obs = torch.empty((N, env.out_dim), device=DEV)
    ret = torch.empty(N, dtype=torch.float64, device=DEV)
    te = torch.empty(N, dtype=torch.uint8, device=DEV)
    tr = torch.empty(N, dtype=torch.uint8, device=DEV)
    tl = torch.empty(N, dtype=torch.int32, device=DEV)
    acc = env.new_inner_steps()
    env.step_into(torch.from_numpy(plist[0]).to(DEV), obs, ret, te, tr, tl, inner_steps=acc)
    torch.cuda.synchronize()
    assert int(acc.sum().item()) == int(tl.to(torch.int64).sum().item())


INFO_CASES = [
    ("fancy_ProDMP/HoleReacher-v0", None, {}, 1000),
    ("fancy_ProMP/HoleReacher-v0", None, {}, 203),                      # velocity controller
    ("fancy_DMP/HoleReacher-v0", REPLAN, {}, 640),                      # replanning (TimeAwareObservation)
    ("fancy_ProDMP/HoleReacher-v0", None, {"allow_self_collision": True}, 256),
]


@pytest.mark.parametrize("g", [1, 4])
@pytest.mark.parametrize("info_level", [1, 2])
@pytest.mark.parametrize("ci", range(len(INFO_CASES)))
def test_hp_info_rows_equal_logging_kernel(ci, info_level, g, monkeypatch):
    """k_episode_hp's INFO instantiation (verbose-2 per-step arrays: plan rows from the producer, the
    other rows from the consumers, the last reward and the padding after trajectory_length from the
    producer at the end) against the logging k_episode (FGX_V2=0): every per-step array, the outputs and
    the device state bit for bit, NaN padding included, with NaN / inf parameters in some envs."""
    env_id, over, kw, N = INFO_CASES[ci]
    monkeypatch.setenv("FGX_HP_G", str(g))
    if info_level >= 2:
        monkeypatch.setenv("FGX_HP", "1")   # (the verbose-2 rows: k_episode_v2h by default)
    a = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=info_level, **kw)
    b = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=info_level, **kw)
    assert a.episode_kernel() == "k_episode_hp"
    np.testing.assert_array_equal(np_(a.reset(seed=6)[0]), np_(b.reset(seed=6)[0]))
    rng = np.random.default_rng(ci + 10 * info_level)
    lengths = set()
    for it in range(5):
        p = (rng.standard_normal((N, a.n_params)) * 2).astype(np.float32)
        p[it::29] = np.nan
        p[1 + it::31, 3] = np.inf
        p = torch.from_numpy(p).to(DEV)
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
    assert len(lengths) > 5


def test_hp_info_reward_aggregation(monkeypatch):
    """reward_aggregation=np.max reads the device step_rewards of k_episode_hp's INFO instantiation
    (info_level 0 requests only step_rewards): equal to the logging kernel's."""
    over = {"black_box_kwargs": {"reward_aggregation": np.max}}
    N = 512
    a = fgx.make("fancy_ProDMP/HoleReacher-v0", num_envs=N, device=DEV, mp_config_override=over, info_level=0)
    b = fgx.make("fancy_ProDMP/HoleReacher-v0", num_envs=N, device=DEV, mp_config_override=over, info_level=0)
    assert a.episode_kernel() == "k_episode_hp"
    a.reset(seed=3)
    b.reset(seed=3)
    rng = np.random.default_rng(3)
    for _ in range(3):
        p = torch.from_numpy(rng.standard_normal((N, a.n_params), dtype=np.float32)).to(DEV)
        monkeypatch.delenv("FGX_V2", raising=False)
        ra = a.step(p)
        monkeypatch.setenv("FGX_V2", "0")
        rb = b.step(p)
        monkeypatch.delenv("FGX_V2")
        for x, y in zip(ra[:4], rb[:4]):
            np.testing.assert_array_equal(np_(x), np_(y))


def test_hp_fast_fk_near_thresholds(monkeypatch):
    """info_level 0 takes the collision booleans from an error-bounded approximate FK and recomputes a
    lane exactly where a decision is within its bound (fgx_hp.h: hp_fast_collision, hp_link_wall_rb).
    Zero-velocity plans (ProMP, velocity controller, zero weights) hold each env at a pose built to sit
    on a decision's threshold for the whole segment: arms lying within 1e-17 .. 1e-12 of the ground
    (the wall test's skip rule and its end-point comparisons), links folded back to within 1e-13 ..
    1e-11 rad (ccw values around the self-collision test's 1e-12), the collinear reset pose, squares
    with touching segments; beside envs with random plans.  Bit-identical to k_episode."""
    env_id, N = "fancy_ProMP/HoleReacher-v0", 1024
    probe = fgx.make(env_id, num_envs=8, device=DEV, info_level=0)
    P = probe.n_params
    del probe
    st = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
    st.reset(seed=3)
    q = np_(st.get_state()["q"]).copy()
    del st
    poses = [[np.pi / 2, 0, 0, 0, 0], [np.pi / 2, np.pi / 2, np.pi / 2, np.pi / 2, np.pi / 2],
             [np.pi / 2, -np.pi / 2, -np.pi / 2, -np.pi / 2, -np.pi / 2]]
    for t in (0.0, 1e-17, 1e-16, 4e-16, 1e-15, 3e-15, 1e-14, 3e-14, 1e-13, 1e-12):
        for sgn in (1.0, -1.0):
            poses.append([sgn * t, 0, 0, 0, 0])                    # along +x, just above / below the ground
            poses.append([np.pi - sgn * t, 0, 0, 0, 0])            # along -x
            poses.append([sgn * t, 0, 0, np.pi / 2, 0])            # three links on the ground, two rising
    for dlt in (1e-13, 3e-13, 7e-13, 1e-12, 1.3e-12, 2e-12, 1e-11):
        for sgn in (1.0, -1.0):
            poses.append([np.pi / 2, sgn * (np.pi - dlt), 0, 0, 0])       # link 1 folded back onto link 0
            poses.append([np.pi / 2, 0.3, sgn * (np.pi - dlt), 0, 0])
            poses.append([np.pi / 2, 0, 0, sgn * (np.pi - dlt), sgn * dlt])
    poses = np.array(poses)
    n_pose = len(poses)
    assert n_pose < N // 2
    q[:n_pose] = poses
    rng = np.random.default_rng(11)
    plist = []
    for b in range(2):
        p = rng.standard_normal((N, P)).astype(np.float32)
        p[:n_pose] = 0.0                      # zero velocity: the pose holds for every sample
        plist.append(p)
    a, tla = _steps(env_id, None, {}, N, 2, plist, True, monkeypatch, g=1, set_q=q)
    b, tlb = _steps(env_id, None, {}, N, 2, plist, False, monkeypatch, set_q=q)
    _same(a, b)
    # the poses decide both ways: some collide at once, some hold for the whole segment
    assert (tla[0][:n_pose] == 1).any() and (tla[0][:n_pose] == 200).any()
