"""k_episode_pair (fgx_kernels.h episode_body PAIR: two lanes per HoleReacher env, the FK sincos and
the collision tests divided between them) against k_episode (one env per lane).

FGX_EPISODE_KERNEL=classic forces k_episode for the same calls, so every output and the whole
device state must agree bit for bit: every MP kind and HoleReacher reward function, the allow_*
switches, replanning, learned tau (per-env plans), partial waves, arms past the joint limits and
bent into every collision, NaN parameters, and the device inner-step counter.  The oracle checks of
HoleReacher in test_gpu_parity.py / test_gpu_configs.py run on the pair kernel (the default).
"""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx

from test_gpu_jp import _same, _state
from test_gpu_parity import DEV, kernel_is, np_

pytestmark = pytest.mark.gpu

# (env id, mp_config_override, env kwargs, envs, BB steps)
CASES = [
    ("fancy_ProDMP/HoleReacher-v0", None, {}, 1000, 3),                               # config 3's MP
    ("fancy_ProMP/HoleReacher-v0", None, {"rew_fct": "vel_acc"}, 333, 3),
    ("fancy_DMP/HoleReacher-v0", None, {"rew_fct": "unbounded"}, 257, 3),
    ("fancy_ProDMP/HoleReacher-v0", None, {"allow_self_collision": True}, 128, 2),
    ("fancy_ProMP/HoleReacher-v0", None, {"allow_wall_collision": True}, 65, 2),
    ("fancy_ProDMP/HoleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}}, {}, 200, 8),
    ("fancy_ProMP/HoleReacher-v0", {"phase_generator_kwargs": {"learn_tau": True}}, {}, 300, 2),
    ("fancy_ProDMP/HoleReacher-v0", None, {"rew_fct": "vel_acc", "allow_self_collision": True}, 4097, 2),
]


def _run(env_id, over, kw, N, n_bb, kernel, seed, params, monkeypatch, set_state=None):
    monkeypatch.setenv("FGX_EPISODE_KERNEL", kernel)
    env = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=0, **kw)
    assert kernel_is(env.episode_kernel(), "k_episode" if kernel == "classic" else "k_episode_pair")
    out = [np_(env.reset(seed=seed)[0])]
    if set_state is not None:
        env.set_state(**set_state)
    for b in range(n_bb):
        obs, ret, te, tr, info = env.step(torch.from_numpy(params[b]).to(DEV))
        out += [np_(obs), np_(ret), np_(te), np_(tr), np_(info["trajectory_length"]),
                np_(info["final_observation"])]
        out += list(_state(env).values())
    return out


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_pair_equals_classic_kernel(ci, monkeypatch):
    env_id, over, kw, N, n_bb = CASES[ci]
    probe = fgx.make(env_id, num_envs=N, device=DEV, info_level=0, mp_config_override=over, **kw)
    rng = np.random.default_rng(90 + ci)
    scale = 2.0 if "learn_tau" not in str(over) else 1.0
    params = [(scale * rng.standard_normal((N, probe.n_params))).astype(np.float32) for _ in range(n_bb)]
    if over and "learn_tau" in str(over):
        for p in params:
            p[:, 0] = rng.uniform(0.2, 2.0, N)   # tau in the action space
    a = _run(env_id, over, kw, N, n_bb, "pair", 700 + ci, params, monkeypatch)
    b = _run(env_id, over, kw, N, n_bb, "classic", 700 + ci, params, monkeypatch)
    _same(a, b)


def test_pair_equals_classic_random_states_and_nan(monkeypatch):
    """Arms in arbitrary poses (joints past +-pi: the joint-limit collision; bent arms: segment
    crossings; links below ground next to the hole edges), every env at a different step, NaN / inf /
    huge parameters."""
    env_id, N = "fancy_ProDMP/HoleReacher-v0", 640
    probe = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
    rng = np.random.default_rng(17)
    probe.reset(seed=3)
    st = _state(probe)
    q = rng.uniform(-3.6, 3.6, st["q"].shape)
    q[:, 0] = rng.uniform(-0.5, 3.6, N)
    qd = rng.uniform(-3, 3, st["qd"].shape)
    steps = (np.arange(N) * 7 % 200).astype(np.int32)
    p = (3.0 * rng.standard_normal((3, N, probe.n_params))).astype(np.float32)
    p[0, 5, 2] = np.nan
    p[0, 77, 0] = np.inf
    p[1, 300, :] = 3e4
    ss = dict(q=q, qd=qd, steps=steps)
    a = _run(env_id, None, {}, N, 3, "pair", 11, list(p), monkeypatch, set_state=ss)
    b = _run(env_id, None, {}, N, 3, "classic", 11, list(p), monkeypatch, set_state=ss)
    _same(a, b)
    assert (a[5] < 200).any()   # collisions end some of these episodes early


def test_pair_inner_steps_counter(monkeypatch):
    """The even lane of each pair counts its env's trajectory length (one atomic per wave)."""
    monkeypatch.setenv("FGX_EPISODE_KERNEL", "pair")
    env_id, N = "fancy_ProDMP/HoleReacher-v0", 1000
    env = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
    assert env.episode_kernel() == "k_episode_pair"
    env.reset(seed=1)
    params = torch.randn((N, env.n_params), device=DEV) * 2
    obs = torch.empty((N, env.out_dim), device=DEV)
    ret = torch.empty(N, dtype=torch.float64, device=DEV)
    te = torch.empty(N, dtype=torch.uint8, device=DEV)
    tr = torch.empty(N, dtype=torch.uint8, device=DEV)
    tl = torch.empty(N, dtype=torch.int32, device=DEV)
    acc = env.new_inner_steps()
    tot = 0
    for _ in range(2):
        env.step_into(params, obs, ret, te, tr, tl, None, inner_steps=acc)
        tot += int(tl.sum().item())
    assert int(acc.sum().item()) == tot
