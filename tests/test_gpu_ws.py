"""k_episode_ws (fgx_ws.h, producer / consumer wave pairs) against k_episode, bit for bit.

FGX_EPISODE_KERNEL=ws forces the wave-specialised kernel wherever it applies; every output and
the whole device state must equal k_episode's (FGX_EPISODE_KERNEL=classic) for partial
workgroups, desynchronised lanes (reset_mask, restored steps), replanning phases, NaN / inf
parameters, per-joint gains, condition_on_desired and non-default basis counts.
"""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx

from test_gpu_jp import CASES, _run, _same, _state
from test_gpu_parity import DEV, kernel_is

pytestmark = pytest.mark.gpu

WS_CASES = CASES + [
    ("fancy_ProMP/LongSimpleReacher-v0", None, 65536 + 100, 2),
    ("fancy_ProDMP/SimpleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(64)}}, 300, 6),
]


@pytest.mark.parametrize("ci", range(len(WS_CASES)))
def test_ws_equals_classic_kernel(ci):
    env_id, over, N, n_bb = WS_CASES[ci]
    probe = fgx.make(env_id, num_envs=N, device=DEV, info_level=0, mp_config_override=over)
    rng = np.random.default_rng(70 + ci)
    params = [rng.standard_normal((N, probe.n_params), dtype=np.float32) for _ in range(n_bb)]
    _same(_run(env_id, over, N, n_bb, "ws", 500 + ci, params),
          _run(env_id, over, N, n_bb, "classic", 500 + ci, params))


def test_ws_equals_classic_nan_and_restored_steps():
    env_id, N = "fancy_ProMP/LongSimpleReacher-v0", 1000
    probe = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
    rng = np.random.default_rng(6)
    p = rng.standard_normal((3, N, probe.n_params)).astype(np.float32)
    p[0, 3, 4] = np.nan
    p[0, 70, 0] = np.inf
    p[0, 130, :] = 3e4
    p[1, 200, 7] = -np.inf
    probe.reset(seed=9)
    st = _state(probe)
    steps = (np.arange(N) * 7 % 200).astype(np.int32)
    ss = dict(q=st["q"], qd=rng.uniform(-2, 2, st["qd"].shape), steps=steps)
    a = _run(env_id, None, N, 3, "ws", 9, list(p), set_state=ss, mask_after_first=False)
    b = _run(env_id, None, N, 3, "classic", 9, list(p), set_state=ss, mask_after_first=False)
    _same(a, b)
    assert np.isnan(a[2][3]) and np.isfinite(a[2][5])


def test_episode_kernel_selection():
    """fgx_episode_kernel reports the measured choice (fgx_dispatch.h episode_kernel_choice)."""
    rp = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}}
    cases = [("fancy_ProMP/LongSimpleReacher-v0", None, 65536, 0, "k_episode"),      # the metric config
             ("fancy_ProMP/LongSimpleReacher-v0", None, 65536, 2, "k_episode_v2"),   # per-step info arrays
             ("fancy_ProMP/LongSimpleReacher-v0", None, 32768, 0, "k_episode_jl"),   # metric shards
             ("fancy_ProMP/LongSimpleReacher-v0", None, 8192, 0, "k_episode_jl"),
             ("fancy_ProMP/LongSimpleReacher-v0", None, 98304, 0, "k_episode_jl"),   # half-full 2nd round
             ("fancy_DMP/LongSimpleReacher-v0", None, 32768, 0, "k_episode_jl"),     # config 4 shard
             ("fancy_ProDMP/SimpleReacher-v0", rp, 8192, 0, "k_episode_jl"),         # config 5 shard
             ("fancy_ProMP/SimpleReacher-v0", None, 65536, 0, "k_episode_jl"),       # 2 links: every size
             ("fancy_ProDMP/HoleReacher-v0", None, 4096, 0, "k_episode_hp"),     # producer / consumer pipeline
             ("fancy_ProDMP/HoleReacher-v0", None, 4000, 1, "k_episode_hp"),     # info level 1: its rows instantiation
             ("fancy_ProDMP/HoleReacher-v0", None, 4096, 2, "k_episode_v2h"),    # verbose-2 rows, whole workgroups
             ("fancy_ProDMP/HoleReacher-v0", None, 4000, 2, "k_episode")]         # verbose-2 rows, a partial one
    for env_id, over, N, lvl, want in cases:
        env = fgx.make(env_id, num_envs=N, device=DEV, info_level=0, mp_config_override=over)
        assert kernel_is(env.episode_kernel(lvl), want), (env_id, N, lvl)
