"""k_episode_w2 (fgx_kernels.h: the k_episode body compiled for two resident waves per SIMD, used for
5-link SimpleReacher past one round of waves) against k_episode: FGX_EPISODE_KERNEL=w2 / =classic
force either for the same call; every output and the whole device state agree bit for bit
(replanning, condition_on_desired, restored per-env steps, the velocity controller and the
caller-given trajectory path included), and the dispatch picks it past one round."""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx

from test_gpu_jp import _run, _same
from test_gpu_parity import DEV, np_

pytestmark = pytest.mark.gpu

W2_CASES = [
    ("fancy_ProMP/LongSimpleReacher-v0", None, 1000, 3),
    ("fancy_DMP/LongSimpleReacher-v0", None, 333, 2),
    ("fancy_ProDMP/LongSimpleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(40),
                                                                "condition_on_desired": True}}, 300, 6),
    ("fancy_ProMP/LongSimpleReacher-v0", {"controller_kwargs": {"controller_type": "velocity"}}, 256, 2),
]


@pytest.mark.parametrize("ci", range(len(W2_CASES)))
def test_w2_equals_classic_kernel(ci):
    env_id, over, N, n_bb = W2_CASES[ci]
    probe = fgx.make(env_id, num_envs=N, device=DEV, info_level=0, mp_config_override=over)
    rng = np.random.default_rng(40 + ci)
    params = [rng.standard_normal((N, probe.n_params), dtype=np.float32) for _ in range(n_bb)]
    _same(_run(env_id, over, N, n_bb, "w2", 300 + ci, params),
          _run(env_id, over, N, n_bb, "classic", 300 + ci, params))


def test_w2_dispatch_past_one_round(monkeypatch):
    monkeypatch.delenv("FGX_EPISODE_KERNEL", raising=False)
    n_round = 4 * 64 * torch.cuda.get_device_properties(DEV).multi_processor_count
    env = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=2 * n_round, device=DEV, info_level=0)
    assert env.episode_kernel() == "k_episode_w2"
    assert env.episode_kernel(info_level=2) == "k_episode_v2"   # per-step arrays: fgx_v2.h
    env1 = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=n_round, device=DEV, info_level=0)
    assert env1.episode_kernel() == "k_episode"
    # full-size run vs the forced k_episode on a strided subset of outputs
    env.reset(seed=0)
    params = torch.randn((2 * n_round, env.n_params), device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    obs, ret, te, tr, info = env.step(params)
    monkeypatch.setenv("FGX_EPISODE_KERNEL", "classic")
    env2 = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=2 * n_round, device=DEV, info_level=0)
    assert env2.episode_kernel() == "k_episode"
    env2.reset(seed=0)
    obs2, ret2, te2, tr2, info2 = env2.step(params)
    assert torch.equal(ret, ret2) and torch.equal(obs, obs2) and torch.equal(tr, tr2)
    assert torch.equal(info["final_observation"], info2["final_observation"])
