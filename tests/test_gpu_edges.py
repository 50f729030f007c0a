"""Edge sizes of the batch.  An empty batch is rejected (fgx_create: n_envs must be positive, a
ValueError on the Python side); a single env — one active lane of one wave, so no fast 8-sample
block of k_episode is taken and k_episode_jl runs one env in a partial wave — matches the oracle
with either episode kernel forced."""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from oracle import batched

from test_gpu_parity import DEV, NAME, assert_ulps, close, ctrl_of, np_, oracle_kwargs, spec_of, split_tables

pytestmark = pytest.mark.gpu


def test_empty_batch_rejected():
    with pytest.raises(ValueError):
        fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=0, device=DEV)


@pytest.mark.parametrize("kern", ["classic", "jl"])
@pytest.mark.parametrize("env_id", ["fancy_ProMP/LongSimpleReacher-v0", "fancy_ProDMP/SimpleReacher-v0",
                                    "fancy_DMP/LongSimpleReacher-v0"])
def test_single_env_vs_oracle(env_id, kern, monkeypatch):
    monkeypatch.setenv("FGX_EPISODE_KERNEL", kern)
    N = 1
    env = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
    assert env.episode_kernel() == ("k_episode_jl" if kern == "jl" else "k_episode")
    spec = spec_of(env)
    tabs = split_tables(spec, np_(env.tables()))
    ob = batched.BatchedBB(NAME[env_id.split("/")[1]], N, ctrl_of(env), mp_spec=spec, tables=tabs,
                           **oracle_kwargs(env))
    close(np_(env.reset(seed=5)[0]), ob.reset(seed=5))
    rng = np.random.default_rng(9)
    for _ in range(2):
        p = rng.standard_normal((N, env.n_params), dtype=np.float32)
        obs, ret, te, tr, info = env.step(torch.from_numpy(p).to(DEV))
        r_obs, r_ret, r_te, r_tr, r_info = ob.step(p)
        np.testing.assert_array_equal(np_(info["trajectory_length"]), r_info["trajectory_length"])
        np.testing.assert_array_equal(np_(te), r_te)
        np.testing.assert_array_equal(np_(tr), r_tr)
        assert_ulps(np_(ret), r_ret, 16)
        close(np_(obs), r_obs)
