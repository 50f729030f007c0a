"""Edge sizes of the batch.  An empty batch is rejected (fgx_create: n_envs must be positive, a
ValueError on the Python side); a single env — one active lane of one wave, so no fast 8-sample
block of k_episode is taken and k_episode_jl runs one env in a partial wave — matches the oracle
with either episode kernel forced."""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from oracle import batched

from test_gpu_parity import DEV, kernel_is, NAME, assert_ulps, close, ctrl_of, np_, oracle_kwargs, spec_of, split_tables, oracle_tables_dict

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
    assert kernel_is(env.episode_kernel(), "k_episode_jl" if kern == "jl" else "k_episode")
    spec = spec_of(env)
    tabs = oracle_tables_dict(spec, env)   # the oracle's own tables (== the device's, bit for bit)
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


def test_single_env_matches_vector_env():
    """gym_compat.SingleEnv (what gym.make returns after fgx.register_gymnasium) is one env of the
    vector env without auto-reset: the same observation, return, flags and info row."""
    import numpy as np
    env_id = "fancy_ProMP/LongSimpleReacher-v0"
    one = fgx.SingleEnv(env_id, device=DEV, info_level=2)
    vec = fgx.make(env_id, num_envs=1, device=DEV, autoreset=False, info_level=2)
    o1, _ = one.reset(seed=11)
    ov, _ = vec.reset(seed=11)
    np.testing.assert_array_equal(o1, np_(ov)[0])
    a = np.random.default_rng(0).standard_normal(one.action_space.shape).astype(np.float32)
    for _ in range(2):
        o1, r1, t1, u1, i1 = one.step(a)
        ov, rv, tv, uv, iv = vec.step(torch.from_numpy(a[None]))
        np.testing.assert_array_equal(o1, np_(ov)[0])
        assert r1 == float(rv[0]) and t1 == bool(te_(tv)) and u1 == bool(te_(uv))
        assert i1["trajectory_length"] == int(iv["trajectory_length"][0])
        np.testing.assert_array_equal(i1["step_rewards"], np_(iv["step_rewards"])[0, :i1["trajectory_length"]])


def te_(t):
    return t[0].item()


def test_kernel_sincos_bit_equals_ocml():
    """fgx_trig.h's sincos (the ocml algorithm, small-argument reduction inlined) equals the ocml
    library call bit for bit over random, near-multiple-of-pi/2, huge and special arguments."""
    import ctypes
    import numpy as np
    from fancy_gym_crowd_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(5)
    k = np.arange(-2000, 2000, dtype=np.float64)
    xs = np.concatenate([
        rng.uniform(-7, 7, 400000), rng.uniform(-1e4, 1e4, 200000), rng.uniform(-1e9, 1e9, 50000),
        rng.standard_normal(100000) * 1e-6, k * (np.pi / 2), np.nextafter(k * (np.pi / 2), np.inf),
        np.nextafter(k * (np.pi / 4), -np.inf), np.array([0.0, -0.0, 5e-324, -5e-324, 2.0 ** 30, -(2.0 ** 30),
                                                          np.nextafter(2.0 ** 30, 0), 1e300, -1e300, np.inf,
                                                          -np.inf, np.nan, np.pi / 4, 3 * np.pi / 4])])
    x = torch.from_numpy(xs).to(DEV)
    out = torch.empty(4 * len(xs), dtype=torch.float64, device=DEV)
    assert lib.fgx_selftest_sincos(ctypes.c_void_p(x.data_ptr()), len(xs), ctypes.c_void_p(out.data_ptr()),
                                   None) == 0
    torch.cuda.synchronize()
    o = np_(out).reshape(-1, 4).view(np.int64)
    np.testing.assert_array_equal(o[:, 0], o[:, 2])
    np.testing.assert_array_equal(o[:, 1], o[:, 3])
