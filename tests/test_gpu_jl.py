"""k_episode_jl (fgx_jl.h, one lane per (env, joint)) against k_episode (one env per lane) and the oracle.

The joint-lane kernel serves SimpleReacher + PD with shared basis tables at info_level < 2 (the same
domain as k_episode_jp).  FGX_EPISODE_KERNEL=jl / =classic force either kernel for the same call, so
every output and the whole device state must agree bit for bit: partial waves and workgroups (N not
a multiple of 12 / 48 / 128 envs), lanes at different env steps / replanning phases (per-lane basis
rows instead of scalar loads), NaN / inf / huge parameters (the chunk redo with np.clip's NaN
propagation), per-joint gains, condition_on_desired and the generic basis count; the oracle checks
the jl results independently.
"""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from oracle import batched

from test_gpu_jp import CASES, _run, _same, _state
from test_gpu_parity import DEV, kernel_is, assert_ulps, close, ctrl_of, np_, oracle_kwargs, spec_of, split_tables

pytestmark = pytest.mark.gpu

JL_CASES = CASES + [
    ("fancy_ProMP/LongSimpleReacher-v0", None, 61, 2),       # one partial workgroup, idle lanes
    ("fancy_ProMP/LongSimpleReacher-v0", None, 8193, 2),     # the 8-GPU shard size + 1
    ("fancy_ProMP/LongSimpleReacher-v0", None, 98304, 2),    # dispatched past one round (half-full tail)
    ("fancy_ProMP/SimpleReacher-v0", None, 4097, 2),
    ("fancy_DMP/LongSimpleReacher-v0", {"basis_generator_kwargs": {"num_basis": 3}}, 97, 2),
    ("fancy_ProDMP/LongSimpleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(40)}}, 150, 6),
]


@pytest.mark.parametrize("ci", range(len(JL_CASES)))
def test_jl_equals_classic_kernel(ci):
    env_id, over, N, n_bb = JL_CASES[ci]
    probe = fgx.make(env_id, num_envs=N, device=DEV, info_level=0, mp_config_override=over)
    rng = np.random.default_rng(70 + ci)
    params = [rng.standard_normal((N, probe.n_params), dtype=np.float32) for _ in range(n_bb)]
    _same(_run(env_id, over, N, n_bb, "jl", 500 + ci, params),
          _run(env_id, over, N, n_bb, "classic", 500 + ci, params))


@pytest.mark.parametrize("env_id", ["fancy_ProMP/LongSimpleReacher-v0", "fancy_ProDMP/SimpleReacher-v0"])
def test_jl_equals_classic_nan_and_restored_steps(env_id):
    """NaN / inf / huge parameters and a restored state with every env at a different step
    (segments of every length 1..200; with replanning the plans start on different table rows)."""
    N = 320
    over = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}} if "ProDMP" in env_id else None
    probe = fgx.make(env_id, num_envs=N, device=DEV, info_level=0, mp_config_override=over)
    rng = np.random.default_rng(6)
    p = rng.standard_normal((3, N, probe.n_params)).astype(np.float32)
    p[0, 3, 4] = np.nan
    p[0, 70, 0] = np.inf
    p[0, 130, :] = 3e4
    p[1, 200, 3] = -np.inf
    probe.reset(seed=9)
    st = _state(probe)
    steps = (np.arange(N) * 7 % 200).astype(np.int32)
    qd = rng.uniform(-2, 2, st["qd"].shape)
    ss = dict(q=st["q"], qd=qd, steps=steps)
    a = _run(env_id, over, N, 3, "jl", 9, list(p), set_state=ss, mask_after_first=False)
    b = _run(env_id, over, N, 3, "classic", 9, list(p), set_state=ss, mask_after_first=False)
    _same(a, b)
    assert np.isnan(a[2][3]) and np.isfinite(a[2][5])   # the NaN env's return is NaN


def test_jl_vs_oracle_desynchronised():
    """jl against the oracle with lanes at different env steps (set_state)."""
    import os
    env_id, N = "fancy_ProMP/LongSimpleReacher-v0", 200
    old = os.environ.get("FGX_EPISODE_KERNEL")
    os.environ["FGX_EPISODE_KERNEL"] = "jl"
    try:
        env = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
        assert kernel_is(env.episode_kernel(), "k_episode_jl")
        spec = spec_of(env)
        ob = batched.BatchedBB("LongSimpleReacher", N, ctrl_of(env), mp_spec=spec,
                               **oracle_kwargs(env))
        env.reset(seed=23)
        ob.reset(seed=23)
        steps = (np.arange(N) % 200).astype(np.int32)
        env.set_state(steps=steps)
        ob.env.steps = steps.astype(np.int64)
        rng = np.random.default_rng(9)
        for b in range(2):
            params = rng.standard_normal((N, env.n_params), dtype=np.float32)
            obs, ret, te, tr, info = env.step(torch.from_numpy(params).to(DEV))
            r_obs, r_ret, r_te, r_tr, r_info = ob.step(params)
            np.testing.assert_array_equal(np_(info["trajectory_length"]), r_info["trajectory_length"])
            np.testing.assert_array_equal(np_(tr), r_tr)
            assert_ulps(np_(ret), r_ret, 16)
            close(np_(obs), r_obs)
            np.testing.assert_array_equal(np_(env.get_state()["q"]), ob.env.q)
            np.testing.assert_array_equal(np_(env.get_state()["steps"]), ob.env.steps)
    finally:
        if old is None:
            os.environ.pop("FGX_EPISODE_KERNEL", None)
        else:
            os.environ["FGX_EPISODE_KERNEL"] = old


@pytest.mark.parametrize("kern", ["jl", "classic", "jp", "ws"])
def test_jl_inner_steps_counter(kern):
    """step_into's device inner-step counters (FGX_INNER_SLOTS partial counters, one atomic per wave
    or workgroup, include/fgx.h) sum to the sum of trajectory lengths, for every episode kernel."""
    import os
    env_id, N = "fancy_ProMP/LongSimpleReacher-v0", 1000
    old = os.environ.get("FGX_EPISODE_KERNEL")
    os.environ["FGX_EPISODE_KERNEL"] = kern
    try:
        env = fgx.make(env_id, num_envs=N, device=DEV, info_level=0)
        env.reset(seed=1)
        env.set_state(steps=(np.arange(N) % 200).astype(np.int32))
        params = torch.randn((N, env.n_params), device=DEV)
        obs = torch.empty((N, env.out_dim), device=DEV)
        ret = torch.empty(N, dtype=torch.float64, device=DEV)
        te = torch.empty(N, dtype=torch.uint8, device=DEV)
        tr = torch.empty(N, dtype=torch.uint8, device=DEV)
        tl = torch.empty(N, dtype=torch.int32, device=DEV)
        acc = env.new_inner_steps()
        env.step_into(params, obs, ret, te, tr, tl, None, inner_steps=acc)
        env.step_into(params, obs, ret, te, tr, tl, None, inner_steps=acc)   # accumulates
        torch.cuda.synchronize()
        assert acc.numel() == 128 * 16 and int((acc != 0).sum()) > 1   # spread over the lines
        env.reset(seed=1)
        env.set_state(steps=(np.arange(N) % 200).astype(np.int32))
        tot = 0
        for _ in range(2):
            env.step_into(params, obs, ret, te, tr, tl, None)
            tot += int(tl.sum().item())
        assert int(acc.sum().item()) == tot
    finally:
        if old is None:
            os.environ.pop("FGX_EPISODE_KERNEL", None)
        else:
            os.environ["FGX_EPISODE_KERNEL"] = old


@pytest.mark.parametrize("rw", ["auto", "0", "1"])
@pytest.mark.parametrize("N", [1000, 8192, 32768])
def test_jl_equals_classic_split_autoreset(N, rw, monkeypatch):
    """The auto-reset of truncated envs runs on each jl workgroup's reset wave, beside the joint waves'
    episodes (fgx_jl.h: it overwrites the env state once every joint wave holds it in registers), or
    (FGX_JL_RW=0, and by default past one workgroup per CU) on the reset group after the gather:
    random_start False (the start angle is restored, base_reacher.py:77-93) with envs at every env
    step, so only some envs of a workgroup truncate; jl and k_episode agree bit for bit, state
    included."""
    env_id = "fancy_ProMP/LongSimpleReacher-v0"
    rng = np.random.default_rng(91)
    params = [rng.standard_normal((N, 25), dtype=np.float32) for _ in range(3)]
    outs = []
    if rw != "auto":
        monkeypatch.setenv("FGX_JL_RW", rw)
    for kern in ("jl", "classic"):
        monkeypatch.setenv("FGX_EPISODE_KERNEL", kern)
        env = fgx.make(env_id, num_envs=N, device=DEV, info_level=0, random_start=False)
        out = [np_(env.reset(seed=17)[0])]
        env.set_state(steps=(np.arange(N) % 200).astype(np.int32))
        for p in params:
            obs, ret, te, tr, info = env.step(torch.from_numpy(p).to(DEV))
            out += [np_(obs), np_(ret), np_(te), np_(tr), np_(info["trajectory_length"]),
                    np_(info["final_observation"])]
            out += list(_state(env).values())
        assert kernel_is(env.episode_kernel(), "k_episode_jl" if kern == "jl" else "k_episode")
        outs.append(out)
    _same(outs[0], outs[1])


def test_jl_helper_form_not_in_release_build(monkeypatch):
    """k_episode_jl's helper form (fgx_jl.h HLP; measured slower) is compiled only into
    diagnostics builds (-DFGX_JL_HELPER_FORM): asking the release library for it is an error, not a
    silent fallback to the plain kernel."""
    monkeypatch.setenv("FGX_JL_HELPER", "1")
    monkeypatch.setenv("FGX_EPISODE_KERNEL", "jl")
    env = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=64, device=DEV, info_level=0)
    env.reset(seed=1)
    with pytest.raises(ValueError, match="helper form"):
        env.step(torch.zeros((64, env.n_params), device=DEV))

