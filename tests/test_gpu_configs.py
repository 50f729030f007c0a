"""Every BASELINE.json config at its stated per-GPU size on the device.

For each config the full batch runs on the GPU for >= 2 BB steps (black_box_wrapper.py:170-253)
and a strided subset of >= 256 envs is replayed by the batched oracle (oracle/batched.py), each
oracle env seeded with its GLOBAL index as the device env was (reset(seed=0) -> env i seeded i):
flags and trajectory lengths bit-exact, returns within 16 ulp, observations within 1e-5.  Config 3
(HoleReacher, collisions end episodes early) additionally compares the flags and lengths of the
FULL batch against the oracle, run in worker processes.  Each test also asserts which episode
kernel fgx_dispatch.h:episode_kernel_choice picks at that size (env.episode_kernel()).
"""
import concurrent.futures as cf
import multiprocessing as mproc

import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from oracle import batched
from tests.test_gpu_parity import DEV, kernel_is, NAME, assert_ulps, close, ctrl_of, np_, oracle_kwargs, spec_of, split_tables

pytestmark = pytest.mark.gpu

REPLAN25 = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}}
# (label, env id, override, envs per GPU, BB steps, expected kernel)
CONFIGS = [
    ("config2", "fancy_ProMP/SimpleReacher-v0", None, 4096, 2, "k_episode_jl"),
    ("config3", "fancy_ProDMP/HoleReacher-v0", None, 65536, 2, "k_episode_hp"),
    ("config3_shard", "fancy_ProDMP/HoleReacher-v0", None, 16384, 2, "k_episode_hp"),
    ("config4_shard", "fancy_DMP/LongSimpleReacher-v0", None, 32768, 2, "k_episode_jl"),
    ("config5_shard", "fancy_ProDMP/SimpleReacher-v0", REPLAN25, 8192, 4, "k_episode_jl"),
    ("metric", "fancy_ProMP/LongSimpleReacher-v0", None, 65536, 2, "k_episode"),
    # the metric's strong-scaling shards (65536 / G envs per GPU on G = 2, 4, 8 GPUs)
    ("metric_shard2", "fancy_ProMP/LongSimpleReacher-v0", None, 32768, 2, "k_episode_jl"),
    ("metric_shard4", "fancy_ProMP/LongSimpleReacher-v0", None, 16384, 2, "k_episode_jl"),
    ("metric_shard8", "fancy_ProMP/LongSimpleReacher-v0", None, 8192, 2, "k_episode_jl"),
    # past one round of waves: k_episode_w2 directly against the oracle (config 4 unsharded on one GPU)
    ("config4_one_gpu", "fancy_DMP/LongSimpleReacher-v0", None, 262144, 2, "k_episode_w2"),
    ("metric_x2", "fancy_ProMP/LongSimpleReacher-v0", None, 131072, 2, "k_episode_w2"),
]


def params_seq(N, P, n_bb):
    rng = np.random.default_rng(1234)
    return [rng.standard_normal((N, P), dtype=np.float32) for _ in range(n_bb)]


def subset_oracle(env, name, idx, params, over_kw):
    spec = spec_of(env)
    ob = batched.BatchedBB(name, len(idx), ctrl_of(env), mp_spec=spec,
                           **over_kw)
    o0 = ob._reset_idx(list(range(len(idx))), [int(i) for i in idx])
    return ob, o0


@pytest.mark.parametrize("ci", range(len(CONFIGS)), ids=[c[0] for c in CONFIGS])
def test_config_full_size_vs_oracle_subset(ci):
    label, env_id, over, N, n_bb, kernel = CONFIGS[ci]
    env = fgx.make(env_id, num_envs=N, device=DEV, mp_config_override=over, info_level=0)
    assert kernel_is(env.episode_kernel(), kernel), (label, env.episode_kernel())
    name = NAME[env_id.split("/")[1]]
    idx = np.unique(np.linspace(0, N - 1, 320).astype(np.int64))
    assert len(idx) >= 256
    o_g, _ = env.reset(seed=0)
    ob, o_r = subset_oracle(env, name, idx, None, oracle_kwargs(env))
    close(np_(o_g)[idx], o_r)
    for b, params in enumerate(params_seq(N, env.n_params, n_bb)):
        obs, ret, te, tr, info = env.step(torch.from_numpy(params).to(DEV))
        r_obs, r_ret, r_te, r_tr, r_info = ob.step(params[idx])
        tl = np_(info["trajectory_length"])
        np.testing.assert_array_equal(tl[idx], r_info["trajectory_length"])
        np.testing.assert_array_equal(np_(te)[idx].astype(bool), r_te)
        np.testing.assert_array_equal(np_(tr)[idx].astype(bool), r_tr)
        assert_ulps(np_(ret)[idx], r_ret, 16)
        close(np_(info["final_observation"])[idx], r_info["final_obs"])
        close(np_(obs)[idx], r_obs)
        # whole-batch invariants: lengths within the plan, returns finite, SimpleReacher never
        # terminates, every env of a non-replanning SimpleReacher plan runs to the TimeLimit
        assert tl.min() >= 1 and tl.max() <= env.T
        assert bool(torch.isfinite(ret).all())
        if name != "HoleReacher":
            assert not bool(te.any())
            if over is None:
                assert (tl == env.T).all() and bool(tr.all())


@pytest.mark.timeout(900)
def test_config3_full_batch_flags_and_lengths():
    """fancy_ProDMP/HoleReacher-v0 at 65536 envs: terminated / truncated flags and trajectory
    lengths of EVERY env bit-exact against the oracle for 2 BB steps (collisions end episodes at
    any sample, so this is the config where lengths carry information)."""
    N, n_bb = 65536, 2
    env = fgx.make("fancy_ProDMP/HoleReacher-v0", num_envs=N, device=DEV, info_level=0)
    env.reset(seed=0)
    plist = params_seq(N, env.n_params, n_bb)
    got = []
    for p in plist:
        _, ret, te, tr, info = env.step(torch.from_numpy(p).to(DEV))
        got.append((np_(info["trajectory_length"]), np_(te).astype(bool), np_(tr).astype(bool), np_(ret)))
    spec = spec_of(env)
    tables = None   # each worker's oracle builds its own tables (bit-identical to the device's)
    chunks = 16
    step = N // chunks
    jobs = [("HoleReacher", ctrl_of(env), spec, tables, oracle_kwargs(env), lo, lo + step,
             [p[lo:lo + step] for p in plist]) for lo in range(0, N, step)]
    # worker processes are spawned (fresh interpreters, numpy only); this process holds the GPU
    with cf.ProcessPoolExecutor(max_workers=8, mp_context=mproc.get_context("spawn")) as ex:
        res = dict(ex.map(batched.run_chunk, jobs))
    n_coll = 0
    for b in range(n_bb):
        tl = np.concatenate([res[lo][b][0] for lo in sorted(res)])
        te = np.concatenate([res[lo][b][1] for lo in sorted(res)])
        tr = np.concatenate([res[lo][b][2] for lo in sorted(res)])
        rr = np.concatenate([res[lo][b][3] for lo in sorted(res)])
        np.testing.assert_array_equal(got[b][0], tl)
        np.testing.assert_array_equal(got[b][1], te)
        np.testing.assert_array_equal(got[b][2], tr)
        assert_ulps(got[b][3], rr, 16)
        n_coll += int(te.sum())
    assert n_coll > 1000   # the batch really exercises collisions
