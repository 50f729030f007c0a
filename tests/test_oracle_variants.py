"""Pin the CPU oracle for the widened env set against reference-generated fixtures
(tests/golden/variants.npz, made by tests/golden/make_golden.py "variants"):

* ViaPointReacher  (viapoint_reacher.py; registered envs/__init__.py:669-679)
* HoleReacher rew_fct "vel_acc" / "unbounded" (hole_reacher.py:48-58,
  hr_dist_vel_acc_reward.py, hr_unbounded_reward.py)

Everything bit-exact, including the reference's -inf ViaPointReacher rewards.
"""
import os

import numpy as np
import pytest

from oracle import batched, port
from tests.test_oracle_golden import table_traj

KINDS = {"via": ("ViaPointReacher", {}),
         "hole_velacc": ("HoleReacher", {"rew_fct": "vel_acc"}),
         "hole_unbounded": ("HoleReacher", {"rew_fct": "unbounded"})}


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "variants.npz"))


def test_via_resets(g):
    env = port.Reacher("ViaPointReacher")
    for s in range(64):
        o = env.reset(seed=s)
        np.testing.assert_array_equal(env.q, g["viareset_q0"][s])
        np.testing.assert_array_equal(env.via, g["viareset_via"][s])
        np.testing.assert_array_equal(env.goal, g["viareset_goal"][s])
        np.testing.assert_array_equal(o, g["viareset_obs"][s])
        for r in range(3):
            o = env.reset()
            np.testing.assert_array_equal(env.via, g["viareset_cont_via"][s, r])
            np.testing.assert_array_equal(env.goal, g["viareset_cont_goal"][s, r])
            np.testing.assert_array_equal(o, g["viareset_cont_obs"][s, r])


@pytest.mark.parametrize("kind", list(KINDS))
def test_step_based(g, kind):
    name, kw = KINDS[kind]
    acts = g[f"{kind}_actions"]
    E = acts.shape[1]
    envs = [port.Reacher(name, **kw) for _ in range(E)]
    np.testing.assert_array_equal(np.array([e.reset(seed=i) for i, e in enumerate(envs)]), g[f"{kind}_obs0"])
    for t in range(acts.shape[0]):
        for i, e in enumerate(envs):
            o, r, te, tr, _ = e.step(acts[t, i])
            np.testing.assert_array_equal(o, g[f"{kind}_obs"][t, i])
            assert float(r) == g[f"{kind}_rew"][t, i], (t, i)
            assert bool(te) == g[f"{kind}_term"][t, i]
            assert bool(tr) == g[f"{kind}_trunc"][t, i]
            if te or tr:
                np.testing.assert_array_equal(e.reset(), g[f"{kind}_reset_obs"][t, i])


BB = {"bbvia": ("via", port.Vel), "bbvelacc": ("hole_velacc", lambda: port.PD(1.0, 0.1)),
      "bbunb": ("hole_unbounded", port.Vel)}


@pytest.mark.parametrize("case", list(BB))
def test_black_box(g, case):
    kind, ctrl = BB[case]
    name, kw = KINDS[kind]
    G = {k[len(case) + 1:]: g[k] for k in g.files if k.startswith(case + "_")}
    E, n_bb = G["ret"].shape
    for i in range(E):
        env = port.Reacher(name, **kw)
        bb = port.BlackBoxPort(env, table_traj(G["pos"][i], G["vel"][i]), ctrl())
        np.testing.assert_array_equal(bb.reset(seed=100 + i), G["obs0"][i])
        for b in range(n_bb):
            obs, ret, te, tr, info = bb.step()
            L = info["trajectory_length"]
            assert L == G["tlen"][i, b]
            assert bool(te) == G["term"][i, b] and bool(tr) == G["trunc"][i, b]
            assert ret == G["ret"][i, b], (i, b, ret, G["ret"][i, b])
            np.testing.assert_array_equal(obs, G["obs"][i, b])
            np.testing.assert_array_equal(info["step_actions"], G["actions"][i, b, :L])
            np.testing.assert_array_equal(info["step_observations"], G["step_obs"][i, b, :L])
            np.testing.assert_array_equal(info["step_rewards"], G["step_rew"][i, b, :L])
            np.testing.assert_array_equal(np.array(info["is_collided"], float), G["info_a"][i, b, :L])
            np.testing.assert_array_equal(np.array(info["is_success"], float), G["info_b"][i, b, :L])
            np.testing.assert_array_equal(np.array(info["end_effector"]), G["info_ee"][i, b, :L])
            if te or tr:
                np.testing.assert_array_equal(bb.reset(), G["reset_obs"][i, b])


@pytest.mark.parametrize("case", list(BB))
def test_batched_black_box(g, case):
    """The vectorised oracle (used by the GPU parity tests) on the same fixtures."""
    kind, ctrl = BB[case]
    name, kw = KINDS[kind]
    G = {k[len(case) + 1:]: g[k] for k in g.files if k.startswith(case + "_")}
    E, n_bb = G["ret"].shape
    P, V = G["pos"], G["vel"]

    def traj(params, s0, q, qd):
        rows = s0[:, None] + np.arange(200)[None, :]
        return P[np.arange(E)[:, None], rows], V[np.arange(E)[:, None], rows]

    c = ctrl()
    spec = ("pd", c.p, c.d) if isinstance(c, port.PD) else ("vel",)
    bb = batched.BatchedBB(name, E, spec, traj_fn=traj, info_level=2, env_kwargs=kw)
    np.testing.assert_array_equal(bb._reset_idx(list(range(E)), [100 + i for i in range(E)]), G["obs0"])
    for b in range(n_bb):
        obs, ret, te, tr, info = bb.step(None)
        np.testing.assert_array_equal(info["trajectory_length"], G["tlen"][:, b])
        np.testing.assert_array_equal(te, G["term"][:, b])
        np.testing.assert_array_equal(tr, G["trunc"][:, b])
        np.testing.assert_array_equal(ret, G["ret"][:, b])
        np.testing.assert_array_equal(info["final_obs"], G["obs"][:, b])
        done = te | tr
        np.testing.assert_array_equal(obs[done], G["reset_obs"][:, b][done])
        for i in range(E):
            L = G["tlen"][i, b]
            np.testing.assert_array_equal(info["step_actions"][i, :L], G["actions"][i, b, :L])
            np.testing.assert_array_equal(info["step_observations"][i, :L], G["step_obs"][i, b, :L])
            np.testing.assert_array_equal(info["step_rewards"][i, :L], G["step_rew"][i, b, :L])
            np.testing.assert_array_equal(info["is_collided"][i, :L].astype(float), G["info_a"][i, b, :L])
            np.testing.assert_array_equal(info["is_success"][i, :L].astype(float), G["info_b"][i, b, :L])
            np.testing.assert_array_equal(info["end_effector"][i, :L], G["info_ee"][i, b, :L])
