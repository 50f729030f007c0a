"""Pin the CPU oracle's reset options, fixed SimpleReacher target and reward-aggregation callables
against reference-generated fixtures (tests/golden/options.npz, tests/golden/make_golden.py
"options"):

* reset(options={'random_start': ...}) sequences (base_reacher.py:77-86: a non-random reset
  restores _start_pos, a random one draws and replaces it), SimpleReacher / LongSimpleReacher /
  HoleReacher / ViaPointReacher;
* SimpleReacherEnv(target=...) resets and step-based rollouts (simple_reacher.py:19,93-94);
* BB steps with reward_aggregation np.median and ``lambda x: np.mean(x[::2])``
  (black_box_wrapper.py:252; the reference's own test/test_black_box.py:139-150 uses both).

Everything bit-exact.
"""
import os

import numpy as np
import pytest

from oracle import port
from tests.test_oracle_golden import table_traj

TARGET = (1.25, -0.5)
KINDS = {"simple": ("SimpleReacher", {}), "long": ("LongSimpleReacher", {}), "hole": ("HoleReacher", {}),
         "via": ("ViaPointReacher", {}), "target": ("SimpleReacher", {"target": TARGET}),
         "target_long": ("LongSimpleReacher", {"target": TARGET})}
# (seeded?, options) — the sequence make_golden.py ran; "flip" = the opposite of the env default
RESET_SEQ = [("seed", None), (None, {"random_start": False}), (None, None), (None, {"random_start": "flip"}),
             (None, {"random_start": False}), (None, None), ("seed", {"random_start": False})]


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "options.npz"))


def run_reset_seq(env, s):
    q0, goal, obs = [], [], []
    for sd, opt in RESET_SEQ:
        if opt is not None and opt.get("random_start") == "flip":
            opt = {"random_start": not env.random_start}
        o = env.reset(seed=s if sd else None, options=opt)
        q0.append(env.q.copy()); goal.append(np.array(env.goal, np.float64)); obs.append(o)
    return np.array(q0), np.array(goal), np.array(obs)


@pytest.mark.parametrize("kind", list(KINDS))
def test_reset_option_sequences(g, kind):
    name, kw = KINDS[kind]
    for s in range(16):
        q0, goal, obs = run_reset_seq(port.Reacher(name, **kw), s)
        np.testing.assert_array_equal(q0, g[f"{kind}_reset_q0"][s])
        np.testing.assert_array_equal(goal, g[f"{kind}_reset_goal"][s])
        np.testing.assert_array_equal(obs, g[f"{kind}_reset_obs"][s])


@pytest.mark.parametrize("kind", ["target", "target_long"])
def test_fixed_target_step_based(g, kind):
    name, kw = KINDS[kind]
    acts = g[f"{kind}_actions"]
    envs = [port.Reacher(name, **kw) for _ in range(acts.shape[1])]
    np.testing.assert_array_equal(np.array([e.reset(seed=i) for i, e in enumerate(envs)]), g[f"{kind}_obs0"])
    for t in range(acts.shape[0]):
        for i, e in enumerate(envs):
            o, r, te, tr, _ = e.step(acts[t, i])
            np.testing.assert_array_equal(o, g[f"{kind}_obs"][t, i])
            assert float(r) == g[f"{kind}_rew"][t, i]


AGG = {"aggmedian": ("LongSimpleReacher", lambda: port.PD(0.6, 0.075), np.median),
       "aggeven": ("HoleReacher", lambda: port.PD(1.0, 0.1), lambda x: np.mean(x[::2]))}


@pytest.mark.parametrize("case", list(AGG))
def test_reward_aggregation_callables(g, case):
    name, ctrl, agg = AGG[case]
    E, n_bb = g[f"{case}_ret"].shape
    for i in range(E):
        env = port.Reacher(name)
        bb = port.BlackBoxPort(env, table_traj(g[f"{case}_pos"][i], g[f"{case}_vel"][i]), ctrl(),
                               reward_aggregation=agg)
        np.testing.assert_array_equal(bb.reset(seed=100 + i), g[f"{case}_obs0"][i])
        for b in range(n_bb):
            obs, ret, te, tr, info = bb.step()
            assert info["trajectory_length"] == g[f"{case}_tlen"][i, b]
            assert ret == g[f"{case}_ret"][i, b], (i, b)
            np.testing.assert_array_equal(obs, g[f"{case}_obs"][i, b])
            if te or tr:
                np.testing.assert_array_equal(bb.reset(), g[f"{case}_reset_obs"][i, b])
