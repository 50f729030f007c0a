"""Generate the golden fixtures under tests/golden/ from the REFERENCE source.

Test infrastructure only (never imported by the product path).

What this does
--------------
* Imports the reference's own env / controller / black-box modules straight from
  ``/root/reference/fancy_gym`` (read-only, nothing is copied):
    - ``envs/classic_control/simple_reacher/simple_reacher.py`` (SimpleReacherEnv, MPWrapper)
    - ``envs/classic_control/hole_reacher/hole_reacher.py``   (HoleReacherEnv, MPWrapper)
    - ``black_box/black_box_wrapper.py``                       (BlackBoxWrapper.step/reset)
    - ``black_box/controller/{pd,vel}_controller.py``
    - ``utils/wrappers.py``                                    (TimeAwareObservation)
* ``gymnasium`` and ``mp_pytorch`` are not installed in this image.  A minimal
  stand-in for the gymnasium *API surface those modules touch* is written to a
  temp dir at run time (Env/Wrapper/ObservationWrapper, spaces.Box with
  gymnasium's dtype casting, seeding.np_random = Generator(PCG64(SeedSequence(s))),
  TimeLimit).  It restates gymnasium 0.29 semantics [EXT-H]; it contains no
  reference code.  ``mp_pytorch`` is replaced by a *stub trajectory generator*
  that returns caller-given desired trajectories: the MP math itself is not
  in the container, so these goldens pin everything *given a
  desired trajectory* (env, controller, clip, BB loop, replanning bookkeeping,
  TimeAwareObservation, reset RNG streams).

Outputs (small .npz files):
    resets.npz, step_based.npz, bb_simple.npz, bb_long.npz, bb_hole_vel.npz,
    bb_hole_pd.npz, bb_replan.npz                     ("base")
    variants.npz  ViaPointReacher + HoleReacher rew_fct vel_acc / unbounded ("variants")
    options.npz   reset(options={'random_start'}), SimpleReacher(target=...), reward_aggregation
                  callables ("options")

Run:  python tests/golden/make_golden.py [base] [variants]   (needs /root/reference; not on the GPU box)
"""
import os
import sys
import tempfile
import textwrap
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

# ----------------------------------------------------------------------------- shim
_SHIM = {
    "gymnasium/__init__.py": """
        from . import spaces, utils, core, wrappers
        from .core import Env, Wrapper, ObservationWrapper
    """,
    "gymnasium/core.py": """
        import numpy as np
        from typing import Any
        ObsType = Any
        ActType = Any
        from .utils import seeding

        class Env:
            _np_random = None
            spec = None
            def reset(self, *, seed=None, options=None):
                if seed is not None:
                    self._np_random, _ = seeding.np_random(seed)
            @property
            def np_random(self):
                if self._np_random is None:
                    self._np_random, _ = seeding.np_random()
                return self._np_random
            @property
            def unwrapped(self):
                return self
            def close(self):
                pass

        class Wrapper(Env):
            def __init__(self, env):
                self.env = env
                self._action_space = None
                self._observation_space = None
            def __getattr__(self, name):
                if name.startswith('_'):
                    raise AttributeError(name)
                return getattr(self.env, name)
            @property
            def action_space(self):
                return self.env.action_space if self._action_space is None else self._action_space
            @action_space.setter
            def action_space(self, s):
                self._action_space = s
            @property
            def observation_space(self):
                return self.env.observation_space if self._observation_space is None else self._observation_space
            @observation_space.setter
            def observation_space(self, s):
                self._observation_space = s
            @property
            def spec(self):
                return self.env.spec
            @property
            def unwrapped(self):
                return self.env.unwrapped
            @property
            def np_random(self):
                return self.env.np_random
            def step(self, action):
                return self.env.step(action)
            def reset(self, *, seed=None, options=None):
                return self.env.reset(seed=seed, options=options)

        class ObservationWrapper(Wrapper):
            def reset(self, *, seed=None, options=None):
                obs, info = self.env.reset(seed=seed, options=options)
                return self.observation(obs), info
            def step(self, action):
                obs, r, te, tr, info = self.env.step(action)
                return self.observation(obs), r, te, tr, info
    """,
    "gymnasium/spaces/__init__.py": """
        import numpy as np
        class Box:
            # gymnasium 0.29: bounds are stored in the space dtype (default float32)
            def __init__(self, low, high, shape=None, dtype=np.float32):
                self.dtype = np.dtype(dtype)
                if shape is None:
                    shape = np.shape(low) if np.ndim(low) else np.shape(high)
                self.shape = tuple(shape)
                self.low = np.broadcast_to(np.asarray(low, dtype=float), self.shape).astype(self.dtype)
                self.high = np.broadcast_to(np.asarray(high, dtype=float), self.shape).astype(self.dtype)
        class Dict(dict):
            pass
        def flatten(space, x):
            raise NotImplementedError
        def flatten_space(space):
            raise NotImplementedError
    """,
    "gymnasium/utils/__init__.py": """
        from . import seeding
        class RecordConstructorArgs:
            def __init__(self, **kwargs):
                pass
    """,
    "gymnasium/utils/seeding.py": """
        import numpy as np
        def np_random(seed=None):
            seed_seq = np.random.SeedSequence(seed)
            return np.random.Generator(np.random.PCG64(seed_seq)), seed_seq.entropy
    """,
    "gymnasium/wrappers/__init__.py": """
        from ..core import Wrapper
        class TimeLimit(Wrapper):
            def __init__(self, env, max_episode_steps):
                super().__init__(env)
                self._max_episode_steps = max_episode_steps
                self._elapsed_steps = None
            def step(self, action):
                obs, r, te, tr, info = self.env.step(action)
                self._elapsed_steps += 1
                if self._elapsed_steps >= self._max_episode_steps:
                    tr = True
                return obs, r, te, tr, info
            def reset(self, *, seed=None, options=None):
                self._elapsed_steps = 0
                return self.env.reset(seed=seed, options=options)
    """,
    "mp_pytorch/__init__.py": "",
    "mp_pytorch/mp/__init__.py": "",
    "mp_pytorch/mp/mp_interfaces.py": "class MPInterface:\n    pass\n",
    "qpsolvers/__init__.py": "def solve_qp(*a, **k):\n    raise NotImplementedError\n",
}


def _install_shim():
    d = tempfile.mkdtemp(prefix="fgx_golden_shim_")
    for rel, src in _SHIM.items():
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(textwrap.dedent(src))
    sys.path.insert(0, d)
    sys.path.insert(0, REF)
    # skip the heavy package __init__s (they import mujoco/metaworld/...)
    for name, sub in [("fancy_gym", "fancy_gym"), ("fancy_gym.envs", "fancy_gym/envs"),
                      ("fancy_gym.envs.classic_control", "fancy_gym/envs/classic_control")]:
        m = types.ModuleType(name)
        m.__path__ = [os.path.join(REF, sub)]
        sys.modules[name] = m


_install_shim()
import torch  # noqa: E402
from gymnasium.wrappers import TimeLimit  # noqa: E402
from fancy_gym.envs.classic_control.simple_reacher.simple_reacher import SimpleReacherEnv  # noqa: E402
from fancy_gym.envs.classic_control.simple_reacher.mp_wrapper import MPWrapper as SRMPWrapper  # noqa: E402
from fancy_gym.envs.classic_control.hole_reacher.hole_reacher import HoleReacherEnv  # noqa: E402
from fancy_gym.envs.classic_control.hole_reacher.mp_wrapper import MPWrapper as HRMPWrapper  # noqa: E402
from fancy_gym.envs.classic_control.viapoint_reacher.viapoint_reacher import ViaPointReacherEnv  # noqa: E402
from fancy_gym.envs.classic_control.viapoint_reacher.mp_wrapper import MPWrapper as VPMPWrapper  # noqa: E402
from fancy_gym.black_box.black_box_wrapper import BlackBoxWrapper  # noqa: E402
from fancy_gym.black_box.controller.pd_controller import PDController  # noqa: E402
from fancy_gym.black_box.controller.vel_controller import VelController  # noqa: E402
from fancy_gym.utils.wrappers import TimeAwareObservation  # noqa: E402


class _Spec:
    max_episode_steps = 200


TARGET = (1.25, -0.5)   # fixed SimpleReacher target of the "options" fixtures


# registered kwargs: envs/__init__.py:57-65 (SimpleReacher), :658-666 (Long), :682-698 (Hole)
def make_raw(kind):
    if kind == "simple":
        env = SimpleReacherEnv(n_links=2)
    elif kind == "long":
        env = SimpleReacherEnv(n_links=5)
    elif kind.startswith("hole"):
        rew = {"hole": "simple", "hole_velacc": "vel_acc", "hole_unbounded": "unbounded"}[kind]
        env = HoleReacherEnv(n_links=5, random_start=True, allow_self_collision=False,
                             allow_wall_collision=False, hole_width=None, hole_depth=1,
                             hole_x=None, collision_penalty=100, rew_fct=rew)
    elif kind == "via":   # envs/__init__.py:669-679
        env = ViaPointReacherEnv(n_links=5, allow_self_collision=False, collision_penalty=1000)
    elif kind.startswith("target"):   # SimpleReacherEnv(target=...) (simple_reacher.py:19,93-94)
        env = SimpleReacherEnv(n_links=2 if kind == "target" else 5, target=TARGET)
    else:
        raise ValueError(kind)
    env.spec = _Spec()
    return TimeLimit(env, 200)


class StubTrajGen:
    """Stand-in for mp_pytorch: returns rows [t0, t0+T) of caller tables (absolute step index)."""

    class _Phase:
        pass

    def __init__(self, P, pos_table, vel_table, T=200):
        self.P, self.T = P, T
        self.phase_gn = self._Phase()
        self.pos_table, self.vel_table = pos_table, vel_table
        self.calls = []

    def set_duration(self, duration, dt):
        self.duration, self.dt = duration, dt

    def get_params_bounds(self):
        return torch.full((self.P,), -np.inf), torch.full((self.P,), np.inf)

    def set_params(self, p):
        self.params = np.array(p)

    def set_initial_conditions(self, init_time, pos, vel):
        self.init_time = float(init_time)
        self.calls.append((self.init_time, np.array(pos, dtype=np.float64), np.array(vel, dtype=np.float64)))

    def _t0(self):
        return int(round(self.init_time / 0.01))

    def get_traj_pos(self):
        t0 = self._t0()
        return torch.from_numpy(self.pos_table[t0:t0 + self.T].copy())

    def get_traj_vel(self):
        t0 = self._t0()
        return torch.from_numpy(self.vel_table[t0:t0 + self.T].copy())

    def reset(self):
        pass


def smooth_tables(rng, n_rows, dof, amp_pos, amp_vel, offset=None):
    """Random smooth f32 desired pos/vel tables [n_rows, dof] (sums of sinusoids)."""
    t = np.arange(n_rows)[:, None] * 0.01
    pos = np.zeros((n_rows, dof))
    vel = np.zeros((n_rows, dof))
    for _ in range(3):
        w = rng.uniform(0.5, 4.0, dof)
        ph = rng.uniform(0, 2 * np.pi, dof)
        pos += rng.uniform(-amp_pos, amp_pos, dof) * np.sin(w * t + ph)
        vel += rng.uniform(-amp_vel, amp_vel, dof) * np.cos(w * t + ph)
    if offset is not None:
        pos += offset
    return pos.astype(np.float32), vel.astype(np.float32)


# ----------------------------------------------------------------------------- (i) resets
def gen_resets():
    out = {}
    for kind in ("simple", "long", "hole"):
        env = make_raw(kind)
        q0, goal, obs, hole = [], [], [], []
        cq0, cgoal, cobs, chole = [], [], [], []
        for s in range(64):
            o, _ = env.reset(seed=s)
            u = env.unwrapped
            q0.append(u._joint_angles.copy()); goal.append(np.array(u._goal, dtype=np.float64)); obs.append(o)
            if kind == "hole":
                hole.append([u._tmp_x, u._tmp_width, float(u._tmp_depth)])
            # unseeded continuation (VectorEnv autoreset path): 3 more resets
            rq, rg, ro, rh = [], [], [], []
            for _ in range(3):
                o2, _ = env.reset()
                rq.append(u._joint_angles.copy()); rg.append(np.array(u._goal, dtype=np.float64)); ro.append(o2)
                if kind == "hole":
                    rh.append([u._tmp_x, u._tmp_width, float(u._tmp_depth)])
            cq0.append(rq); cgoal.append(rg); cobs.append(ro); chole.append(rh)
        out[f"{kind}_q0"] = np.array(q0)
        out[f"{kind}_goal"] = np.array(goal)
        out[f"{kind}_obs"] = np.array(obs)
        out[f"{kind}_cont_q0"] = np.array(cq0)
        out[f"{kind}_cont_goal"] = np.array(cgoal)
        out[f"{kind}_cont_obs"] = np.array(cobs)
        if kind == "hole":
            out["hole_hole"] = np.array(hole)
            out["hole_cont_hole"] = np.array(chole)
    np.savez_compressed(os.path.join(OUT, "resets.npz"), **out)


# ----------------------------------------------------------------------------- (ii) step-based
def gen_step_based():
    out = {}
    # config 1: fancy/SimpleReacher-v0 step-based; actions uniform(-1000,1000) f32
    specs = [("simple", 8, 2, 1000.0), ("long", 4, 5, 1000.0), ("hole", 6, 5, 0.35 * 2 * np.pi)]
    for kind, E, dof, amp in specs:
        rng = np.random.default_rng(1234)
        acts = rng.uniform(-amp, amp, (200, E, dof))
        if kind == "hole":   # per-env drift so that some arms reach the wall / fold
            acts += rng.uniform(-2.0, 2.0, (1, E, dof))
        acts = acts.astype(np.float32)
        envs = [make_raw(kind) for _ in range(E)]
        obs0 = np.array([e.reset(seed=i)[0] for i, e in enumerate(envs)])
        O, R, TE, TR, RESET = [], [], [], [], []
        for t in range(200):
            o_t, r_t, te_t, tr_t, rs_t = [], [], [], [], []
            for i, e in enumerate(envs):
                o, r, te, tr, _ = e.step(acts[t, i])
                o_t.append(o); r_t.append(float(r)); te_t.append(bool(te)); tr_t.append(bool(tr))
                if te or tr:   # autoreset (unseeded), the reset obs is what a VectorEnv returns
                    o2, _ = e.reset()
                    rs_t.append(o2)
                else:
                    rs_t.append(np.full_like(o, np.nan))
            O.append(o_t); R.append(r_t); TE.append(te_t); TR.append(tr_t); RESET.append(rs_t)
        out[f"{kind}_actions"] = acts
        out[f"{kind}_obs0"] = obs0
        out[f"{kind}_obs"] = np.array(O, dtype=np.float32)
        out[f"{kind}_rew"] = np.array(R)
        out[f"{kind}_term"] = np.array(TE)
        out[f"{kind}_trunc"] = np.array(TR)
        out[f"{kind}_reset_obs"] = np.array(RESET, dtype=np.float32)
    np.savez_compressed(os.path.join(OUT, "step_based.npz"), **out)


# ----------------------------------------------------------------------------- (iii)/(iv) BB
def run_bb(name, kind, controller, E, n_bb, table_fn, replan=None, ctx=True, out_dict=None, bb_kw=None):
    """E envs, reset(seed=100+i), n_bb BB steps each with autoreset; stub MP tables per (env, bb)."""
    rng = np.random.default_rng(4321)
    wrap = {"via": VPMPWrapper}.get(kind, HRMPWrapper if kind.startswith("hole") else SRMPWrapper)
    dof = 2 if kind == "simple" else 5
    recs = {k: [] for k in ("pos", "vel", "obs", "ret", "term", "trunc", "tlen", "actions",
                            "step_obs", "step_rew", "reset_obs", "obs0", "init_time", "init_pos",
                            "init_vel", "info_a", "info_b", "info_ee")}
    for i in range(E):
        raw = make_raw(kind)
        env = wrap(raw)
        if replan is not None:
            env = TimeAwareObservation(env)
        n_rows = 400 if replan is not None else 200
        pos_t, vel_t = table_fn(rng, n_rows, dof)
        tg = StubTrajGen(dof * 5, pos_t, vel_t)
        kw = dict(bb_kw or {})
        if replan is not None:
            kw["replanning_schedule"] = replan
        bb = BlackBoxWrapper(env, trajectory_generator=tg, tracking_controller=controller,
                             duration=2.0, **kw)
        o0, _ = bb.reset(seed=100 + i)
        recs["obs0"].append(o0)
        recs["pos"].append(pos_t); recs["vel"].append(vel_t)
        per = {k: [] for k in recs if k not in ("pos", "vel", "obs0")}
        for b in range(n_bb):
            obs, ret, te, tr, info = bb.step(np.zeros(dof * 5, dtype=np.float32))
            L = info["trajectory_length"]
            per["obs"].append(obs); per["ret"].append(float(ret)); per["term"].append(bool(te))
            per["trunc"].append(bool(tr)); per["tlen"].append(int(L))
            def pad(a, w, dt=np.float64):
                return np.concatenate([np.asarray(a, dtype=dt).reshape(L, -1), np.full((200 - L, w), np.nan, dt)])
            per["actions"].append(pad(info["step_actions"], dof))
            per["step_obs"].append(pad(info["step_observations"], info["step_observations"].shape[-1], np.float32))
            per["step_rew"].append(pad(info["step_rewards"], 1)[:, 0])
            if kind != "simple" and kind != "long":
                per["info_a"].append(pad(np.array(info["is_collided"], dtype=float), 1)[:, 0])
                per["info_b"].append(pad(np.array(info["is_success"], dtype=float), 1)[:, 0])
                per["info_ee"].append(pad(np.array(info["end_effector"]), 2))
            else:
                per["info_a"].append(pad(np.array(info["reward_dist"], dtype=float), 1)[:, 0])
                per["info_b"].append(pad(np.array(info["reward_ctrl"], dtype=float), 1)[:, 0])
                per["info_ee"].append(np.full((200, 2), np.nan))
            c = tg.calls[-1]
            per["init_time"].append(c[0]); per["init_pos"].append(c[1]); per["init_vel"].append(c[2])
            if te or tr:
                o2, _ = bb.reset()
                per["reset_obs"].append(o2)
            else:
                per["reset_obs"].append(np.full_like(obs, np.nan))
        for k, v in per.items():
            recs[k].append(v)
    out = {k: np.array(v) for k, v in recs.items()}
    if out_dict is not None:
        out_dict.update({f"{name}_{k}": v for k, v in out.items()})
        return
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)


def gen_bb():
    def simple_tab(rng, n, dof):
        return smooth_tables(rng, n, dof, 1.0, 3.0)

    def hole_vel_tab(rng, n, dof):
        return smooth_tables(rng, n, dof, 0.5, 1.2)

    def hole_pd_tab(rng, n, dof):
        # random folded targets: drives a mix of wall hits, self-collisions and joint-limit hits
        off = rng.uniform(-3.5, 3.5, dof)
        off[0] = rng.uniform(0.0, np.pi)
        return smooth_tables(rng, n, dof, 0.6, 1.0, offset=off)

    # ProMP/DMP SimpleReacher: PD p=.6 d=.075 (simple_reacher/mp_wrapper.py:11-17)
    run_bb("bb_simple", "simple", PDController(0.6, 0.075), 8, 2, simple_tab)
    run_bb("bb_long", "long", PDController(0.6, 0.075), 4, 2, simple_tab)
    # HoleReacher ProMP/DMP: velocity controller (hole_reacher/mp_wrapper.py:11-23)
    run_bb("bb_hole_vel", "hole", VelController(), 6, 2, hole_vel_tab)
    # HoleReacher ProDMP: motor PD 1.0/0.1 from _BB_DEFAULTS (registry.py:116-120), clipped to +-2pi
    run_bb("bb_hole_pd", "hole", PDController(1.0, 0.1), 8, 2, hole_pd_tab)
    # config 5: SimpleReacher + replanning every 25 steps (TimeAwareObservation inserted)
    run_bb("bb_replan", "simple", PDController(1.0, 0.1), 3, 10, simple_tab,
           replan=lambda pos, vel, obs, action, t: t % 25 == 0)


# ----------------------------------------------------------------------------- (vi) widening
def gen_variants():
    """ViaPointReacher (envs/__init__.py:669-679) and the HoleReacher reward variants
    (hole_reacher.py:48-58: rew_fct "vel_acc" / "unbounded"): resets, step-based rollouts and
    BB steps given a desired trajectory, in one file."""
    out = {}
    env = make_raw("via")
    u = env.unwrapped
    rec = {k: [] for k in ("q0", "via", "goal", "obs", "cont_via", "cont_goal", "cont_obs")}
    for s in range(64):
        o, _ = env.reset(seed=s)
        rec["q0"].append(u._joint_angles.copy()); rec["via"].append(np.array(u._via_point, np.float64))
        rec["goal"].append(np.array(u._goal, np.float64)); rec["obs"].append(o)
        cv, cg, co = [], [], []
        for _ in range(3):
            o2, _ = env.reset()
            cv.append(np.array(u._via_point, np.float64)); cg.append(np.array(u._goal, np.float64)); co.append(o2)
        rec["cont_via"].append(cv); rec["cont_goal"].append(cg); rec["cont_obs"].append(co)
    out.update({f"viareset_{k}": np.array(v) for k, v in rec.items()})
    for kind, E in (("via", 4), ("hole_velacc", 4), ("hole_unbounded", 4)):
        rng = np.random.default_rng(99)
        acts = rng.uniform(-0.35 * 2 * np.pi, 0.35 * 2 * np.pi, (200, E, 5)) + rng.uniform(-2.0, 2.0, (1, E, 5))
        acts = acts.astype(np.float32)
        envs = [make_raw(kind) for _ in range(E)]
        obs0 = np.array([e.reset(seed=i)[0] for i, e in enumerate(envs)])
        O, R, TE, TR, RESET = [], [], [], [], []
        for t in range(200):
            o_t, r_t, te_t, tr_t, rs_t = [], [], [], [], []
            for i, e in enumerate(envs):
                o, r, te, tr, _ = e.step(acts[t, i])
                o_t.append(o); r_t.append(float(r)); te_t.append(bool(te)); tr_t.append(bool(tr))
                rs_t.append(e.reset()[0] if (te or tr) else np.full_like(o, np.nan))
            O.append(o_t); R.append(r_t); TE.append(te_t); TR.append(tr_t); RESET.append(rs_t)
        out[f"{kind}_actions"] = acts
        out[f"{kind}_obs0"] = obs0
        out[f"{kind}_obs"] = np.array(O, dtype=np.float32)
        out[f"{kind}_rew"] = np.array(R)
        out[f"{kind}_term"] = np.array(TE)
        out[f"{kind}_trunc"] = np.array(TR)
        out[f"{kind}_reset_obs"] = np.array(RESET, dtype=np.float32)

    def vel_tab(rng, n, dof):
        return smooth_tables(rng, n, dof, 0.5, 1.2)

    def fold_tab(rng, n, dof):
        off = rng.uniform(-3.5, 3.5, dof)
        off[0] = rng.uniform(0.0, np.pi)
        return smooth_tables(rng, n, dof, 0.6, 1.0, offset=off)

    # ViaPointReacher ProMP/DMP: velocity controller (viapoint_reacher/mp_wrapper.py:11-23)
    run_bb("bbvia", "via", VelController(), 4, 2, vel_tab, out_dict=out)
    run_bb("bbvelacc", "hole_velacc", PDController(1.0, 0.1), 4, 2, fold_tab, out_dict=out)
    run_bb("bbunb", "hole_unbounded", VelController(), 4, 2, vel_tab, out_dict=out)
    np.savez_compressed(os.path.join(OUT, "variants.npz"), **out)


# ----------------------------------------------------------------------------- (vii) options
RESET_SEQ = [("seed", None), (None, {"random_start": False}), (None, None), (None, {"random_start": "flip"}),
             (None, {"random_start": False}), (None, None), ("seed", {"random_start": False})]


def gen_options():
    """reset(options={'random_start': ...}) sequences (base_reacher.py:77-86: a non-random reset
    restores _start_pos, which a random one replaces), SimpleReacher(target=...) resets and
    step-based rollouts, and BB steps with reward_aggregation callables other than np.sum
    (black_box_wrapper.py:252; test/test_black_box.py:139-150 uses np.median and a lambda)."""
    out = {}
    for kind in ("simple", "long", "hole", "via", "target", "target_long"):
        rec = {k: [] for k in ("q0", "goal", "obs")}
        for s in range(16):
            env = make_raw(kind)
            u = env.unwrapped
            q0, goal, obs = [], [], []
            for sd, opt in RESET_SEQ:
                if opt is not None and opt.get("random_start") == "flip":
                    opt = {"random_start": not u.random_start}
                o, _ = env.reset(seed=s if sd else None, options=opt)
                q0.append(u._joint_angles.copy()); goal.append(np.array(u._goal, np.float64)); obs.append(o)
            rec["q0"].append(q0); rec["goal"].append(goal); rec["obs"].append(obs)
        out.update({f"{kind}_reset_{k}": np.array(v) for k, v in rec.items()})
    for kind, E, dof in (("target", 4, 2), ("target_long", 3, 5)):
        rng = np.random.default_rng(5)
        acts = rng.uniform(-100, 100, (60, E, dof)).astype(np.float32)
        envs = [make_raw(kind) for _ in range(E)]
        out[f"{kind}_obs0"] = np.array([e.reset(seed=i)[0] for i, e in enumerate(envs)])
        O, R = [], []
        for t in range(60):
            o_t, r_t = [], []
            for i, e in enumerate(envs):
                o, r, te, tr, _ = e.step(acts[t, i])
                o_t.append(o); r_t.append(float(r))
            O.append(o_t); R.append(r_t)
        out[f"{kind}_actions"] = acts
        out[f"{kind}_obs"] = np.array(O, dtype=np.float32)
        out[f"{kind}_rew"] = np.array(R)

    def simple_tab(rng, n, dof):
        return smooth_tables(rng, n, dof, 1.0, 3.0)

    def hole_pd_tab(rng, n, dof):
        off = rng.uniform(-3.5, 3.5, dof)
        off[0] = rng.uniform(0.0, np.pi)
        return smooth_tables(rng, n, dof, 0.6, 1.0, offset=off)

    run_bb("aggmedian", "long", PDController(0.6, 0.075), 4, 2, simple_tab, out_dict=out,
           bb_kw={"reward_aggregation": np.median})
    run_bb("aggeven", "hole", PDController(1.0, 0.1), 6, 2, hole_pd_tab, out_dict=out,
           bb_kw={"reward_aggregation": lambda x: np.mean(x[::2])})
    np.savez_compressed(os.path.join(OUT, "options.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["base", "variants", "options"]
    if "base" in which:
        gen_resets()
        gen_step_based()
        gen_bb()
    if "variants" in which:
        gen_variants()
    if "options" in which:
        gen_options()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
