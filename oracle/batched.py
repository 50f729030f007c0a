"""Vectorised (over envs) restatement of oracle/port.py + oracle/mp.py — TEST INFRASTRUCTURE ONLY.

Same per-element numpy operations and dtypes as the per-env port (so it is bit-exact with it,
checked by tests/test_oracle_batched.py), but with [N, ...] arrays so that the GPU parity
tests can use thousands of envs.  Resets use one numpy Generator per env (the reference's
RNG, unchanged).  The VectorEnv wrapper semantics are gymnasium 0.29's SyncVectorEnv
[EXT-M]: reset(seed=s) seeds env i with s+i; step() auto-resets finished envs in the same call
and returns the reset observation, the finished one going to ``final_obs``.
"""
import numpy as np

from . import mp as mpm
from .port import MAX_EPISODE_STEPS, Reacher

f32 = np.float32
DT32 = f32(0.01)


def _seqsum(sq, as32):
    """np.sum over the last axis of a [N, n <= 8] array in numpy's pairwise_sum order (umath
    loops_utils.h): left to right for n < 8, at n = 8 the eight accumulators combined as
    ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) (f32 when as32)."""
    n = sq.shape[1]
    dt = f32 if as32 else np.float64
    if n == 8:
        r = [sq[:, j].astype(dt) for j in range(8)]
        return (((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))).astype(dt)
    assert n < 8
    c = sq[:, 0].astype(f32) if as32 else sq[:, 0] + 0.0
    for j in range(1, n):
        c = (c + sq[:, j]).astype(dt)
    return c


def _norm2(v):
    """np.linalg.norm of each row of a [M, 2] array (per-row call: BLAS ordering kept)."""
    return np.array([np.linalg.norm(r) for r in v], dtype=np.float64)


class BatchedReacher:
    def __init__(self, name, N, random_start=None, **overrides):
        self.N = N
        self.envs = [Reacher(name, random_start, **overrides) for _ in range(N)]   # RNG + reset sampling
        e0 = self.envs[0]
        self.kind, self.n, self.dt = e0.kind, e0.n, e0.dt
        self.obs_dim = e0.obs_dim
        self.act_low, self.act_high = e0.act_low, e0.act_high
        self.mask = e0.context_mask()
        self.q = np.zeros((N, self.n))
        self.qd = np.zeros((N, self.n))
        self.qd_f32 = np.zeros(N, bool)      # qd holds a float32 *array* in the reference
        self.goal = np.zeros((N, 2))
        self.joints = np.zeros((N, self.n + 1, 2))
        self.steps = np.zeros(N, np.int64)
        if self.kind == "hole":
            self.hole_x = np.zeros(N)
            self.hole_w = np.zeros(N)
            self.hole_d = float(e0.init_depth)
            self.rew_factors = e0.rew_factors
            self.rew_fct = e0.rew_fct
            self.allow_self, self.allow_wall = e0.allow_self, e0.allow_wall
            self.rf_collided = np.zeros(N, bool)      # vel_acc reward function state
            self.rf_coll_dist = np.zeros(N)
            self.ee_save = np.zeros((N, 2))           # unbounded reward function state
        if self.kind == "via":
            self.via = np.zeros((N, 2))
            self.allow_self, self.penalty = e0.allow_self, e0.penalty

    def reset(self, idx, seeds=None, options=None):
        """Reset envs idx (list); returns obs [len(idx), obs_dim] f32."""
        out = []
        for j, i in enumerate(idx):
            e = self.envs[i]
            o = e.reset(None if seeds is None else int(seeds[j]), options)
            self.q[i] = e.q
            self.qd[i] = e.qd
            self.qd_f32[i] = False
            self.goal[i] = e.goal
            self.steps[i] = 0
            if self.kind == "hole":
                self.hole_x[i], self.hole_w[i] = e.hole_x, e.hole_w
                self.rf_collided[i] = False
                self.rf_coll_dist[i] = 0.0
            if self.kind == "via":
                self.via[i] = e.via
            out.append(o)
        self._fk()
        return np.array(out, dtype=f32).reshape(len(idx), self.obs_dim)

    def _fk(self):
        ang = np.cumsum(self.q, axis=1)
        xy = np.stack([np.cos(ang), np.sin(ang)], axis=-1)
        self.joints[:, 1:] = 0.0 + np.cumsum(xy, axis=1)

    @property
    def ee(self):
        return self.joints[:, self.n]

    def obs(self):
        cols = [np.cos(self.q), np.sin(self.q), self.qd]
        if self.kind == "hole":
            cols.append(self.hole_w[:, None])
        if self.kind == "via":
            cols.append(self.ee - self.via)
        cols += [self.ee - self.goal, self.steps[:, None].astype(np.float64)]
        return np.concatenate(cols, axis=1).astype(f32)

    def _self_collision(self):
        lim = np.any(self.q > np.pi, axis=1) | np.any(self.q < -np.pi, axis=1)
        J = self.joints

        def ccw(A, B, C):
            return (C[:, 1] - A[:, 1]) * (B[:, 0] - A[:, 0]) - (B[:, 1] - A[:, 1]) * (C[:, 0] - A[:, 0]) > 1e-12
        hit = np.zeros(self.N, bool)
        for i in range(self.n):
            for j in range(i + 2, self.n):
                A, B, C, D = J[:, i], J[:, i + 1], J[:, j], J[:, j + 1]
                hit |= (ccw(A, C, D) != ccw(B, C, D)) & (ccw(A, B, C) != ccw(A, B, D))
        return lim | hit

    def _wall_collision(self):
        s = np.linspace(0, 1, 100)
        acc = np.cumsum(self.q, axis=1)
        x = np.cos(acc)[:, :, None] * s
        y = np.sin(acc)[:, :, None] * s
        px = np.empty_like(x)
        py = np.empty_like(y)
        px[:, 0], py[:, 0] = x[:, 0], y[:, 0]
        for i in range(1, self.n):
            px[:, i] = x[:, i] + px[:, i - 1, -1:]
            py[:, i] = y[:, i] + py[:, i - 1, -1:]
        px = px + 0.0
        py = py + 0.0
        left = (self.hole_x - self.hole_w / 2)[:, None, None]
        right = (self.hole_x + self.hole_w / 2)[:, None, None]
        c1 = np.any((px < left) & (py < 0), axis=(1, 2))
        c2 = np.any((px > right) & (py < 0), axis=(1, 2))
        c3 = np.any((px > left) & (px < right) & (py < -self.hole_d), axis=(1, 2))
        return c1 | c2 | c3

    def step(self, a, act, a_is_f32):
        """One inner step for envs where act[i]; a [N, n] (f64, or f32 values if a_is_f32).

        Returns obs [N, obs_dim] f32, reward [N] f64, terminated [N] bool, truncated [N] bool,
        info dict of [N] arrays (values undefined where ~act).
        """
        N, n = self.N, self.n
        q, qd = self.q.copy(), self.qd.copy()
        info = {}
        if self.kind == "simple":
            if a_is_f32:
                inc = (DT32 * a.astype(f32)).astype(np.float64)
            else:
                inc = self.dt * a
            qd = qd + inc
            q = q + self.dt * qd
        else:
            a32 = a.astype(f32) if a_is_f32 else None
            if a_is_f32:
                acc64 = (a32.astype(np.float64) - qd) / self.dt
                acc32 = ((a32 - qd.astype(f32)) / DT32).astype(f32)
                use32 = self.qd_f32
                qd = a32.astype(np.float64)
                q = q + (DT32 * a32).astype(np.float64)
            else:
                acc64 = (a - qd) / self.dt
                acc32 = None
                use32 = np.zeros(N, bool)
                qd = a.copy()
                q = q + self.dt * qd
        self.q = np.where(act[:, None], q, self.q)
        self.qd = np.where(act[:, None], qd, self.qd)
        self._fk()
        steps = self.steps
        if self.kind == "simple":
            if a_is_f32:
                ctrl = _seqsum(a.astype(f32) ** 2, True).astype(np.float64)
            else:
                ctrl = _seqsum(a ** 2, False)
            dist = np.zeros(N)
            need = act & (steps >= 199)
            if np.any(need):
                dist[need] = -_norm2(self.ee[need] - self.goal[need])
            if a_is_f32:
                # int 0 - float32 -> float32; float64 - float32 -> float64 (NEP 50)
                reward = np.where(need, dist - ctrl, -ctrl)
            else:
                reward = dist - ctrl
            info["reward_dist"] = dist
            info["reward_ctrl"] = ctrl
            term = np.zeros(N, bool)
        elif self.kind == "via":
            coll = np.zeros(N, bool) if self.allow_self else self._self_collision()
            if a_is_f32:   # 5e-8 * float32 scalar stays float32 (NEP 50)
                pen_ctrl = (f32(5e-8) * _seqsum(a.astype(f32) ** 2, True)).astype(f32).astype(np.float64)
            else:
                pen_ctrl = 5e-8 * _seqsum(a ** 2, False)
            reward = np.full(N, -np.inf)
            success = np.zeros(N, bool)
            for i in np.nonzero(act)[0]:
                if coll[i]:
                    d = np.linalg.norm(self.ee[i] - self.goal[i])
                    reward[i] = (-self.penalty - d ** 2) - pen_ctrl[i]
                elif steps[i] == 100:
                    success[i] = np.linalg.norm(self.ee[i] - self.via[i]) < 0.005
                elif steps[i] == 199:
                    success[i] = np.linalg.norm(self.ee[i] - self.goal[i]) < 0.005
            info["is_success"] = success
            info["is_collided"] = coll
            info["end_effector"] = self.ee.copy()
            term = coll
        else:
            if a_is_f32:
                sq64 = acc64 * acc64
                acc_cost = np.where(use32, _seqsum((acc32 * acc32).astype(f32), True).astype(np.float64),
                                    _seqsum(sq64, False))
                self.qd_f32 = np.where(act, True, self.qd_f32)
            else:
                acc_cost = _seqsum(acc64 * acc64, False)
            success = np.zeros(N, bool)
            if self.rew_fct == "simple":
                coll = ((np.zeros(N, bool) if self.allow_self else self._self_collision())
                        | (np.zeros(N, bool) if self.allow_wall else self._wall_collision()))
                special = act & ((steps == 199) | coll)
                reward = acc_cost * self.rew_factors[1]      # fma(0,-100,fma(acc,-5e-8,-0.0))
                if np.any(special):
                    idx = np.nonzero(special)[0]
                    dist = _norm2(self.ee[idx] - self.goal[idx])
                    for j, i in enumerate(idx):
                        feats = np.array((dist[j] ** 2, acc_cost[i], int(coll[i])))
                        reward[i] = np.dot(feats, self.rew_factors)
                        success[i] = dist[j] < 0.005 and not coll[i]
            elif self.rew_fct == "vel_acc":
                # qd after the step is the action (float32 values when a_is_f32)
                vel_cost = (_seqsum(a.astype(f32) ** 2, True).astype(np.float64) if a_is_f32
                            else _seqsum(a ** 2, False))
                fresh = act & ~self.rf_collided
                now = ((np.zeros(N, bool) if self.allow_self else self._self_collision())
                       | (np.zeros(N, bool) if self.allow_wall else self._wall_collision()))
                self.rf_collided = np.where(fresh, now, self.rf_collided)
                for i in np.nonzero(fresh)[0]:
                    self.rf_coll_dist[i] = np.linalg.norm(self.ee[i] - self.goal[i])
                coll = self.rf_collided.copy()
                reward = np.zeros(N)
                for i in np.nonzero(act)[0]:
                    dist_cost, collision_cost, time_cost = 0, 0, 0
                    if steps[i] == 199:
                        dist = np.linalg.norm(self.ee[i] - self.goal[i])
                        success[i] = dist < 0.005 and not coll[i]
                        dist_cost = dist ** 2
                        collision_cost = coll[i] * self.rf_coll_dist[i] ** 2
                        time_cost = 199 - int(steps[i])
                    reward[i] = np.dot(np.array((dist_cost, vel_cost[i], acc_cost[i], collision_cost, time_cost)),
                                       self.rew_factors)
            else:   # unbounded
                coll = ((np.zeros(N, bool) if self.allow_self else self._self_collision())
                        | (np.zeros(N, bool) if self.allow_wall else self._wall_collision()))
                save = act & ((steps == 180) | coll)
                self.ee_save = np.where(save[:, None], self.ee, self.ee_save)
                reward = acc_cost * self.rew_factors[1]      # fma(acc, -5e-6, 0 * 1)
                for i in np.nonzero(act & ((steps == 199) | coll))[0]:
                    dist = np.linalg.norm(self.ee_save[i] - self.goal[i])
                    if coll[i]:
                        dr = 0.25 * np.exp(-dist)
                    elif self.ee[i, 1] > 0:
                        dr = np.exp(-dist)
                    else:
                        dr = 1 - self.ee_save[i, 1]
                    success[i] = not coll[i]
                    reward[i] = np.dot(np.array((dr, acc_cost[i])), self.rew_factors)
            info["is_success"] = success
            info["is_collided"] = coll
            info["end_effector"] = self.ee.copy()
            term = coll
        self.steps = np.where(act, steps + 1, steps)
        trunc = self.steps >= MAX_EPISODE_STEPS
        return self.obs(), reward, term & act, trunc & act, info


class BatchedBB:
    """Vectorised BlackBoxWrapper over N envs with VectorEnv autoreset semantics.

    ctrl: ('pd', p, d) or ('vel',).  mp_spec: oracle.mp.MPSpec, or traj_fn(params, s0, q, qd)
    returning desired (pos, vel) [N, T, dof] f32.
    """

    def __init__(self, name, N, ctrl, mp_spec=None, traj_fn=None, replan_period=0,
                 max_planning_times=np.inf, condition_on_desired=False, info_level=0,
                 time_aware=None, tables=None, env_kwargs=None, learned=None, schedule=None,
                 reward_aggregation=np.sum):
        self.env = BatchedReacher(name, N, **(env_kwargs or {}))
        self.reward_aggregation = reward_aggregation   # black_box_wrapper.py:252
        self.N = N
        self.ctrl = ctrl
        self.spec = mp_spec
        self.replan = replan_period
        self.schedule = schedule          # object with .batch(obs [N, D] f64, t [N]) -> bool [N]
        do_replan = replan_period > 0 or schedule is not None
        self.do_replan = do_replan
        sub = bool(learned and learned.get("sub_traj"))
        self.time_aware = (do_replan or sub) if time_aware is None else time_aware
        self.return_context = not do_replan and not sub
        self.max_planning_times = max_planning_times
        self.condition_on_desired = condition_on_desired
        self.info_level = info_level
        if learned is not None:   # per-env tau / delay (make_env_helpers.py:115-126)
            lk = dict(learned)
            traj_fn = lambda params, s0, q, qd: mpm.trajectory_learned(
                mp_spec, params, s0, q, qd, learn_tau=lk.get("learn_tau", False) or sub,
                learn_delay=lk.get("learn_delay", False), sub_traj=sub,
                tau_bound=lk.get("tau_bound"), delay_bound=lk.get("delay_bound"))
        if traj_fn is None:
            self.T = mp_spec.T
            self.tables = tables if tables is not None else mpm.build_tables(
                mp_spec, (MAX_EPISODE_STEPS if do_replan else 0) + self.T + 2)
            traj_fn = lambda params, s0, q, qd: mpm.trajectory(mp_spec, self.tables, params, s0, q, qd)
        self.traj_fn = traj_fn
        self.traj_steps = np.zeros(N, np.int64)
        self.plan_steps = np.zeros(N, np.int64)
        self.cond_pos = None
        self.cond_vel = None
        self.has_cond = np.zeros(N, bool)

    def _full(self, o, t_aware):
        if self.time_aware:
            o = np.concatenate([o.astype(np.float64), (t_aware / MAX_EPISODE_STEPS)[:, None]], axis=1)
        return o

    def observation(self, o):
        if self.return_context:
            o = o[:, self.env.mask]
        return o.astype(f32)

    def _reset_idx(self, idx, seeds=None, options=None):
        o = self.env.reset(idx, seeds, options)
        self.traj_steps[idx] = 0
        self.plan_steps[idx] = 0
        self.has_cond[idx] = False
        return self.observation(self._full(o, np.zeros(len(idx))))

    def reset(self, seed=None, options=None):
        idx = list(range(self.N))
        seeds = None if seed is None else [seed + i for i in idx]
        return self._reset_idx(idx, seeds, options)

    def step(self, params):
        env, N, n = self.env, self.N, self.env.n
        q_c = env.q.copy()
        qd_c = env.qd.copy()
        if self.condition_on_desired and np.any(self.has_cond):
            q_c[self.has_cond] = self.cond_pos[self.has_cond]
            qd_c[self.has_cond] = self.cond_vel[self.has_cond]
        s0 = self.traj_steps if self.do_replan else np.zeros(N, np.int64)
        out = self.traj_fn(params, s0, q_c, qd_c)
        pos, vel = out[0], out[1]
        T = pos.shape[1]
        plan_len = out[2] if len(out) > 2 else np.full(N, T)
        act = np.ones(N, bool)
        rewards = np.zeros((N, T))
        tlen = np.zeros(N, np.int64)
        last_obs = np.zeros((N, env.obs_dim + int(self.time_aware)))
        term = np.zeros(N, bool)
        trunc = np.zeros(N, bool)
        self.plan_steps += 1
        if self.info_level >= 2:
            acts_log = np.full((N, T, n), np.nan)
            obs_log = np.full((N, T, env.obs_dim + int(self.time_aware)), np.nan, f32)
            info_log = {}
        a_is_f32 = self.ctrl[0] in ("vel", "pos")
        for t in range(T):
            if self.ctrl[0] == "pd":
                p, d = self.ctrl[1], self.ctrl[2]
                a = p * (pos[:, t] - env.q) + d * (vel[:, t] - env.qd)
            elif self.ctrl[0] == "pos":          # pos_controller.py:8-9
                a = pos[:, t]
            else:                                 # vel_controller.py:8-9
                a = vel[:, t]
            a = np.clip(a, env.act_low, env.act_high)
            o, r, te, tr, info = env.step(a if not a_is_f32 else a.astype(np.float64), act, a_is_f32)
            o = self._full(o, env.steps.astype(np.float64))
            rewards[act, t] = r[act]
            last_obs[act] = o[act]
            if self.info_level >= 2:
                acts_log[act, t] = np.asarray(a, np.float64)[act]
                obs_log[act, t] = o[act]
                for k, v in info.items():
                    if k not in info_log:
                        info_log[k] = np.zeros((N, T) + np.shape(v)[1:], np.asarray(v).dtype)
                    info_log[k][act, t] = np.asarray(v)[act]
            tlen[act] = t + 1
            term[act] = te[act]
            trunc[act] = tr[act]
            replan_now = np.zeros(N, bool)
            if self.schedule is not None:
                replan_now = self.schedule.batch(o, t + 1 + self.traj_steps) & (self.plan_steps < self.max_planning_times)
            elif self.replan > 0:
                replan_now = ((t + 1 + self.traj_steps) % self.replan == 0) & (self.plan_steps < self.max_planning_times)
            stop = act & (te | tr | replan_now | (t + 1 >= plan_len))
            if self.condition_on_desired and np.any(stop):
                if self.cond_pos is None:
                    self.cond_pos = np.zeros((N, n), f32)
                    self.cond_vel = np.zeros((N, n), f32)
                self.cond_pos[stop] = pos[stop, t]
                self.cond_vel[stop] = vel[stop, t]
                self.has_cond |= stop
            act = act & ~stop
            if not np.any(act):
                break
        self.traj_steps += tlen
        ret = np.array([self.reward_aggregation(rewards[i, :tlen[i]]) for i in range(N)], np.float64)
        obs = self.observation(last_obs)
        final_obs = obs.copy()
        done = term | trunc
        if np.any(done):
            idx = list(np.nonzero(done)[0])
            obs[idx] = self._reset_idx(idx)
        out_info = {"trajectory_length": tlen, "final_obs": final_obs, "done": done}
        if self.info_level >= 2:
            out_info.update(positions=pos, velocities=vel, step_actions=acts_log,
                            step_observations=obs_log, step_rewards=rewards)
            out_info.update(info_log)
        return obs, ret, term, trunc, out_info


def run_chunk(args):
    """Flags / lengths / returns of global envs [lo, hi) (env i seeded i) over a list of BB-step
    parameter blocks: the unit of work of the tests' process-parallel full-batch checks."""
    name, ctrl, spec, tables, kw, lo, hi, plist = args
    ob = BatchedBB(name, hi - lo, ctrl, mp_spec=spec, tables=tables, **kw)
    ob._reset_idx(list(range(hi - lo)), list(range(lo, hi)))
    out = []
    for p in plist:
        _, r_ret, r_te, r_tr, r_info = ob.step(p)
        out.append((r_info["trajectory_length"], r_te, r_tr, r_ret))
    return lo, out
