"""Batched black-box / step-based reacher envs on one MI355X, returning torch-ROCm tensors.

The Python surface mirrors what a user of the reference gets from
``gymnasium.vector.SyncVectorEnv([lambda: gym.make('fancy_ProMP/...')] * N)``:
  reset(seed, options) -> (obs [N, obs_dim] f32, info)          (black_box_wrapper.py:258-267)
  step(actions)        -> (obs, reward [N] f64, terminated [N] bool, truncated [N] bool, info)
                                                                  (black_box_wrapper.py:170-253)
with gymnasium 0.29 vector semantics [EXT-M]: reset(seed=s) seeds env i with s + i; finished
envs are auto-reset inside step(), their last observation is in info['final_observation'] and
the info of their last step in info['final_info'] (boolean masks '_final_observation' /
'_final_info').

info levels (BlackBoxWrapper.step assembles its info per verbosity, black_box_wrapper.py:185-249;
the reference's step(action, verbose=2) default means a gym.make user always gets level 2):
  0  trajectory_length only (the fast path; bench.py)
  1  + the env's per-step info lists: reward_dist / reward_ctrl (SimpleReacher,
     simple_reacher.py:56-70) or is_collided / is_success / end_effector (Hole / ViaPoint)
  2  + positions, velocities, step_actions, step_observations, step_rewards   (default)
Per-step arrays are [N, T, ...], NaN (0 for flags) after each env's trajectory_length.

All compute runs in libfgx.so (HIP) on the tensors' device; there is no CPU fallback.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .registry import resolve


class Box:
    """Minimal gymnasium.spaces.Box stand-in (bounds in the space dtype, as gymnasium stores them)."""

    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        shape = tuple(shape) if shape is not None else np.shape(low)
        self.shape = shape
        self.low = np.broadcast_to(np.asarray(low, float), shape).astype(self.dtype)
        self.high = np.broadcast_to(np.asarray(high, float), shape).astype(self.dtype)

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        lo, hi = self.low.astype(float), self.high.astype(float)
        out = np.where(np.isfinite(lo) & np.isfinite(hi), rng.uniform(np.nan_to_num(lo), np.nan_to_num(hi)),
                       rng.standard_normal(self.shape))
        return out.astype(self.dtype)

    def __repr__(self):
        return f"Box({self.shape}, {self.dtype})"


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class _Engine:
    """Owns one libfgx handle (one device)."""

    def __init__(self, cfg, num_envs, device):
        self.lib = _lib.load()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("fancy_gym_crowd_amd runs on a ROCm GPU device (cuda:N); there is no CPU path")
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        torch.cuda.set_device(idx)
        self.cfg = cfg
        h = ctypes.c_void_p()
        _lib.check(self.lib.fgx_create(ctypes.byref(cfg), int(num_envs), int(idx), ctypes.byref(h)))
        self.h = h
        d = _lib.FgxDims()
        _lib.check(self.lib.fgx_get_dims(h, ctypes.byref(d)))
        self.dims = d

    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.fgx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FinalInfo:
    """info['final_info'] of gymnasium 0.29's SyncVectorEnv [EXT-M]: entry i is the info dict env i
    produced on the step that ended its episode (the reference's BlackBoxWrapper.step infos:
    trajectory_length, the per-step lists cut at trajectory_length, the full desired plan), None
    for envs that did not finish.  Entries are built on access (numpy, host), so step() itself
    stays free of host synchronisation."""

    _FULL = ("positions", "velocities")   # black_box_wrapper.py:245-246: the whole plan

    def __init__(self, done, per_env):
        self._done_t = done
        self._done = None
        self._per_env = per_env
        self._host = None

    def _sync(self):
        if self._done is None:
            self._done = self._done_t.detach().cpu().numpy().astype(bool)
            self._host = {k: v.detach().cpu().numpy() for k, v in self._per_env.items()}
        return self._done

    def __len__(self):
        return int(self._done_t.shape[0])

    def __getitem__(self, i):
        done = self._sync()
        if not done[i]:
            return None
        if "trajectory_length" not in self._host:   # step-based envs: no per-step info is kept
            return {}
        L = int(self._host["trajectory_length"][i])
        out = {}
        for k, v in self._host.items():
            if k == "trajectory_length":
                out[k] = L
            elif k in self._FULL:
                out[k] = v[i]
            else:
                out[k] = v[i, :L]
        return out

    def __iter__(self):
        return (self[i] for i in range(len(self)))


class ResetNeeded(RuntimeError):
    """step() before reset() (gymnasium's OrderEnforcing wrapper, error.ResetNeeded [EXT-M])."""


def _order_check(env):
    if env._needs_reset:
        raise ResetNeeded("Cannot call env.step() before calling env.reset()")


class BlackBoxVectorEnv:
    """N black-box envs (one BB step = one whole (sub-)episode) on one GPU."""

    def __init__(self, env_id, num_envs, device="cuda", mp_config_override=None, info_level=None,
                 autoreset=True, seed_offset=0, **env_kwargs):
        cfg, meta = resolve(env_id, mp_config_override, **env_kwargs)
        if meta["mp_type"] is None:
            raise ValueError(f"{env_id} is a step-based id; use StepVectorEnv / make()")
        self.meta = meta
        self.num_envs = int(num_envs)
        self.info_level = meta["verbose"] if info_level is None else int(info_level)
        if self.info_level not in (0, 1, 2):
            raise ValueError("info_level must be 0, 1 or 2")
        self.autoreset = bool(autoreset)
        self.seed_offset = int(seed_offset)
        self._needs_reset = True
        self._eng = _Engine(cfg, num_envs, device)
        d = self._eng.dims
        self.dof, self.T, self.n_params = d.dof, d.T, d.n_params
        self.obs_dim, self.out_dim, self.full_dim = d.obs_dim, d.out_obs_dim, d.obs_dim + cfg.time_aware
        self.device = self._eng.device
        self.single_action_space = Box(-np.inf, np.inf, (self.n_params,), np.float32)
        self.action_space = Box(-np.inf, np.inf, (self.num_envs, self.n_params), np.float32)
        self.single_observation_space = self._obs_space(cfg)
        self.observation_space = Box(np.broadcast_to(self.single_observation_space.low, (self.num_envs, self.out_dim)),
                                     np.broadcast_to(self.single_observation_space.high, (self.num_envs, self.out_dim)))
        self._alloc()

    def _obs_space(self, cfg):
        return observation_space(cfg)

    def _alloc(self):
        N, dev = self.num_envs, self.device
        self._obs = torch.empty((N, self.out_dim), dtype=torch.float32, device=dev)
        self._fobs = torch.empty((N, self.out_dim), dtype=torch.float32, device=dev)
        self._ret = torch.empty(N, dtype=torch.float64, device=dev)
        self._te = torch.empty(N, dtype=torch.uint8, device=dev)
        self._tr = torch.empty(N, dtype=torch.uint8, device=dev)
        self._len = torch.empty(N, dtype=torch.int32, device=dev)

    # ------------------------------------------------------------------ gymnasium-style API
    def reset(self, *, seed=None, options=None):
        """seed: int (env i gets seed + seed_offset + i) or one seed per env; options:
        'random_start' (base_reacher.py:77-80) and 'reset_mask' ([N] bool: reset only those envs,
        the others' rows of obs hold their current observation)."""
        obs = torch.empty((self.num_envs, self.out_dim), dtype=torch.float32, device=self.device)
        _reset_engine(self, seed, options, obs)
        return obs, {}

    def _needs_step_rewards(self):
        """A reward_aggregation other than sum / mean reads the per-step rewards."""
        return self.meta["reward_aggregation"] not in ("sum", "mean")

    def _info_buffers(self):
        """Per-step info arrays of the info level (module docstring).  The device writes them
        time- and component-major ([T, N] and [T, X, N], so that every wave store covers 64
        consecutive envs, include/fgx.h fgx_info); the caller sees [N, T, ...] views.  A
        reward_aggregation other than sum / mean also needs step_rewards."""
        generic_agg = self._needs_step_rewards()
        if self.info_level == 0 and not generic_agg:
            return None, {}
        N, T, n, dev = self.num_envs, self.T, self.dof, self.device
        # every row is written by the kernel (NaN / 0 after trajectory_length): no fill here
        e = lambda *shape, dt=torch.float32: torch.empty(shape, dtype=dt, device=dev)   # noqa: E731
        raw = {}
        info = _lib.FgxInfo()
        if self.info_level >= 2:
            raw.update(positions=e(T, n, N), velocities=e(T, n, N), step_actions=e(T, n, N, dt=torch.float64),
                       step_observations=e(T, self.full_dim, N))
            info.positions, info.velocities = raw["positions"].data_ptr(), raw["velocities"].data_ptr()
            info.step_actions, info.step_obs = raw["step_actions"].data_ptr(), raw["step_observations"].data_ptr()
        if self.info_level >= 2 or generic_agg:
            raw["step_rewards"] = e(T, N, dt=torch.float64)
            info.step_rewards = raw["step_rewards"].data_ptr()
        if self.info_level >= 1:
            if self.meta["kind"] in ("hole", "via"):
                raw["is_collided"] = e(T, N, dt=torch.uint8)
                raw["is_success"] = e(T, N, dt=torch.uint8)
                raw["end_effector"] = e(T, 2, N, dt=torch.float64)
                info.is_collided, info.is_success = raw["is_collided"].data_ptr(), raw["is_success"].data_ptr()
                info.end_effector = raw["end_effector"].data_ptr()
            else:
                raw["reward_dist"] = e(T, N, dt=torch.float64)
                raw["reward_ctrl"] = e(T, N, dt=torch.float64)
                info.reward_dist, info.reward_ctrl = raw["reward_dist"].data_ptr(), raw["reward_ctrl"].data_ptr()
        return info, {k: (v.transpose(0, 1) if v.dim() == 2 else v.permute(2, 0, 1)) for k, v in raw.items()}

    def _check_actions(self, actions):
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.float32:
            a = a.to(torch.float32)
        if tuple(a.shape) != (self.num_envs, self.n_params):
            raise ValueError(f"actions must have shape {(self.num_envs, self.n_params)}, got {tuple(a.shape)}")
        return a.contiguous()

    def step(self, actions):
        _order_check(self)
        a = self._check_actions(actions)
        N = self.num_envs
        obs = torch.empty((N, self.out_dim), dtype=torch.float32, device=self.device)
        fobs = torch.empty_like(obs)
        ret = torch.empty(N, dtype=torch.float64, device=self.device)
        # (bool tensors: the library writes bytes 0 / 1, so .bool() below is free, no conversion kernel)
        te = torch.empty(N, dtype=torch.bool, device=self.device)
        tr = torch.empty(N, dtype=torch.bool, device=self.device)
        tl = torch.empty(N, dtype=torch.int32, device=self.device)
        info_s, bufs = self._info_buffers()
        _lib.check(self._eng.lib.fgx_step(self._eng.h, _ptr(a), _ptr(obs), _ptr(ret), _ptr(te), _ptr(tr), _ptr(tl),
                                          _ptr(fobs), ctypes.byref(info_s) if info_s is not None else None,
                                          int(self.autoreset), self._eng.stream()))
        return self._package(obs, ret, te, tr, tl, fobs, bufs)

    def step_trajectory(self, des_pos, des_vel):
        """BB step with caller-supplied desired trajectories [N, T, dof] f32 (no MP evaluation)."""
        _order_check(self)
        N, T, n = self.num_envs, self.T, self.dof
        p = torch.as_tensor(des_pos, device=self.device).to(torch.float32).contiguous()
        v = torch.as_tensor(des_vel, device=self.device).to(torch.float32).contiguous()
        if tuple(p.shape) != (N, T, n) or tuple(v.shape) != (N, T, n):
            raise ValueError(f"desired trajectories must be {(N, T, n)}")
        obs = torch.empty((N, self.out_dim), dtype=torch.float32, device=self.device)
        fobs = torch.empty_like(obs)
        ret = torch.empty(N, dtype=torch.float64, device=self.device)
        # (bool tensors: the library writes bytes 0 / 1, so .bool() below is free, no conversion kernel)
        te = torch.empty(N, dtype=torch.bool, device=self.device)
        tr = torch.empty(N, dtype=torch.bool, device=self.device)
        tl = torch.empty(N, dtype=torch.int32, device=self.device)
        info_s, bufs = self._info_buffers()
        _lib.check(self._eng.lib.fgx_step_traj(self._eng.h, _ptr(p), _ptr(v), _ptr(obs), _ptr(ret), _ptr(te),
                                               _ptr(tr), _ptr(tl), _ptr(fobs),
                                               ctypes.byref(info_s) if info_s is not None else None,
                                               int(self.autoreset), self._eng.stream()))
        if self.info_level >= 2:
            bufs["positions"], bufs["velocities"] = p, v
        return self._package(obs, ret, te, tr, tl, fobs, bufs)

    def _package(self, obs, ret, te, tr, tl, fobs, bufs):
        """(obs, return, terminated, truncated, info) as gymnasium 0.29's SyncVectorEnv assembles
        them from the envs' BlackBoxWrapper.step results (black_box_wrapper.py:241-253).

        info holds every per-env key for all envs, with gymnasium's '_key' masks marking the envs
        whose step info gymnasium would report there (those that did not finish: a finished env's
        step info moves to info['final_info'][i], its last observation to
        info['final_observation'][i])."""
        term, trunc = te.bool(), tr.bool()
        agg = self.meta["reward_aggregation"]
        if agg == "mean":
            ret = torch.where(tl > 0, ret / tl.to(torch.float64), ret)   # (tl 0: an invalid plan's return)
        elif agg in _DEVICE_AGG:   # np.max / np.min / np.median of rewards[:t+1] on the device
            ret = torch.where(tl > 0, _DEVICE_AGG[agg](bufs["step_rewards"], tl), ret)
        elif callable(agg):
            # any other callable on rewards[:t+1] (black_box_wrapper.py:252): user Python, applied
            # per env on the host -- a device sync and O(N) interpreter work per step
            rew = bufs["step_rewards"].detach().cpu().numpy()
            L = tl.detach().cpu().numpy()
            r0 = ret.detach().cpu().numpy()
            ret = torch.tensor([float(agg(rew[i, :L[i]])) if L[i] > 0 else float(r0[i]) for i in range(self.num_envs)],
                               dtype=torch.float64, device=self.device)
        if agg not in ("sum", "mean") and self.info_level < 2:
            bufs = {k: v for k, v in bufs.items() if k != "step_rewards"}
        per_env = {"trajectory_length": tl}
        per_env.update(bufs)
        info = dict(per_env)
        if self.autoreset:
            done = term | trunc
            keep = ~done
            for k in per_env:
                info["_" + k] = keep
            info["final_observation"] = fobs
            info["_final_observation"] = done
            info["final_info"] = FinalInfo(done, per_env)
            info["_final_info"] = done
        else:
            ones = torch.ones_like(term)
            for k in per_env:
                info["_" + k] = ones
            info["final_observation"] = fobs
        return obs, ret, term, trunc, info

    def trajectory(self, actions):
        """Desired (pos, vel) [N, T, dof] of the next plan (BlackBoxWrapper.get_trajectory)."""
        a = self._check_actions(actions)
        N, T, n = self.num_envs, self.T, self.dof
        pos = torch.empty((N, T, n), dtype=torch.float32, device=self.device)
        vel = torch.empty_like(pos)
        _lib.check(self._eng.lib.fgx_trajectory(self._eng.h, _ptr(a), _ptr(pos), _ptr(vel), self._eng.stream()))
        return pos, vel

    # ------------------------------------------------------------------ fast path (bench)
    def step_into(self, actions, obs, ret, te, tr, tl, fobs=None, inner_steps=None):
        """Allocation-free BB step into preallocated buffers (no shape checks of the env buffers; for
        benchmarks).  inner_steps: optional zero-initialised int64 [_lib.INNER_STEPS_LEN] device
        partial counters (new_inner_steps() allocates them): their sum += the sum of trajectory
        lengths.  A failed launch raises (fgx_step's return code is checked)."""
        _order_check(self)
        info = None
        if inner_steps is not None:
            # the kernels add to line (wave % 128) * 16 of the array: a shorter one would be written past
            if inner_steps.dtype != torch.int64 or inner_steps.numel() < _lib.INNER_STEPS_LEN:
                raise ValueError(f"inner_steps must be int64 with >= {_lib.INNER_STEPS_LEN} entries (new_inner_steps())")
            info = _lib.FgxInfo()
            info.inner_steps = inner_steps.data_ptr()
            info = ctypes.byref(info)
        _lib.check(self._eng.lib.fgx_step(self._eng.h, ctypes.c_void_p(actions.data_ptr()),
                                          ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(ret.data_ptr()),
                                          ctypes.c_void_p(te.data_ptr()), ctypes.c_void_p(tr.data_ptr()),
                                          ctypes.c_void_p(tl.data_ptr()),
                                          ctypes.c_void_p(fobs.data_ptr()) if fobs is not None else None, info,
                                          int(self.autoreset), self._eng.stream()))

    def new_inner_steps(self):
        """Zeroed device partial counters for step_into(inner_steps=...); total = .sum()."""
        return torch.zeros(_lib.INNER_STEPS_LEN, dtype=torch.int64, device=self.device)

    # ------------------------------------------------------------------ state / tables
    def get_state(self):
        N, n, dev = self.num_envs, self.dof, self.device
        q = torch.empty((N, n), dtype=torch.float64, device=dev)
        qd = torch.empty_like(q)
        goal = torch.empty((N, 2), dtype=torch.float64, device=dev)
        hole = torch.empty((N, 3), dtype=torch.float64, device=dev)
        steps = torch.empty(N, dtype=torch.int32, device=dev)
        _lib.check(self._eng.lib.fgx_get_state(self._eng.h, _ptr(q), _ptr(qd), _ptr(goal), _ptr(hole), _ptr(steps),
                                               self._eng.stream()))
        return dict(q=q, qd=qd, goal=goal, hole=hole, steps=steps)

    def set_state(self, q=None, qd=None, goal=None, hole=None, steps=None):
        def prep(x, dt):
            return None if x is None else torch.as_tensor(x, device=self.device).to(dt).contiguous()
        q, qd, goal, hole = (prep(x, torch.float64) for x in (q, qd, goal, hole))
        steps = prep(steps, torch.int32)
        _lib.check(self._eng.lib.fgx_set_state(self._eng.h, _ptr(q), _ptr(qd), _ptr(goal), _ptr(hole), _ptr(steps),
                                               self._eng.stream()))

    def episode_kernel(self, info_level=None):
        """Name of the HIP kernel step() launches (fgx_episode_kernel): k_episode, k_episode_jp,
        k_episode_ws, k_episode_jl, k_episode_w2, k_episode_pair, k_episode_v2, k_episode_v2h or k_episode_hp
        (HoleReacher up to info_level 1); all nine produce bit-identical results.  Whenever some per-step
        array is written (info_level >= 1, or a reward_aggregation that reads step_rewards) the launch
        takes k_episode_hp (HoleReacher below the verbose-2 rows), k_episode_v2 (SimpleReacher + PD),
        k_episode_v2h (the direct envs at a multiple of 256 envs) or the logging k_episode."""
        lvl = self.info_level if info_level is None else int(info_level)
        if self._needs_step_rewards():
            lvl = max(lvl, 1)
        k = self._eng.lib.fgx_episode_kernel(self._eng.h, lvl)
        if k < 0:
            _lib.check(k)
        return _lib.EPISODE_KERNELS[k]

    def tables(self):
        d = self._eng.dims
        out = torch.empty((d.table_rows, d.table_stride), dtype=torch.float32, device=self.device)
        _lib.check(self._eng.lib.fgx_get_tables(self._eng.h, _ptr(out), self._eng.stream()))
        return out

    def close(self):
        self._eng.close()


class StepVectorEnv:
    """N step-based reacher envs ('fancy/SimpleReacher-v0' ...), actions applied unclipped."""

    def __init__(self, env_id, num_envs, device="cuda", autoreset=True, seed_offset=0, **env_kwargs):
        cfg, meta = resolve(env_id, None, **env_kwargs)
        if meta["mp_type"] is not None:
            raise ValueError(f"{env_id} is a black-box id; use BlackBoxVectorEnv")
        self.meta = meta
        self.num_envs = int(num_envs)
        self.autoreset = bool(autoreset)
        self.seed_offset = int(seed_offset)
        self._needs_reset = True
        self._eng = _Engine(cfg, num_envs, device)
        d = self._eng.dims
        self.dof, self.obs_dim = d.dof, d.obs_dim
        self.device = self._eng.device
        bound = float(cfg.act_high)
        self.single_action_space = Box(-bound, bound, (self.dof,), np.float32)
        self.single_observation_space = observation_space(cfg)

    def reset(self, *, seed=None, options=None):
        obs = torch.empty((self.num_envs, self.obs_dim), dtype=torch.float32, device=self.device)
        _reset_engine(self, seed, options, obs)
        return obs, {}

    def step(self, actions):
        _order_check(self)
        a = torch.as_tensor(actions, device=self.device).to(torch.float32).contiguous()
        N = self.num_envs
        if tuple(a.shape) != (N, self.dof):
            raise ValueError(f"actions must have shape {(N, self.dof)}")
        obs = torch.empty((N, self.obs_dim), dtype=torch.float32, device=self.device)
        fobs = torch.empty_like(obs)
        rew = torch.empty(N, dtype=torch.float64, device=self.device)
        # (bool tensors: the library writes bytes 0 / 1, so .bool() below is free, no conversion kernel)
        te = torch.empty(N, dtype=torch.bool, device=self.device)
        tr = torch.empty(N, dtype=torch.bool, device=self.device)
        _lib.check(self._eng.lib.fgx_step_raw(self._eng.h, _ptr(a), _ptr(obs), _ptr(rew), _ptr(te), _ptr(tr),
                                              _ptr(fobs), int(self.autoreset), self._eng.stream()))
        term, trunc = te.bool(), tr.bool()
        done = term | trunc
        info = {"final_observation": fobs, "_final_observation": done}
        if self.autoreset:
            info["final_info"] = FinalInfo(done, {})
            info["_final_info"] = done
        return obs, rew, term, trunc, info

    def get_state(self):
        return BlackBoxVectorEnv.get_state(self)

    def set_state(self, q=None, qd=None, goal=None, hole=None, steps=None):
        """fgx_set_state (checkpoint restore / tests), as BlackBoxVectorEnv.set_state."""
        return BlackBoxVectorEnv.set_state(self, q, qd, goal, hole, steps)

    def close(self):
        self._eng.close()


def _masked_rows(step_rewards, tl, fill):
    """[N, T] view of the time-major rewards with the samples at or after trajectory_length set to
    `fill` (the kernel writes NaN there)."""
    T = step_rewards.shape[1]
    valid = torch.arange(T, device=step_rewards.device)[None, :] < tl.to(torch.int64)[:, None]
    return torch.where(valid, step_rewards, torch.full_like(step_rewards, fill)), valid


def _agg_max(step_rewards, tl):
    return _masked_rows(step_rewards, tl, -np.inf)[0].amax(dim=1)   # NaN propagates as in np.max


def _agg_min(step_rewards, tl):
    return _masked_rows(step_rewards, tl, np.inf)[0].amin(dim=1)


def _agg_median(step_rewards, tl):
    """np.median of rewards[:L] per row: the mean of the two middle order statistics ((a + b) / 2,
    or a / 1 for odd L -- numpy's mean of the partitioned middle), NaN if any reward is NaN."""
    x, valid = _masked_rows(step_rewards, tl, np.inf)
    has_nan = (torch.isnan(step_rewards) & valid).any(dim=1)
    xs = torch.sort(torch.nan_to_num(x, nan=np.inf), dim=1).values   # pads (+inf) sort after the samples
    L = tl.to(torch.int64).clamp(min=1)
    lo = xs.gather(1, ((L - 1) // 2)[:, None])[:, 0]
    hi = xs.gather(1, (L // 2)[:, None])[:, 0]
    med = torch.where(L % 2 == 1, lo, (lo + hi) / 2.0)
    return torch.where(has_nan, torch.full_like(med, np.nan), med)


# reductions of rewards[:t+1] run on the device (black_box_wrapper.py:252)
_DEVICE_AGG = {np.max: _agg_max, np.amax: _agg_max, np.min: _agg_min, np.amin: _agg_min, np.median: _agg_median}


def _reset_engine(env, seed, options, obs):
    """fgx_reset for either env class: seeds (int -> seed + seed_offset + i, or one per env),
    options 'random_start' / 'reset_mask' (checked against num_envs before any device read)."""
    N, dev = env.num_envs, env.device
    seeds = None
    if seed is not None:
        if isinstance(seed, (list, tuple, np.ndarray, torch.Tensor)):
            arr = np.asarray(seed.cpu() if isinstance(seed, torch.Tensor) else seed).reshape(-1)
            if arr.shape[0] != N:
                raise ValueError(f"seed list has {arr.shape[0]} entries for {N} envs")
            seeds = torch.as_tensor(arr.astype(np.uint64).astype(np.int64), device=dev)
        else:
            seeds = torch.arange(N, dtype=torch.int64, device=dev) + (int(seed) + env.seed_offset)
        seeds = seeds.contiguous()
    options = options or {}
    mask = None
    if options.get("reset_mask") is not None:
        mask = torch.as_tensor(options["reset_mask"], device=dev).reshape(-1).to(torch.uint8).contiguous()
        if mask.numel() != N:
            raise ValueError(f"reset_mask has {mask.numel()} entries for {N} envs")
    rs = options.get("random_start")
    rs = -1 if rs is None else int(bool(rs))
    _lib.check(env._eng.lib.fgx_reset(env._eng.h, _ptr(seeds), _ptr(mask), rs, _ptr(obs), env._eng.stream()))
    env._needs_reset = False


def math_isnan(x):
    return x != x


def observation_space(cfg):
    """The observation Box of one env of a resolved config: the env's state bounds (base_reacher.py
    observation_space: pi for cos / sin, inf otherwise), + TimeAwareObservation's [0, 1] entry
    (utils/wrappers.py:49-63), context-masked for a black-box id (black_box_wrapper.py:90-95)."""
    n = int(cfg.n_links)
    extra = {_lib.ENV_SIMPLE: 0, _lib.ENV_HOLE: 1, _lib.ENV_VIA: 2}[cfg.env_kind]   # width | via - ee
    bound = np.hstack([[np.pi] * n, [np.pi] * n, [np.inf] * n, [np.inf] * extra, [np.inf] * 2, [np.inf]])
    low, high = -bound, bound
    if cfg.time_aware:
        low, high = np.append(low, 0.0), np.append(high, 1.0)
    if cfg.return_context:
        rs = [bool(cfg.random_start)] * (3 * n)
        if cfg.env_kind == _lib.ENV_HOLE:
            rs = rs + [math_isnan(cfg.hole_width)]
        elif cfg.env_kind == _lib.ENV_VIA:
            rs = rs + [math_isnan(cfg.via_x)] * 2
        mask = rs + [True, True, False]
        low, high = low[np.array(mask)], high[np.array(mask)]
    return Box(low, high, dtype=np.float32)


def action_space(cfg, n_params):
    """The action Box of one env: the MP parameters (unbounded; learned tau / delay clipped inside the
    step as the reference's get_trajectory does) or, for a step-based id, the env's torque / velocity
    bounds in float32 (base_reacher_torque.py:16-18, base_reacher_direct.py:16-18)."""
    if cfg.mp_kind != _lib.MP_NONE:
        return Box(-np.inf, np.inf, (int(n_params),), np.float32)
    bound = float(cfg.act_high)
    return Box(-bound, bound, (int(cfg.n_links),), np.float32)
