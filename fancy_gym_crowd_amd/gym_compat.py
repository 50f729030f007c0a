"""gymnasium reachability: ``gym.make('fancy_ProMP/LongSimpleReacher-v0')`` over the engine.

The reference registers its ids with gymnasium (envs/registry.py:245-254, ``gym.register(id=...,
entry_point=bb_env_constructor, ...)``), so user code reaches a black-box env through
``gym.make``.  ``register_gymnasium()`` does the same for every id of this package's registry
(``fancy/<Name>-v0`` and ``fancy_{ProMP,DMP,ProDMP}/<Name>-v0``), each backed by ``SingleEnv``: ONE
env of the id as a gymnasium Env (numpy in / out, no auto-reset -- the semantics of the reference's
``gym.make`` result) on a GPU handle.  Batched code should keep using ``fgx.make(id, num_envs=N)``.
gymnasium is not installed in this image: ``register_gymnasium()`` then returns False and nothing is
registered; ``SingleEnv`` itself needs no gymnasium.
"""
import functools

import numpy as np
import torch


class SingleEnv:
    """One env of a registered id with the gymnasium Env API (reset / step / spaces / close).

    reset(seed=s, options=...) -> (obs, info); step(action) -> (obs, reward, terminated, truncated,
    info) with numpy arrays and Python scalars; the per-env info keys of the vector env, row 0."""

    metadata = {"render_modes": []}
    render_mode = None

    def __init__(self, env_id, device="cuda:0", **kwargs):
        from . import make
        self._env = make(env_id, num_envs=1, device=device, autoreset=False, **kwargs)
        self.env_id = env_id
        self.black_box = hasattr(self._env, "n_params")
        self.observation_space = getattr(self._env, "single_observation_space", None)
        self.action_space = self._env.single_action_space

    @property
    def unwrapped(self):
        return self

    def reset(self, *, seed=None, options=None):
        obs, info = self._env.reset(seed=seed, options=options)
        return obs[0].detach().cpu().numpy(), {}

    def step(self, action):
        a = torch.as_tensor(np.asarray(action, dtype=np.float32)).reshape(1, -1)
        obs, rew, te, tr, info = self._env.step(a)
        out = {}
        for k, v in info.items():
            if k.startswith("_") or k in ("final_observation", "final_info"):
                continue
            if isinstance(v, torch.Tensor):
                x = v[0].detach().cpu().numpy()
                out[k] = x.item() if x.ndim == 0 else x
        if "trajectory_length" in out:   # per-step lists end at trajectory_length (black_box_wrapper.py:241)
            L = int(out["trajectory_length"])
            for k, v in list(out.items()):
                if k not in ("trajectory_length", "positions", "velocities") and isinstance(v, np.ndarray) \
                        and v.ndim >= 1 and v.shape[0] >= L:
                    out[k] = v[:L]
        return (obs[0].detach().cpu().numpy(), float(rew[0]), bool(te[0]), bool(tr[0]), out)

    def close(self):
        self._env.close()


def _to_gym_box(b, gym_module):
    """the engine's Box stand-in as a `gym_module.spaces.Box` (same low / high / shape / dtype)"""
    return gym_module.spaces.Box(low=b.low, high=b.high, shape=b.shape, dtype=b.dtype)


def gym_spaces(env_id, gym_module, mp_config_override=None, **env_kwargs):
    """(observation_space, action_space) of one env of `env_id` as `gym_module.spaces.Box` instances
    (same low / high / shape / dtype as the engine's own Box stand-in), from the resolved config
    alone (no device work).  gymnasium's env checker requires spaces derived from gymnasium.spaces.Space."""
    from .registry import resolve
    from .vector_env import action_space, observation_space
    cfg, meta = resolve(env_id, mp_config_override, **env_kwargs)
    return (_to_gym_box(observation_space(cfg), gym_module),
            _to_gym_box(action_space(cfg, meta.get("n_params", 0)), gym_module))


def registered_ids():
    from .registry import _BB_IDS, ENV_SPECS
    return sorted(ENV_SPECS) + sorted(_BB_IDS)


def register_gymnasium(device="cuda:0", gym_module=None):
    """Register every id with gymnasium (entry point: SingleEnv on `device`); False when gymnasium
    is not importable.  gym_module: a stand-in with gymnasium's ``register`` / ``Env`` (tests)."""
    gym = gym_module
    if gym is None:
        try:
            import gymnasium as gym
        except ImportError:
            return False
    def _init(self, env_id, device="cuda:0", **kwargs):
        # every make() kwarg (mp_config_override, info_level, env kwargs, ...) goes to the engine once,
        # as bb_env_constructor takes them (envs/registry.py:280-309)
        SingleEnv.__init__(self, env_id, device, **kwargs)
        # gymnasium's PassiveEnvChecker rejects spaces that are not gymnasium.spaces.Space instances:
        # the spaces of the env just built, converted (never a second resolve of the kwargs)
        self.observation_space = _to_gym_box(self.observation_space, gym)
        self.action_space = _to_gym_box(self.action_space, gym)

    base = type("GymSingleEnv", (SingleEnv, gym.Env), {"__init__": _init})
    for env_id in registered_ids():
        # the engine keeps the registry's TimeLimit itself (the truncated flag), so gymnasium adds none
        gym.register(id=env_id, entry_point=functools.partial(base, env_id, device))
    return True
