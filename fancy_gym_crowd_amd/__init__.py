"""fancy_gym_crowd_amd — MI355X-native vectorised black-box rollout engine for fancy_gym's reachers.

Drop-in for the reference's black-box path (fancy_gym/black_box/black_box_wrapper.py):

    import fancy_gym_crowd_amd as fgx
    env = fgx.make('fancy_ProMP/LongSimpleReacher-v0', num_envs=65536, device='cuda:0')
    obs, info = env.reset(seed=0)
    obs, ret, terminated, truncated, info = env.step(params)    # params [N, 25] f32 tensor

``make`` resolves the id and ``mp_config_override`` exactly as the reference's
``gym.make`` -> ``bb_env_constructor`` -> ``make_bb`` chain (envs/registry.py:280-309,
utils/make_env_helpers.py:68-136) and returns a batched env whose every step runs in
hand-written HIP kernels (libfgx.so) on the GPU.
"""
from .registry import (ALL_MOVEMENT_PRIMITIVE_ENVIRONMENTS, ENV_SPECS, KNOWN_MPS,  # noqa: F401
                       MOVEMENT_PRIMITIVE_ENVIRONMENTS_FOR_NS, REPLAN_CLOSE, ReplanAny, ReplanAt,
                       ReplanEvery, ReplanNormPeriod, TrajValidity, nested_update, register, resolve,
                       upgrade)

__all__ = ["make", "BlackBoxVectorEnv", "StepVectorEnv", "ReplanEvery", "ReplanAt", "ReplanNormPeriod",
           "ReplanAny", "REPLAN_CLOSE", "TrajValidity", "register", "register_gymnasium", "SingleEnv", "upgrade", "resolve",
           "ALL_MOVEMENT_PRIMITIVE_ENVIRONMENTS", "KNOWN_MPS"]


def make(env_id, num_envs=1, device="cuda", mp_config_override=None, **kwargs):
    """gym.make-style constructor of a batched env (BlackBoxVectorEnv or StepVectorEnv)."""
    from .registry import parse_id
    from .vector_env import BlackBoxVectorEnv, StepVectorEnv
    _, mp_type, _ = parse_id(env_id)
    if mp_type is None:
        if mp_config_override:
            raise ValueError("mp_config_override given for a step-based env id")
        return StepVectorEnv(env_id, num_envs, device=device, **kwargs)
    return BlackBoxVectorEnv(env_id, num_envs, device=device, mp_config_override=mp_config_override, **kwargs)


def register_gymnasium(device="cuda:0", gym_module=None):
    """gym.make('fancy_ProMP/...') reachability (envs/registry.py:245-254): see gym_compat."""
    from .gym_compat import register_gymnasium as _reg
    return _reg(device, gym_module)


def __getattr__(name):
    if name == "SingleEnv":
        from .gym_compat import SingleEnv
        return SingleEnv
    if name in ("BlackBoxVectorEnv", "StepVectorEnv", "Box", "ResetNeeded"):
        from . import vector_env
        return getattr(vector_env, name)
    raise AttributeError(name)
