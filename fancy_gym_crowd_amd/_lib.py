"""ctypes binding of libfgx.so (include/fgx.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be loaded,
``lib()`` raises.  torch is imported first so that libfgx.so binds to the HIP runtime torch
already loaded (both carry the SONAME libamdhip64.so.7): device pointers and streams from
torch are then valid in libfgx.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfgx.so")

FGX_ABI_VERSION = 8
INNER_STEPS_LEN = 128 * 16   # include/fgx.h FGX_INNER_STEPS_LEN (partial counters, sum them)
ENV_SIMPLE, ENV_HOLE, ENV_VIA = 0, 1, 2
REW_SIMPLE, REW_VEL_ACC, REW_UNBOUNDED = 0, 1, 2
SCHED_EVERY, SCHED_AT, SCHED_NORM_PERIOD = 0, 1, 2
MP_NONE, MP_PROMP, MP_DMP, MP_PRODMP = 0, 1, 2, 3
PHASE_LINEAR, PHASE_EXP = 0, 1
CTRL_PD, CTRL_VEL, CTRL_POS = 0, 1, 2
VALID_TAU, VALID_DELAY, VALID_POS = 1, 2, 4
INVALID_OBS_ZEROS, INVALID_OBS_CURRENT = 0, 1
ERRORS = {-1: "FGX_E_INVALID", -2: "FGX_E_HIP", -3: "FGX_E_NOMEM", -4: "FGX_E_UNSUPPORTED"}


class FgxConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "abi_version", "env_kind", "n_links", "random_start", "allow_self_collision",
        "allow_wall_collision", "mp_kind", "phase_kind", "n_basis", "zero_start", "zero_goal",
        "ctrl_kind", "T", "max_episode_steps", "replan_period", "max_planning_times",
        "condition_on_desired", "time_aware", "return_context", "num_basis_outside")] + [
        (n, ctypes.c_double) for n in (
            "dt", "duration", "tau", "delay", "alpha_phase", "bandwidth", "weights_scale",
            "goal_scale", "alpha", "pc_length", "p_gain", "d_gain", "act_low", "act_high",
            "hole_width", "hole_depth", "hole_x", "collision_penalty")] + [
        (n, ctypes.c_int32) for n in (
            "rew_fct", "learn_tau", "learn_delay", "learn_sub_trajectories")] + [
        (n, ctypes.c_double) for n in (
            "tau_bound_lo", "tau_bound_hi", "delay_bound_lo", "delay_bound_hi",
            "via_x", "via_y", "target_x", "target_y")] + [
        ("sched_n", ctypes.c_int32), ("sched_kind", ctypes.c_int32 * 4), ("sched_k", ctypes.c_int32 * 4),
        ("sched_i0", ctypes.c_int32 * 4), ("sched_i1", ctypes.c_int32 * 4),
        ("sched_mul", ctypes.c_double * 4), ("sched_div", ctypes.c_double * 4),
        ("n_gains", ctypes.c_int32), ("reserved1", ctypes.c_int32),
        ("p_gains", ctypes.c_double * 8), ("d_gains", ctypes.c_double * 8)] + [
        (n, ctypes.c_int32) for n in ("valid_flags", "invalid_obs", "invalid_terminated", "invalid_truncated")] + [
        (n, ctypes.c_double) for n in ("invalid_reward", "valid_tau_lo", "valid_tau_hi", "valid_delay_lo",
                                       "valid_delay_hi")] + [
        ("valid_pos_lo", ctypes.c_double * 8), ("valid_pos_hi", ctypes.c_double * 8),
        ("basis_dt", ctypes.c_double)]


class FgxDims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_envs", "dof", "obs_dim", "ctx_dim", "out_obs_dim", "n_params", "T", "table_rows",
        "table_stride")] + [("reserved", ctypes.c_int32 * 7)]


class FgxInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "positions", "velocities", "step_actions", "step_obs", "step_rewards", "is_collided",
        "is_success", "end_effector", "reward_dist", "reward_ctrl", "inner_steps")]


EXPORTS = {
    "fgx_last_error": (ctypes.c_char_p, []),
    "fgx_abi_version": (ctypes.c_int, []),
    "fgx_build_id": (ctypes.c_char_p, []),
    "fgx_create": (ctypes.c_int, [ctypes.POINTER(FgxConfig), ctypes.c_int64, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_void_p)]),
    "fgx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "fgx_get_dims": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(FgxDims)]),
    "fgx_reset": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_int32] + [ctypes.c_void_p] * 2),
    "fgx_step": (ctypes.c_int, [ctypes.c_void_p] * 8 + [ctypes.POINTER(FgxInfo), ctypes.c_int32,
                                                         ctypes.c_void_p]),
    "fgx_step_traj": (ctypes.c_int, [ctypes.c_void_p] * 9 + [ctypes.POINTER(FgxInfo), ctypes.c_int32,
                                                              ctypes.c_void_p]),
    "fgx_trajectory": (ctypes.c_int, [ctypes.c_void_p] * 5),
    "fgx_step_raw": (ctypes.c_int, [ctypes.c_void_p] * 7 + [ctypes.c_int32, ctypes.c_void_p]),
    "fgx_get_state": (ctypes.c_int, [ctypes.c_void_p] * 7),
    "fgx_set_state": (ctypes.c_int, [ctypes.c_void_p] * 7),
    "fgx_get_tables": (ctypes.c_int, [ctypes.c_void_p] * 3),
    "fgx_episode_kernel": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "fgx_selftest_sincos": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
}
EPISODE_KERNELS = {0: "k_episode", 1: "k_episode_jp", 2: "k_episode_ws", 3: "k_episode_jl", 4: "k_episode_w2",
                   5: "k_episode_pair", 6: "k_episode_v2", 7: "k_episode_v2h",
                   8: "k_episode_hp"}

_LIB = None


class FgxError(RuntimeError):
    pass


def load(path=None):
    """Load libfgx.so and declare every exported symbol (no GPU needed).  FGX_LIB names another
    build of the same ABI (kernel experiments; its build id is not checked); the default is the
    in-tree library, whose build id must match the in-tree sources (_build.source_hash)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("FGX_LIB") or LIB_PATH
    import torch  # noqa: F401  (bind to torch's HIP runtime, see module docstring)
    if not os.path.exists(path):
        raise FgxError(f"libfgx.so not built ({path}); run __graft_entry__.build() — there is no CPU fallback")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    abi = lib.fgx_abi_version()
    if abi != FGX_ABI_VERSION:
        raise FgxError("libfgx ABI version mismatch")
    if path == LIB_PATH:   # build provenance: the in-tree library must match the in-tree sources
        from . import _build
        want, got = _build.source_hash(), lib.fgx_build_id().decode()
        if got != want:
            raise FgxError(f"libfgx.so was built from other sources (build id {got}, sources {want}); "
                           "run __graft_entry__.build()")
    _LIB = lib
    return lib


def check(rc):
    if rc != 0:
        msg = _LIB.fgx_last_error().decode() if _LIB is not None else ""
        kind = ERRORS.get(rc, str(rc))
        if rc in (-1, -4):
            raise ValueError(f"{kind}: {msg}")
        raise FgxError(f"{kind}: {msg}")
    return rc
