"""CPU-only checks of the boundary and the host layer (no kernel is launched here).

Re-expresses the reference's structural tests (test/test_black_box.py, test/test_fancy_registry.py)
for the reacher path: id registration, config merge, action / context space sizes, error types.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import fancy_gym_crowd_amd as fgx
from fancy_gym_crowd_amd import _lib, registry

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ensure_built():
    from fancy_gym_crowd_amd import _build
    _build.build()   # no-op when the library's build id matches the sources


def test_library_exports_every_declared_symbol():
    _ensure_built()
    header = open(os.path.join(ROOT, "include", "fgx.h")).read()
    declared = set(re.findall(r"^\s*(?:int|const char\*)\s+(fgx_\w+)\s*\(", header, re.M))
    assert declared, "no declarations parsed"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = declared - exported
    assert not missing, f"declared in include/fgx.h but not exported: {missing}"
    assert declared == set(_lib.EXPORTS), "ctypes binding out of sync with include/fgx.h"
    # arity of every declaration == arity of the ctypes binding
    for name in declared:
        m = re.search(r"^\s*(?:int|const char\*)\s+" + name + r"\s*\(([^)]*)\)", header, re.S | re.M)
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(_lib.EXPORTS[name][1]), name


def test_library_loads_and_reports_abi():
    _ensure_built()
    lib = _lib.load()
    assert lib.fgx_abi_version() == _lib.FGX_ABI_VERSION
    # build provenance: the loaded library was compiled from exactly the tracked sources
    from fancy_gym_crowd_amd import _build
    assert lib.fgx_build_id().decode() == _build.source_hash() == _build.built_id()
    # argument validation happens before any device work
    cfg = _lib.FgxConfig()
    cfg.abi_version = 999
    h = ctypes.c_void_p()
    assert lib.fgx_create(ctypes.byref(cfg), 4, 0, ctypes.byref(h)) == -1
    assert b"abi" in lib.fgx_last_error()


def test_config_struct_layout_matches_header():
    # 20 int32, 18 doubles, (ABI 2) 4 int32 and 8 doubles, (ABI 3) 17 int32 + pad and 8 doubles,
    # (ABI 4) 2 int32 and 16 doubles, (ABI 6) 4 int32 and 21 doubles
    # (ABI 8) + basis_dt
    assert ctypes.sizeof(_lib.FgxConfig) == (20 * 4 + 18 * 8 + 4 * 4 + 8 * 8 + 17 * 4 + 4 + 8 * 8 + 2 * 4 + 16 * 8
                                             + 4 * 4 + 21 * 8 + 8)
    assert ctypes.sizeof(_lib.FgxInfo) == 11 * 8


def test_ctypes_layout_equals_c_compiler_layout(tmp_path):
    """Every field offset of the ctypes mirrors equals offsetof() of include/fgx.h under gcc."""
    import subprocess
    src = tmp_path / "layout.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "fgx.h"', 'int main(void) {']
    for cname, cls in (("fgx_config", _lib.FgxConfig), ("fgx_dims", _lib.FgxDims), ("fgx_info", _lib.FgxInfo)):
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines += ['return 0;', '}']
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-I", inc, str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                            check=True).stdout.splitlines())
    for cname, cls in (("fgx_config", _lib.FgxConfig), ("fgx_dims", _lib.FgxDims), ("fgx_info", _lib.FgxInfo)):
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_registry_ids():
    # registry.py:243 -> '{ns}_{mp}/{name}'
    for mp in fgx.KNOWN_MPS:
        for name in ("SimpleReacher-v0", "LongSimpleReacher-v0", "HoleReacher-v0", "ViaPointReacher-v0"):
            assert f"fancy_{mp}/{name}" in fgx.ALL_MOVEMENT_PRIMITIVE_ENVIRONMENTS[mp]
    assert len(fgx.ALL_MOVEMENT_PRIMITIVE_ENVIRONMENTS["all"]) == 12
    assert fgx.MOVEMENT_PRIMITIVE_ENVIRONMENTS_FOR_NS["fancy"]["ProDMP"]


def test_nested_update_type_key_replaces():
    base = {"controller_kwargs": {"controller_type": "motor", "p_gains": 1.0, "d_gains": 0.1}}
    out = fgx.nested_update(base, {"controller_kwargs": {"controller_type": "velocity"}})
    assert out["controller_kwargs"] == {"controller_type": "velocity"}
    out = fgx.nested_update({"a": {"b": 1, "c": 2}}, {"a": {"c": 3}})
    assert out == {"a": {"b": 1, "c": 3}}


@pytest.mark.parametrize("mp,name,n_params,ctrl,p,d", [
    ("ProMP", "SimpleReacher-v0", 10, _lib.CTRL_PD, 0.6, 0.075),
    ("ProMP", "LongSimpleReacher-v0", 25, _lib.CTRL_PD, 0.6, 0.075),
    ("DMP", "LongSimpleReacher-v0", 30, _lib.CTRL_PD, 0.6, 0.075),
    ("ProDMP", "SimpleReacher-v0", 12, _lib.CTRL_PD, 1.0, 0.1),
    ("ProMP", "HoleReacher-v0", 25, _lib.CTRL_VEL, None, None),
    ("DMP", "HoleReacher-v0", 30, _lib.CTRL_VEL, None, None),
    ("ProDMP", "HoleReacher-v0", 30, _lib.CTRL_PD, 1.0, 0.1),
    ("ProMP", "ViaPointReacher-v0", 25, _lib.CTRL_VEL, None, None),
    ("DMP", "ViaPointReacher-v0", 30, _lib.CTRL_VEL, None, None),
    ("ProDMP", "ViaPointReacher-v0", 30, _lib.CTRL_PD, 1.0, 0.1),
])
def test_resolved_configs(mp, name, n_params, ctrl, p, d):
    c, meta = fgx.resolve(f"fancy_{mp}/{name}")
    assert meta["n_params"] == n_params                         # test_black_box.py:168-193
    assert c.ctrl_kind == ctrl
    if p is not None:
        assert (c.p_gain, c.d_gain) == (p, d)
    assert c.T == 200 and c.duration == 2.0                     # make_env_helpers.py:110-113
    assert c.tau == (1.5 if mp == "ProDMP" else 2.0)
    if mp == "DMP":
        assert c.weights_scale == (500 if "Hole" in name else 50)
        assert c.alpha_phase == (2.5 if "Hole" in name else 2)
    if mp == "ProMP":
        assert c.zero_start == 1 and c.n_basis == 5
        assert c.weights_scale == (2 if "Hole" in name else 1)
    if "Hole" in name:
        assert c.act_high == float(np.float32(2 * np.pi))       # Box(float32) bound
        assert np.isnan(c.hole_width) and np.isnan(c.hole_x) and c.hole_depth == 1.0
        assert c.collision_penalty == 100
    if "ViaPoint" in name:   # envs/__init__.py:669-679, viapoint_reacher.py:15-16
        assert c.env_kind == _lib.ENV_VIA and c.random_start == 0 and c.collision_penalty == 1000
        assert np.isnan(c.via_x) and np.isnan(c.target_x)


def test_hole_reward_function_option():
    c, _ = fgx.resolve("fancy_ProMP/HoleReacher-v0", rew_fct="vel_acc")
    assert c.rew_fct == _lib.REW_VEL_ACC
    c, _ = fgx.resolve("fancy_ProMP/HoleReacher-v0", rew_fct="unbounded")
    assert c.rew_fct == _lib.REW_UNBOUNDED
    with pytest.raises(ValueError):   # hole_reacher.py:57-58
        fgx.resolve("fancy_ProMP/HoleReacher-v0", rew_fct="foo")


def test_replanning_schedule_compiles_to_period():
    c, _ = fgx.resolve("fancy_ProDMP/SimpleReacher-v0",
                       {"black_box_kwargs": {"replanning_schedule": lambda pos, vel, obs, action, t: t % 25 == 0}})
    assert c.replan_period == 25 and c.time_aware == 1 and c.return_context == 0
    with pytest.raises(NotImplementedError):
        fgx.resolve("fancy_ProDMP/SimpleReacher-v0",
                    {"black_box_kwargs": {"replanning_schedule":
                                          lambda pos, vel, obs, action, t: t in (3, 50, 60, 61, 90)}})
    with pytest.raises(NotImplementedError):
        fgx.resolve("fancy_ProDMP/SimpleReacher-v0",
                    {"black_box_kwargs": {"replanning_schedule": lambda pos, vel, obs, action, t: pos[0] > 0.5}})


def test_errors_mirror_reference():
    with pytest.raises(ValueError):   # unknown controller type (controller_factory.py:22-24)
        fgx.resolve("fancy_ProMP/SimpleReacher-v0", {"controller_kwargs": {"controller_type": "foo"}})
    with pytest.raises(ValueError):   # unknown trajectory generator (trajectory_generator_factory.py:19-21)
        fgx.resolve("fancy_ProMP/SimpleReacher-v0", {"trajectory_generator_kwargs": {"trajectory_generator_type": "x"}})
    with pytest.raises(ValueError):   # sub-trajectories + replanning (make_env_helpers.py:91-92)
        fgx.resolve("fancy_ProMP/SimpleReacher-v0", {"black_box_kwargs": {
            "learn_sub_trajectories": True, "replanning_schedule": lambda *a: False}})
    with pytest.raises(ValueError):
        fgx.resolve("fancy_XYZ/SimpleReacher-v0")


def test_context_space_sizes():
    # test_black_box.py:153-165: BB obs shape == context_mask.sum()
    for name, ctx in (("SimpleReacher-v0", 8), ("LongSimpleReacher-v0", 17), ("HoleReacher-v0", 18)):
        c, _ = fgx.resolve(f"fancy_ProMP/{name}")
        n = c.n_links
        full = 3 * n + 3 if "Simple" in name else 3 * n + 4
        assert ctx == full - 1
    # ViaPointReacher (random_start False): via - ee and goal - ee only
    from oracle import port
    assert int(port.Reacher("ViaPointReacher").context_mask().sum()) == 4


def test_schedule_clause_compilation():
    from fancy_gym_crowd_amd import registry
    c, _ = fgx.resolve("fancy_ProMP/LongSimpleReacher-v0", {"black_box_kwargs": {"replanning_schedule": fgx.REPLAN_CLOSE}})
    assert c.sched_n == 2 and c.replan_period == 0 and c.time_aware == 1 and c.return_context == 0
    assert list(c.sched_kind[:2]) == [_lib.SCHED_EVERY, _lib.SCHED_NORM_PERIOD]
    assert (c.sched_i0[1], c.sched_i1[1], c.sched_mul[1], c.sched_div[1]) == (0, 2, 10.0, 4.0)
    # plain lambdas firing at a few fixed steps compile to AT clauses
    cl = registry._compile_schedule(lambda pos, vel, obs, action, t: t in (30, 120), 200)
    assert [k[:2] for k in cl] == [(_lib.SCHED_AT, 30), (_lib.SCHED_AT, 120)]
    # the clause objects behave like the reference's lambdas
    obs = np.array([0.3, -0.8, 0.1])
    ref = lambda t: t % 10 == 0 or t % max(int(np.linalg.norm(obs[:2]) ** 2 * 10 / 4), 1) == 0  # noqa: E731
    for t in range(1, 201):
        assert fgx.REPLAN_CLOSE(None, None, obs, None, t) == ref(t)
    with pytest.raises(ValueError):
        fgx.ReplanAny(*[fgx.ReplanEvery(k) for k in (2, 3, 5, 7, 11)])


def test_per_joint_gains_resolution():
    c, _ = fgx.resolve("fancy_ProMP/LongSimpleReacher-v0",
                       {"controller_kwargs": {"p_gains": (1, 2, 3, 4, 5), "d_gains": 0.1}})
    assert c.n_gains == 5 and list(c.p_gains[:5]) == [1, 2, 3, 4, 5] and list(c.d_gains[:5]) == [0.1] * 5
    c, _ = fgx.resolve("fancy_ProMP/LongSimpleReacher-v0")
    assert c.n_gains == 0 and (c.p_gain, c.d_gain) == (0.6, 0.075)
    with pytest.raises(ValueError):   # (2,) gains do not broadcast against 5 joints
        fgx.resolve("fancy_ProMP/LongSimpleReacher-v0", {"controller_kwargs": {"p_gains": (1.0, 2.0)}})


class _StandInSpaces:
    """gymnasium.spaces stand-in: Space base class and Box(low, high, shape, dtype)."""

    class Space:
        pass

    class Box(Space):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape)
            self.low = np.broadcast_to(np.asarray(low), self.shape).astype(self.dtype)
            self.high = np.broadcast_to(np.asarray(high), self.shape).astype(self.dtype)


def test_register_gymnasium_with_stand_in():
    """envs/registry.py:245-254: every id reaches gym.make; without gymnasium nothing is registered.
    The registered envs' spaces are gymnasium spaces (the PassiveEnvChecker's requirement)."""
    import types
    from fancy_gym_crowd_amd import gym_compat
    calls = []
    stand_in = types.SimpleNamespace(Env=object, register=lambda **kw: calls.append(kw), spaces=_StandInSpaces)
    assert fgx.register_gymnasium(gym_module=stand_in) is True
    ids = [c["id"] for c in calls]
    assert "fancy_ProMP/LongSimpleReacher-v0" in ids and "fancy/HoleReacher-v0" in ids
    assert len(ids) == len(set(ids)) == 4 + 12
    assert all(callable(c["entry_point"]) for c in calls)
    for env_id in ids:   # what GymSingleEnv.__init__ installs, for every id (step-based ones included)
        obs, act = gym_compat.gym_spaces(env_id, stand_in)
        assert isinstance(obs, _StandInSpaces.Space) and isinstance(act, _StandInSpaces.Space)
        assert obs.dtype == np.float32 and act.dtype == np.float32
    obs, act = gym_compat.gym_spaces("fancy_ProMP/LongSimpleReacher-v0", stand_in)
    assert obs.shape == (17,) and act.shape == (25,)          # test_black_box.py:153-193 sizes
    obs, act = gym_compat.gym_spaces("fancy/HoleReacher-v0", stand_in)
    assert obs.shape == (19,) and act.shape == (5,)
    assert act.high[0] == np.float32(2 * np.pi) and np.isinf(obs.high[-1])
    try:
        import gymnasium  # noqa: F401
    except ImportError:
        assert fgx.register_gymnasium() is False


def test_gym_make_entry_point_forwards_kwargs(monkeypatch):
    """gym.make(id, mp_config_override=..., info_level=..., **env_kwargs) through the registered entry
    point: every kwarg reaches the engine once (bb_env_constructor, envs/registry.py:280-309) and the
    gymnasium spaces are the built env's own, converted (so an override that changes the parameter
    count changes the action space)."""
    import types
    from fancy_gym_crowd_amd import gym_compat
    from fancy_gym_crowd_amd.vector_env import Box, action_space, observation_space
    made = []

    def fake_make(env_id, num_envs=1, device="cuda", mp_config_override=None, info_level=None, autoreset=True,
                  **env_kwargs):
        cfg, meta = fgx.resolve(env_id, mp_config_override, **env_kwargs)
        made.append(dict(env_id=env_id, override=mp_config_override, info_level=info_level, env_kwargs=env_kwargs))
        n = meta.get("n_params", 0)
        return types.SimpleNamespace(n_params=n, single_observation_space=observation_space(cfg),
                                     single_action_space=Box(-np.inf, np.inf, (n,), np.float32)
                                     if meta["mp_type"] else action_space(cfg, n))

    monkeypatch.setattr(fgx, "make", fake_make)
    calls = []
    stand_in = types.SimpleNamespace(Env=object, register=lambda **kw: calls.append(kw), spaces=_StandInSpaces)
    assert fgx.register_gymnasium(gym_module=stand_in) is True
    entry = {c["id"]: c["entry_point"] for c in calls}
    over = {"basis_generator_kwargs": {"num_basis": 7}}
    env = entry["fancy_ProMP/LongSimpleReacher-v0"](mp_config_override=over, info_level=1, seed_offset=0)
    assert made[-1]["override"] == over and made[-1]["info_level"] == 1
    assert isinstance(env.action_space, _StandInSpaces.Space) and env.action_space.shape == (35,)
    assert isinstance(env.observation_space, _StandInSpaces.Space) and env.observation_space.shape == (17,)
    env = entry["fancy/HoleReacher-v0"](n_links=3)
    assert made[-1]["env_kwargs"] == {"n_links": 3} and env.action_space.shape == (3,)


def test_num_basis_outside_resolution():
    """basis_generator_kwargs num_basis_outside (mp_pytorch NormalizedRBF / ProDMP generators)."""
    c, _ = fgx.resolve("fancy_DMP/SimpleReacher-v0", {"basis_generator_kwargs": {"num_basis_outside": 1}})
    assert c.num_basis_outside == 1
    c, _ = fgx.resolve("fancy_ProDMP/HoleReacher-v0")
    assert c.num_basis_outside == 0
    with pytest.raises(ValueError):   # num_basis - 2 o - 1 must stay >= 1
        fgx.resolve("fancy_DMP/SimpleReacher-v0", {"basis_generator_kwargs": {"num_basis_outside": 2}})
    with pytest.raises(TypeError):    # the zero-padding generator has no such argument
        fgx.resolve("fancy_ProMP/SimpleReacher-v0", {"basis_generator_kwargs": {"num_basis_outside": 1}})


def test_oracle_centres_with_basis_outside():
    """centres = unbounded phase of linspace(-o d, tau + o d, n), d = tau / (n - 2o - 1)"""
    from oracle import mp
    for phase in ("linear", "exp"):
        s = mp.MPSpec("dmp", 2, 7, phase, 2.0, basis_outside=2, alpha_phase=3.0)
        c, _ = mp.centers64(s)
        d = 2.0 / (7 - 4 - 1)
        u = np.linspace(-2 * d, 2.0 + 2 * d, 7) / 2.0
        np.testing.assert_allclose(c, u if phase == "linear" else np.exp(-3.0 * u), rtol=1e-15)
        c0, _ = mp.centers64(mp.replace(s, basis_outside=0))
        np.testing.assert_array_equal(c0, mp.centers64(mp.MPSpec("dmp", 2, 7, phase, 2.0, alpha_phase=3.0))[0])


def test_table_exp_restatement_is_bit_exact(tmp_path):
    """csrc/fgx_exp.h (the basis tables' exp) compiled for the host equals oracle/mp.py:exp64 bit for
    bit: the same IEEE operations in the same order (no fma on either side)."""
    from oracle import mp
    src = tmp_path / "e.cpp"
    src.write_text('#include "fgx_exp.h"\n'
                   'extern "C" void run(const double* x, double* y, long n) {\n'
                   '  for (long i = 0; i < n; ++i) y[i] = fgx::fgx_exp(x[i]);\n}\n')
    so = tmp_path / "libe.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-D__host__=", "-D__device__=", "-shared", "-fPIC",
                    "-I", os.path.join(ROOT, "fancy_gym_crowd_amd", "csrc"), str(src), "-o", str(so)], check=True)
    lib = ctypes.CDLL(str(so))
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(-760, 720, 400000), rng.uniform(-40, 40, 400000), rng.uniform(-1, 1, 100000),
                        [0.0, -0.0, np.inf, -np.inf, np.nan, 709.78, 709.79, 709.8, -745.1, -745.2, -746.0, -708.4,
                         -700.0, -1e-300, 5e-324]])
    y = np.empty_like(x)
    lib.run(x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(x.size))
    ref = mp.exp64(x)
    np.testing.assert_array_equal(y.view(np.int64), ref.view(np.int64))
    fin = np.isfinite(ref) & (ref > 1e-300)
    with np.errstate(over="ignore"):
        assert (np.abs(ref[fin] - np.exp(x[fin])) <= np.spacing(np.exp(x[fin]))).all()   # within 1 ulp of numpy


def test_link_counts_resolve():
    """n_links 1..8 (base_reacher.py:17-39 takes any count; bb_env_constructor forwards env kwargs,
    envs/registry.py:280-281); outside the engine's range a ValueError."""
    for n in range(1, 9):
        c, meta = fgx.resolve("fancy_ProMP/SimpleReacher-v0", n_links=n)
        assert c.n_links == n and meta["n_params"] == 5 * n
        c, meta = fgx.resolve("fancy_ProDMP/ViaPointReacher-v0", n_links=n)
        assert meta["n_params"] == 6 * n
    with pytest.raises(ValueError):
        fgx.resolve("fancy_ProMP/SimpleReacher-v0", n_links=9)
    with pytest.raises(IndexError):   # the reference's wall check cannot index one squeezed link
        fgx.resolve("fancy_ProMP/HoleReacher-v0", n_links=1)
    c, _ = fgx.resolve("fancy_ProMP/HoleReacher-v0", n_links=1, allow_wall_collision=True)
    assert c.n_links == 1 and c.allow_wall_collision == 1


def test_prodmp_basis_dt_resolution():
    """basis_generator_kwargs dt (basis_generator_factory.py:8-23 forwards it to the ProDMP generator)."""
    c, _ = fgx.resolve("fancy_ProDMP/SimpleReacher-v0")
    assert c.basis_dt == c.dt == 0.01
    c, _ = fgx.resolve("fancy_ProDMP/HoleReacher-v0", {"basis_generator_kwargs": {"dt": 0.005}})
    assert c.basis_dt == 0.005
    with pytest.raises(TypeError):   # the RBF generators take no dt
        fgx.resolve("fancy_ProMP/SimpleReacher-v0", {"basis_generator_kwargs": {"dt": 0.005}})
    from oracle import mp
    # the oracle's row map: rint(t_i / bdt) on the fine grid (j(i) = 2 i for bdt = dt / 2)
    s = mp.MPSpec("prodmp", 2, 5, "exp", 1.5, alpha=10.0, basis_dt=0.005)
    j = mp.prodmp_delay_index(s, np.arange(50) * 0.01)
    np.testing.assert_array_equal(j, 2 * np.arange(50))
    t = mp.build_tables(s, 50)
    f = mp.prodmp_fine64(s, 99)
    np.testing.assert_array_equal(t["pb"], f["pb"][::2].astype(np.float32))


def test_validity_bound_semantics_follow_nep50():
    """TrajValidity compares the raw float32 action with a Python-float bound as numpy >= 2 does
    (NEP 50: in float32).  0.3 is not an f32 value: f32(0.3) > 0.3 in float64, == in float32."""
    assert int(np.__version__.split(".")[0]) >= 2
    val = fgx.TrajValidity(tau=(0.1, 0.3))
    pos = np.zeros((200, 2), np.float32)
    at = np.float32(0.3)
    assert float(at) > 0.3                                   # float64: above the bound
    assert val(np.array([at, 0.0], np.float32), pos, pos)[0]   # float32 (NEP 50): on it -> valid
    up = np.nextafter(at, np.float32(1.0))
    assert not val(np.array([up, 0.0], np.float32), pos, pos)[0]
    lo = np.float32(0.1)                                     # f32(0.1) > 0.1: the lower bound the same way
    assert val(np.array([lo, 0.0], np.float32), pos, pos)[0]
    assert not val(np.array([np.nextafter(lo, np.float32(0.0)), 0.0], np.float32), pos, pos)[0]


def test_episode_kernel_lists_agree():
    """fgx_episode_kernel's ids: include/fgx.h, INTEGRATION.md's entry-point table and the host's name
    map (_lib.EPISODE_KERNELS) list the same kernels under the same numbers."""
    import os
    import re
    from fancy_gym_crowd_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "fgx.h")).read()
    doc = hdr[hdr.index("/* The kernel fgx_step launches"):hdr.index("int fgx_episode_kernel(")]
    in_hdr = {int(k): v for k, v in re.findall(r"(\d+) = (k_episode\w*)", " ".join(doc.split()))}
    integ = open(os.path.join(root, "INTEGRATION.md")).read()
    row = [ln for ln in integ.splitlines() if ln.startswith("| `fgx_episode_kernel`")][0]
    in_doc = {}
    for k, v in re.findall(r"(\d+) (k_episode\w*|jp|ws|jl)", row):
        in_doc[int(k)] = {"jp": "k_episode_jp", "ws": "k_episode_ws", "jl": "k_episode_jl"}.get(v, v)
    assert in_hdr == _lib.EPISODE_KERNELS, (in_hdr, _lib.EPISODE_KERNELS)
    assert in_doc == _lib.EPISODE_KERNELS, (in_doc, _lib.EPISODE_KERNELS)


def test_design_lists_every_kernel():
    """Every __global__ kernel in csrc/ appears in DESIGN.md (its kernel table or a section of §4)."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "fancy_gym_crowd_amd", "csrc")
    names = set()
    for f in os.listdir(csrc):
        if f.endswith((".h", ".hip")):
            for line in open(os.path.join(csrc, f)):
                if "__global__" in line:
                    names |= set(re.findall(r"void (k_[a-z0-9_]+)", line))
    design = open(os.path.join(root, "DESIGN.md")).read()
    assert names and {"k_episode", "k_episode_hp", "k_traj_run"} <= names
    missing = sorted(n for n in names if not re.search(r"\b%s\b" % n, design))
    assert not missing, missing
