"""Structural invariants of the MP path that the reference's own tests pin (CPU, oracle side),
plus exactness of the reciprocal division the kernels use.

Reference tests re-expressed: test/test_black_box.py:168-193 (action dims), :219-262 (flat
linear-phase tail after tau), test/test_replanning_sequencing.py:64-109 (T = round(tau/dt)
samples after t0).  Numeric parity of the MP values to mp_pytorch is unpinned (oracle/mp.py).
"""
import numpy as np
import pytest

from oracle import fp32, mp


@pytest.mark.parametrize("kind,dof,nb", [("promp", 2, 5), ("promp", 5, 5), ("dmp", 5, 5), ("prodmp", 2, 5),
                                         ("promp", 1, 1), ("dmp", 3, 2), ("prodmp", 5, 1)])
def test_param_count(kind, dof, nb):
    spec = mp.MPSpec(kind, dof, nb)
    assert spec.n_params == dof * nb + (dof if kind != "promp" else 0)


@pytest.mark.parametrize("tau", [0.25, 0.5, 0.75, 1.0])
def test_linear_phase_flat_after_tau(tau):
    spec = mp.MPSpec("promp", 1, 5, "linear", tau, zero_start=1, duration=2.0)
    tabs = mp.build_tables(spec, spec.T + 2)
    rng = np.random.default_rng(0)
    for _ in range(5):
        p = rng.standard_normal((1, spec.n_params), dtype=np.float32)
        pos, vel = mp.trajectory(spec, tabs, p, 0, np.zeros((1, 1)), np.zeros((1, 1)))
        pos, vel = pos[0, :, 0], vel[0, :, 0]
        k = int(np.round(tau / spec.dt))
        assert len(pos) == spec.T == 200                     # T = round(duration / dt)
        assert np.all(pos[k:] == pos[-1])                    # test_black_box.py:256
        assert np.all(vel[k:] == vel[-1])                    # test_black_box.py:257
        assert np.all(pos[:k - 1] != pos[-1])                # test_black_box.py:260


def test_prodmp_starts_at_initial_condition():
    spec = mp.MPSpec("prodmp", 2, 5, "exp", 1.5, alpha=10.0)
    tabs = mp.build_tables(spec, spec.T + 2)
    q0 = np.array([[0.3, -0.2]])
    qd0 = np.array([[1.0, 0.5]])
    p = np.random.default_rng(1).standard_normal((1, spec.n_params), dtype=np.float32)
    pos, vel = mp.trajectory(spec, tabs, p, 0, q0, qd0)
    # first sample is one dt after t0: q(dt) ~ q0 + dt * qd0
    np.testing.assert_allclose(pos[0, 0], q0[0] + 0.01 * qd0[0], atol=2e-3)
    np.testing.assert_allclose(vel[0, 0], qd0[0], atol=0.2)


def test_replan_shift_uses_absolute_rows():
    spec = mp.MPSpec("promp", 2, 5, "linear", 2.0, zero_start=1)
    tabs = mp.build_tables(spec, 200 + spec.T + 2)
    p = np.random.default_rng(2).standard_normal((1, spec.n_params), dtype=np.float32)
    a, _ = mp.trajectory(spec, tabs, p, 0, np.zeros((1, 2)), np.zeros((1, 2)))
    b, _ = mp.trajectory(spec, tabs, p, 25, np.zeros((1, 2)), np.zeros((1, 2)))
    np.testing.assert_array_equal(a[0, 25:], b[0, :175])   # plan at t0 = 25*dt continues the grid


def _div_rcp(x, d):
    r = (np.float32(1.0) / np.float32(d)).astype(np.float32)
    q = (x * r).astype(np.float32)
    e = fp32.fma32(-q, d, x)
    return fp32.fma32(e, r, q)


def test_division_by_reciprocal_is_exact():
    """Kernels divide by table constants with div_rcp (fgx_device.h); it must equal x / d."""
    divisors = set()
    for i in range(0, 600):
        t0, t1 = np.float32(i * 0.01), np.float32((i + 1) * 0.01)
        divisors.add(float(np.float32(t1 - t0)))
    divisors.update([float(np.float32(x)) for x in (1.5, 2.0, 1.0, 0.25, 0.5, 0.75, 3.0)])
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(200_000) * rng.choice([1e-4, 1e-2, 1.0, 1e2, 1e4], 200_000)).astype(np.float32)
    for d in divisors:
        d32 = np.float32(d)
        np.testing.assert_array_equal(_div_rcp(x, d32), (x / d32).astype(np.float32))


def test_f64_division_by_reciprocal_is_exact():
    """div_rcp64 (fgx_device.h) for the env dt: RN(x / 0.01) == fma(fma(-q, d, x), r, q)."""
    from fractions import Fraction as F

    def fma(a, b, c):
        return float(F(a) * F(b) + F(c))
    d = 0.01
    r = 1.0 / d
    rng = np.random.default_rng(7)
    xs = list(rng.standard_normal(4000) * rng.choice([1e-6, 1e-3, 1.0, 1e3, 1e6], 4000))
    xs += [i * 0.01 for i in range(1, 500)] + [float(i) for i in range(1, 500)]
    for x in xs:
        q = x * r
        assert fma(fma(-q, d, x), r, q) == x / d, x


# ---------------------------------------------------------------- learned tau / delay (oracle side)
def _learned(kind, phase, extra, lk, seed=0):
    spec = mp.MPSpec(kind, 1, 5, phase, 1.5 if kind == "prodmp" else 2.0,
                     zero_start=1 if kind == "promp" else 0, alpha=10.0)
    p = np.random.default_rng(seed).standard_normal((1, spec.n_params + len(extra))).astype(np.float32)
    p[0, :len(extra)] = extra
    pos, vel, L = mp.trajectory_learned(spec, p, 0, np.zeros((1, 1)), np.zeros((1, 1)), **lk)
    return pos[0, :L[0], 0], vel[0, :L[0], 0], int(L[0])


@pytest.mark.parametrize("kind", ["promp", "prodmp"])
@pytest.mark.parametrize("tau", [0.25, 0.5, 0.75, 1.0])
def test_learn_tau_structure(kind, tau):
    """test_black_box.py:219-255 on the restated MP: length 200, flat after tau (linear phase),
    active section differs from the end."""
    pos, vel, L = _learned(kind, "linear" if kind == "promp" else "exp", [tau], dict(learn_tau=True))
    k = int(np.round(tau / 0.01))
    assert L == 200
    if kind == "promp":
        assert np.all(pos[k:] == pos[-1]) and np.all(vel[k:] == vel[-1])
    assert np.all(pos[:k - 1] != pos[-1]) and np.all(vel[:k - 2] != vel[-1])


@pytest.mark.parametrize("kind", ["promp", "prodmp"])
@pytest.mark.parametrize("delay", [0, 0.25, 0.5, 0.75])
def test_learn_delay_structure(kind, delay):
    """test_black_box.py:258-307 (ProMP, linear phase; ProDMP, exp phase): constant during the
    delay, moving after it."""
    pos, vel, L = _learned(kind, "linear" if kind == "promp" else "exp", [delay], dict(learn_delay=True))
    k = int(np.round(delay / 0.01))
    assert L == 200
    assert np.all(pos[:max(1, k - 1)] == pos[0]) and np.all(vel[:max(1, k - 2)] == vel[0])
    assert np.all(pos[max(1, k):] != pos[0]) and np.all(vel[max(1, k)] != vel[0])


@pytest.mark.parametrize("kind", ["promp", "prodmp"])
@pytest.mark.parametrize("tau", [0.25, 0.5, 0.75, 1.0])
@pytest.mark.parametrize("delay", [0.25, 0.5, 0.75, 1.0])
def test_learn_tau_and_delay_structure(kind, tau, delay):
    """test_black_box.py:310-368 (ProMP linear / ProDMP exp phase)."""
    if 2.0 < delay + tau:
        return
    pos, vel, L = _learned(kind, "linear" if kind == "promp" else "exp", [tau, delay],
                           dict(learn_tau=True, learn_delay=True))
    kt, kd = int(np.round(tau / 0.01)), int(np.round(delay / 0.01))
    kj = kt + kd
    if kind == "promp":   # flat end only for the linear phase
        assert np.all(pos[kj:] == pos[-1]) and np.all(vel[kj:] == vel[-1])
    assert np.all(pos[:kd - 1] == pos[0]) and np.all(vel[:kd - 2] == vel[0])
    ap, av = pos[kd:kj - 1], vel[kd:kj - 2]
    assert np.all(ap != pos[-1]) and np.all(ap != pos[0])
    assert np.all(av != vel[-1]) and np.all(av != vel[0])


@pytest.mark.parametrize("kind", ["promp", "dmp"])
def test_sub_trajectory_length(kind):
    """test_replanning_sequencing.py:99-107: length == round(tau / dt), tau clipped to [2dt, D]."""
    for tau in (0.013, 0.02, 0.37, 1.234, 2.0, 7.0):
        _, _, L = _learned(kind, "exp", [tau], dict(sub_traj=True, learn_tau=True))
        t = float(np.clip(np.float32(tau), np.float32(0.02), np.float32(2.0)))
        assert L == int(np.round(t / 0.01))
