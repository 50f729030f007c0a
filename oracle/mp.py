"""Movement-primitive math (ProMP / DMP / ProDMP) — TEST INFRASTRUCTURE ONLY.

Restates the published algorithms of the third-party ``mp_pytorch<=0.1.3`` (pyproject.toml:30),
which is NOT vendored under /root/reference and not installed: numeric parity to mp_pytorch is
**parity unpinned** (SURVEY.md §8c).  What *is* pinned by the reference's own tests
(test/test_black_box.py:168-368, test/test_replanning_sequencing.py:64-364) — parameter
counts, T = round(duration/dt) samples with the t0 sample dropped, flat position after tau
for the linear phase — is re-checked by tests/test_mp_structure.py.

This module is the *specification* the HIP kernels implement (fgx_kernels.hip) and the CPU
check they are compared with.  Conventions (reference call sites in brackets):

time grid   absolute step index i >= 0, t_i = i*dt (f64); a plan that starts at env step s0
            uses rows i = s0+1 .. s0+T  [black_box_wrapper.py:120-128: init_time = s0*dt,
            set_duration(duration, dt) -> T = round(duration/dt) samples after t0]
phase       linear: x = clip((t-delay)/tau, 0, 1); exp: x = exp(-alpha_x * max(t-delay, 0)/tau)
            [factory/phase_generator_factory.py:11-14]
basis       normalized RBF, centres = unbounded phase of linspace(delay - o d, delay + tau + o d, n),
            d = tau / (n - 2o - 1), o = num_basis_outside (default 0), bandwidth
            h_j = bw / (c_{j+1}-c_j)^2 (last repeated), phi_j = exp(-h_j (x-c_j)^2 / 2) / sum;
            zero padding builds n_b + z_s + z_g RBFs and keeps columns z_s..z_s+n_b-1
            [factory/basis_generator_factory.py:10-17]
tables      every table value is computed in f64 and rounded once to f32 (mp_pytorch computes
            in torch f32 on the CPU; f64-then-round is the deliberate, documented choice), with
            exp64 (= csrc/fgx_exp.h) as the exp, so the device tables equal these bit for bit
ProMP       pos_k[d] = fma-chain_j(Phi[i][j], w[d][j]) with Phi = f32(weights_scale*phi);
            vel_k = f32(f32(pos_{k+1}-pos_k) / dt32_i), dt32_i = f32(f32(t_{i+1}) - f32(t_i)),
            vel_{T-1} = vel_{T-2}.  params = w, dof-major (w[d][j] = params[d*n_b + j]).
DMP         tau^2 y'' = alpha(beta(g-y) - tau y') + f, beta = alpha/4, f = x*phi.w' (w' =
            f32(w*weights_scale)), semi-implicit Euler in scaled time in f32:
            acc = alpha*(beta*(g-y) - z) + f_k; z += sdt*acc; y += sdt*z; vel = z/tau;
            y_0 = f32(q0), z_0 = f32(f32(qd0)*tau).  params = [w (dof-major), g (dof)].
ProDMP      q(s) = c1 y1(s) + c2 y2(s) + Phi_p(s).[w; g], y1 = exp(-alpha s/2), y2 = s y1,
            Phi_p/Phi_v from the cumulative-trapezoid variation-of-parameters integrals on the
            grid s_j = j*bdt/tau up to s = 6 (pre_compute_length_factor; bdt = the basis
            generator's dt, default the env dt), looked up at the rounded grid index; (c1, c2) solved from q(s0) = q0, q'(s0) = tau*qd0 (2x2
            Wronskian).  params = per-dof blocks [w_d (n_b), g_d] (num_basis_g = n_b + 1).
"""
from dataclasses import dataclass, field, replace

import numpy as np

from .fp32 import fma32, fma_chain32

f32 = np.float32


@dataclass
class MPSpec:
    kind: str = "promp"            # promp | dmp | prodmp
    dof: int = 2
    n_basis: int = 5
    phase: str = "linear"          # linear | exp
    tau: float = 2.0
    delay: float = 0.0
    alpha_phase: float = 3.0
    bandwidth: float = 3.0
    zero_start: int = 0
    zero_goal: int = 0
    basis_outside: int = 0         # num_basis_outside (centres beyond the phase's [0, 1])
    weights_scale: float = 1.0
    goal_scale: float = 1.0
    alpha: float = 25.0            # DMP / ProDMP spring constant
    pc_length: float = 6.0         # ProDMP pre_compute_length_factor
    dt: float = 0.01
    duration: float = 2.0
    extra: dict = field(default_factory=dict)
    T_override: int = 0            # learn_sub_trajectories: T = round(tau / dt) per env
    basis_dt: float = 0.0          # ProDMP basis generator dt (its precompute grid); 0 = the env dt

    @property
    def bdt(self):
        return self.basis_dt or self.dt

    @property
    def T(self):
        return self.T_override or int(round(self.duration / self.dt))

    @property
    def n_params(self):
        if self.kind == "promp":
            return self.dof * self.n_basis
        return self.dof * (self.n_basis + 1)


# ----------------------------------------------------------------------------- exp of the tables
_L2E = 1.4426950408889634
_LN2_HI = 6.93147180369123816490e-01
_LN2_LO = 1.90821492927058770002e-10
_EXP_C = [1.6059043836821613e-10, 2.08767569878681e-09, 2.505210838544172e-08, 2.755731922398589e-07,
          2.7557319223985893e-06, 2.48015873015873e-05, 0.0001984126984126984, 0.001388888888888889,
          0.008333333333333333, 0.041666666666666664, 0.16666666666666666, 0.5]


def exp64(x):
    """The tables' exp (csrc/fgx_exp.h:fgx_exp), operation for operation: Cody-Waite reduction with
    fdlibm's two-part ln 2, degree-13 Taylor polynomial in Horner form with separate IEEE mul / add
    (numpy ufuncs never fuse), exact scaling by 2^k (subnormal results: exact ldexp, then one
    multiplication by 2^-600).  Deterministic on both sides, so device tables == oracle tables bit
    for bit; a few f64 ulp from the true exp (the tables then round to f32).  mp_pytorch itself
    evaluates torch f32 exp: parity to it stays unpinned either way."""
    x = np.asarray(x, np.float64)
    with np.errstate(over="ignore", invalid="ignore"):
        xs = np.where(np.isfinite(x), np.clip(x, -746.0, 709.8), 0.0)
        k = np.rint(xs * _L2E)
        r = (xs - k * _LN2_HI) - k * _LN2_LO
        p = np.full_like(r, _EXP_C[0])
        for c in _EXP_C[1:]:
            p = p * r + c
        p = p * r + 1.0
        p = p * r + 1.0
        ki = k.astype(np.int32)
        small = ki < -1000
        y = np.where(small, np.ldexp(p, np.where(small, ki + 600, 0)) * 2.0 ** -600, np.ldexp(p, np.where(small, 0, ki)))
    y = np.where(x > 709.8, np.inf, y)
    y = np.where(x < -746.0, 0.0, y)
    return np.where(np.isnan(x), x, y)


# ----------------------------------------------------------------------------- phase / basis
def phase64(spec, t):
    lin = np.maximum((np.asarray(t, np.float64) - spec.delay) / spec.tau, 0.0)
    if spec.phase == "linear":
        return np.minimum(lin, 1.0)
    return exp64(-spec.alpha_phase * lin)


def centers64(spec):
    n = spec.n_basis + spec.zero_start + spec.zero_goal
    o = spec.basis_outside                # centres at the unbounded phase of
    # linspace(delay - o d, delay + tau + o d, n), d = tau / (n - 2o - 1): u_j = (j - o) / (n - 2o - 1)
    u = (np.arange(n, dtype=np.float64) - o) / (n - 2 * o - 1) if n > 1 else np.zeros(1)
    c = u if spec.phase == "linear" else exp64(-spec.alpha_phase * u)
    if n > 1:
        d = np.empty(n)
        d[:-1] = c[1:] - c[:-1]
        d[-1] = d[-2]
    else:
        d = np.ones(1)
    h = spec.bandwidth / (d ** 2)
    return c, h


def _seqsum_last(a):
    """numpy's reduction order over the last axis for n < 8 is a plain left-to-right loop."""
    n = a.shape[-1]
    if n >= 8:
        return np.sum(a, axis=-1)
    s = a[..., 0] + 0.0
    for j in range(1, n):
        s = s + a[..., j]
    return s


def rbf64(spec, x):
    """Normalized RBF values in f64, zero-padding columns removed: [..., n_basis]."""
    c, h = centers64(spec)
    d = np.asarray(x, np.float64)[..., None] - c
    e = exp64((-h) * (d * d) / 2)
    phi = e / _seqsum_last(e)[..., None]
    return phi[..., spec.zero_start:spec.zero_start + spec.n_basis]


# ----------------------------------------------------------------------------- tables
def prodmp_fine64(spec, n_rows):
    """ProDMP precompute on the fine grid s_j = j*bdt/tau (f64), rows 0..n_rows-1 (bdt: the basis
    generator's dt, basis_generator_factory.py:8-23 passes it through; default the env dt)."""
    h = spec.bdt / spec.tau
    J = int(round(spec.pc_length / h)) + 1
    J = max(J, n_rows)
    s = np.arange(J, dtype=np.float64) * h
    a = spec.alpha
    x = exp64(-spec.alpha_phase * s)                       # exp phase at t = s*tau (+delay)
    phi = rbf64(spec, x)                                   # [J, nb]
    e = exp64(a * s / 2)
    dp1 = (s * e * x)[:, None] * phi
    dp2 = (e * x)[:, None] * phi
    p1 = np.zeros_like(dp1)
    p2 = np.zeros_like(dp2)
    for j in range(1, J):                                  # cumulative trapezoid
        p1[j] = p1[j - 1] + h * (dp1[j - 1] + dp1[j]) / 2
        p2[j] = p2[j - 1] + h * (dp2[j - 1] + dp2[j]) / 2
    y1 = exp64(-a * s / 2)
    y2 = s * y1
    dy1 = -a / 2 * y1
    dy2 = -a / 2 * y2 + y1
    q1 = (a * s / 2 - 1) * e + 1
    q2 = a / 2 * (e - 1)
    pb = np.concatenate([p2 * y2[:, None] - p1 * y1[:, None], (q2 * y2 - q1 * y1)[:, None]], 1)
    vb = np.concatenate([p2 * dy2[:, None] - p1 * dy1[:, None], (q2 * dy2 - q1 * dy1)[:, None]], 1)
    return dict(pb=pb[:n_rows], vb=vb[:n_rows], y1=y1[:n_rows], y2=y2[:n_rows],
                dy1=dy1[:n_rows], dy2=dy2[:n_rows])


def build_tables(spec, n_rows):
    """Shared per-config tables by absolute step index i in [0, n_rows) (all f32)."""
    i = np.arange(n_rows + 1, dtype=np.float64)
    t = i * spec.dt
    if spec.kind == "promp":
        phi = rbf64(spec, phase64(spec, t[:n_rows]))
        t32 = t.astype(f32)
        return dict(phi=(spec.weights_scale * phi).astype(f32),
                    dt32=(t32[1:] - t32[:-1]).astype(f32))
    if spec.kind == "dmp":
        x = phase64(spec, t[:n_rows])
        psi = (x[:, None] * rbf64(spec, x)).astype(f32)
        s32 = np.maximum((t - spec.delay) / spec.tau, 0.0).astype(f32)
        return dict(psi=psi, sdt=(s32[1:] - s32[:-1]).astype(f32))
    if spec.kind == "prodmp":
        if spec.delay or spec.bdt != spec.dt:   # row i = fine-grid row j(i)
            j = prodmp_delay_index(spec, t[:n_rows])
            fine = prodmp_fine64(spec, int(j.max()) + 1)
            fine = {k: v[j] for k, v in fine.items()}
        else:                                   # j(i) = i
            fine = prodmp_fine64(spec, n_rows)
        return {k: v.astype(f32) for k, v in fine.items()}
    raise ValueError(spec.kind)


def prodmp_delay_index(spec, t):
    """ProDMP with a delay or its own basis dt: fine-grid index of time t on the left-bounded
    linear phase, rint(max((t - delay) / tau, 0) / (bdt / tau)) — mp_pytorch's ProDMP basis looks
    its precomputed rows up at the rounded scaled-time index of the (delay-shifted, clamped at 0)
    linear phase.  Parity unpinned like the rest of this module; what the reference's tests pin
    for a ProDMP delay (constant position and velocity before the delay, moving after,
    test_black_box.py:267-307) is re-checked in tests/test_mp_structure.py."""
    u = np.maximum((np.asarray(t, np.float64) - spec.delay) / spec.tau, 0.0)
    return np.rint(u / (spec.bdt / spec.tau)).astype(np.int64)


# ----------------------------------------------------------------------------- trajectories
def split_params(spec, params):
    p = np.asarray(params, f32).reshape(-1, spec.n_params)
    nb, D = spec.n_basis, spec.dof
    if spec.kind == "promp":
        return p.reshape(-1, D, nb), None
    if spec.kind == "dmp":
        return p[:, :D * nb].reshape(-1, D, nb), p[:, D * nb:]
    blk = p.reshape(-1, D, nb + 1)
    return blk[:, :, :nb], blk[:, :, nb]


def trajectory(spec, tables, params, s0, q0, qd0):
    """Desired (pos, vel) [N, T, dof] f32 for N envs whose plans start at env steps s0[N].

    q0/qd0 are the env's current (f64) joint state used as initial conditions.
    """
    N = np.asarray(params).reshape(-1, spec.n_params).shape[0]
    s0 = np.broadcast_to(np.asarray(s0, np.int64), (N,))
    T, D = spec.T, spec.dof
    rows = s0[:, None] + 1 + np.arange(T)[None, :]                  # [N, T]
    w, g = split_params(spec, params)
    tau32 = f32(spec.tau)
    if spec.kind == "promp":
        phi = tables["phi"][rows]                                     # [N, T, nb]
        pos = fma_chain32(phi[:, :, None, :], w[:, None, :, :])       # [N, T, D]
        dt32 = tables["dt32"][rows[:, :-1]][:, :, None]
        vel = np.empty_like(pos)
        vel[:, :-1] = (pos[:, 1:] - pos[:, :-1]) / dt32
        vel[:, -1] = vel[:, -2]
        return pos, vel
    if spec.kind == "dmp":
        ws = (w * f32(spec.weights_scale)).astype(f32)
        gs = (g * f32(spec.goal_scale)).astype(f32)
        f = fma_chain32(tables["psi"][rows][:, :, None, :], ws[:, None, :, :])    # [N, T, D]
        sdt = tables["sdt"][rows]                                     # [N, T]
        alpha, beta = f32(spec.alpha), f32(spec.alpha / 4)
        y = np.asarray(q0, np.float64).reshape(N, D).astype(f32)
        z = (np.asarray(qd0, np.float64).reshape(N, D).astype(f32) * tau32).astype(f32)
        pos = np.empty((N, T, D), f32)
        vel = np.empty((N, T, D), f32)
        for k in range(T):
            pos[:, k], vel[:, k] = y, z / tau32
            if k == T - 1:
                break
            acc = alpha * (beta * (gs - y) - z) + f[:, k]
            z = z + sdt[:, k, None] * acc
            y = y + sdt[:, k, None] * z
        return pos, vel
    if spec.kind == "prodmp":
        ws = (w * f32(spec.weights_scale)).astype(f32)
        gs = (g * f32(spec.goal_scale)).astype(f32)
        wg = np.concatenate([ws, gs[:, :, None]], axis=2)             # [N, D, nb+1]
        tb = tables
        b = s0
        y1b, y2b, dy1b, dy2b = tb["y1"][b], tb["y2"][b], tb["dy1"][b], tb["dy2"][b]
        det = (y1b * dy2b - y2b * dy1b).astype(f32)
        P = fma_chain32(tb["pb"][b][:, None, :], wg)                  # [N, D]
        V = fma_chain32(tb["vb"][b][:, None, :], wg)
        q0f = np.asarray(q0, np.float64).reshape(N, D).astype(f32)
        v0f = np.asarray(qd0, np.float64).reshape(N, D).astype(f32)
        A = q0f - P
        B = (v0f * tau32).astype(f32) - V
        c1 = ((dy2b[:, None] * A - y2b[:, None] * B) / det[:, None]).astype(f32)
        c2 = ((y1b[:, None] * B - dy1b[:, None] * A) / det[:, None]).astype(f32)
        coef = np.concatenate([wg, c1[:, :, None], c2[:, :, None]], axis=2)    # [N, D, nb+3]
        Hp = np.concatenate([tb["pb"][rows], tb["y1"][rows][..., None], tb["y2"][rows][..., None]], 2)
        Hv = np.concatenate([tb["vb"][rows], tb["dy1"][rows][..., None], tb["dy2"][rows][..., None]], 2)
        pos = fma_chain32(Hp[:, :, None, :], coef[:, None, :, :])
        vel = (fma_chain32(Hv[:, :, None, :], coef[:, None, :, :]) / tau32).astype(f32)
        return pos, vel
    raise ValueError(spec.kind)


# ----------------------------------------------------------------------------- learned tau / delay
def learned_params(spec, params, learn_tau, learn_delay, tau_bound, delay_bound):
    """Split params [tau?, delay?, w...] after BlackBoxWrapper.get_trajectory's clip to the
    float32 action-space bounds (black_box_wrapper.py:115-119; bounds from
    make_env_helpers.py:118-126 via the phase generator's tau_bound / delay_bound)."""
    p = np.asarray(params, f32)
    p = p.reshape(p.shape[0], -1)
    lo = np.full(p.shape[1], -np.inf, f32)
    hi = np.full(p.shape[1], np.inf, f32)
    i = 0
    if learn_tau:
        lo[0], hi[0] = f32(tau_bound[0]), f32(tau_bound[1])
        i = 1
    if learn_delay:
        lo[i], hi[i] = f32(delay_bound[0]), f32(delay_bound[1])
        i += 1
    p = np.clip(p, lo, hi)
    N = p.shape[0]
    tau = p[:, 0].astype(np.float64) if learn_tau else np.full(N, spec.tau)
    delay = p[:, 1 if learn_tau else 0].astype(np.float64) if learn_delay else np.full(N, spec.delay)
    return tau, delay, p[:, i:]


def trajectory_learned(spec, params, s0, q0, qd0, learn_tau=False, learn_delay=False, sub_traj=False,
                       tau_bound=None, delay_bound=None):
    """Per-env phase (learned tau / delay): per-env tables built exactly as build_tables with the
    env's (tau, delay), then `trajectory`.  With learn_sub_trajectories the plan has
    T_e = round(tau_e / dt) samples (duration=None, black_box_wrapper.py:107-113; the length is
    pinned by test_replanning_sequencing.py:99-107).  Returns pos, vel [N, T, dof] (NaN beyond
    T_e) and T_e [N]."""
    tau_bound = tau_bound or (2 * spec.dt, spec.duration)
    delay_bound = delay_bound or (0.0, spec.duration - 2 * spec.dt)
    tau, delay, w = learned_params(spec, params, learn_tau, learn_delay, tau_bound, delay_bound)
    N, D = w.shape[0], spec.dof
    s0 = np.broadcast_to(np.asarray(s0, np.int64), (N,))
    q0 = np.asarray(q0, np.float64).reshape(N, D)
    qd0 = np.asarray(qd0, np.float64).reshape(N, D)
    Tmax = spec.T
    pos = np.full((N, Tmax, D), np.nan, f32)
    vel = np.full((N, Tmax, D), np.nan, f32)
    lens = np.zeros(N, np.int64)
    for i in range(N):
        sp = replace(spec, tau=float(tau[i]), delay=float(delay[i]))
        if sub_traj:
            sp = replace(sp, T_override=int(np.round(tau[i] / spec.dt)))
        Ti = sp.T
        tabs = build_tables(sp, int(s0[i]) + Ti + 2)
        p_, v_ = trajectory(sp, tabs, w[i:i + 1], s0[i:i + 1], q0[i:i + 1], qd0[i:i + 1])
        pos[i, :Ti], vel[i, :Ti] = p_[0], v_[0]
        lens[i] = Ti
    return pos, vel, lens
