"""Decision margins of config 3's collision tests (CPU, oracle only; a design measurement).

Runs the batched oracle (oracle/batched.py) on fancy_ProDMP/HoleReacher-v0 with the bench's
synthetic parameters, records q of every counted sample, and reports how far each boolean the
consumers of k_episode_hp compute (hole_reacher.py:126-179, base_reacher.py:105-119) lies from its
threshold: the 24 ccw values of the self-collision test against 1e-12 (classic_control/utils.py:1-2)
and the wall test's submerged links.  This sizes an error-bounded approximate FK: a decision is
taken from approximate joint positions only when its margin exceeds the bound.

    python tools/hp_margins.py [N] [BB steps]
"""
import sys
import types

import numpy as np

sys.path.insert(0, ".")
from oracle import batched, mp  # noqa: E402
from fancy_gym_crowd_amd import registry  # noqa: E402


def spec_from_cfg(c):
    kind = {1: "promp", 2: "dmp", 3: "prodmp"}[c.mp_kind]
    return mp.MPSpec(kind=kind, dof=c.n_links, n_basis=c.n_basis, phase="linear" if c.phase_kind == 0 else "exp",
                     tau=c.tau, delay=c.delay, alpha_phase=c.alpha_phase, bandwidth=c.bandwidth,
                     zero_start=c.zero_start, zero_goal=c.zero_goal, basis_outside=c.num_basis_outside,
                     weights_scale=c.weights_scale, goal_scale=c.goal_scale, alpha=c.alpha, pc_length=c.pc_length,
                     dt=c.dt, duration=c.duration, basis_dt=c.basis_dt if c.mp_kind == 3 else 0.0)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n_bb = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    c, meta = registry.resolve("fancy_ProDMP/HoleReacher-v0")
    spec = spec_from_cfg(c)
    ctrl = ("pd", c.p_gain, c.d_gain) if c.ctrl_kind == 0 else {1: ("vel",), 2: ("pos",)}[c.ctrl_kind]
    ob = batched.BatchedBB("HoleReacher", N, ctrl, mp_spec=spec)
    ob._reset_idx(list(range(N)), list(range(N)))
    rec = []
    env = ob.env
    orig = env.step

    def step(a, act, a_is_f32):
        out = orig(a, act, a_is_f32)
        rec.append((env.q[act].copy(), env.hole_x[act].copy(), env.hole_w[act].copy()))
        return out
    env.step = step
    rng = np.random.default_rng(1234)
    n_params = spec.dof * spec.n_basis + (spec.dof if spec.kind != "promp" else 0)
    tls = []
    for _ in range(n_bb):
        p = rng.standard_normal((N, n_params), dtype=np.float32)
        _, _, te, tr, info = ob.step(p)
        tls.append(info["trajectory_length"])
    q = np.concatenate([r[0] for r in rec])
    hx = np.concatenate([r[1] for r in rec])
    hw = np.concatenate([r[2] for r in rec])
    hd = env.hole_d
    S, n = q.shape
    ang = np.cumsum(q, axis=1)
    J = np.zeros((S, n + 1, 2))
    J[:, 1:, 0] = np.cumsum(np.cos(ang), axis=1)
    J[:, 1:, 1] = np.cumsum(np.sin(ang), axis=1)
    # f32 FK (the approximate path): error vs the f64 joints
    a32 = np.cumsum(q.astype(np.float32), axis=1, dtype=np.float32)
    J32 = np.zeros((S, n + 1, 2), np.float32)
    J32[:, 1:, 0] = np.cumsum(np.cos(a32), axis=1, dtype=np.float32)
    J32[:, 1:, 1] = np.cumsum(np.sin(a32), axis=1, dtype=np.float32)
    e32 = np.abs(J32.astype(np.float64) - J).max(axis=(1, 2))

    def ccw(A, B, C):
        return (C[:, 1] - A[:, 1]) * (B[:, 0] - A[:, 0]) - (B[:, 1] - A[:, 1]) * (C[:, 0] - A[:, 0])
    m = np.full(S, np.inf)
    for i in range(n):
        for j in range(i + 2, n):
            A, B, C, D = J[:, i], J[:, i + 1], J[:, j], J[:, j + 1]
            for v in (ccw(A, C, D), ccw(B, C, D), ccw(A, B, C), ccw(A, B, D)):
                m = np.minimum(m, np.abs(v - 1e-12))
    sub = (J[:, :-1, 1] < 0) | (J[:, 1:, 1] < 0)
    print(f"samples {S}  envs {N}  BB steps {n_bb}  mean length {np.mean(np.concatenate(tls)):.1f}")
    print(f"max |q| {np.abs(q).max():.3f}  max sum|q| {np.abs(q).sum(1).max():.3f}")
    print(f"f32 FK error: max {e32.max():.2e}  p99 {np.quantile(e32, 0.99):.2e}")
    for M in (1e-3, 1e-4, 2e-5, 1e-5, 1e-6, 1e-8, 1e-11):
        print(f"ccw margin < {M:g}: {np.mean(m < M):.2e} of samples")
    print(f"samples with a submerged link: {np.mean(sub.any(1)):.3f}; links submerged per sample {sub.sum(1).mean():.3f}")
    ks = np.arange(S)
    print("ccw margin < 2e-5 by sample index within the record (first 8 records):",
          [float(np.mean(m[r0:r0 + len(rec[0][0])] < 2e-5)) for r0 in (0,)])
    # min |y| of the joints (the wall test's skip test margin)
    y = J[:, 1:, 1]
    for M in (1e-4, 1e-5, 1e-6):
        print(f"some joint with |y| < {M:g}: {np.mean((np.abs(y) < M).any(1)):.2e}")


if __name__ == "__main__":
    main()


def wave_stats(N=1024, n_bb=1):
    """Per (64-env wave, sample): how often at least one lane has a submerged link (the exact wall
    test) or a ccw value within M of its threshold."""
    c, meta = registry.resolve("fancy_ProDMP/HoleReacher-v0")
    spec = spec_from_cfg(c)
    ctrl = ("pd", c.p_gain, c.d_gain)
    ob = batched.BatchedBB("HoleReacher", N, ctrl, mp_spec=spec)
    ob._reset_idx(list(range(N)), list(range(N)))
    env = ob.env
    orig = env.step
    rec = []

    def step(a, act, a_is_f32):
        out = orig(a, act, a_is_f32)
        rec.append((env.q.copy(), act.copy()))
        return out
    env.step = step
    rng = np.random.default_rng(1234)
    p = rng.standard_normal((N, spec.dof * spec.n_basis + spec.dof), dtype=np.float32)
    ob.step(p)
    n = spec.dof
    W = N // 64
    sub_w, unc_w, both_w, act_w = 0, {1e-13: 0, 3e-13: 0, 1e-12: 0}, 0, 0
    for q, act in rec:
        ang = np.cumsum(q, axis=1)
        J = np.zeros((N, n + 1, 2))
        J[:, 1:, 0] = np.cumsum(np.cos(ang), axis=1)
        J[:, 1:, 1] = np.cumsum(np.sin(ang), axis=1)
        sub = (J[:, 1:, 1] < 1e-14).any(1) & act   # (joint 0 is the origin in both paths)
        m = np.full(N, np.inf)
        for i in range(n):
            for j in range(i + 2, n):
                A, B, C, D = J[:, i], J[:, i + 1], J[:, j], J[:, j + 1]
                for X, Y, Z in ((A, C, D), (B, C, D), (A, B, C), (A, B, D)):
                    v = (Z[:, 1] - X[:, 1]) * (Y[:, 0] - X[:, 0]) - (Y[:, 1] - X[:, 1]) * (Z[:, 0] - X[:, 0])
                    m = np.minimum(m, np.abs(v - 1e-12))
        aw = act.reshape(W, 64).any(1)
        act_w += aw.sum()
        sub_w += sub.reshape(W, 64).any(1).sum()
        for M in unc_w:
            unc_w[M] += ((m < M) & act).reshape(W, 64).any(1).sum()
    print(f"wave-samples {act_w}: some lane submerged {sub_w / act_w:.3f}; "
          + ", ".join(f"some ccw within {M:g}: {v / act_w:.2e}" for M, v in unc_w.items()))


if __name__ == "__main__" and len(sys.argv) > 3:
    wave_stats(int(sys.argv[1]))
