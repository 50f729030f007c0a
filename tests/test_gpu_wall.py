"""Adversarial HoleReacher wall-check geometry: the device's link_wall (fgx_device.h: end-point
shortcut for links that cross no hole edge, crossing estimates taken without evaluating points when
they are far from every sample index, verified estimates, binary searches) against the reference's
100-points-per-link test (hole_reacher.py:126-179, oracle/batched.py:_wall_collision).

Hole edges are placed within a few ulps of a link's sample points (crossings at, or a rounding away
from, an integer index: the cases the estimate cannot decide alone), links hang vertically /
horizontally (|cos| or |sin| of ~1e-17, exactly 0), end points sit on an edge; one zero-velocity raw
step per configuration, terminated flags (= wall collisions; self-collision off) bit-exact.
"""
import numpy as np
import pytest
import torch

import fancy_gym_crowd_amd as fgx
from oracle import batched
from tests.test_gpu_parity import DEV, np_

pytestmark = pytest.mark.gpu


def _fk(q):
    ang = np.cumsum(q, axis=1)
    c, s = np.cos(ang), np.sin(ang)
    jx = np.concatenate([np.zeros((len(q), 1)), 0.0 + np.cumsum(c, axis=1)], axis=1)
    jy = np.concatenate([np.zeros((len(q), 1)), 0.0 + np.cumsum(s, axis=1)], axis=1)
    return c, s, jx, jy


def _configs(N, rng):
    q = rng.uniform(-2.0, 2.0, (N, 5))
    q[:, 0] = rng.uniform(0.2, np.pi - 0.2, N)       # the arm starts upwards: few links submerged
    m = N // 8
    q[:m, 1] = -np.pi / 2 - q[:m, 0]                  # a link hanging exactly "vertical" (cos ~ 6e-17)
    q[m:2 * m, 1] = -q[m:2 * m, 0]                    # a horizontal link (cumulative angle exactly 0)
    c, s, jx, jy = _fk(q)
    # the edge goes onto a submerged link (one with an end below the ground) where there is one
    sub = np.minimum(jy[:, :-1], jy[:, 1:]) < 0.0
    k = np.where(sub.any(axis=1), np.argmax(sub * rng.uniform(0.5, 1.0, (N, 5)), axis=1), rng.integers(0, 5, N))
    j = rng.integers(0, 100, N)
    lin = np.where(j == 99, 1.0, j * (1.0 / 99.0))
    r = np.arange(N)
    px = c[r, k] * lin + jx[r, k]                     # the reference's sample point x of link k
    w = rng.choice([0.15, 0.3, 0.5], N)
    side = rng.integers(0, 3, N)                      # left edge on the point, right edge, or end point
    target = np.where(side == 2, jx[r, k], px)
    hx = np.where(side == 1, target - w / 2, target + w / 2)
    ulps = rng.integers(-3, 4, N)
    hx = hx + ulps * np.spacing(np.abs(hx))
    return q, hx, w


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_wall_check_adversarial_edges(seed):
    N = 16384
    rng = np.random.default_rng(seed)
    q, hx, w = _configs(N, rng)
    env = fgx.make("fancy/HoleReacher-v0", num_envs=N, device=DEV, allow_self_collision=True)
    env.reset(seed=seed)
    hole = np.stack([hx, w, np.ones(N)], axis=1)
    env.set_state(q=q, qd=np.zeros((N, 5)), hole=hole, steps=np.zeros(N, np.int32))
    ob = batched.BatchedReacher("HoleReacher", N, allow_self_collision=True)
    ob.reset(list(range(N)), list(range(N)))
    ob.q, ob.qd = q.copy(), np.zeros((N, 5))
    ob.hole_x, ob.hole_w = hx.copy(), w.copy()
    ob.steps = np.zeros(N, np.int64)
    ob._fk()
    a = np.zeros((N, 5), np.float32)
    _, _, te, _, _ = env.step(torch.from_numpy(a))
    _, _, te_r, _, _ = ob.step(a.astype(np.float64), np.ones(N, bool), True)
    te = np_(te).astype(bool)
    bad = np.nonzero(te != te_r)[0]
    assert bad.size == 0, f"{bad.size} flags differ, e.g. env {bad[:5]}: device {te[bad[:5]]}"
    assert 0.1 < te_r.mean() < 0.9   # both outcomes well represented
