"""k_traj_run DMP workgroup shapes (FGX_TRAJ_GE / _RC) give bit-identical trajectories: the default
shape against fewer envs per group with longer pieces, 65536 (and a partial 1001) envs."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fancy_gym_crowd_amd as fgx  # noqa: E402


def traj(env_id, N, ge=None, rc=None):
    for k in ("FGX_TRAJ_GE", "FGX_TRAJ_RC", "FGX_TRAJ_NT"):
        os.environ.pop(k, None)
    if ge:
        os.environ.update({"FGX_TRAJ_GE": ge, "FGX_TRAJ_RC": rc, "FGX_TRAJ_NT": "1"})
    env = fgx.make(env_id, num_envs=N, device="cuda", info_level=0)
    env.reset(seed=3)
    g = torch.Generator(device="cpu").manual_seed(5)
    params = torch.randn((N, env.n_params), generator=g).cuda()
    pos = torch.empty((N, env.T, env.dof), device="cuda")
    vel = torch.empty_like(pos)
    lib, h = env._eng.lib, env._eng.h
    rc_ = lib.fgx_trajectory(h, *[ctypes.c_void_p(x.data_ptr()) for x in (params, pos, vel)], env._eng.stream())
    torch.cuda.synchronize()
    assert rc_ == 0, rc_
    return pos.cpu(), vel.cpu()


for env_id in ("fancy_DMP/LongSimpleReacher-v0", "fancy_DMP/HoleReacher-v0"):
    for N in (65536, 1001):
        a = traj(env_id, N)
        for ge, rc in (("6", "80"), ("4", "200"), ("3", "200"), ("2", "200")):
            b = traj(env_id, N, ge, rc)
            ok = torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
            print(env_id, N, ge, rc, "identical" if ok else "DIFFERENT", flush=True)
            assert ok
