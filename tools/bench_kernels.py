"""Per-kernel timing of every BASELINE config on one MI355X (diagnostics for DESIGN.md).

Prints one JSON line per measurement: config, envs, kernel time (HIP events on the launch
stream), inner env-steps/s, algorithmic bytes and GB/s where meaningful.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import fancy_gym_crowd_amd as fgx  # noqa: E402

dev = torch.device("cuda", 0)


def timed(fn, reps=20, warm=3):
    """Seconds per call: the reps calls captured in one HIP graph and replayed between two
    events, so that host launch overhead (ctypes) does not show up as GPU time."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
    except Exception:   # not capturable: eager launches
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3   # seconds per call


def episode(env_id, N, over=None, label=None, reps=20, env_kwargs=None):
    env = fgx.make(env_id, num_envs=N, device=dev, info_level=0, mp_config_override=over, **(env_kwargs or {}))
    env.reset(seed=0)
    P = env.n_params
    params = torch.from_numpy(np.random.default_rng(1234).standard_normal((N, P), dtype=np.float32)).to(dev)
    obs = torch.empty((N, env.out_dim), device=dev)
    fobs = torch.empty_like(obs)
    ret = torch.empty(N, dtype=torch.float64, device=dev)
    te = torch.empty(N, dtype=torch.uint8, device=dev)
    tr = torch.empty(N, dtype=torch.uint8, device=dev)
    tl = torch.empty(N, dtype=torch.int32, device=dev)
    acc = env.new_inner_steps()
    t = timed(lambda: env.step_into(params, obs, ret, te, tr, tl, fobs, inner_steps=acc), reps=reps)
    acc.zero_()
    env.step_into(params, obs, ret, te, tr, tl, fobs, inner_steps=acc)
    torch.cuda.synchronize()
    inner = int(acc.sum().item())
    print(json.dumps(dict(kernel=env.episode_kernel(), config=label or env_id, envs=N, kernel_us=t * 1e6,
                          inner_steps_per_call=inner, inner_steps_per_s=inner / t,
                          mean_traj_len=inner / N)), flush=True)


def trajectory(env_id, N, force_valu=False, over=None, kernel=None):
    """fgx_trajectory at N envs: k_traj_mfma, or (a replanning schedule that never fires before T, or
    `over`) k_traj_run / k_traj_valu (FGX_TRAJ_VALU=1)"""
    if over is None and force_valu:
        over = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(200)}}
    env = fgx.make(env_id, num_envs=N, device=dev, info_level=0, mp_config_override=over or None)
    env.reset(seed=0)
    params = torch.randn((N, env.n_params), device=dev)
    T, n = env.T, env.dof
    pos = torch.empty((N, T, n), device=dev)
    vel = torch.empty_like(pos)
    lib, h = env._eng.lib, env._eng.h
    import ctypes
    args = [ctypes.c_void_p(x.data_ptr()) for x in (params, pos, vel)]
    t = timed(lambda: lib.fgx_trajectory(h, *args, env._eng.stream()))   # current (capture) stream
    bytes_ = N * (env.n_params * 4 + 2 * T * n * 4)
    K = 8
    flops = N * n * T * 2 * 2 * K          # two K=8 GEMMs (pos + next/vel) incl. zero padding
    if kernel is None:
        vk = bool(over) or env_id.startswith("fancy_DMP/")
        kernel = ("k_traj_valu" if os.environ.get("FGX_TRAJ_VALU") else "k_traj_run") if vk else "k_traj_mfma"
    print(json.dumps(dict(kernel=kernel, config=env_id, envs=N, over="replan" if over else None,
                          traj_ge=os.environ.get("FGX_TRAJ_GE"), traj_rc=os.environ.get("FGX_TRAJ_RC"),
                          traj_nt=os.environ.get("FGX_TRAJ_NT"), traj_sep=os.environ.get("FGX_TRAJ_SEP"),
                          traj_align=os.environ.get("FGX_TRAJ_ALIGN"), traj_threads=os.environ.get("FGX_TRAJ_THREADS"),
                          traj_pipe=os.environ.get("FGX_TRAJ_PIPE"),
                          kernel_us=t * 1e6, GBps=bytes_ / t / 1e9, hbm_frac=bytes_ / t / 8e12,
                          mfma_TFLOPs=flops / t / 1e12, mfma_frac_f32=flops / t / 157.3e12)), flush=True)


def traj_run_scan():
    """k_traj_run vs k_traj_valu on the plans k_traj_mfma does not take (65536 envs), then the
    workgroup-shape A/B (FGX_TRAJ_GE / FGX_TRAJ_RC)"""
    rp = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(200)}}
    cases = [("fancy_DMP/LongSimpleReacher-v0", {}), ("fancy_DMP/HoleReacher-v0", {}),
             ("fancy_ProMP/LongSimpleReacher-v0", rp), ("fancy_ProDMP/HoleReacher-v0", rp)]
    for valu in (False, True):
        if valu:
            os.environ["FGX_TRAJ_VALU"] = "1"
        for env_id, over in cases:
            trajectory(env_id, 65536, over=over)
        os.environ.pop("FGX_TRAJ_VALU", None)
    def run(env_id, over, **kv):
        for k in ("FGX_TRAJ_GE", "FGX_TRAJ_RC", "FGX_TRAJ_NT", "FGX_TRAJ_SEP", "FGX_TRAJ_ALIGN"):
            os.environ.pop(k, None)
        os.environ.update({"FGX_TRAJ_" + k: v for k, v in kv.items()})
        trajectory(env_id, 65536, over=over)
    for env_id, over in cases[:2]:   # DMP: chunk rows, 128-B aligned pieces or not, store kind
        for rc in ("32", "40", "64"):
            for al in ("1", "0"):
                for nt in ("0", "1"):
                    run(env_id, over, GE="12", RC=rc, ALIGN=al, NT=nt)
    for env_id, over in cases[2:]:   # ProMP / ProDMP: whole runs through one region, group size, store kind
        for ge in ("6", "8", "10", "12", "16"):
            for nt in ("0", "1"):
                run(env_id, over, GE=ge, RC="200", SEP="1", NT=nt)
        run(env_id, over, GE="16", RC="64", SEP="0", NT="1")
        run(env_id, over, GE="16", RC="64", SEP="0", NT="1", ALIGN="0")
    for env_id, over in cases:   # the defaults again, end of session
        run(env_id, over)
    for k in ("FGX_TRAJ_GE", "FGX_TRAJ_RC", "FGX_TRAJ_NT", "FGX_TRAJ_SEP", "FGX_TRAJ_ALIGN"):
        os.environ.pop(k, None)


def mfma_ab(env_id="fancy_ProMP/LongSimpleReacher-v0", N=65536, reps=20):
    """The MP contraction on the matrix cores vs fused on the VALU: (a) fgx_step = k_episode, the
    contraction as f32 fma chains inside the episode loop; (b) fgx_trajectory (k_traj_mfma: the
    basis GEMM on v_mfma_f32_32x32x2_f32, plans [N, T, dof] to HBM) + fgx_step_traj
    (k_episode<MP_GIVEN>: the same episode reading the plans).  Same returns bit for bit."""
    import ctypes
    res = {}
    for mode in ("fused_valu", "mfma_plans"):
        env = fgx.make(env_id, num_envs=N, device=dev, info_level=0)
        env.reset(seed=0)
        T, n = env.T, env.dof
        params = torch.from_numpy(np.random.default_rng(1234).standard_normal((N, env.n_params), dtype=np.float32)).to(dev)
        obs = torch.empty((N, env.out_dim), device=dev)
        ret = torch.empty(N, dtype=torch.float64, device=dev)
        te = torch.empty(N, dtype=torch.uint8, device=dev)
        tr = torch.empty(N, dtype=torch.uint8, device=dev)
        tl = torch.empty(N, dtype=torch.int32, device=dev)
        pos = torch.empty((N, T, n), device=dev)
        vel = torch.empty_like(pos)
        lib, h = env._eng.lib, env._eng.h
        p = [ctypes.c_void_p(x.data_ptr()) for x in (params, pos, vel, obs, ret, te, tr, tl)]
        if mode == "fused_valu":
            fn = lambda: lib.fgx_step(h, p[0], p[3], p[4], p[5], p[6], p[7], None, None, 1, env._eng.stream())  # noqa: E731
        else:
            def fn():
                lib.fgx_trajectory(h, p[0], p[1], p[2], env._eng.stream())
                lib.fgx_step_traj(h, p[1], p[2], p[3], p[4], p[5], p[6], p[7], None, None, 1, env._eng.stream())
        t = timed(fn, reps=reps)
        env.reset(seed=0)
        fn()
        torch.cuda.synchronize()
        res[mode] = ret.cpu().numpy().copy()
        print(json.dumps(dict(kernel=mode, config=env_id, envs=N, us_per_bb_step=t * 1e6,
                              inner_steps_per_s=float(tl.sum().item()) / t)), flush=True)
        del env
    print(json.dumps(dict(kernel="mfma_ab", returns_bit_equal=bool(np.array_equal(
        res["fused_valu"].view(np.int64), res["mfma_plans"].view(np.int64))))), flush=True)


def step_raw(env_id, N, final_obs=True):
    """k_step_raw through fgx_step_raw as StepVectorEnv.step calls it (with final_obs)."""
    env = fgx.make(env_id, num_envs=N, device=dev, info_level=0)
    env.reset(seed=0)
    n, od = env.dof, env.obs_dim
    a = (torch.rand((N, n), device=dev) * 2 - 1) * 10
    obs = torch.empty((N, od), device=dev)
    fobs = torch.empty((N, od), device=dev)
    rew = torch.empty(N, dtype=torch.float64, device=dev)
    te = torch.empty(N, dtype=torch.uint8, device=dev)
    tr = torch.empty(N, dtype=torch.uint8, device=dev)
    import ctypes
    lib, h = env._eng.lib, env._eng.h
    args = [ctypes.c_void_p(x.data_ptr()) for x in (a, obs, rew, te, tr)]
    fo = ctypes.c_void_p(fobs.data_ptr()) if final_obs else None
    t = timed(lambda: lib.fgx_step_raw(h, *args, fo, 1, env._eng.stream()), reps=50)
    # algorithmic bytes per env-step: action in; q, qd, goal, steps, flags (+ hole x / width /
    # depth for Hole / ViaPoint) read and written; obs (+ final obs), reward, two flags out
    # (the PCG64 state moves only on the 1-in-200 auto-reset)
    hole = 0 if env_id.startswith("fancy/Simple") or env_id.startswith("fancy/LongSimple") else 24
    state = 2 * n * 8 + 16 + 8 + hole
    b = N * (n * 4 + 2 * state + od * 4 * (2 if final_obs else 1) + 8 + 2)
    print(json.dumps(dict(kernel="k_step_raw", config=env_id, envs=N, final_obs=final_obs, kernel_us=t * 1e6,
                          steps_per_s=N / t, bytes_per_env_step=b // N, GBps=b / t / 1e9, hbm_frac=b / t / 8e12,
                          build=fgx._lib.load().fgx_build_id().decode())), flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["episode", "traj", "raw"]
    if "bw" in which:   # what plain torch kernels reach on this box (write / copy streams)
        for mb in (524, 2048):
            n = mb * (1 << 20) // 4
            a = torch.empty(n, device=dev)
            b = torch.empty(n, device=dev)
            t = timed(lambda: a.fill_(1.0), reps=20)
            print(json.dumps(dict(kernel="torch fill_", MB=mb, us=t * 1e6, write_GBps=n * 4 / t / 1e9)), flush=True)
            t = timed(lambda: b.copy_(a), reps=20)
            print(json.dumps(dict(kernel="torch copy_", MB=mb, us=t * 1e6, GBps=2 * n * 4 / t / 1e9)), flush=True)
            del a, b
    if "hole" in which:   # HoleReacher cost split: full, no wall check, no self-collision check
        episode("fancy_ProDMP/HoleReacher-v0", 65536, label="config3", reps=5)
        episode("fancy_ProDMP/HoleReacher-v0", 65536, label="config3 allow_wall_collision", reps=5,
                env_kwargs={"allow_wall_collision": True})
        episode("fancy_ProDMP/HoleReacher-v0", 65536, label="config3 allow_self_collision", reps=5,
                env_kwargs={"allow_self_collision": True})
    if "hp3" in which:   # config 3 with the default kernel (A/B of library builds)
        for n in (65536, 32768):
            episode("fancy_ProDMP/HoleReacher-v0", n, label="config3", reps=10)
    if "hp" in which:   # config 3: k_episode_hp (both workgroup shapes) against k_episode / k_episode_pair
        import os
        for n in (65536, 32768, 16384, 131072):
            for label, env_set in (("hp", {}), ("hp G=1", {"FGX_HP_G": "1"}), ("hp G=4", {"FGX_HP_G": "4"}),
                                   ("classic", {"FGX_EPISODE_KERNEL": "classic"}),
                                   ("pair", {"FGX_EPISODE_KERNEL": "pair"})):
                if label == "hp":
                    continue
                for k in ("FGX_HP_G", "FGX_EPISODE_KERNEL"):
                    os.environ.pop(k, None)
                os.environ.update(env_set)
                episode("fancy_ProDMP/HoleReacher-v0", n, label=f"config3 {label}", reps=5)
        for k in ("FGX_HP_G", "FGX_EPISODE_KERNEL"):
            os.environ.pop(k, None)
    if "jlh" in which:   # the 8-GPU shard sizes: k_episode_jl vs its helper form, alternated three times
        for _ in range(3):
            for n in (8192, 16384, 32768):
                for h in ("0", "1", "2"):
                    os.environ["FGX_EPISODE_KERNEL"] = "jl"
                    os.environ["FGX_JL_HELPER"] = h
                    episode("fancy_ProMP/LongSimpleReacher-v0", n, label=f"metric jl helper={h}")
        for k in ("FGX_EPISODE_KERNEL", "FGX_JL_HELPER"):
            os.environ.pop(k, None)
    if "hpinfo" in which:   # config 3's verbose-2 / info-level-1 public step(): k_episode_hp vs v2h vs logging
        import os
        for lvl in (2, 1):
            for label, env_set in (("hp", {"FGX_HP": "1"}), ("v2h", {"FGX_HP": "0"}), ("logging", {"FGX_V2": "0"})):
                for k in ("FGX_HP", "FGX_V2"):
                    os.environ.pop(k, None)
                os.environ.update(env_set)
                env = fgx.make("fancy_ProDMP/HoleReacher-v0", num_envs=65536, device=dev, info_level=lvl)
                env.reset(seed=0)
                params = torch.from_numpy(np.random.default_rng(1234).standard_normal((65536, env.n_params),
                                                                                      dtype=np.float32)).to(dev)
                for _ in range(2):
                    info = env.step(params)[4]
                torch.cuda.synchronize()
                ib = sum(v.untyped_storage().nbytes() for kk, v in info.items() if isinstance(v, torch.Tensor)
                         and v.dim() >= 2 and v.shape[1] == env.T)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    env.step(params)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 5 * 1e3
                print(json.dumps(dict(kernel=env.episode_kernel(), label=f"config3 step(info_level={lvl}) {label}",
                                      envs=65536, us_per_step=us, info_bytes=ib,
                                      info_GBps=ib / us / 1e3)), flush=True)
                del env, info
                torch.cuda.empty_cache()
        for k in ("FGX_HP", "FGX_V2"):
            os.environ.pop(k, None)
    log_ids = [e for w, e in (("log", None), ("logsimple", "fancy_ProMP/LongSimpleReacher-v0"),
                              ("loghole", "fancy_ProDMP/HoleReacher-v0")) if w in which]
    if log_ids:   # info_level=2 (verbose 2 per-step arrays) through the public step(); logsimple /
        # loghole: one env id only (PMC passes keep one kernel)
        ids = ("fancy_ProMP/LongSimpleReacher-v0", "fancy_ProDMP/HoleReacher-v0") if None in log_ids else log_ids
        for env_id in ids:
            env = fgx.make(env_id, num_envs=65536, device=dev, info_level=2)
            env.reset(seed=0)
            params = torch.randn((65536, env.n_params), device=dev)
            for _ in range(2):
                info = env.step(params)[4]
            torch.cuda.synchronize()
            # bytes the kernel writes per step into the per-step info arrays (their full [T, X, N] extents)
            ib = sum(v.untyped_storage().nbytes() for k, v in info.items() if isinstance(v, torch.Tensor)
                     and v.dim() >= 2 and v.shape[1] == env.T)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                env.step(params)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 5 * 1e3
            print(json.dumps(dict(kernel="step(info_level=2)", config=env_id, envs=65536, us_per_step=us,
                                  info_bytes=ib, info_GBps_step_wall=ib / us / 1e3)), flush=True)
            del env
            torch.cuda.empty_cache()
    if "levels" in which:   # the public step() at info_level 0 / 1 / 2 (what the logging kernel's stores cost)
        for lvl in (0, 1, 2):
            env = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=65536, device=dev, info_level=lvl)
            env.reset(seed=0)
            params = torch.randn((65536, env.n_params), device=dev)
            for _ in range(2):
                env.step(params)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                env.step(params)
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps(dict(kernel="step(info_level=%d)" % lvl, config="fancy_ProMP/LongSimpleReacher-v0",
                                  envs=65536, us_per_step=e0.elapsed_time(e1) / 5 * 1e3,
                                  episode_kernel=env.episode_kernel())), flush=True)
            del env
            torch.cuda.empty_cache()
    if "scan" in which:   # metric env over the envs-per-GPU axis (occupancy / tail effects)
        for n in (4096, 8192, 16384, 32768, 49152, 65536, 81920, 98304, 131072, 262144):
            episode("fancy_ProMP/LongSimpleReacher-v0", n, label="scan: ProMP LongSimpleReacher", reps=10)
        for n in (16384, 32768, 65536, 131072):
            episode("fancy_DMP/LongSimpleReacher-v0", n, label="scan: DMP LongSimpleReacher", reps=10)
    if "scanmp" in which:   # every MP kind and link count over the envs-per-GPU axis
        rp = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}}
        for env_id, over in (("fancy_ProDMP/LongSimpleReacher-v0", None), ("fancy_ProMP/SimpleReacher-v0", None),
                             ("fancy_DMP/SimpleReacher-v0", None), ("fancy_ProDMP/SimpleReacher-v0", None),
                             ("fancy_ProDMP/SimpleReacher-v0", rp)):
            for n in (4096, 16384, 32768, 49152, 65536, 131072):
                episode(env_id, n, over=over, label="scan: " + env_id + (" replan25" if over else ""), reps=10)
    if "scanlite" in which:
        for n in (16384, 32768, 49152, 65536, 131072):
            episode("fancy_ProMP/LongSimpleReacher-v0", n, label="scan: ProMP LongSimpleReacher", reps=10)
    if "metric" in which:
        episode("fancy_ProMP/LongSimpleReacher-v0", 65536, label="metric: ProMP LongSimpleReacher")
    if "shards" in which:   # the metric's strong-scaling shards (1/2/4/8 GPUs) and configs 2 / 4 / 5
        for n in (65536, 32768, 16384, 8192):
            episode("fancy_ProMP/LongSimpleReacher-v0", n, label=f"shard {n}: ProMP LongSimpleReacher")
        episode("fancy_ProMP/SimpleReacher-v0", 4096, label="config2: ProMP SimpleReacher")
        episode("fancy_DMP/LongSimpleReacher-v0", 32768, label="config4: DMP LongSimpleReacher (1/8 shard)")
        episode("fancy_ProDMP/SimpleReacher-v0", 8192,
                over={"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}},
                label="config5: ProDMP SimpleReacher replan 25 (1/8 shard)")
    if "big" in which:   # k_episode past one round (two resident waves per SIMD or not)
        for n in (65536, 131072, 262144):
            episode("fancy_ProMP/LongSimpleReacher-v0", n, label=f"big {n}: ProMP LongSimpleReacher", reps=10)
        for env_id in ("fancy_DMP/LongSimpleReacher-v0", "fancy_ProDMP/LongSimpleReacher-v0"):
            for n in (65536, 131072):
                episode(env_id, n, label=f"big {n}: {env_id}", reps=10)
    if "probe" in which:   # metric env at one full k_episode round and at the 2-GPU shard (PMC probes)
        episode("fancy_ProMP/LongSimpleReacher-v0", 65536, label="probe 65536", reps=10)
        episode("fancy_ProMP/LongSimpleReacher-v0", 32768, label="probe 32768", reps=10)
    if "episode" in which:
        episode("fancy_ProMP/LongSimpleReacher-v0", 65536, label="metric: ProMP LongSimpleReacher")
        episode("fancy_ProMP/LongSimpleReacher-v0", 262144, label="ProMP LongSimpleReacher x4 envs")
        episode("fancy_ProMP/SimpleReacher-v0", 4096, label="config2: ProMP SimpleReacher")
        episode("fancy_ProDMP/HoleReacher-v0", 65536, label="config3: ProDMP HoleReacher", reps=5)
        episode("fancy_DMP/LongSimpleReacher-v0", 32768, label="config4: DMP LongSimpleReacher (1/8 shard)")
        episode("fancy_ProDMP/SimpleReacher-v0", 8192,
                over={"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(25)}},
                label="config5: ProDMP SimpleReacher replan 25 (1/8 shard)")
    if "traj" in which:
        for force in (False, True):
            trajectory("fancy_ProMP/LongSimpleReacher-v0", 65536, force)
            trajectory("fancy_ProDMP/HoleReacher-v0", 65536, force)
    if "trajrun" in which:
        traj_run_scan()
    if "config3" in which:   # k_episode_hp at four (65536) and one (32768) groups per workgroup
        episode("fancy_ProDMP/HoleReacher-v0", 65536, label="config3: ProDMP HoleReacher", reps=10)
        episode("fancy_ProDMP/HoleReacher-v0", 32768, label="config3 half: ProDMP HoleReacher", reps=10)
    if "dmpshape" in which:   # k_traj_run DMP: fewer envs per group for longer pieces (whole runs at GE <= 3)
        for _ in range(2):
            for ge, rc in (("12", "40"), ("6", "80"), ("6", "100"), ("4", "200"), ("3", "200"), ("2", "200")):
                for k in ("FGX_TRAJ_GE", "FGX_TRAJ_RC", "FGX_TRAJ_NT"):
                    os.environ.pop(k, None)
                os.environ.update({"FGX_TRAJ_GE": ge, "FGX_TRAJ_RC": rc, "FGX_TRAJ_NT": "1"})
                trajectory("fancy_DMP/LongSimpleReacher-v0", 65536)
        for k in ("FGX_TRAJ_GE", "FGX_TRAJ_RC", "FGX_TRAJ_NT"):
            os.environ.pop(k, None)
        trajectory("fancy_DMP/LongSimpleReacher-v0", 65536)
    if "dmp" in which:   # DMP trajectory: the default shape against explicit ones
        for kv in ({}, {"FGX_TRAJ_GE": "6"}, {"FGX_TRAJ_GE": "8"}, {"FGX_TRAJ_GE": "10"},
                   {"FGX_TRAJ_RC": "32"}, {"FGX_TRAJ_GE": "8", "FGX_TRAJ_RC": "32"}, {}):
            for k in ("FGX_TRAJ_GE", "FGX_TRAJ_RC", "FGX_TRAJ_NT", "FGX_TRAJ_SEP", "FGX_TRAJ_ALIGN", "FGX_TRAJ_THREADS",
                      "FGX_TRAJ_PIPE"):
                os.environ.pop(k, None)
            os.environ.update(kv)
            trajectory("fancy_DMP/LongSimpleReacher-v0", 65536)
        for k in ("FGX_TRAJ_GE", "FGX_TRAJ_RC", "FGX_TRAJ_NT", "FGX_TRAJ_SEP", "FGX_TRAJ_ALIGN"):
            os.environ.pop(k, None)
    if "trajrun1" in which:   # one pass of each k_traj_run case (PMC runs): DMP x2, ProMP / ProDMP replanning
        rp = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(200)}}
        for env_id, over in (("fancy_DMP/LongSimpleReacher-v0", None), ("fancy_DMP/HoleReacher-v0", None),
                             ("fancy_ProMP/LongSimpleReacher-v0", rp), ("fancy_ProDMP/HoleReacher-v0", rp)):
            trajectory(env_id, 65536, over=over)
    if "raw" in which:   # config 1 (step-based SimpleReacher) and the other step ids at 1M envs
        for env_id in ("fancy/SimpleReacher-v0", "fancy/LongSimpleReacher-v0", "fancy/HoleReacher-v0",
                       "fancy/ViaPointReacher-v0"):
            step_raw(env_id, 1 << 20)
        step_raw("fancy/SimpleReacher-v0", 1 << 20, final_obs=False)
    if "mfmaab" in which:
        mfma_ab()
        mfma_ab("fancy_ProDMP/LongSimpleReacher-v0")
    if "raw1" in which:   # config 1 alone (PMC passes)
        step_raw("fancy/SimpleReacher-v0", 1 << 20)
