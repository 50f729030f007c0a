"""Episode-kernel scan: every eligible kernel (FGX_EPISODE_KERNEL = classic | jp | ws | jl) forced over
env counts per GPU for one workload; one JSON line per (kernel, envs) with the kernel time per BB step
(HIP events around a HIP-graph replay of `reps` BB steps, bench.py's timed region).

  python tools/kernel_scan.py [env_id] [kernels] [envs,...]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import fancy_gym_crowd_amd as fgx  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "fancy_ProMP/LongSimpleReacher-v0"
kernels = (sys.argv[2] if len(sys.argv) > 2 else "classic,jp,jl").split(",")
sizes = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "8192,16384,32768,65536").split(",")]
over = None
if "replan" in os.environ.get("SCAN_OVER", ""):
    over = {"black_box_kwargs": {"replanning_schedule": fgx.ReplanEvery(int(os.environ["SCAN_OVER"][6:]))}}
dev = torch.device("cuda", 0)
reps = 20

for N in sizes:
    for kname in kernels:
        os.environ["FGX_EPISODE_KERNEL"] = kname
        env = fgx.make(env_id, num_envs=N, device=dev, info_level=0, mp_config_override=over)
        got = env.episode_kernel()
        env.reset(seed=0)
        params = torch.from_numpy(np.random.default_rng(1234).standard_normal((N, env.n_params),
                                                                              dtype=np.float32)).to(dev)
        obs = torch.empty((N, env.out_dim), device=dev)
        fobs = torch.empty_like(obs)
        ret = torch.empty(N, dtype=torch.float64, device=dev)
        te = torch.empty(N, dtype=torch.uint8, device=dev)
        tr = torch.empty(N, dtype=torch.uint8, device=dev)
        tl = torch.empty(N, dtype=torch.int32, device=dev)
        acc = env.new_inner_steps()
        cnt = None if os.environ.get("SCAN_NO_COUNT") else acc   # the device inner-step counter (atomics)
        stream = torch.cuda.Stream(dev)
        with torch.cuda.stream(stream):
            for _ in range(3):
                env.step_into(params, obs, ret, te, tr, tl, fobs, inner_steps=cnt)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for _ in range(reps):
                    env.step_into(params, obs, ret, te, tr, tl, fobs, inner_steps=cnt)
            torch.cuda.synchronize()
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                acc.zero_()
                e0.record(stream)
                g.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) * 1e3 / reps
                best = t if best is None else min(best, t)
        inner = int(acc.sum().item()) / reps if cnt is not None else float(tl.sum().item())
        print(json.dumps(dict(env=env_id, envs=N, forced=kname, kernel=got, us_per_bb_step=round(best, 2),
                              counter=cnt is not None,
                              inner_steps_per_s=inner / (best * 1e-6), ret0=float(ret[0]))), flush=True)
        del g, env
        torch.cuda.synchronize()
