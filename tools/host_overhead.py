"""Diagnose host-side overhead of one BB step (GPU box)."""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
import fancy_gym_crowd_amd as fgx  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = torch.device("cuda", 0)
env = fgx.make("fancy_ProMP/LongSimpleReacher-v0", num_envs=N, device=dev, info_level=0)
env.reset(seed=0)
params = torch.randn((N, env.n_params), device=dev)
obs = torch.empty((N, env.out_dim), device=dev)
fobs = torch.empty_like(obs)
ret = torch.empty(N, dtype=torch.float64, device=dev)
te = torch.empty(N, dtype=torch.uint8, device=dev)
tr = torch.empty(N, dtype=torch.uint8, device=dev)
tl = torch.empty(N, dtype=torch.int32, device=dev)
for _ in range(5):
    env.step_into(params, obs, ret, te, tr, tl, fobs)
torch.cuda.synchronize()


def timeit(label, fn, K=50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{label:40s} host {1e6 * (t1 - t0) / K:9.1f} us/call   wall {1e6 * (t2 - t0) / K:9.1f} us/call", flush=True)


lib = env._eng.lib
h = env._eng.h
s = env._eng.stream()
args = [ctypes.c_void_p(t.data_ptr()) for t in (params, obs, ret, te, tr, tl, fobs)]
timeit("step_into", lambda: env.step_into(params, obs, ret, te, tr, tl, fobs))
timeit("raw ctypes fgx_step", lambda: lib.fgx_step(h, *args, None, 1, s))
timeit("current_stream()", lambda: env._eng.stream())
timeit("tl.sum()", lambda: tl.sum())
ev = torch.cuda.Event(enable_timing=True)
timeit("event.record()", lambda: ev.record())
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    lib.fgx_step(h, *args, None, 1, s)
e1.record()
torch.cuda.synchronize()
print("gpu time per step (events over 20):", e0.elapsed_time(e1) / 20 * 1e3, "us")
