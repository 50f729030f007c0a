"""Per-section clocks of k_episode from the diagnostics build (-DFGX_STAMPS, _build.build_variant).

  FGX_LIB=tools/ab/libfgx_stamps.so [FGX_EPISODE_KERNEL=jl] python tools/stamps.py [env_id] [envs]

k_episode_jl: 0 entry, 1 after the prologue, 2 after the fast chunk pipeline, 3 after the generic
chunks, 4 after the gather barriers, 5 after the return and epilogue (wave 0 of each workgroup).

Lane 0 of every wave records s_memtime at: 0 kernel entry, 1 after the prologue (table staging,
state load, trajectory init), 2 after the fast blocks, 3 after the generic samples, 4 after the
return, 5 after the epilogue (outputs, auto-reset, state store).  Prints one JSON line with the
median / mean cycles of each section over the waves and the spread of wave start / end times.
"""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import fancy_gym_crowd_amd as fgx  # noqa: E402
from fancy_gym_crowd_amd import _lib  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "fancy_ProMP/LongSimpleReacher-v0"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
dev = torch.device("cuda", 0)
env = fgx.make(env_id, num_envs=N, device=dev, info_level=0)
env.reset(seed=0)
params = torch.from_numpy(np.random.default_rng(1234).standard_normal((N, env.n_params), dtype=np.float32)).to(dev)
obs = torch.empty((N, env.out_dim), device=dev)
fobs = torch.empty_like(obs)
ret = torch.empty(N, dtype=torch.float64, device=dev)
te = torch.empty(N, dtype=torch.uint8, device=dev)
tr = torch.empty(N, dtype=torch.uint8, device=dev)
tl = torch.empty(N, dtype=torch.int32, device=dev)
for _ in range(4):
    env.step_into(params, obs, ret, te, tr, tl, fobs)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
env.step_into(params, obs, ret, te, tr, tl, fobs)
e1.record()
torch.cuda.synchronize()
kern_us = e0.elapsed_time(e1) * 1e3
lib = _lib.load()
fn = lib.fgx_dbg_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
kern = env.episode_kernel()
JL = kern in ("k_episode_jl", "k_episode_jl_pc")
wpb = 8 if kern == "k_episode_jl_pc" else 4   # stamped waves per workgroup (joint waves [+ producers])
import os  # noqa: E402
if JL and os.environ.get("FGX_JL_HELPER", "0") in ("1", "2"):   # one stamped joint wave per workgroup
    W = (N + 64 // env._eng.cfg.n_links - 1) // (64 // env._eng.cfg.n_links)
elif JL:
    epb = 4 * (64 // env._eng.cfg.n_links)
    W = (N + epb - 1) // epb * wpb
else:
    W = (N + 63) // 64
buf = np.zeros(W * 16, dtype=np.uint64)
assert fn(buf.ctypes.data, W * 16) == 0
full = buf.reshape(W, 16).astype(np.int64)
if JL and wpb == 8:   # the joint (consumer) waves carry the sections; producers: points only
    prod = full[(np.arange(W) % 8) >= 4]
    full = full[(np.arange(W) % 8) < 4]
    W = full.shape[0]
st = full[:, :6]
rt = full[:, 6:8]   # s_memrealtime (100 MHz, one clock for the GPU)
extra = full[:, 8:]  # further shader-clock points (0 = not stamped by this kernel)
names = (["prologue", "fast_chunks", "slow_chunks", "gather", "return_epilogue"] if JL else
         ["prologue", "fast_blocks", "generic_samples", "return", "epilogue"])
sec = np.diff(st, axis=1)
out = {"env": env_id, "envs": N, "kernel": env.episode_kernel(), "waves": W,
       "cycles_median": {n: int(np.median(sec[:, i])) for i, n in enumerate(names)},
       "cycles_mean": {n: float(sec[:, i].mean()) for i, n in enumerate(names)},
       "wave_total_median": int(np.median(st[:, 5] - st[:, 0])),
       "kernel_us_events": kern_us}
tot = st[:, 5] - st[:, 0]
order = np.argsort(tot)
slow, fast = order[-max(1, W // 10):], order[:max(1, W // 10)]
out["slowest10pct_cycles_median"] = {n: int(np.median(sec[slow, i])) for i, n in enumerate(names)}
out["fastest10pct_cycles_median"] = {n: int(np.median(sec[fast, i])) for i, n in enumerate(names)}
out["slowest10pct_xcd_hist"] = np.bincount(((slow // 4) % 8), minlength=8).tolist()
out["total_cycles_pctl"] = [int(np.percentile(tot, p)) for p in (0, 10, 50, 90, 100)]
if JL:   # the epilogue runs in wave 0 of each workgroup
    out["cycles_median_wave0"] = {n: int(np.median(sec[::4, i])) for i, n in enumerate(names)}
# s_memtime counters are per XCD (workgroup b runs on XCD b % 8): start / end spread inside each
# XCD, and the clock rate implied by the XCD's first start to last end over the event time
xcd = (np.arange(W) // 4) % 8
per = []
for x in range(8):
    m = xcd == x
    if m.any():
        per.append(dict(xcd=x, start_spread=int(st[m, 0].max() - st[m, 0].min()),
                        end_spread=int(st[m, 5].max() - st[m, 5].min()),
                        span=int(st[m, 5].max() - st[m, 0].min())))
out["per_xcd"] = per
rstart, rend = rt[:, 0] - rt[:, 0].min(), rt[:, 1] - rt[:, 0].min()
out["realtime_us"] = {"start_max": float(rstart.max() / 100), "start_median": float(np.median(rstart) / 100),
                      "end_min": float(rend.min() / 100), "end_median": float(np.median(rend) / 100),
                      "end_max": float(rend.max() / 100),
                      "wave_duration_median": float(np.median(rend - rstart) / 100)}
out["shader_ticks_per_us"] = float(np.median((st[:, 5] - st[:, 0]) / np.maximum(1, rt[:, 1] - rt[:, 0]) * 100))
out["ticks_per_us_upper_bound"] = max(p["span"] for p in per) / kern_us
# extra points 8..15: median cycles since kernel entry, per wave slot of the workgroup (jl: 4 waves)
ws = 4 if JL else 1
pts = {}
for i in range(8):
    col = extra[:, i]
    if (col != 0).any():
        pts[str(8 + i)] = {f"wave{w}": int(np.median((col - st[:, 0])[w::ws][col[w::ws] != 0]))
                           for w in range(ws) if (col[w::ws] != 0).any()}
if pts:
    out["points_since_entry"] = pts
    out["point5_since_entry"] = {f"wave{w}": int(np.median((st[:, 5] - st[:, 0])[w::ws])) for w in range(ws)}
print(json.dumps(out), flush=True)
