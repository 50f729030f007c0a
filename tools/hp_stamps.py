"""Per-role section clocks of k_episode_hp (diagnostics build -DFGX_STAMPS: fgx_hp.h FGX_HP_PUT).

  FGX_LIB=tools/ab/libfgx_stamps.so python tools/hp_stamps.py [envs] [G]

Row blockIdx * (1 + NC) G + w of the stamp buffer: 0 loop start, 1 loop end (shader clock), 8 cycles waiting
at the chunk barriers, 9 the producer's iteration count, 10 the role (0 producer, 1 / 2 consumers),
11 / 12 the producer's resolve / produce cycles (consumers: 11 the cycles in hp_fast_collision).
Prints one JSON line per role: median loop cycles, barrier cycles, their ratio.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import fancy_gym_crowd_amd as fgx  # noqa: E402
from fancy_gym_crowd_amd import _lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
G = int(os.environ.get("FGX_HP_G", "4" if N >= 65536 else "1"))
dev = torch.device("cuda", 0)
env = fgx.make("fancy_ProDMP/HoleReacher-v0", num_envs=N, device=dev, info_level=0)
assert env.episode_kernel() == "k_episode_hp"
env.reset(seed=0)
params = torch.from_numpy(np.random.default_rng(1234).standard_normal((N, env.n_params), dtype=np.float32)).to(dev)
obs = torch.empty((N, env.out_dim), device=dev)
fobs = torch.empty_like(obs)
ret = torch.empty(N, dtype=torch.float64, device=dev)
te = torch.empty(N, dtype=torch.uint8, device=dev)
tr = torch.empty(N, dtype=torch.uint8, device=dev)
tl = torch.empty(N, dtype=torch.int32, device=dev)
for _ in range(3):
    env.step_into(params, obs, ret, te, tr, tl, fobs)
torch.cuda.synchronize()
lib = _lib.load()
fn = lib.fgx_dbg_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
NW = 3   # waves per group: producer, C0, C1
W = (N + 64 * G - 1) // (64 * G) * NW * G
buf = np.zeros(W * 16, dtype=np.uint64)
assert fn(buf.ctypes.data, W * 16) == 0
st = buf.reshape(W, 16).astype(np.int64)
role = np.arange(W) % (NW * G) // G
loop = st[:, 1] - st[:, 0]
for r, name in enumerate(("producer", "consumer0", "consumer1")[:NW]):
    m = role == r
    print(json.dumps({"envs": N, "G": G, "role": name, "waves": int(m.sum()),
                      "loop_cycles_median": int(np.median(loop[m])), "barrier_cycles_median": int(np.median(st[m, 8])),
                      "barrier_share": float(np.median(st[m, 8] / np.maximum(loop[m], 1))),
                      "iterations_median": int(np.median(st[m, 9])) if r == 0 else None,
                      # producer: resolve / produce cycles; consumers: cycles in hp_fast_collision
                      "s11_median": int(np.median(st[m, 11])), "s12_median": int(np.median(st[m, 12]))}), flush=True)
